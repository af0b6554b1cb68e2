"""TEST INFRASTRUCTURE: seed corpora for the libFuzzer targets (tests/fuzz).

Starting from an empty corpus libFuzzer needs minutes to grow inputs long
enough to reach a call (a k=10 encode of 4 KiB columns needs ~40 KB of
input). These seeds put one input per operation and shape class in place:
lengths 0, 1, 31, 32, 4096 + 5 and 16384 (the harnesses' maximum), k and rows
at 1, a mid value and 16, every misalignment class.

  python tests/fuzz/seeds.py diff DIR    ec_diff_fuzz.c's input layout
  python tests/fuzz/seeds.py ec DIR      the reference's ec_fuzz_test.c layout
  python tests/fuzz/seeds.py raid DIR    the reference's raid_fuzz_test.c layout
"""
import os
import random
import sys

LENS = (0, 1, 31, 32, 4096 + 5, 16384)


def _payload(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def diff_seeds(rng):
    """ec_diff_fuzz.c: op, len (2 B, big-endian), k-1, rows-1, offset, sel, payload."""
    nops = 11
    for op in range(nops):
        for ln in LENS:
            for k, rows in ((1, 1), (10, 4), (16, 16)):
                off, sel = rng.randrange(16), rng.randrange(256)
                head = bytes([op, ln >> 8, ln & 0xFF, k - 1, rows - 1, off, sel])
                # payload shorter than the call needs: ec_diff_fuzz cycles it
                yield head + _payload(rng, min(4096, 64 + k * rows + ln))


def ec_seeds(rng):
    """ec_fuzz_test.c:322-348: selector, then the helper's own header."""
    for sel in range(8):
        for ln in LENS:
            for k, rows in ((1, 1), (10, 4), (16, 16)):
                if sel < 2:  # init tables: k, rows, coefficients
                    body = bytes([k - 1, rows - 1]) + _payload(rng, k * rows)
                elif sel < 4:  # encode: len, k, rows, coefficients, k * len data
                    body = bytes([ln >> 8, ln & 0xFF, k - 1, rows - 1]) + _payload(rng, k * rows + k * ln)
                elif sel < 6:  # dot product: len, vlen, 32 * vlen tables, vlen * len data
                    body = bytes([ln >> 8, ln & 0xFF, k - 1]) + _payload(rng, 32 * k + k * ln)
                else:  # mad: len, vec, vec_i, 32 * vec tables, src, dest
                    body = bytes([ln >> 8, ln & 0xFF, k - 1, rng.randrange(256)]) + _payload(rng, 32 * k + 2 * ln)
                yield bytes([sel]) + body


def raid_seeds(rng):
    """raid_fuzz_test.c:61-117: selector, vects byte (3 + b % 14 vectors), len
    (2 B), then vects * len bytes of vectors."""
    for sel in range(8):
        for ln in (32, 64, 1000, 4096, 16384):
            for b in (0, 1, 7, 13):
                vects = 3 + b % 14
                yield bytes([sel, b, ln >> 8, ln & 0xFF]) + _payload(rng, vects * ln)


def write(kind, out):
    rng = random.Random(1234)
    os.makedirs(out, exist_ok=True)
    gen = {"diff": diff_seeds, "ec": ec_seeds, "raid": raid_seeds}[kind]
    n = 0
    for n, seed in enumerate(gen(rng), 1):
        with open(os.path.join(out, f"seed{n:04d}"), "wb") as f:
            f.write(seed)
    return n


if __name__ == "__main__":
    print(write(sys.argv[1], sys.argv[2]))
