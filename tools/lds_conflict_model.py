"""Expected LDS cycles of one wave-wide ds_read_b64 lookup into a table of
random-indexed 8-byte entries (MI355X_MICROARCH.md §LDS: ds_read_b64 serves
lanes 0-31 and 32-63 as two groups, one LDS cycle per group when conflict-free;
bank of byte address a = (a/4) mod 64, so an 8-byte entry e occupies bank pair
(base/8 + e) mod 32; each extra distinct entry on a busy bank pair in a group
costs one more cycle). Monte Carlo over uniformly random lane indices.

Schemes: a table of 2^b entries in one copy (the fused CRC64 kernel's byte
tables: b = 8; the field tables: b = 5), and the "partial replication" the
round-5 verdict proposed — R copies, lane subset c of each group reading copy
c laid out in its own 32/R bank pairs (or at a bank-skewed base over all 32).
Usage: python3 tools/lds_conflict_model.py [trials]
"""
import random
import sys


def cycles(bits, copies, layout, trials, rng):
    n = 1 << bits
    total = 0
    for _ in range(trials):
        worst_groups = 0
        for _g in range(2):  # two 32-lane groups per instruction
            slots = {}
            for lane in range(32):
                c = lane * copies // 32
                e = rng.randrange(n)
                if copies == 1:
                    slot = e % 32
                elif layout == "disjoint":  # copy c confined to bank pairs [c*32/R, (c+1)*32/R)
                    w = 32 // copies
                    slot = c * w + e % w
                else:  # "skewed": copy c starts 32/R bank pairs later
                    slot = (e + c * (32 // copies)) % 32
                slots.setdefault(slot, set()).add((c, e))
            worst_groups += max(len(s) for s in slots.values())
        total += worst_groups
    return total / trials  # LDS cycles per wave-instruction (conflict-free: 2)


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    rng = random.Random(1)
    print("scheme,entries,copies,layout,lds_cycles_per_wave_instr,vs_conflict_free,conflict_share")
    for bits, copies, layout in [(5, 1, "-"), (6, 1, "-"), (7, 1, "-"), (8, 1, "-"),
                                 (8, 2, "disjoint"), (8, 4, "disjoint"), (8, 2, "skewed"), (8, 4, "skewed")]:
        c = cycles(bits, copies, layout, trials, rng)
        print(f"{bits}-bit,{1 << bits},{copies},{layout},{c:.3f},{c / 2:.3f},{1 - 2 / c:.3f}")


if __name__ == "__main__":
    main()
