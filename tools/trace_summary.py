#!/usr/bin/env python3
"""Summarise a rocprofv3 --memory-copy-trace --kernel-trace run of
tools/host_call_trace.py: records are split into calls at gaps > 2 ms
between consecutive records (the script sleeps 20 ms between
configurations, and its calls are back to back), and each call prints its
span, the busy time of H2D copies, D2H copies and kernels, how long H2D and
D2H copies ran at the same time, and the copy sizes.

usage: tools/trace_summary.py DIR   (the -d directory of the rocprofv3 run)
"""
import csv
import glob
import os
import sys


def load(pattern):
    rows = []
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            rows += list(csv.DictReader(f))
    return rows


def busy(iv):
    """Total length of the union of intervals."""
    tot, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def overlap(x, y):
    """Length of union(x) intersected with union(y)."""
    return busy(x) + busy(y) - busy(x + y)


def main(d):
    copies = load(os.path.join(d, "**", "*memory_copy_trace.csv"))
    kernels = load(os.path.join(d, "**", "*kernel_trace.csv"))
    ev = []
    for r in copies:
        direction = r.get("Direction", "")
        kind = "h2d" if "HOST_TO_DEVICE" in direction else "d2h" if "DEVICE_TO_HOST" in direction else "other"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, int(r.get("Bytes", 0) or 0)))
    for r in kernels:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", 0))
    ev.sort()
    calls, cur = [], []
    for e in ev:
        if cur and e[0] - max(x[1] for x in cur) > 2_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
    if cur:
        calls.append(cur)
    for i, c in enumerate(calls):
        t0, t1 = min(x[0] for x in c), max(x[1] for x in c)
        h = [(a, b) for a, b, k, _ in c if k == "h2d"]
        dd = [(a, b) for a, b, k, _ in c if k == "d2h"]
        kk = [(a, b) for a, b, k, _ in c if k == "kernel"]
        sizes = sorted({n for _, _, k, n in c if k in ("h2d", "d2h")})
        print(f"group {i}: {len(c)} records span {(t1 - t0) / 1e3:.1f} us; h2d {len(h)} busy "
              f"{busy(h) / 1e3:.1f} us; d2h {len(dd)} busy {busy(dd) / 1e3:.1f} us; kernels {len(kk)} "
              f"busy {busy(kk) / 1e3:.1f} us; h2d||d2h {overlap(h, dd) / 1e3:.1f} us; sizes {sizes[:6]}")


if __name__ == "__main__":
    main(sys.argv[1])
