#!/usr/bin/env python3
"""Steady-state per-launch duration of one kernel from a rocprofv3
`--kernel-trace --output-format csv` run (the *_kernel_trace.csv it writes).

rocprofv3's own `--stats` summary averages EVERY dispatch of a kernel,
including bench.py's warm-up launches (the first launch of a process runs
~20 % slow). bench.py's roofline divides by the average of the K timed
launches only (HIP events around them), so the comparable profile figure is
the average over the last K dispatches of the kernel: this tool drops the
first `--skip` dispatches (bench.py's --warmup) and keeps `--keep` (its
--steps; default: all remaining).

usage: tools/kernel_stats.py TRACE_DIR_OR_CSV KERNEL_SUBSTRING [--skip W] [--keep K]
                             [--bytes B] [--out FILE] [--trace-out FILE] [--command CMD]
Prints (and writes with --out) a CSV: kernel, dispatches, skipped, kept,
avg/median/min/max ns of the kept dispatches and, given --bytes (algorithmic
bytes per launch), the achieved GB/s and the fraction of 8 TB/s.
"""
import argparse
import csv
import glob
import os
import statistics
import sys


def dispatches(path, needle):
    files = [path] if path.endswith(".csv") else sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"),
                                                                  recursive=True))
    rows = []
    for f in files:
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if needle in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--keep", type=int, default=0)
    ap.add_argument("--bytes", type=float, default=0.0)
    ap.add_argument("--peak", type=float, default=8000.0, help="GB/s")
    ap.add_argument("--out")
    ap.add_argument("--trace-out", help="also write every dispatch of the kernel (the rows averaged, and the "
                                        "warm-up ones marked) as a compact CSV: the evidence behind --out")
    ap.add_argument("--command", default="")
    ap.add_argument("--config", default="", help='e.g. "workload=encode k=10 p=4 len=1048576 stripes=1024" '
                                                 "(bench.py matches its own configuration against it)")
    a = ap.parse_args(argv)
    rows = dispatches(a.trace, a.kernel)
    if len(rows) <= a.skip:
        print(f"kernel_stats: {len(rows)} dispatches of {a.kernel!r}, nothing after skipping {a.skip}",
              file=sys.stderr)
        return 1
    names = sorted({r["Kernel_Name"] for r in rows})
    kept = rows[a.skip:]
    if a.keep:
        kept = kept[:a.keep]
    ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kept]
    avg = statistics.fmean(ns)
    out = [["# config: " + a.config], ["# command", a.command], ["# trace", a.trace],
           ["kernel", " | ".join(names)], ["dispatches", len(rows)], ["skipped_warmup", a.skip],
           ["kept", len(kept)], ["avg_ns", round(avg, 1)], ["median_ns", statistics.median(ns)],
           ["min_ns", min(ns)], ["max_ns", max(ns)],
           ["first_dispatch_ns", int(rows[0]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])]]
    if a.bytes:
        gbs = a.bytes / avg
        out += [["bytes_per_launch", int(a.bytes)], ["achieved_gb_s", round(gbs, 1)],
                ["frac_of_peak", round(gbs / a.peak, 4)], ["peak_gb_s", a.peak]]
    w = csv.writer(sys.stdout)
    w.writerows(out)
    if a.out:
        with open(a.out, "w", newline="") as fh:
            csv.writer(fh).writerows(out)
    if a.trace_out:
        kept_ids = {id(r) for r in kept}
        with open(a.trace_out, "w", newline="") as fh:
            t = csv.writer(fh)
            t.writerow([f"# per-dispatch rocprofv3 kernel trace of {a.kernel!r} behind "
                        f"{os.path.basename(a.out) if a.out else 'the summary'}; config: {a.config}"])
            t.writerow(["dispatch", "start_ns", "end_ns", "duration_ns", "averaged", "kernel"])
            for r in rows:
                s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                t.writerow([r.get("Dispatch_Id", ""), s0, e0, e0 - s0, int(id(r) in kept_ids),
                            r["Kernel_Name"].split("(")[0].replace("void ", "")])
    return 0


if __name__ == "__main__":
    sys.exit(main())
