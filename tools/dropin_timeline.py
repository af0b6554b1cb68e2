#!/usr/bin/env python3
"""Per-call timeline of the synchronous drop-in call from a rocprofv3
--hip-trace --kernel-trace run of tools/dropin_bench (one thread): for every
timed call, the host API intervals and the kernel's device interval on one
clock, reduced to medians.

  python3 tools/dropin_timeline.py DIR KERNEL_SUBSTR [--skip N]

Fields (medians over calls, microseconds):
  call_us                one launch start to the next (the per-call period)
  launch_api_us          hipLaunchKernel duration
  launch_to_start_us     hipLaunchKernel start -> kernel start on the device
  kernel_us              kernel duration
  end_to_next_launch_us  kernel end -> next launch start (completion
                         detection, the return to the caller, the caller's
                         loop; negative when the host sees the mailbox before
                         the kernel's end timestamp)
  other_api_us_per_call  every other HIP API call inside one call period, by
                         name (median total per call)
"""
import csv
import statistics
import sys


def main(argv):
    d, sub = argv[1], argv[2]
    skip = int(argv[argv.index("--skip") + 1]) if "--skip" in argv else 10
    api = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
    ker = [r for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")) if sub in r["Kernel_Name"]]
    launches = [r for r in api if r["Function"] == "hipLaunchKernel"]
    by_corr = {r["Correlation_Id"]: r for r in launches}
    rows = []
    for k in ker:
        l = by_corr.get(k["Correlation_Id"])
        if l:
            rows.append((int(l["Start_Timestamp"]), int(l["End_Timestamp"]),
                         int(k["Start_Timestamp"]), int(k["End_Timestamp"])))
    rows.sort()
    rows = rows[skip:]
    med = lambda xs: statistics.median(xs) / 1e3  # noqa: E731
    out = {
        "calls": len(rows) - 1,
        "call_us": med([b[0] - a[0] for a, b in zip(rows, rows[1:])]),
        "launch_api_us": med([r[1] - r[0] for r in rows]),
        "launch_to_start_us": med([r[2] - r[0] for r in rows]),
        "kernel_us": med([r[3] - r[2] for r in rows]),
        "end_to_next_launch_us": med([b[0] - a[3] for a, b in zip(rows, rows[1:])]),
    }
    # other API calls inside one call period, by name (median total per call)
    per = {}
    for i, (a, b) in enumerate(zip(rows, rows[1:])):
        for r in api:
            s = int(r["Start_Timestamp"])
            if a[0] <= s < b[0] and r["Function"] != "hipLaunchKernel":
                per.setdefault(r["Function"], [0] * (len(rows) - 1))[i] += int(r["End_Timestamp"]) - s
    out["other_api_us_per_call"] = {f: round(med(v), 3) for f, v in per.items()}
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv)
