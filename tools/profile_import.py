#!/usr/bin/env python3
"""Turn one workload's rocprofv3 runs of a gpurun session into the committed
profile files bench.py looks its roofline cross-checks up in (DESIGN.md §6,
"Profiles and bench lines of one session").

usage: tools/profile_import.py NAME WORKLOAD OUTDIR ROUND [BENCH_ARGS...]

OUTDIR holds, from the same session:
  trbench_NAME.json   the bench line printed under `rocprofv3 --kernel-trace`
  tr_NAME/            that run's kernel trace
  fetch_NAME/ write_NAME/   the two --pmc passes (FETCH_SIZE, WRITE_SIZE)
Writes OUTDIR/{ROUND}_{NAME}_kernel_steady.csv (the timed dispatches'
average, tools/kernel_stats.py), {ROUND}_{NAME}_kernel_trace.csv (every
dispatch) and {ROUND}_pmc_{NAME}.csv (tools/pmc_csv.py), and copies them
into profiles/{ROUND}/ of this tree, so a bench line run after it in the same
session cites them. The kernel is the one the bench line names
(roofline.kernel), matched against rocprof's full names."""
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import kernel_stats  # noqa: E402


def norm(name):
    name = name.replace("(anonymous namespace)::", "").replace(" ", "")
    name = name[4:] if name.startswith("void") else name
    return name.split("(")[0]


def main():
    name, workload, out, rnd = sys.argv[1:5]
    bargs = sys.argv[5:]
    line = [l for l in open(os.path.join(out, f"trbench_{name}.json")) if l.startswith("{")][-1]
    d = json.loads(line)
    rf, cfg = d["roofline"], d["config"]
    label = rf["kernel"].replace(" ", "")
    names = set()
    for f in kernel_stats.glob.glob(os.path.join(out, f"tr_{name}", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in kernel_stats.csv.DictReader(fh):
                if norm(r["Kernel_Name"]) == label:
                    names.add(r["Kernel_Name"])
    if len(names) != 1:
        sys.exit(f"profile_import {name}: kernel {label!r} matched {sorted(names)}")
    full = names.pop()
    config = (f"workload={workload} k={cfg['k']} p={cfg['p']} len={cfg['shard_bytes']} "
              f"stripes={cfg['stripes_per_gpu']}")
    cmd = "python3 bench.py --no-cpu-baseline " + " ".join(bargs)
    steady = os.path.join(out, f"{rnd}_{name}_kernel_steady.csv")
    trace = os.path.join(out, f"{rnd}_{name}_kernel_trace.csv")
    rc = kernel_stats.main([os.path.join(out, f"tr_{name}"), full, "--skip", str(d["warmup"]), "--keep",
                            str(d["steps"]), "--bytes", str(rf["bytes_per_launch"]), "--config", config,
                            "--command", "rocprofv3 --kernel-trace --stats --output-format csv -- " + cmd,
                            "--out", steady, "--trace-out", trace])
    if rc:
        sys.exit(rc)
    pmc = os.path.join(out, f"{rnd}_pmc_{name}.csv")
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_csv.py"), pmc, config,
                    cmd + " --steps 2 --warmup 1", os.path.join(out, f"fetch_{name}"),
                    os.path.join(out, f"write_{name}"), full], check=True)
    dst = os.path.join(REPO, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for f in (steady, trace, pmc):
        shutil.copy(f, dst)


if __name__ == "__main__":
    main()
