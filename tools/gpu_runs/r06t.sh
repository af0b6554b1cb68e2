#!/bin/bash
# r06t: CRC64 and CRC32C combines as one wave per shard (shuffle tree, no barriers): every CRC test,
# then the checksum and fused lines with their steady traces (combine kernel beside).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06t; mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "crc" > $O/pytest_crc.txt 2>&1 || { tail -40 $O/pytest_crc.txt; exit 1; }
tail -2 $O/pytest_crc.txt
for wl in crc64 encode-crc64 crc encode-crc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$wl -o t -- $B --workload $wl > $O/trbench_$wl.json 2>> $O/log.txt || { echo FAIL tr $wl; tail $O/log.txt; exit 1; }
  timeout -k 10 300 $B --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail $O/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$wl.json') if l.startswith('{')][-1]); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], r['frac'])"
  python3 - "$O/tr_$wl" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "crc" in r["Name"][:60]:
            print("  ", r["Name"][:50], r["Calls"], r["AverageNs"])
PY
done
