#!/bin/bash
# NOTE: the R06_* switch this script sets existed only in the experiment's working tree (removed after
# the A/B; the shipped library ignores it), so re-running it today times the shipped kernel in every arm.
# r06aa: device update (C4 shape) with 128-thread workgroups and/or the 32 KiB LDS occupancy cap
# (R06_UPD=128 / 128c / 256c) against the shipped 256 threads, no cap; parity tests under 128c;
# three interleaved rounds.
set -o pipefail
O=gpurun_out/r06aa; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
R06_UPD=128c timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "update" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for round in 0 1 2; do
  for v in 256 256c 128 128c; do
    if [ $v = 256 ]; then unset R06_UPD; else export R06_UPD=$v; fi
    timeout -k 10 200 python bench.py --workload update --k 20 --p 6 --len 4194304 --stripes 64 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'round': $round, 'variant': '$v', 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac'], 'value': d['value']}))" | tee -a $O/ab.jsonl
  done
done
