#!/bin/bash
# NOTE: the R06_* switch this script sets existed only in the experiment's working tree (removed after
# the A/B; the shipped library ignores it), so re-running it today times the shipped kernel in every arm.
# r06ab: the v16 encode (passes of <= 4 rows) with 128-lane workgroups (2 KiB tiles) under a
# 32 KiB (R06_V16_B=128) or 16 KiB (128h) LDS occupancy cap, against the shipped 256 lanes /
# 32 KiB: parity tests under 128, then C2 / C3 decode / pq_gen / xor_gen lines, three interleaved
# rounds.
set -o pipefail
O=gpurun_out/r06ab; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
R06_V16_B=128 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or xor_fast_path or load_groups or batch_encode or decode or pq_gen or xor_gen" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for round in 0 1 2; do
for wl in encode decode pq_gen xor_gen; do
  for v in 256 128 128h; do
    if [ $v = 256 ]; then unset R06_V16_B; else export R06_V16_B=$v; fi
    timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'round': $round, 'workload': '$wl', 'variant': '$v', 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac']}))" | tee -a $O/ab.jsonl
  done
done
done
