#!/bin/bash
# NOTE: the R06_* switch this script sets existed only in the experiment's working tree (removed after
# the A/B; the shipped library ignores it), so re-running it today times the shipped kernel in every arm.
# r06af: occupancy cap of the 128-lane RAID-gen encode (passes of 1-2 rows): dynamic LDS per
# workgroup 16 / 24 / 32 (shipped) / 40 / 48 KiB (R06_CAP), three interleaved rounds.
set -o pipefail
O=gpurun_out/r06af; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for round in 0 1 2; do
for wl in xor_gen pq_gen; do
  for c in 16384 24576 32768 40960 49152; do
    R06_CAP=$c timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'round': $round, 'workload': '$wl', 'cap': $c, 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac']}))" | tee -a $O/ab.jsonl
  done
done
done
