#!/bin/bash
# NOTE: the R06_* switch this script sets existed only in the experiment's working tree (removed after
# the A/B; the shipped library ignores it), so re-running it today times the shipped kernel in every arm.
# r06v: fused encode + CRC64 at C2: 512-lane workgroups sharing one table copy forced to 4 waves
# per SIMD (128 VGPRs, 14 spilled; R06_FUSED_NV=2) against the shipped 256-lane, 3-wave kernel
# (=1), three interleaved rounds, same box; CRC64 fused tests under both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06v; mkdir -p $O
for nv in 2 1; do
  R06_FUSED_NV=$nv timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "encode_crc64" > $O/pytest_$nv.txt 2>&1 || { tail -40 $O/pytest_$nv.txt; exit 1; }
  tail -1 $O/pytest_$nv.txt
done
for r in 0 1 2; do
  for nv in 2 1; do
    R06_FUSED_NV=$nv timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload encode-crc64 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); r=d['roofline']; print(json.dumps({'round': $r, 'nv': $nv, 'ms_per_step': d['ms_per_step'], 'frac': r['frac']}))" | tee -a $O/ab.jsonl
  done
done
