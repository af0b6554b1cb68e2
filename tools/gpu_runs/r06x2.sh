#!/bin/bash
# r06x2: memory skeletons of the C4 update (7 read, 6 written), C3 decode (10 -> 3) and pq_gen
# (10 -> 2) at 128 / 256 threads per workgroup, two rounds.
set -o pipefail
O=gpurun_out/r06x2; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 0 1; do
  for shape in "C4 update" "C3 decode" "pq_gen" "C2 encode"; do
    BLOCKS=256,128 timeout -k 10 300 python3 tools/skel_probe.py 10 "$shape" >> $O/skel_blocks.jsonl 2>> $O/skel.err || { tail $O/skel.err; exit 1; }
  done
done
echo done
