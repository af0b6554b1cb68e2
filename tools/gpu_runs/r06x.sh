#!/bin/bash
# r06x: k20p6 / k20p8 memory skeletons at 128 / 256 / 512 threads per workgroup (2 / 4 / 8 KiB
# tiles), two rounds.
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 0 1; do
  for shape in "k20p6" "k20p8"; do
    BLOCKS=256,128,512 timeout -k 10 300 python3 tools/skel_probe.py 10 "$shape" >> $O/skel_blocks.jsonl 2>> $O/skel.err || { tail $O/skel.err; exit 1; }
  done
done
echo done
