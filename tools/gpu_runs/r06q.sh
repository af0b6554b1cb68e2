#!/bin/bash
# r06q: memory skeleton with a pad between consecutive shards (do the shards' mutual
# alignments limit the many-stream shapes?), two rounds.
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or kernel_label or batch_encode" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 0 1; do
  for shape in "C2" "k20p6" "k20p8" "xor_gen" "copy" "k10p8"; do
    PAD=0,256,2048,4096,12288,65536,69632,1052672 timeout -k 10 300 python3 tools/skel_probe.py 10 "$shape" >> $O/skel_pad.jsonl 2>> $O/skel.err || { tail $O/skel.err; exit 1; }
  done
done
echo done
