#!/bin/bash
# r06w: the library's default encode over k in {4..32} x p in {1..8}, 1 MiB shards, ~14 GiB per
# launch (tools/wide_probe matrix mode): bench.py's layout two rounds, then each stripe's shards
# back to back one round; the kernels the passes launched counted.
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O; export TMPDIR=/tmp
ISAL_HIP_LOG=2 timeout -k 10 500 ./tools/wide_probe 10 2 1 matrix > $O/matrix_l1.jsonl 2> $O/matrix.err || { tail $O/matrix.err; exit 1; }
sort $O/matrix.err | uniq -c > $O/kernels.txt
timeout -k 10 400 ./tools/wide_probe 10 1 0 matrix > $O/matrix_l0.jsonl 2> $O/matrix0.err || { tail $O/matrix0.err; exit 1; }
echo done
