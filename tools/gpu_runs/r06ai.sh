#!/bin/bash
# r06ai: the product-table encode at 256 lanes (library kernel) and 128 lanes (2 KiB tiles) under
# dynamic-LDS occupancy caps, k20p8 / k20p6 / k16p8 / k10p8, two rounds (tools/wide_probe lanes mode).
set -o pipefail
O=gpurun_out/r06ai; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 ./tools/wide_probe 10 2 1 lanes > $O/lanes.jsonl 2> $O/lanes.err || { tail $O/lanes.err; exit 1; }
echo done
