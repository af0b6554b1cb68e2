#!/bin/bash
# r06aj: is the product-table kernel's dynamic-LDS cap (at equal occupancy) a real effect or the
# first-measured configuration of each shape? cap 0 / 16 KiB / 20 KiB / 0 / 16 KiB / 0 in that order,
# 256 lanes, two rounds.
set -o pipefail
O=gpurun_out/r06aj; mkdir -p $O; export TMPDIR=/tmp
LANES_ORDER=1 timeout -k 10 600 ./tools/wide_probe 10 2 1 lanes > $O/order.jsonl 2> $O/order.err || { tail $O/order.err; exit 1; }
echo done
