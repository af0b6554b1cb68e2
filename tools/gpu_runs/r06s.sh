#!/bin/bash
# r06s: ec_encode_ldsx<P, 2> under occupancy caps (dynamic LDS) beside the library's encode,
# bench.py's shard layout then the back-to-back layout, two rounds each.
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 ./tools/wide_probe 10 2 1 > $O/probe_l1.jsonl 2> $O/probe.err || { cat $O/probe.err; exit 1; }
timeout -k 10 400 ./tools/wide_probe 10 2 0 > $O/probe_l0.jsonl 2>> $O/probe.err || { cat $O/probe.err; exit 1; }
echo done
