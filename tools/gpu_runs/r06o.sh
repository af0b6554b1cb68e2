#!/bin/bash
# r06o: LDS product tables: loads in pairs / prefetched pairs / per-wave LDS-DMA ring beside the v_perm encode.
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 ./tools/wide_probe 10 2 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; tail -5 $O/probe.jsonl; exit 1; }
echo done
