#!/bin/bash
# r06l: LDS product tables: every pass width 3-8 x source group 1-5 beside the library's v_perm encode.
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 ./tools/wide_probe 10 2 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; tail -5 $O/probe.jsonl; exit 1; }
echo done
