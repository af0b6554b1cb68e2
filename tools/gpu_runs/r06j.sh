#!/bin/bash
# r06j: wide encode passes with LDS product tables (tools/wide_probe) vs the library kernels.
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 400 ./tools/wide_probe 10 2 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; tail -5 $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
