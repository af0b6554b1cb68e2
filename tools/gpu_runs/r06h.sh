#!/bin/bash
# r06h: CRC64 checksum-only: compute-only (no HBM) variants vs the library kernel.
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 ./tools/crc64_probe 10 1024 2 lib lib128 nomem2 nomem1 nomem4 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; exit 1; }
cat $O/probe.jsonl
