#!/bin/bash
# r06c: CRC64 checksum-only variants (tools/crc64_probe), C2 shape.
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 ./tools/crc64_probe 10 1024 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; exit 1; }
cat $O/probe.jsonl
