#!/bin/bash
# r06e: CRC64 checksum-only: rolling register batches vs the library kernel (tools/crc64_probe).
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 300 ./tools/crc64_probe 10 1024 3 lib lib128 roll2_4 roll2_2 roll2_3 roll1_4 roll2_6 roll3_2 roll2_4_128 roll2_2_128 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; exit 1; }
cat $O/probe.jsonl
