#!/bin/bash
# r06g: CRC64 checksum-only: byte-table variants vs the library kernel (tools/crc64_probe).
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 300 ./tools/crc64_probe 10 1024 3 lib lib128 bytes2_4_1 bytes2_4_2 bytes1_4_2 bytes2_2_2 bytes3_2_2 bytes2_4_2_128 bytes4_2_2 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; exit 1; }
cat $O/probe.jsonl
