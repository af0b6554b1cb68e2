#!/bin/bash
# r06d: SQ counters of the CRC64 checksum-only pass: library kernel vs LDS-DMA ring (tools/crc64_probe).
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O; cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
P="./tools/crc64_probe 2 1024 1 lib lib128 ring4_2 ring8_2"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o p1 -- $P > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/p2 -o p2 -- $P > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- ./tools/crc64_probe 10 1024 1 lib lib128 ring4_2 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
find $O -name "*.csv" | head -20
