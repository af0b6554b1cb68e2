#!/bin/bash
# Fused encode+CRC / checksum-only tuning sweep: source-chain location x tiles
# per workgroup. Usage (via gpurun): bash tools/crc_sweep.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-sweep}
mkdir -p "$OUT"
for chain in reg lds; do
        for tt in 4 8 16 32; do
                echo "chain=$chain tt=$tt" | tee -a "$OUT/sweep.txt"
                ISAL_HIP_CRC_SRC_CHAIN=$chain ISAL_HIP_CRC_TILES=$tt timeout -k 10 120 \
                        python bench.py --workload encode-crc --no-cpu-baseline --steps 10 --warmup 3 \
                        > "$OUT/ec_${chain}_$tt.log" 2>&1 || exit $?
                python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])" "$OUT/ec_${chain}_$tt.log" | tee -a "$OUT/sweep.txt"
        done
done
for tt in 4 8 16 32; do
        echo "crc tt=$tt" | tee -a "$OUT/sweep.txt"
        ISAL_HIP_CRC_TILES=$tt timeout -k 10 120 python bench.py --workload crc --no-cpu-baseline --steps 10 --warmup 3 \
                > "$OUT/crc_$tt.log" 2>&1 || exit $?
        python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['roofline']['launch_ms'], d['roofline']['frac'])" "$OUT/crc_$tt.log" | tee -a "$OUT/sweep.txt"
done
