# CRC block geometry sweep: ISAL_HIP_CRC_TILES (4 KiB tiles chained per
# workgroup item) for the checksum-only and fused kernels, C2 shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
for w in crc crc64 encode-crc encode-crc64; do
  for tt in 16 32 64 128; do
    ISAL_HIP_CRC_TILES=$tt timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $O/b_${w}_$tt.json 2> $O/b_${w}_$tt.err || { echo FAIL $w $tt; tail $O/b_${w}_$tt.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${w}_$tt.json').read().strip().splitlines()[-1]); print('$w', $tt, d['value'], d['roofline']['frac'], d['roofline']['launch_ms'], d['self_check'])" | tee -a $O/sweep.txt
  done
done
