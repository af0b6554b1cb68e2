# CRC32C checksum-only: batch of 8 tiles (111 VGPRs, 4 waves/SIMD, shipped) vs
# 6 (93, 5) vs 4 (71, 7); two interleaved rounds, C2 shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
for r in 1 2; do
  for cfg in "b8:$PWD/isa-l_amd/lib/libisal_hip.so" "b6:$PWD/isa-l_amd/build/ab_b6/libisal_hip.so" "b4:$PWD/isa-l_amd/build/ab_b4/libisal_hip.so"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    ISAL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload crc > $O/b_${r}_${name}.json 2> $O/b_${r}_${name}.err || { echo FAIL $name; tail $O/b_${r}_${name}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${r}_${name}.json').read().strip().splitlines()[-1]); print('r$r $name crc', d['value'], d['roofline']['frac'], d['roofline']['launch_ms'], d['self_check'])" | tee -a $O/ab.txt
  done
done
