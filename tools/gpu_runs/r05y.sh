# Fused encode + CRC64 (C2, slice 3): 3 waves/SIMD, one 256-lane group per
# workgroup (shipped) vs 4 waves with two lane groups sharing the tables (14
# VGPRs spilled); two interleaved rounds. First the CRC parity tests on the
# shipped tree (checksum-only CRC32C now loads 4 tiles per batch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "crc" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for cfg in "w3:$PWD/isa-l_amd/lib/libisal_hip.so" "w4nv2:$PWD/isa-l_amd/build/ab_nv2/libisal_hip.so"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    ISAL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload encode-crc64 > $O/b_${r}_${name}.json 2> $O/b_${r}_${name}.err || { echo FAIL $name; tail $O/b_${r}_${name}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${r}_${name}.json').read().strip().splitlines()[-1]); print('r$r $name encode-crc64', d['value'], d['roofline']['frac'], d['roofline']['launch_ms'], d['self_check'])" | tee -a $O/ab.txt
  done
done
