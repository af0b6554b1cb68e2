# CRC kernels: first data batch issued before the LDS table copy, and the
# table copy batched (4 loads per thread in flight) — tests and a same-box A/B
# against the previous library (ISAL_HIP_LIB), two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "crc" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for cfg in "prev:$PWD/isa-l_amd/build/ab_prev/libisal_hip.so" "new:$PWD/isa-l_amd/lib/libisal_hip.so"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    for w in crc crc64 encode-crc encode-crc64; do
      ISAL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $O/b_${r}_${name}_$w.json 2> $O/b_${r}_${name}_$w.err || { echo FAIL $name $w; tail $O/b_${r}_${name}_$w.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${r}_${name}_$w.json').read().strip().splitlines()[-1]); print('r$r $name $w', d['value'], d['roofline']['frac'], d['roofline']['launch_ms'], d['self_check'])" | tee -a $O/ab.txt
    done
  done
done
