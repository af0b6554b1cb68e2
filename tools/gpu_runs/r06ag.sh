#!/bin/bash
# r06ag: drop-in encodes of 7-8 rows on the LDS product tables (ec_encode_karg_ldsx): drop-in and
# kernel-argument tests, 3 minutes of the differential fuzz on the kernels, then per-call latency and
# 16-thread throughput for k10 p8 / k10 p7 / k20 p8, product tables (default) vs v_perm
# (ISAL_HIP_ENC_LDSX=0), two interleaved rounds.
set -o pipefail
O=gpurun_out/r06ag; mkdir -p $O/corpus $O/artifacts; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dropin or kernel_args or karg or concurrent or selftest" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
python3 tests/fuzz/seeds.py diff $O/corpus > /dev/null || exit 1
ISAL_HIP_BACKEND=gpu timeout -k 10 300 /bin/sh -c '"$@"; exit $?' sh ./isa-l_amd/build/fuzzgpu/ec_diff_fuzz_gpu -max_total_time=180 -max_len=300000 -print_final_stats=1 -rss_limit_mb=2048 -malloc_limit_mb=2048 -artifact_prefix=$O/artifacts/ $O/corpus > $O/fuzz.txt 2>&1 || { tail -40 $O/fuzz.txt; exit 1; }
grep "^stat::number_of_executed_units\|^stat::peak_rss" $O/fuzz.txt; rm -rf $O/corpus
for round in 1 2; do
  for shape in "10 8 1048576 64" "10 7 1048576 64" "20 8 1048576 32"; do
    for x in d 0; do
      for t in 1 16; do
        if [ $x = d ]; then unset ISAL_HIP_ENC_LDSX; else export ISAL_HIP_ENC_LDSX=0; fi
        r=$(timeout -k 10 60 ./tools/dropin_bench $shape $t 2) || { echo FAIL $shape $x $t; exit 1; }
        echo "r$round ldsx=$x t=$t $r" | tee -a $O/dropin_ab.txt
      done
    done
  done
done
