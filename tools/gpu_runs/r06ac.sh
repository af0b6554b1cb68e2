#!/bin/bash
# r06ac: the differential fuzz target (tests/fuzz/ec_diff_fuzz.c: every input one engine call and
# the same oracle call, outputs / return codes / canaries compared) on the final library with every
# call on the kernels, 10 minutes.
set -o pipefail
O=gpurun_out/r06ac; mkdir -p $O/corpus $O/artifacts; export TMPDIR=/tmp
python3 tests/fuzz/seeds.py diff $O/corpus > /dev/null || exit 1
ISAL_HIP_BACKEND=gpu timeout -k 10 700 /bin/sh -c '"$@"; exit $?' sh ./isa-l_amd/build/fuzzgpu/ec_diff_fuzz_gpu -max_total_time=600 -max_len=300000 -print_final_stats=1 -rss_limit_mb=2048 -malloc_limit_mb=2048 -artifact_prefix=$O/artifacts/ $O/corpus > $O/fuzz.txt 2>&1 || { tail -40 $O/fuzz.txt; exit 1; }
grep "^stat::" $O/fuzz.txt; rm -rf $O/corpus
echo done
