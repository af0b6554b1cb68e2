# Kernarg preloading (-mllvm -amdgpu-kernarg-preload-count=16 on ec_kernels.hip,
# isa-l_amd/lib_pre/libisal_hip.so) against the shipped library: parity of the
# preloaded build, then a same-box A/B, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05as; mkdir -p $O
PRE=$PWD/isa-l_amd/lib_pre/libisal_hip.so
ISAL_HIP_LIB=$PRE timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or xor_fast_path or load_groups or batch_encode_update or c2_c3_full_size or raid_vs_reference or batch_check or dropin or karg or verify" > $O/pytest_pre.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_pre.txt; exit 1; }
tail -n 1 $O/pytest_pre.txt
for r in 1 2; do
  while read name args; do
    for v in base pre; do
      if [ $v = pre ]; then export ISAL_HIP_LIB=$PRE; else unset ISAL_HIP_LIB; fi
      timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > $O/b_${name}_${v}_r$r.json 2> $O/b.err || { echo FAIL $name $v; tail $O/b.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${name}_${v}_r$r.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$name', '$v', 'round=$r', d['value'], d.get('ms_per_step'), r.get('frac'), d.get('self_check'))" | tee -a $O/ab.txt
    done
  done <<'LIST'
c2
decode --workload decode
xor_gen --workload xor_gen
pq_gen --workload pq_gen
pq_check --workload pq_check
update --workload update --k 20 --p 6 --len 4194304 --stripes 64
k10p6 --k 10 --p 6
k20p6 --k 20 --p 6 --len 4194304 --stripes 64
dropin --workload dropin
LIST
done
unset ISAL_HIP_LIB
