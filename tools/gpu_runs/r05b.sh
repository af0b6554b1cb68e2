set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05b
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "k0_empty or result_visible or completion_paths or raid_check_routes or dropin_kernel_args or concurrent_callers or ordered_after or update_equals" > gpurun_out/r05b/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/r05b/pytest.txt; exit 1; }
tail -3 gpurun_out/r05b/pytest.txt
for op in encode pq_check; do
  timeout -k 10 300 python bench.py --workload dropin --dropin-op $op > gpurun_out/r05b/dropin_$op.json 2> gpurun_out/r05b/dropin_$op.err || { echo DROPIN FAIL $op; tail -20 gpurun_out/r05b/dropin_$op.err; exit 1; }
done
ISAL_HIP_KARG_DONE=0 timeout -k 10 300 python bench.py --workload dropin > gpurun_out/r05b/dropin_encode_nomail.json 2> gpurun_out/r05b/dropin_encode_nomail.err || exit 1
python3 -c "
import json
for f in ['dropin_encode','dropin_pq_check','dropin_encode_nomail']:
    d=json.load(open('gpurun_out/r05b/'+f+'.json')); print(f, [(r['threads'], r['us_per_call'], r['gib_s']) for r in d['threads']])
"
