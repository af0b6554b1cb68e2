set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a/smoke.txt 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r05a/smoke.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "k0_empty or result_visible or completion_paths or raid_check_routes or batch_check or dropin_kernel_args or concurrent_callers or ordered_after or raid_vs_reference or raid_pq_large or golden_encode" > gpurun_out/r05a/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 gpurun_out/r05a/pytest.txt; exit 1; }
tail -3 gpurun_out/r05a/pytest.txt
for op in encode pq_gen pq_check; do
  timeout -k 10 300 python bench.py --workload dropin --dropin-op $op > gpurun_out/r05a/dropin_$op.json 2> gpurun_out/r05a/dropin_$op.err || { echo DROPIN FAIL $op; tail -20 gpurun_out/r05a/dropin_$op.err; exit 1; }
done
for w in pq_gen xor_gen pq_check; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/r05a/bench_$w.json 2> gpurun_out/r05a/bench_$w.err || { echo BENCH FAIL $w; tail -20 gpurun_out/r05a/bench_$w.err; exit 1; }
done
cat gpurun_out/r05a/*.json | cut -c1-400
