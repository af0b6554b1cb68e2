# Round-5 tree after pruning: smoke, the whole GPU suite, the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE FAIL; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; grep -v "^  File" $O/pytest.txt | tail -40; exit 1; }
tail -4 $O/pytest.txt
timeout -k 10 900 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAIL; tail -20 $O/bench_c2.err; exit 1; }
cut -c1-600 $O/bench_c2.json
