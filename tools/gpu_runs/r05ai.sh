# Final tree: smoke, the whole GPU suite (with the device-resident abort test).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05ai}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE FAIL; tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread --durations=10 > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -16 $O/pytest.txt
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAIL; tail $O/bench_default.err; exit 1; }
tail -n 1 $O/bench_default.json
