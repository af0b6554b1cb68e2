# Final tree: the whole GPU suite (the driver's command, plus timing flags)
# and smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05s}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE FAIL; tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
