# The GPU suite with each test's peak RSS logged (which test sets the suite's peak); OUT= names the output directory.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05aj}; mkdir -p $O
export ISAL_TEST_RSS_LOG=$O/rss.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
awk 'BEGIN{p=0} {if ($2 > p + 256) print; if ($2 > p) p = $2}' $O/rss.txt
