# Which pages make the full-size C2/C3 test's RSS: anonymous, file-backed or shmem.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05ak; mkdir -p $O
export ISAL_TEST_RSS_LOG=$O/rss.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "golden_encode or c2_c3_full_size or raid6_batch_full_size" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
cat $O/rss.txt
