# Full-size RAID-6 batch parity + check test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 500 --timeout-method thread -k "raid6_batch_full_size or batch_check" --durations=5 > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest.txt; exit 1; }
tail -12 $O/pytest.txt
