# Completion-tree group size sweep (tools/launch_probe.hip); drop-in tests on
# the tree with the in-flight fix.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "dropin or k0_empty or raid_check or batch_check" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 240 tools/launch_probe 3000 > $O/launch_probe.jsonl 2> $O/launch_probe.err || { echo PROBE FAIL; cat $O/launch_probe.err; exit 1; }
grep group_min $O/launch_probe.jsonl
