# Launch + completion floor by kernel-argument size / stream kind / grid
# (tools/launch_probe.hip); the two slow RAID conformance programs forced onto
# the kernels; the encode shapes' memory skeletons (tools/skel_probe.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 120 tools/launch_probe 3000 > $O/launch_probe.jsonl 2> $O/launch_probe.err || { echo PROBE FAIL; cat $O/launch_probe.err; exit 1; }
cat $O/launch_probe.jsonl
timeout -k 10 300 python3 tools/skel_probe.py 10 > $O/skel_probe.jsonl 2> $O/skel_probe.err || { echo SKEL FAIL; tail $O/skel_probe.err; exit 1; }
cat $O/skel_probe.jsonl
ISAL_SLOW_CONFORMANCE=1 timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread "tests/test_gpu_parity.py::test_reference_test_programs[xor_check_test-gpu]" "tests/test_gpu_parity.py::test_reference_test_programs[pq_check_test-gpu]" > $O/slow_conformance.txt 2>&1 || { echo CONF FAIL; tail -30 $O/slow_conformance.txt; exit 1; }
tail -5 $O/slow_conformance.txt
