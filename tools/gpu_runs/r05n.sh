# Adaptive drop-in lane width: tests + same-box A/B against forced 4- and
# 16-byte lanes; launch/completion floor v2 (tree / per-group slots); encode
# memory skeletons incl. the 1:1 copy.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
D=tools/dropin_bench
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "dropin or raid_check or batch_check or k0_empty or concurrent_callers" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for cfg in "adaptive:" "narrow:ISAL_HIP_KARG_NARROW=1" "wide:ISAL_HIP_KARG_NARROW=0"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    for t in 1 4 8 16; do
      echo -n "r$r $name t=$t " >> $O/dropin_ab.txt
      env $envs timeout -k 10 60 $D 10 4 1048576 64 $t 2 >> $O/dropin_ab.txt 2>&1 || { echo FAIL dropin $name $t; tail $O/dropin_ab.txt; exit 1; }
    done
  done
done
cat $O/dropin_ab.txt
timeout -k 10 180 tools/launch_probe 3000 > $O/launch_probe.jsonl 2> $O/launch_probe.err || { echo PROBE FAIL; cat $O/launch_probe.err; exit 1; }
timeout -k 10 300 python3 tools/skel_probe.py 10 > $O/skel_probe.jsonl 2> $O/skel_probe.err || { echo SKEL FAIL; tail $O/skel_probe.err; exit 1; }
cat $O/launch_probe.jsonl $O/skel_probe.jsonl
