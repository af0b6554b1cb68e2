# Mailbox calls on a non-blocking stream while the default stream is idle:
# tests + same-box A/B against the previous library (blocking stream).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
D=tools/dropin_bench
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "dropin or raid_check or batch_check or k0_empty or concurrent_callers or ordered_after or update_equals" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for cfg in "blocking:isa-l_amd/build/ab_prev" "nbquery:"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    for t in 1 4 16; do
      echo -n "r$r $name t=$t " >> $O/dropin_ab.txt
      LD_LIBRARY_PATH=$lib timeout -k 10 60 $D 10 4 1048576 64 $t 2 >> $O/dropin_ab.txt 2>&1 || { echo FAIL dropin $name $t; tail $O/dropin_ab.txt; exit 1; }
    done
    for op in xor_gen pq_check; do
      echo -n "r$r $name op=$op t=1 " >> $O/dropin_ab.txt
      LD_LIBRARY_PATH=$lib timeout -k 10 60 $D 10 4 1048576 64 1 2 0 $op >> $O/dropin_ab.txt 2>&1 || { echo FAIL dropin $name $op; tail $O/dropin_ab.txt; exit 1; }
    done
  done
done
cut -c1-190 $O/dropin_ab.txt
