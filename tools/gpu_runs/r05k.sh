# Default KARG_NARROW threshold cases; per-call cost of the reference's RAID
# check tests' calls forced onto the kernels (host memory); hip-trace of the
# mailbox drop-in call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
D=tools/dropin_bench
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "dropin_kernel_args" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for mem in host pinned; do
  for op in xor_check pq_check xor_gen pq_gen; do
    for be in gpu auto; do
      echo -n "mem=$mem backend=$be " >> $O/raid_calls.txt
      DROPIN_MEM=$mem ISAL_HIP_BACKEND=$be timeout -k 10 60 $D 16 1 1024 64 1 2 0 $op >> $O/raid_calls.txt 2>&1 || { echo FAIL $mem $op $be; tail $O/raid_calls.txt; exit 1; }
    done
  done
done
cat $O/raid_calls.txt
for op in encode pq_gen xor_gen pq_check xor_check; do
  for t in 1 16; do
    echo -n "device op=$op t=$t " >> $O/dropin_ops.txt
    timeout -k 10 60 $D 10 4 1048576 64 $t 2 0 $op >> $O/dropin_ops.txt 2>&1 || { echo FAIL dropin $op $t; tail $O/dropin_ops.txt; exit 1; }
  done
done
cat $O/dropin_ops.txt
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/hip_mail -o run -- $D 10 4 1048576 64 1 1 2000 > $O/hip_mail.txt 2>&1 || { echo FAIL hip_mail; tail $O/hip_mail.txt; exit 1; }
DROPIN_MEM=host ISAL_HIP_BACKEND=gpu timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/hip_xorcheck -o run -- $D 16 1 1024 64 1 1 2000 xor_check > $O/hip_xorcheck.txt 2>&1 || { echo FAIL hip_xorcheck; tail $O/hip_xorcheck.txt; exit 1; }
tail -2 $O/hip_mail.txt $O/hip_xorcheck.txt
