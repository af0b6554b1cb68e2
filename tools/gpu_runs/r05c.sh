set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
D=tools/dropin_bench
for cfg in "mail narrow:ISAL_HIP_KARG_DONE=1 ISAL_HIP_KARG_NARROW=1" "mail wide:ISAL_HIP_KARG_DONE=1 ISAL_HIP_KARG_NARROW=0" "sync narrow:ISAL_HIP_KARG_DONE=0 ISAL_HIP_KARG_NARROW=1" "sync wide:ISAL_HIP_KARG_DONE=0 ISAL_HIP_KARG_NARROW=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  for t in 1 16; do
    echo -n "$name t=$t " >> $O/summary.txt
    env $envs timeout -k 10 120 $D 10 4 1048576 64 $t 2 >> $O/summary.txt 2>&1 || exit 1
  done
done
for cfg in "mail:ISAL_HIP_KARG_DONE=1" "sync:ISAL_HIP_KARG_DONE=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run -- $D 10 4 1048576 64 1 1 2000 > $O/prof_$name.txt 2>&1 || exit 1
done
cat $O/summary.txt
find $O -name "*kernel_stats.csv" | while read f; do echo $f; cat $f | cut -c1-200; done
