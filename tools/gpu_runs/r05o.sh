# Launch floor v3 (blocking vs non-blocking + hipStreamQuery(0)); adaptive
# lane width at threshold 12.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
D=tools/dropin_bench
timeout -k 10 180 tools/launch_probe 3000 > $O/launch_probe.jsonl 2> $O/launch_probe.err || { echo PROBE FAIL; cat $O/launch_probe.err; exit 1; }
cat $O/launch_probe.jsonl
for r in 1 2; do
  for cfg in "adaptive:" "wide:ISAL_HIP_KARG_NARROW=0"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    for t in 1 8 16; do
      echo -n "r$r $name t=$t " >> $O/dropin_ab.txt
      env $envs timeout -k 10 60 $D 10 4 1048576 64 $t 2 >> $O/dropin_ab.txt 2>&1 || { echo FAIL dropin $name $t; tail $O/dropin_ab.txt; exit 1; }
    done
  done
done
cut -c1-200 $O/dropin_ab.txt
