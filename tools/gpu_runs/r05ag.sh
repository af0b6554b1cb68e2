# ec_encode_v16 with every scalar argument loaded before the item loop (new)
# vs the shipped kernel (prev): two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05ag; mkdir -p $O
for r in 1 2; do
  for cfg in "prev:$PWD/isa-l_amd/build/ab_prev/libisal_hip.so" "new:$PWD/isa-l_amd/lib/libisal_hip.so"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    for w in xor_gen pq_gen encode decode; do
      ISAL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $O/b_${r}_${name}_$w.json 2> $O/b_${r}_${name}_$w.err || { echo FAIL $name $w; tail $O/b_${r}_${name}_$w.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${r}_${name}_$w.json').read().strip().splitlines()[-1]); print('r$r $name $w', d['value'], d['roofline']['frac'], d['roofline']['launch_ms'], d['self_check'])" | tee -a $O/ab.txt
    done
  done
done
