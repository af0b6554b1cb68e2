# Headline bench with the CPU baselines pinned round-robin over L3 domains
# (twice), plus the spread's topology; memory skeletons incl. the update shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
python3 -c "import sys; sys.path.insert(0,'tools'); import cpu_ref_baseline as c; print(c.usable_cores(), c._physical_cpus(c.usable_cores()))" > $O/cpus.txt
for i in 1 2; do
  timeout -k 10 600 python3 bench.py > $O/bench_c2_$i.json 2> $O/bench_c2_$i.err || { echo FAIL c2; tail $O/bench_c2_$i.err; exit 1; }
done
timeout -k 10 300 python3 tools/skel_probe.py 10 > $O/skel_probe.jsonl 2> $O/skel_probe.err || { echo SKEL FAIL; tail $O/skel_probe.err; exit 1; }
cat $O/cpus.txt
for i in 1 2; do python3 -c "
import json; d=json.loads(open('$O/bench_c2_$i.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d['roofline'].get('frac_of_copy_ceiling'), d['cpu_baseline']['value'], d['cpu_baseline']['single_core_gib_s'], d['cpu_baseline_simd_port']['value'], d['cpu_baseline_simd_port_cold']['value'])"; done
