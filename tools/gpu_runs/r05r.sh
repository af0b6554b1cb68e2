# (1) verify with the stored rows loaded before the fold (P <= 3): tests and a
# same-box A/B against the previous library; (2) headline bench with the CPU
# baselines pinned round-robin over L3 domains; (3) memory skeletons incl. the
# update shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
D=tools/dropin_bench
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "raid or check or verify" > $O/pytest.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for cfg in "prev:isa-l_amd/build/ab_prev" "early:"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    for op in pq_check xor_check; do
      echo -n "r$r $name op=$op t=1 " >> $O/verify_ab.txt
      LD_LIBRARY_PATH=$lib timeout -k 10 60 $D 10 4 1048576 64 1 2 0 $op >> $O/verify_ab.txt 2>&1 || { echo FAIL $name $op; tail $O/verify_ab.txt; exit 1; }
    done
    echo -n "r$r $name op=pq_check t=16 " >> $O/verify_ab.txt
    LD_LIBRARY_PATH=$lib timeout -k 10 60 $D 10 4 1048576 64 16 2 0 pq_check >> $O/verify_ab.txt 2>&1 || { echo FAIL $name t16; exit 1; }
  done
done
cut -c1-200 $O/verify_ab.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload pq_check > $O/bench_pq_check.json 2> $O/bench_pq_check.err || { echo FAIL pq_check bench; tail $O/bench_pq_check.err; exit 1; }
python3 -c "import sys; sys.path.insert(0,'tools'); import cpu_ref_baseline as c; print(c.usable_cores(), c._physical_cpus(c.usable_cores()))" > $O/cpus.txt
timeout -k 10 600 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo FAIL c2; tail $O/bench_c2.err; exit 1; }
timeout -k 10 300 python3 tools/skel_probe.py 10 > $O/skel_probe.jsonl 2> $O/skel_probe.err || { echo SKEL FAIL; tail $O/skel_probe.err; exit 1; }
cat $O/cpus.txt
for f in $O/bench_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}
print('$f', d['value'], r['frac'], r.get('frac_of_copy_ceiling'), c.get('value'), c.get('single_core_gib_s'), (d.get('cpu_baseline_simd_port') or {}).get('value'), (d.get('cpu_baseline_simd_port_cold') or {}).get('value'))"; done
