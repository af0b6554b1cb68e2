# Tiles per workgroup (ISAL_HIP_EXP_TILES, experiment): parity with 2 and 4,
# then the skeleton with 1/2/4 tiles and a same-box A/B of xor_gen, pq_gen,
# decode and C2, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05aq; mkdir -p $O
for t in 2 4; do
  ISAL_HIP_EXP_TILES=$t timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or batch_encode_update or c2_c3_full_size or raid_vs_reference or batch_check or raid6_batch_full" > $O/pytest_t$t.txt 2>&1 || { echo PYTEST FAIL $t; tail -30 $O/pytest_t$t.txt; exit 1; }
  tail -1 $O/pytest_t$t.txt
done
for s in xor_gen pq_gen "C2 encode" "C3 decode"; do
  TILES=1,2,4 timeout -k 10 120 python -u tools/skel_probe.py 10 "$s" >> $O/skel_tiles.jsonl 2>> $O/err.txt || { echo SKEL FAIL; exit 1; }
done
for r in 1 2; do
  while read name args; do
    for t in 1 2 4; do
      ISAL_HIP_EXP_TILES=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > $O/b_${name}_t${t}_r$r.json 2> $O/b.err || { echo FAIL $name $t; tail $O/b.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${name}_t${t}_r$r.json').read().strip().splitlines()[-1]); print('$name', 'tiles=$t', 'round=$r', d['value'], d['roofline']['frac'], d['self_check'])" | tee -a $O/ab.txt
    done
  done <<'LIST'
xor_gen --workload xor_gen
pq_gen --workload pq_gen
decode --workload decode
c2
LIST
done
python3 -c "
import json
for l in open('$O/skel_tiles.jsonl'):
    d = json.loads(l); print(d['shape'], d['tiles_per_wg'], d['lds_bytes'], d['pointer_table'], d['frac_of_8tbs'])
"
