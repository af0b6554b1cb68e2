# Memory skeletons with and without the batch encode's device pointer table,
# and the RAID/C2 encodes on the same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 400 python3 tools/skel_probe.py 10 > $O/skel_probe.jsonl 2> $O/skel_probe.err || { echo SKEL FAIL; tail $O/skel_probe.err; exit 1; }
for w in xor_gen pq_gen encode; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $O/b_$w.json 2> $O/b_$w.err || { echo FAIL $w; tail $O/b_$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['roofline']['frac'], d['roofline']['kernel'], d['self_check'])"
done
python3 -c "
import json
for l in open('$O/skel_probe.jsonl'):
    d=json.loads(l); print(d['shape'], d['lds_bytes'], d['pointer_table'], d['frac_of_8tbs'])"
