# Host-resident (page-locked) pipelines on the final tree: encode (C2 stripes)
# and update (C4 shape), PCIe-bound.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05ah; mkdir -p $O
timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload e2e-encode --steps 200 --warmup 10 > $O/b_e2e_encode.json 2> $O/b_e2e_encode.err || { echo FAIL enc; tail $O/b_e2e_encode.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload e2e-update --k 20 --p 6 --len 4194304 --steps 200 --warmup 10 > $O/b_e2e_update.json 2> $O/b_e2e_update.err || { echo FAIL upd; tail $O/b_e2e_update.err; exit 1; }
for f in $O/b_e2e_*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['unit'], d.get('ms_per_step'), d['parity_check_last_stripe'], d['config']['workload'][:120])"; done
