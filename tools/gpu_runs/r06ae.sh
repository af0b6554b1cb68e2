#!/bin/bash
# r06ae: the remaining BASELINE configs on the final tree: C5 (1,048,576 stripes on one GPU,
# decode round trip), the host-resident pipelines (C2 stripes encode, C4 update; PCIe-bound)
# and C1 (host CPU route).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06ae; mkdir -p $O
timeout -k 10 400 python3 bench.py --no-cpu-baseline --total-stripes 1048576 --steps 2 --warmup 1 > $O/b_c5.json 2> $O/b_c5.err || { echo FAIL c5; tail $O/b_c5.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload e2e-encode --steps 200 --warmup 10 > $O/b_e2e_encode.json 2> $O/b_e2e_encode.err || { echo FAIL enc; tail $O/b_e2e_encode.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload e2e-update --k 20 --p 6 --len 4194304 --steps 200 --warmup 10 > $O/b_e2e_update.json 2> $O/b_e2e_update.err || { echo FAIL upd; tail $O/b_e2e_update.err; exit 1; }
timeout -k 10 400 python3 bench.py --workload c1 > $O/b_c1.json 2> $O/b_c1.err || { echo FAIL c1; tail $O/b_c1.err; exit 1; }
for f in $O/b_*.json; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['unit'], d.get('ms_per_step'), d.get('self_check'), d.get('parity_check_last_stripe'))"; done
