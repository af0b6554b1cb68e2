#!/bin/bash
# r06p: ec_encode_ldsx with double-buffered source groups (the probe's ldsx_pf2 in the library):
# parity tests, then bench lines LDSX forced (=1) / off (=0) over 5-8 row shapes, two interleaved rounds.
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or kernel_label or batch_encode" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for round in 0 1; do
for shape in "--k 20 --p 8 --len 4194304 --stripes 64" "--k 20 --p 6 --len 4194304 --stripes 64" "--k 20 --p 5 --len 4194304 --stripes 64" "--k 16 --p 8 --len 1048576 --stripes 512" "--k 16 --p 6 --len 1048576 --stripes 512" "--k 13 --p 6 --len 1048576 --stripes 512" "--k 12 --p 5 --len 1048576 --stripes 512" "--k 10 --p 8" "--k 10 --p 7" "--k 10 --p 6" "--k 10 --p 5"; do
  for x in 1 0; do
    export ISAL_HIP_ENC_LDSX=$x
    timeout -k 10 200 python bench.py $shape --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'round': $round, 'shape': '$shape', 'ldsx': '$x', 'kernel': d['roofline']['kernel'], 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac'], 'value': d['value']}))" | tee -a $O/bench_ab.jsonl
  done
done
done
