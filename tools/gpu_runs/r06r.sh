#!/bin/bash
# r06r: product tables forced on 4-row passes (C2): parity tests, then C2 / k12p4 bench lines
# LDSX=1 vs default, three interleaved rounds.
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or kernel_label or batch_encode or selftest or registry" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for round in 0 1 2; do
for shape in "--k 10 --p 4" "--k 12 --p 4 --len 1048576 --stripes 1024"; do
  for x in 1 d; do
    if [ $x = d ]; then unset ISAL_HIP_ENC_LDSX; else export ISAL_HIP_ENC_LDSX=$x; fi
    timeout -k 10 200 python bench.py $shape --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'round': $round, 'shape': '$shape', 'ldsx': '$x', 'kernel': d['roofline']['kernel'], 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac'], 'value': d['value']}))" | tee -a $O/bench_ab.jsonl
  done
done
done
