#!/bin/bash
# r06m: LDS product tables with the measured policy (7-8 rows, or 5-6 rows over k >= 16; groups of 2):
# parity tests, bench lines LDSX default / off.
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or kernel_label or batch_encode or pipe_host or multi_device" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for shape in "--k 20 --p 8 --len 4194304 --stripes 64" "--k 20 --p 6 --len 4194304 --stripes 64" "--k 16 --p 8 --len 1048576 --stripes 512" "--k 10 --p 8" "--k 10 --p 7" "--k 10 --p 6" "--k 10 --p 4"; do
  for x in d 0; do
    if [ $x = d ]; then unset ISAL_HIP_ENC_LDSX; else export ISAL_HIP_ENC_LDSX=0; fi
    timeout -k 10 200 python bench.py $shape --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'shape': '$shape', 'ldsx': '$x', 'kernel': d['roofline']['kernel'], 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac'], 'value': d['value']}))" | tee -a $O/bench_ab.jsonl
  done
done
