#!/bin/bash
# r06k: LDS product tables for the wide passes: probe, parity tests, bench lines with LDSX on / off.
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 ./tools/wide_probe 10 1 > $O/probe.jsonl 2> $O/probe.err || { cat $O/probe.err; tail -5 $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or kernel_label or batch_encode or pipe_host or multi_device" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for shape in "--k 20 --p 8 --len 4194304 --stripes 64" "--k 20 --p 6 --len 4194304 --stripes 64" "--k 10 --p 8" "--k 10 --p 6"; do
  for x in 1 0; do
    ISAL_HIP_ENC_LDSX=$x timeout -k 10 200 python bench.py $shape --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'shape': '$shape', 'ldsx': '$x', 'kernel': d['roofline']['kernel'], 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac']}))" | tee -a $O/bench_ab.jsonl
  done
done
