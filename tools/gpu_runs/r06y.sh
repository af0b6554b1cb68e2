#!/bin/bash
# NOTE: the R06_* switch this script sets existed only in the experiment's working tree (removed after
# the A/B; the shipped library ignores it), so re-running it today times the shipped kernel in every arm.
# r06y: ec_encode_ldsx with 128-thread workgroups (2 KiB tiles; R06_LDSX_B=128) against 256
# (4 KiB, shipped): parity tests with the tables forced under 128, then bench lines, two
# interleaved rounds.
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
R06_LDSX_B=128 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xor_fast_path or load_groups or batch_encode" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for round in 0 1; do
for shape in "--k 20 --p 8 --len 4194304 --stripes 64" "--k 20 --p 6 --len 4194304 --stripes 64" "--k 20 --p 5 --len 4194304 --stripes 64" "--k 16 --p 8 --len 1048576 --stripes 512" "--k 16 --p 6 --len 1048576 --stripes 512" "--k 10 --p 8" "--k 10 --p 7"; do
  for b in 128 256; do
    R06_LDSX_B=$b timeout -k 10 200 python bench.py $shape --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print(json.dumps({'round': $round, 'shape': '$shape', 'block': $b, 'launch_ms': d['roofline']['launch_ms'], 'frac': d['roofline']['frac']}))" | tee -a $O/bench_ab.jsonl
  done
done
done
