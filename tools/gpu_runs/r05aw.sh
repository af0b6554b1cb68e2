# CRC32C checksum-only with NI interleaved chains per lane (ISAL_HIP_EXP_CRC32=
# NI*10+B; 0 = the shipped single chain with double-buffered loads): parity of
# each variant, then a same-box A/B, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05aw; mkdir -p $O
V="24 22 32 41 14"
for v in $V; do
  ISAL_HIP_EXP_CRC32=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "crc_golden or encode_crc_vs_oracle or encode_crc_tiles or encode_crc_c2" > $O/pytest_$v.txt 2>&1 || { echo PYTEST FAIL $v; tail -30 $O/pytest_$v.txt; exit 1; }
  tail -n 1 $O/pytest_$v.txt
done
for r in 1 2; do
  for v in 0 $V; do
    ISAL_HIP_EXP_CRC32=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload crc > $O/b_crc_${v}_r$r.json 2> $O/b.err || { echo FAIL $v; tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_crc_${v}_r$r.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('crc', 'exp=$v', 'round=$r', d['value'], d.get('ms_per_step'), r.get('frac'), d.get('self_check'))" | tee -a $O/ab.txt
  done
done
