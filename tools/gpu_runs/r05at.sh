# CRC64 checksum-only with NI interleaved chains per lane (ISAL_HIP_EXP_CRC2=
# NI*10+B: B tiles of each of NI items loaded together; RUN=r05au): parity, then a same-box A/B
# against the shipped kernel (0), two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r05at}; mkdir -p $O
for v in ${PAR:-2 4}; do
  ISAL_HIP_EXP_CRC2=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "crc64_golden or test_crc64_vs_oracle or test_crc64_c2_full_size" > $O/pytest_$v.txt 2>&1 || { echo PYTEST FAIL $v; tail -30 $O/pytest_$v.txt; exit 1; }
  tail -n 1 $O/pytest_$v.txt
done
for r in 1 2; do
  for v in ${AB:-0 2 4}; do
    ISAL_HIP_EXP_CRC2=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload crc64 > $O/b_crc64_${v}_r$r.json 2> $O/b.err || { echo FAIL $v; tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_crc64_${v}_r$r.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('crc64', 'exp=$v', 'round=$r', d['value'], d.get('ms_per_step'), r.get('frac'), d.get('self_check'))" | tee -a $O/ab.txt
  done
done
