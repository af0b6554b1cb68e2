# Separate CRC64 block geometry per pass (checksum-only 128 tiles, fused 64):
# every CRC test, then default vs ISAL_HIP_CRC_TILES=64 (the previous shared
# geometry), same box, two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05bb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "crc" > $O/pytest_crc.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_crc.txt; exit 1; }
tail -n 1 $O/pytest_crc.txt
for r in 1 2; do
  for wl in crc64 encode-crc64; do
    for v in default 64; do
      if [ $v = 64 ]; then export ISAL_HIP_CRC_TILES=64; else unset ISAL_HIP_CRC_TILES; fi
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $wl > $O/b_${wl}_${v}_r$r.json 2> $O/b.err || { echo FAIL $wl $v; tail $O/b.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${wl}_${v}_r$r.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$wl', 'tiles=$v', 'round=$r', d['value'], d.get('ms_per_step'), r.get('frac'), d.get('self_check'))" | tee -a $O/ab.txt
    done
  done
done
unset ISAL_HIP_CRC_TILES
