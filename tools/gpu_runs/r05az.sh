# CRC64 checksum-only (two chains per lane) and fused encode + CRC64: tiles
# per item (ISAL_HIP_CRC_TILES; 64 = default), same box, two interleaved
# rounds. OUT= / TILES= / WL= (workloads) override.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05az}; mkdir -p $O
for r in 1 2; do
  for wl in ${WL:-crc64}; do
  for tt in ${TILES:-64 32 128 256}; do
    ISAL_HIP_CRC_TILES=$tt timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $wl > $O/b_${wl}_tt${tt}_r$r.json 2> $O/b.err || { echo FAIL $tt; tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${wl}_tt${tt}_r$r.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$wl', 'tiles=$tt', 'round=$r', d['value'], d.get('ms_per_step'), r.get('frac'), d.get('self_check'))" | tee -a $O/ab.txt
  done
  done
done
