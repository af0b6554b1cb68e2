#!/bin/bash
# r06z: the round's final evidence, one workload at a time in ONE session: its kernel
# trace and HBM-traffic passes, converted into profiles/r06/ (tools/profile_import.py),
# then its bench line, which cites those files. PART=a: GPU suite, smoke, C2 headline
# (with the CPU baseline); PART=b/c: the other workloads; PART=d: the C4 update again
# after its kernel changed; PART=e: full suite, smoke and the RAID-gen lines after theirs did;
# PART=f: the decode line again (kernel name now carries the lane count, as rocprofv3 prints it).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PART=${1:-a}
O=gpurun_out/r06z$PART; mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
one() {  # NAME WORKLOAD ARGS...
  local name=$1 wl=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$name -o t -- $B --workload $wl "$@" > $O/trbench_$name.json 2>> $O/log.txt || { echo FAIL tr $name; tail $O/log.txt; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$name -o p -- $B --workload $wl "$@" --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL fetch $name; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$name -o p -- $B --workload $wl "$@" --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL write $name; return 1; }
  python3 tools/profile_import.py $name $wl $O r06 --workload $wl "$@" >> $O/log.txt 2>&1 || { echo FAIL import $name; tail $O/log.txt; return 1; }
  if [ $name = c2 ]; then BL="python3 bench.py"; else BL=$B; fi
  timeout -k 10 600 $BL --workload $wl "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { echo FAIL bench $name; tail $O/bench_$name.err; return 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$name.json') if l.startswith('{')][-1]); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['frac'], r.get('profile_launch_ms'), r.get('kernel_stats_source'), r.get('traffic'), r.get('traffic_source'))"
}
if [ $PART = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
  tail -3 $O/pytest.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
  tail -2 $O/smoke.txt
  one c2 encode || exit 1
elif [ $PART = b ]; then
  one c3 decode || exit 1
  one c4 update --k 20 --p 6 --len 4194304 --stripes 64 || exit 1
  one k10p6 encode --k 10 --p 6 || exit 1
  one k10p8 encode --k 10 --p 8 || exit 1
  one k16p8 encode --k 16 --p 8 --len 1048576 --stripes 512 || exit 1
  one k20p6 encode --k 20 --p 6 --len 4194304 --stripes 64 || exit 1
  one k20p8 encode --k 20 --p 8 --len 4194304 --stripes 64 || exit 1
elif [ $PART = e ]; then  # after the 128-lane encode for 1-2 row passes: full suite, smoke, RAID-gen lines
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
  tail -3 $O/pytest.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
  one pq_gen pq_gen || exit 1
  one xor_gen xor_gen || exit 1
elif [ $PART = f ]; then  # the decode again after the v16 kernels gained their lane-count template argument
  one c3 decode || exit 1
elif [ $PART = d ]; then  # after the 128-lane update kernel
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "update or selftest or c4 or pipe" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
  tail -1 $O/pytest.txt
  one c4 update --k 20 --p 6 --len 4194304 --stripes 64 || exit 1
else
  one pq_gen pq_gen || exit 1
  one xor_gen xor_gen || exit 1
  one pq_check pq_check || exit 1
  one crc crc || exit 1
  one crc64 crc64 || exit 1
  one encrc encode-crc || exit 1
  one encrc64 encode-crc64 || exit 1
  timeout -k 10 300 $B --workload dropin > $O/bench_dropin.json 2> $O/bench_dropin.err || { echo FAIL dropin; tail $O/bench_dropin.err; exit 1; }
  tail -c 400 $O/bench_dropin.json
fi
echo done
