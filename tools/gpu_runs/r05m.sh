# Final-tree bench lines for every workload (headline with the CPU baseline on
# the usable cores), the encode memory skeletons on the same box, and rocprof
# traces + HBM traffic of the RAID kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05m}; mkdir -p $O
B="python3 bench.py"
timeout -k 10 600 $B > $O/bench_c2.json 2> $O/bench_c2.err || { echo FAIL c2; tail $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 300 python3 tools/skel_probe.py 10 > $O/skel_probe.jsonl 2> $O/skel_probe.err || { echo SKEL FAIL; tail $O/skel_probe.err; exit 1; }
while read name args; do
  timeout -k 10 300 $B --no-cpu-baseline $args > $O/bench_$name.json 2> $O/bench_$name.err || { echo FAIL $name; tail $O/bench_$name.err; exit 1; }
done <<'LIST'
decode --workload decode
update --workload update --k 20 --p 6 --len 4194304 --stripes 64
k10p6 --k 10 --p 6
k10p8 --k 10 --p 8
k20p6 --k 20 --p 6 --len 4194304 --stripes 64
k20p8 --k 20 --p 8 --len 4194304 --stripes 64
pq_gen --workload pq_gen
xor_gen --workload xor_gen
pq_check --workload pq_check
encrc --workload encode-crc
encrc64 --workload encode-crc64
crc --workload crc
crc64 --workload crc64
dropin --workload dropin
LIST
while read name args; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$name -o t -- $B --no-cpu-baseline $args >> $O/log.txt 2>&1 || { echo FAIL tr $name; tail $O/log.txt; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$name -o p -- $B --no-cpu-baseline $args --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL fetch $name; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$name -o p -- $B --no-cpu-baseline $args --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL write $name; exit 1; }
done <<'LIST'
pq_gen --workload pq_gen
xor_gen --workload xor_gen
pq_check --workload pq_check
LIST
for f in $O/bench_*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('kernel'), d['self_check'])")"; done
