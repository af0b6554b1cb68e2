# Round-5 profiles of the shipped tree: steady-state traces (+ --stats
# summaries), HBM traffic and SQ counters of the main shapes; first-call cost.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for i in 1 2 3; do timeout -k 10 60 tools/first_call isa-l_amd/lib/libisal_hip.so 10 4 1048576 >> $O/first_call.jsonl 2>&1 || exit 1; done
while read name args; do
  echo "== $name" >> $O/log.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$name -o t -- $B $args >> $O/log.txt 2>&1 || { echo FAIL tr $name; tail $O/log.txt; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$name -o p -- $B $args --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL fetch $name; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$name -o p -- $B $args --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL write $name; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_$name -o p -- $B $args --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL sq $name; exit 1; }
done <<'LIST'
c2 --workload encode
c3 --workload decode
c4 --workload update --k 20 --p 6 --len 4194304 --stripes 64
k10p6 --k 10 --p 6
k10p8 --k 10 --p 8
k20p6 --k 20 --p 6 --len 4194304 --stripes 64
k20p8 --k 20 --p 8 --len 4194304 --stripes 64
encrc --workload encode-crc
encrc64 --workload encode-crc64
crc --workload crc
crc64 --workload crc64
LIST
python3 tools/pmc_summary.py $O/sq_* > $O/sq_summary.txt
cat $O/first_call.jsonl
