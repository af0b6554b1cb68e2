# Counters + steady-state traces: fused encode+CRC64 formulations (before the
# round-5 pruning removes the field/hybrid variants), CRC64-only, C2 encode,
# k20p6 (default, LDS-DMA ring of 4), RAID workloads' HBM traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
B="python3 bench.py --no-cpu-baseline"
run() {  # name timeout env... -- cmd
  local name=$1 t=$2; shift 2
  echo "== $name" >> $O/log.txt
  env "$@" >> $O/log.txt 2>&1 || { echo "FAIL $name"; tail -20 $O/log.txt; exit 1; }
}
for cfg in "sl3:ISAL_HIP_CRC64_SLICE=3" "sl1:ISAL_HIP_CRC64_SLICE=1" "sl0:ISAL_HIP_CRC64_SLICE=0"; do
  n=${cfg%%:*}; e=${cfg#*:}
  run pmc_$n 120 $e timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_encrc64_$n -o p -- $B --workload encode-crc64 --steps 2 --warmup 1
  run tr_$n 300 $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_encrc64_$n -o t -- $B --workload encode-crc64
done
run pmc_crc64 120 X=1 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_crc64 -o p -- $B --workload crc64 --steps 2 --warmup 1
run tr_crc64 300 X=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_crc64 -o t -- $B --workload crc64
run pmc_c2 120 X=1 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_c2 -o p -- $B --steps 2 --warmup 1
run pmc_encrc 120 X=1 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_encrc -o p -- $B --workload encode-crc --steps 2 --warmup 1
run tr_encrc 300 X=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_encrc -o t -- $B --workload encode-crc
for g in 0 4; do
  run pmc_k20p6_g$g 120 ISAL_HIP_ENC_GLDS=$g timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_k20p6_g$g -o p -- $B --k 20 --p 6 --len 4194304 --stripes 64 --steps 2 --warmup 1
done
for w in pq_gen xor_gen pq_check; do
  run fetch_$w 120 X=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$w -o p -- $B --workload $w --steps 2 --warmup 1
  run write_$w 120 X=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$w -o p -- $B --workload $w --steps 2 --warmup 1
  run tr_$w 300 X=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$w -o t -- $B --workload $w
done
python3 tools/pmc_summary.py $O/pmc_encrc64_sl3 $O/pmc_encrc64_sl1 $O/pmc_encrc64_sl0 $O/pmc_crc64 $O/pmc_c2 $O/pmc_encrc $O/pmc_k20p6_g0 $O/pmc_k20p6_g4 > $O/sq_summary.txt
cat $O/sq_summary.txt
