# SQ counters of the xor_gen encode vs its memory skeleton (one pass each).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05af; mkdir -p $O
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_xor -o p -- python3 bench.py --no-cpu-baseline --workload xor_gen --steps 2 --warmup 1 > $O/log.txt 2>&1 || { echo FAIL xor; tail $O/log.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_skel -o p -- python3 tools/skel_probe.py 2 xor_gen >> $O/log.txt 2>&1 || { echo FAIL skel; tail $O/log.txt; exit 1; }
python3 tools/pmc_summary.py $O/sq_xor > $O/sq_xor.txt && python3 tools/pmc_summary.py $O/sq_skel > $O/sq_skel.txt
grep -A9 "ec_encode_v16<1" $O/sq_xor.txt; grep -A9 "skel_tiles" $O/sq_skel.txt
