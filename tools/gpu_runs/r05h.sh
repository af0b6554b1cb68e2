# Fused encode + CRC64: pre-shifted 5-bit field tables (SL 4) vs the default
# byte tables pipelined into the GF rows (SL 3): parity, same-box A/B, trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
ISAL_HIP_CRC64_SLICE=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "encode_crc64" > $O/pytest_sl4.txt 2>&1 || { echo PYTEST FAIL; grep -v "^  File" $O/pytest_sl4.txt | tail -30; exit 1; }
tail -2 $O/pytest_sl4.txt
for r in 1 2 3; do
  for sl in 3 4; do
    ISAL_HIP_CRC64_SLICE=$sl timeout -k 10 300 python bench.py --workload encode-crc64 --no-cpu-baseline > $O/b.json 2>$O/b.err || { echo BENCH FAIL; tail $O/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b.json')); r=d['roofline']
print(json.dumps({'round':$r,'slice':$sl,'frac':r['frac'],'launch_ms':r['launch_ms'],'ms_per_step':d['ms_per_step'],'kernel':r['kernel'],'self_check':d['self_check']}))" >> $O/ab.jsonl
  done
done
for k in 8 20; do
  for sl in 3 4; do
    ISAL_HIP_CRC64_SLICE=$sl timeout -k 10 300 python bench.py --workload encode-crc64 --k $k --no-cpu-baseline > $O/b.json 2>$O/b.err || { echo BENCH FAIL; tail $O/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b.json')); r=d['roofline']
print(json.dumps({'k':$k,'slice':$sl,'frac':r['frac'],'launch_ms':r['launch_ms'],'kernel':r['kernel'],'self_check':d['self_check']}))" >> $O/ab.jsonl
  done
done
ISAL_HIP_CRC64_SLICE=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_sl4 -o t -- python3 bench.py --workload encode-crc64 --no-cpu-baseline > $O/tr.log 2>&1 || exit 1
ISAL_HIP_CRC64_SLICE=4 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/pmc_sl4 -o p -- python3 bench.py --workload encode-crc64 --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/pmc_sl4 > $O/sq_sl4.txt
cat $O/ab.jsonl
