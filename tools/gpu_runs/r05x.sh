# Fused encode + CRC32C: 4 waves/SIMD with 4 VGPRs spilled (shipped) vs 3
# waves without spills; two interleaved rounds. Then the CRC32C checksum-only
# kernel (batch 4) re-profiled: steady trace + HBM traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
for r in 1 2; do
  for cfg in "w4:$PWD/isa-l_amd/lib/libisal_hip.so" "w3:$PWD/isa-l_amd/build/ab_w3/libisal_hip.so"; do
    name=${cfg%%:*}; lib=${cfg#*:}
    ISAL_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload encode-crc > $O/b_${r}_${name}.json 2> $O/b_${r}_${name}.err || { echo FAIL $name; tail $O/b_${r}_${name}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${r}_${name}.json').read().strip().splitlines()[-1]); print('r$r $name encode-crc', d['value'], d['roofline']['frac'], d['roofline']['launch_ms'], d['self_check'])" | tee -a $O/ab.txt
  done
done
B="python3 bench.py --no-cpu-baseline --workload crc"
timeout -k 10 300 $B > $O/bench_crc.json 2> $O/bench_crc.err || { echo FAIL crc bench; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_crc -o t -- $B >> $O/log.txt 2>&1 || { echo FAIL tr; tail $O/log.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_crc -o p -- $B --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL fetch; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_crc -o p -- $B --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL write; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_crc.json').read().strip().splitlines()[-1]); print('crc', d['value'], d['roofline']['frac'], d['self_check'])"
