# CRC64 checksum-only with two interleaved chains per lane (the new default):
# every CRC test, the bench line, its steady-state trace and HBM traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05av; mkdir -p $O
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "crc" > $O/pytest_crc.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_crc.txt; exit 1; }
tail -n 1 $O/pytest_crc.txt
timeout -k 10 300 $B --workload crc64 > $O/bench_crc64.json 2> $O/bench.err || { echo BENCH FAIL; tail $O/bench.err; exit 1; }
cat $O/bench_crc64.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_crc64 -o t -- $B --workload crc64 > $O/log.txt 2>&1 || { echo FAIL tr; tail $O/log.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_crc64 -o p -- $B --workload crc64 --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL fetch; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_crc64 -o p -- $B --workload crc64 --steps 2 --warmup 1 >> $O/log.txt 2>&1 || { echo FAIL write; exit 1; }
python3 tools/kernel_stats.py $O/tr_crc64 crc64_shards_pre --skip 5 --keep 20 --bytes 15032385536 --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --no-cpu-baseline --workload crc64" --out $O/crc64_kernel_steady.csv --trace-out $O/crc64_kernel_trace.csv
