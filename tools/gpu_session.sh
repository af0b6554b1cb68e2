#!/bin/bash
# One GPU-box session: parity tests, benches, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_session.sh TAG [steps...]
#   steps: tests bench crc prof pmc decode update e2e probe
# Every GPU step runs under its own timeout and the chain stops at the first
# failure; outputs land in gpurun_out/TAG/.
# Round 6 pruned the A/B steps whose variant knobs round 5 removed (their
# arms would now run the same kernel): hybrid pipe64 pipe32 prepipe pre8 order
# xcd encstore occ ldsmin updocc c2ab grid dropinspin crc64step slice64 fastcrc
# crcp prestand encrc64sweep crcstep. Their results stay in profiles/ and
# DESIGN.md §2b; tools/gpu_runs/ keeps the commands as they were run.
set -o pipefail
TAG=${1:-run}
shift
STEPS=${*:-tests bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1

run() {  # name seconds cmd...
        local name=$1 secs=$2
        shift 2
        echo "[$(date +%T)] $name: $*"
        timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
        local rc=$?
        tail -3 "$OUT/$name.log"
        if [ $rc -ne 0 ]; then
                echo "[$(date +%T)] $name FAILED rc=$rc"
                tail -40 "$OUT/$name.log"
                exit $rc
        fi
}

for s in $STEPS; do
        case $s in
        tests)
                run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread
                grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" "$OUT/pytest_gpu.log" > "$OUT/pytest_gpu_summary.txt" || true
                ;;
        benchtests)
                run pytest_gpu_bench 600 python -u -m pytest tests -m gpu -x -v -k "bench" --timeout 300 --timeout-method thread
                ;;
        stage)
                # how a synchronous host-resident call can move pageable shards (tools/stage_probe.c)
                run stage_probe 300 tools/stage_probe
                ;;
        tail)
                run pytest_gpu_tail 900 python -u -m pytest tests -m gpu -x -v -k "fuzz or bench or multi_device or pinned or hip_failure or large_host" --timeout 300 --timeout-method thread
                ;;
        faulttests)
                run pytest_gpu_fault 600 python -u -m pytest tests -m gpu -x -v -k "hip_failure or large_host_call or multi_device or pinned_host" --timeout 300 --timeout-method thread
                ;;
        fuzzgpu)
                # differential fuzzing of the shipped library on the kernels (tests/fuzz)
                python3 tests/fuzz/seeds.py diff "$OUT/fuzz_corpus" > /dev/null
                ISAL_HIP_BACKEND=gpu run fuzz_gpu 200 isa-l_amd/build/fuzzgpu/ec_diff_fuzz_gpu -max_total_time=90 -max_len=300000 -print_final_stats=1 -print_pcs=0 -rss_limit_mb=0 "$OUT/fuzz_corpus"
                rm -rf "$OUT/fuzz_corpus"
                ;;
        gpus2)
                # the driver's N>1 form on this one-GPU box: two gloo ranks share the GPU
                run bench_gpus2_gloo 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline
                ;;
        gpus8)
                # rehearsal of the driver's N=8 launch forms on this one-GPU box: eight gloo
                # ranks share the GPU (RCCL needs one GPU per rank), 128 stripes per rank
                run bench_gpus8_gloo 300 python bench.py --gpus 8 --dist-backend gloo --stripes 128 --no-cpu-baseline
                run bench_gpus4_torchrun_gloo 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --dist-backend gloo --stripes 128 --no-cpu-baseline
                run bench_c5_gpus8_gloo 300 python bench.py --gpus 8 --dist-backend gloo --total-stripes 8192 --stripes 128 --steps 2 --warmup 1 --no-cpu-baseline
                ;;
        steady)
                # C2 headline kernel: per-dispatch trace, steady-state average of the
                # K timed launches (tools/kernel_stats.py), beside the bench line
                run bench_c2 300 python bench.py --no-cpu-baseline
                cp "$OUT/bench_c2.log" "$OUT/bench_c2.json"
                run rocprof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python3 bench.py --no-cpu-baseline
                run steady_c2 60 python3 tools/kernel_stats.py "$OUT/prof_c2" "ec_encode_v16<4" --skip 5 --keep 20 --bytes 15032385536 --out "$OUT/c2_encode_kernel_steady.csv" --config "workload=encode k=10 p=4 len=1048576 stripes=1024" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline"
                ;;
        headline)
                # the round's headline evidence for one tree: C2 line (with the CPU
                # baseline), its rocprofv3 trace + steady-state summary, PMC traffic;
                # C3 decode the same way
                run bench_c2 300 python bench.py
                cp "$OUT/bench_c2.log" "$OUT/bench_c2.json"
                run rocprof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python3 bench.py --no-cpu-baseline
                run steady_c2 60 python3 tools/kernel_stats.py "$OUT/prof_c2" "ec_encode_v16<4" --skip 5 --keep 20 --bytes 15032385536 --out "$OUT/c2_encode_kernel_steady.csv" --config "workload=encode k=10 p=4 len=1048576 stripes=1024" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline"
                run pmc_fetch_c2 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c2" -o f -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1
                run pmc_write_c2 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_c2" -o w -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1
                python3 tools/pmc_csv.py "$OUT/pmc_c2_encode.csv" "workload=encode k=10 p=4 len=1048576 stripes=1024" "python bench.py --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_c2" "$OUT/pmc_write_c2" ec_encode_v16
                run pmc_sq_c2 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_sq_c2" -o s -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
                run bench_decode 300 python bench.py --workload decode --cpu-seconds 5
                cp "$OUT/bench_decode.log" "$OUT/bench_decode.json"
                run rocprof_decode 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_decode" -o decode -- python3 bench.py --workload decode --no-cpu-baseline
                run steady_decode 60 python3 tools/kernel_stats.py "$OUT/prof_decode" "ec_encode_v16<3" --skip 5 --keep 20 --bytes 13958643712 --out "$OUT/decode_encode_kernel_steady.csv" --config "workload=decode k=10 p=4 len=1048576 stripes=1024" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --workload decode --no-cpu-baseline"
                run pmc_fetch_decode 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_decode" -o f -- python3 bench.py --workload decode --no-cpu-baseline --steps 3 --warmup 1
                run pmc_write_decode 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_decode" -o w -- python3 bench.py --workload decode --no-cpu-baseline --steps 3 --warmup 1
                python3 tools/pmc_csv.py "$OUT/pmc_decode.csv" "workload=decode k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload decode --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_decode" "$OUT/pmc_write_decode" ec_encode_v16
                run bench_c2_final 300 python bench.py --no-cpu-baseline
                cp "$OUT/bench_c2_final.log" "$OUT/bench_c2_final.json"
                ;;
        wide)
                # wide-stripe encode: device-resident shapes beyond C2's p = 4
                for shape in ${WIDE_SHAPES:-"20 6 4194304 64" "10 8 1048576 1024" "10 6 1048576 1024" "10 4 1048576 1024"}; do
                        set -- ${shape//_/ }
                        tag=k$1p$2
                        args="--workload encode --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline"
                        bytes=$(( ($1 + $2) * $3 * $4 ))
                        run bench_$tag 300 python bench.py $args
                        cp "$OUT/bench_$tag.log" "$OUT/bench_$tag.json"
                        run rocprof_$tag 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$tag" -o $tag -- python3 bench.py $args
                        run steady_$tag 60 python3 tools/kernel_stats.py "$OUT/prof_$tag" ec_encode_ --skip 5 --keep 20 --bytes $bytes --out "$OUT/${tag}_encode_kernel_steady.csv" --config "workload=encode k=$1 p=$2 len=$3 stripes=$4" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py $args"
                        run pmc_fetch_$tag 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$tag" -o f -- python3 bench.py $args --steps 3 --warmup 1
                        run pmc_write_$tag 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$tag" -o w -- python3 bench.py $args --steps 3 --warmup 1
                        python3 tools/pmc_csv.py "$OUT/pmc_$tag.csv" "workload=encode k=$1 p=$2 len=$3 stripes=$4" "python bench.py $args --steps 3 --warmup 1" "$OUT/pmc_fetch_$tag" "$OUT/pmc_write_$tag" ec_encode_
                        run pmc_sq_$tag 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_sq_$tag" -o s -- python3 bench.py $args --steps 2 --warmup 1
                done
                ;;
        xor)
                # encode 0/1 fast path (ISAL_HIP_ENC_XOR): parity tests, then A/B per shape
                run pytest_gpu_xor 600 python -u -m pytest tests -m gpu -x -v -k "xor_fast_path or config_c2 or random_shapes or raid or maximum_stripe" --timeout 300 --timeout-method thread
                for r in 1 2; do
                        for shape in ${XOR_SHAPES:-10_4_1048576_1024 20_6_4194304_64 10_8_1048576_1024 10_6_1048576_1024}; do
                                set -- ${shape//_/ }
                                for x in 0 1; do
                                        ISAL_HIP_ENC_XOR=$x run bench_k$1p$2_x${x}_r$r 300 python bench.py --workload encode --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline
                                done
                        done
                done
                ;;
        lds)
                # encode low table halves from LDS (ISAL_HIP_ENC_LDS): parity tests, then A/B per shape
                run pytest_gpu_lds 600 python -u -m pytest tests -m gpu -x -v -k "xor_fast_path or config_c2 or random_shapes or raid or maximum_stripe or decode" --timeout 300 --timeout-method thread
                for r in 1 2; do
                        for shape in ${XOR_SHAPES:-10_4_1048576_1024 20_6_4194304_64 10_8_1048576_1024 10_6_1048576_1024}; do
                                set -- ${shape//_/ }
                                for x in 0 1; do
                                        ISAL_HIP_ENC_LDS=$x run bench_k$1p$2_lds${x}_r$r 300 python bench.py --workload encode --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline
                                done
                        done
                done
                run bench_decode 300 python bench.py --workload decode --no-cpu-baseline
                ISAL_HIP_ENC_LDS=0 run bench_decode_lds0 300 python bench.py --workload decode --no-cpu-baseline
                ;;
        group)
                # encode load group forced (ISAL_HIP_ENC_GROUP) x LDS halves, wide shapes
                ISAL_HIP_ENC_GROUP=5 run pytest_gpu_group5 600 python -u -m pytest tests -m gpu -x -q -k "xor_fast_path or load_groups" --timeout 300 --timeout-method thread
                for r in 1 2; do
                        for v in ${GROUP_CASES:-10_8_1048576_1024_10_d 10_8_1048576_1024_5_d 10_8_1048576_1024_5_1 10_8_1048576_1024_10_1 20_6_4194304_64_10_d 20_6_4194304_64_5_d 20_6_4194304_64_4_d 10_4_1048576_1024_10_d 10_4_1048576_1024_5_d}; do
                                set -- ${v//_/ }
                                lds=$6; [ "$lds" = d ] && lds=
                                ISAL_HIP_ENC_GROUP=$5 ISAL_HIP_ENC_LDS=$lds run bench_k$1p$2_g$5_l$6_r$r 300 python bench.py --workload encode --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline
                        done
                done
                ;;
        narrow)
                # drop-in kernel-argument encode with 4-byte lanes (ISAL_HIP_KARG_NARROW) A/B
                run pytest_gpu_narrow 600 python -u -m pytest tests -m gpu -x -q -k "dropin or concurrent or golden or xor_fast_path" --timeout 300 --timeout-method thread
                for r in 1 2; do
                        for x in 0 1; do
                                for t in 1 4 16; do
                                        ISAL_HIP_KARG_NARROW=$x run dropin_n${x}_t${t}_r$r 120 tools/dropin_bench 10 4 1048576 64 $t 3
                                done
                                ISAL_HIP_KARG_NARROW=$x run dropin_n${x}_small_r$r 120 tools/dropin_bench 10 4 4096 64 1 3
                                ISAL_HIP_KARG_NARROW=$x run dropin_n${x}_4m_r$r 120 tools/dropin_bench 10 4 4194304 16 1 3
                        done
                done
                ;;
        wide5)
                # 6-8 row passes in load groups of 5 (ISAL_HIP_ENC_WIDE5) A/B
                run pytest_gpu_wide5 600 python -u -m pytest tests -m gpu -x -q -k "xor_fast_path or load_groups or random_shapes or maximum_stripe or decode" --timeout 300 --timeout-method thread
                for r in 1 2; do
                        for shape in ${WIDE5_SHAPES:-10_6_1048576_1024 10_7_1048576_1024 10_8_1048576_1024 20_6_4194304_64 20_8_4194304_64 15_6_1048576_1024 30_6_1048576_512}; do
                                set -- ${shape//_/ }
                                for x in 0 1; do
                                        ISAL_HIP_ENC_WIDE5=$x run bench_k$1p$2_w${x}_r$r 300 python bench.py --workload encode --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline
                                done
                        done
                done
                ;;
        labels)
                run pytest_gpu_labels 900 python -u -m pytest tests -m gpu -x -v -k "kernel_label or dropin_kernel_args or smoke" --timeout 300 --timeout-method thread
                ;;
        confirm)
                run pytest_gpu_confirm 600 python -u -m pytest tests -m gpu -x -q -k "xor_fast_path or load_groups or random_shapes or decode or raid or golden or kernel_label or smoke" --timeout 300 --timeout-method thread
                for w in "encode" "decode" "encode --k 20 --p 6 --len 4194304 --stripes 64" "encode --k 10 --p 2" "encode --k 10 --p 8"; do
                        tag=$(echo $w | tr -d ' -' | cut -c1-24)
                        run bench_${tag}_default 300 python bench.py --workload $w --no-cpu-baseline
                done
                ;;
        ldsinfo)
                run lds_info 60 python3 -c "import torch, ctypes; torch.zeros(1, device='cuda'); l = ctypes.CDLL('tools/libcopy_probe.so'); print('lds_per_cu', l.copy_probe_lds_per_cu()); [print('dyn', d, 'blocks_per_cu', l.copy_probe_blocks_per_cu(ctypes.c_ulonglong(d))) for d in (0, 16384, 22528, 27136, 32768, 40960, 65536)]"
                ;;
        fuzzrss)
                # the GPU differential fuzz target for 150 s with libFuzzer's 2 GiB RSS /
                # malloc bounds; its status lines log the process RSS over time
                mkdir -p "$OUT/fuzz_corpus" && python3 tests/fuzz/seeds.py diff "$OUT/fuzz_corpus" > /dev/null
                ISAL_HIP_BACKEND=gpu run fuzz_rss 240 isa-l_amd/build/fuzzgpu/ec_diff_fuzz_gpu -max_total_time=150 -max_len=300000 -print_final_stats=1 -rss_limit_mb=2048 -malloc_limit_mb=2048 -artifact_prefix="$OUT/" "$OUT/fuzz_corpus"
                grep -E "rss:|stat::" "$OUT/fuzz_rss.log" | tail -40 > "$OUT/fuzz_rss_summary.txt" || true
                rm -rf "$OUT/fuzz_corpus"
                ;;
        c5test)
                run pytest_gpu_c5 900 python -u -m pytest tests -m gpu -x -v -s -k "c5_full_workload or two_ranks_on_one_gpu" --timeout 800 --timeout-method thread
                ;;
        sqwide)
                # SQ counters of the wide encodes with and without LDS table halves
                for shape in ${SQ_SHAPES:-20_6_4194304_64 10_8_1048576_1024}; do
                        set -- ${shape//_/ }
                        for x in 0 1; do
                                ISAL_HIP_ENC_LDS=$x run pmc_sq_k$1p$2_lds$x 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_sq_k$1p$2_lds$x" -o s -- python3 bench.py --workload encode --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline --steps 2 --warmup 1
                        done
                done
                ;;
        dropintests)
                run pytest_gpu_dropin 600 python -u -m pytest tests -m gpu -x -v -k "dropin or concurrent or pinned or golden or device or xor_fast_path or smoke or raid" --timeout 300 --timeout-method thread
                ;;
        dropin)
                # the synchronous drop-in call on device-resident C2 stripes, 1/4/16 threads
                for t in 1 4 16; do
                        run dropin_t$t 120 tools/dropin_bench 10 4 1048576 64 $t 3
                done
                run dropin_small_t1 120 tools/dropin_bench 10 4 4096 64 1 3
                run bench_dropin 300 python bench.py --workload dropin
                ISAL_HIP_KARG=0 run bench_dropin_nokarg 300 python bench.py --workload dropin
                run dropin_hiptrace 200 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$OUT/prof_dropin" -o dropin -- tools/dropin_bench 10 4 1048576 64 1 0 400
                ;;
        tests_crc)
                run pytest_gpu_crc 300 python -u -m pytest tests -m gpu -x -v -k "crc" --timeout 200 --timeout-method thread
                ;;
        bench)
                run bench_c2 300 python bench.py
                cp "$OUT/bench_c2.log" "$OUT/bench_c2.json"
                ;;
        crc)
                run bench_encode_crc 300 python bench.py --workload encode-crc
                run bench_crc 300 python bench.py --workload crc --cpu-seconds 5
                ;;
        crc64)
                run pytest_gpu_crc64 300 python -u -m pytest tests -m gpu -x -v -k "crc64" --timeout 200 --timeout-method thread
                run bench_crc64 300 python bench.py --workload crc64 --cpu-seconds 5
                run rocprof_crc64 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_crc64" -o crc64 -- python3 bench.py --workload crc64 --no-cpu-baseline
                run pmc_fetch_crc64 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_crc64" -o f -- python3 bench.py --workload crc64 --no-cpu-baseline --steps 3 --warmup 1
                run pmc_write_crc64 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_crc64" -o w -- python3 bench.py --workload crc64 --no-cpu-baseline --steps 3 --warmup 1
                python3 tools/pmc_csv.py "$OUT/pmc_c2_crc64.csv" "workload=crc64 k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload crc64 --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_crc64" "$OUT/pmc_write_crc64" crc64_shards
                run pmc_lds_crc64 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$OUT/pmc_lds_crc64" -o l -- python3 bench.py --workload crc64 --no-cpu-baseline --steps 2 --warmup 1
                ;;
        encrc64)
                run pytest_gpu_encrc64 300 python -u -m pytest tests -m gpu -x -v -k "encode_crc64" --timeout 200 --timeout-method thread
                run bench_encode_crc64 300 python bench.py --workload encode-crc64 --cpu-seconds 5
                run rocprof_encrc64 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_encrc64" -o encrc64 -- python3 bench.py --workload encode-crc64 --no-cpu-baseline
                run pmc_fetch_encrc64 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_encrc64" -o f -- python3 bench.py --workload encode-crc64 --no-cpu-baseline --steps 3 --warmup 1
                run pmc_write_encrc64 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_encrc64" -o w -- python3 bench.py --workload encode-crc64 --no-cpu-baseline --steps 3 --warmup 1
                python3 tools/pmc_csv.py "$OUT/pmc_c2_encode_crc64.csv" "workload=encode-crc64 k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload encode-crc64 --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_encrc64" "$OUT/pmc_write_encrc64" ec_encode_crc64_v16
                ;;
        abprev)
                # A/B against the previous build kept at isa-l_amd/lib/prev (same box)
                run pytest_gpu_crc 700 python -u -m pytest tests -m gpu -x -v -k "crc" --timeout 200 --timeout-method thread
                for wl in encode-crc encode-crc64; do
                        for r in 1 2; do
                                ISAL_HIP_LIB=isa-l_amd/lib/prev/libisal_hip.so run bench_${wl}_prev$r 300 python bench.py --workload $wl --no-cpu-baseline
                                run bench_${wl}_new$r 300 python bench.py --workload $wl --no-cpu-baseline
                        done
                done
                ;;
        crctt)
                # checksum-only kernels: tiles per workgroup now that they are memory-side bound
                for tt in ${TT_LIST:-16 32 64 128}; do
                        for wl in crc crc64 encode-crc encode-crc64; do
                                ISAL_HIP_CRC_TILES=$tt run bench_${wl}_tt$tt 300 python bench.py --workload $wl --no-cpu-baseline
                        done
                done
                ;;
        smoke)
                run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
                ;;
        memprobe)
                # memory-only kernels with the encode addressing: C2 (10 read + 4 write) and C3 decode (10 + 3)
                run probe_c2 300 isa-l_amd/build/ec_probe 10 4 1048576 1024 5
                run probe_c3 300 isa-l_amd/build/ec_probe 10 3 1048576 1024 5
                ;;
        fusedprof)
                # kernel stats of the fused encode+CRC kernels (default paths) for the roofline lines
                run rocprof_encrc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_encrc" -o encrc -- python3 bench.py --workload encode-crc --no-cpu-baseline
                run rocprof_encrc64 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_encrc64" -o encrc64 -- python3 bench.py --workload encode-crc64 --no-cpu-baseline
                for wl in encode-crc encode-crc64; do
                        run pmc_fetch_$wl 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$wl" -o f -- python3 bench.py --workload $wl --no-cpu-baseline --steps 3 --warmup 1
                        run pmc_write_$wl 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$wl" -o w -- python3 bench.py --workload $wl --no-cpu-baseline --steps 3 --warmup 1
                done
                python3 tools/pmc_csv.py "$OUT/pmc_c2_encode_crc.csv" "workload=encode-crc k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload encode-crc --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_encode-crc" "$OUT/pmc_write_encode-crc" ec_encode_crc_v16
                python3 tools/pmc_csv.py "$OUT/pmc_c2_encode_crc64.csv" "workload=encode-crc64 k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload encode-crc64 --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_encode-crc64" "$OUT/pmc_write_encode-crc64" ec_encode_crc64_v16
                run bench_encode_crc 300 python bench.py --workload encode-crc --cpu-seconds 5
                run bench_encode_crc64 300 python bench.py --workload encode-crc64 --cpu-seconds 5
                ;;
        decode)
                run bench_decode 300 python bench.py --workload decode --no-cpu-baseline
                ;;
        update)
                run bench_update 300 python bench.py --workload update --k 20 --p 6 --len 4194304 --stripes 64 --no-cpu-baseline
                ;;
        e2e)
                run bench_e2e_update 300 python bench.py --workload e2e-update --k 20 --p 6 --len 4194304 --steps 40 --warmup 4
                run bench_e2e_encode 300 python bench.py --workload e2e-encode --steps 200 --warmup 10
                ;;
        prof)
                run rocprof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python3 bench.py --no-cpu-baseline
                cp "$OUT/rocprof_c2.log" "$OUT/bench_c2_under_rocprof.log"
                run rocprof_crc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_crc" -o crc -- python3 bench.py --workload encode-crc --no-cpu-baseline
                run rocprof_crconly 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_crconly" -o crconly -- python3 bench.py --workload crc --no-cpu-baseline
                ;;
        pmc)
                for wl in encode encode-crc crc; do
                        run pmc_fetch_$wl 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$wl" -o f -- python3 bench.py --workload $wl --no-cpu-baseline --steps 3 --warmup 1
                        run pmc_write_$wl 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$wl" -o w -- python3 bench.py --workload $wl --no-cpu-baseline --steps 3 --warmup 1
                done
                python3 tools/pmc_csv.py "$OUT/pmc_c2_encode.csv" "workload=encode k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload encode --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_encode" "$OUT/pmc_write_encode" ec_encode_v16
                python3 tools/pmc_csv.py "$OUT/pmc_c2_encode_crc.csv" "workload=encode-crc k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload encode-crc --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_encode-crc" "$OUT/pmc_write_encode-crc" ec_encode_crc_v16
                python3 tools/pmc_csv.py "$OUT/pmc_c2_crc.csv" "workload=crc k=10 p=4 len=1048576 stripes=1024" "python bench.py --workload crc --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_crc" "$OUT/pmc_write_crc" crc32c_shards
                ;;
        pmc_lds)
                # LDS bank conflicts / VALU pressure of the CRC kernels (one SQ pass each)
                for wl in ${PMC_WORKLOADS:-crc encode-crc encode}; do
                        run pmc_lds_$wl 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$OUT/pmc_lds_$wl" -o l -- python3 bench.py --workload $wl --no-cpu-baseline --steps 2 --warmup 1
                        run pmc_wait_$wl 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INST_CYCLES_VMEM --output-format csv -d "$OUT/pmc_wait_$wl" -o w -- python3 bench.py --workload $wl --no-cpu-baseline --steps 2 --warmup 1
                done
                ;;
        probe)
                run probe 300 isa-l_amd/build/ec_probe
                ;;
        valu)
                # issue rate of v_perm / v_bitop3 / SDWA shifts vs v_add, random ds_read_b64 (tools/valu_probe.hip)
                for w in 2 4 8; do
                        run valu_probe_w$w 120 tools/valu_probe $w
                done
                ;;
        refcpu)
                # the reference's own perf harnesses on the host cores (no GPU)
                run refcpu_encode 200 python3 tools/cpu_ref_baseline.py --which encode
                cp "$OUT/refcpu_encode.log" "$OUT/refcpu_encode.json"
                run refcpu_update 300 python3 tools/cpu_ref_baseline.py --which update
                cp "$OUT/refcpu_update.log" "$OUT/refcpu_update.json"
                ;;
        decodeprof|updateprof)
                if [ $s = decodeprof ]; then
                        wl=decode; args="--workload decode"; kern=ec_encode_v16; cfg="workload=decode k=10 p=4 len=1048576 stripes=1024"
                else
                        wl=update; args="--workload update --k 20 --p 6 --len 4194304 --stripes 64"; kern=ec_update_v16; cfg="workload=update k=20 p=6 len=4194304 stripes=64"
                fi
                run bench_$wl 300 python bench.py $args --cpu-seconds 5
                cp "$OUT/bench_$wl.log" "$OUT/bench_$wl.json"
                run rocprof_$wl 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$wl" -o $wl -- python3 bench.py $args --no-cpu-baseline
                if [ $s = updateprof ]; then
                        run steady_$wl 60 python3 tools/kernel_stats.py "$OUT/prof_$wl" "ec_update_v16<6>" --skip 5 --keep 20 --bytes 3489660928 --out "$OUT/update_update_kernel_steady.csv" --config "$cfg" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py $args --no-cpu-baseline"
                fi
                run pmc_fetch_$wl 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$wl" -o f -- python3 bench.py $args --no-cpu-baseline --steps 3 --warmup 1
                run pmc_write_$wl 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$wl" -o w -- python3 bench.py $args --no-cpu-baseline --steps 3 --warmup 1
                python3 tools/pmc_csv.py "$OUT/pmc_$wl.csv" "$cfg" "python bench.py $args --steps 3 --warmup 1 --no-cpu-baseline" "$OUT/pmc_fetch_$wl" "$OUT/pmc_write_$wl" $kern
                ;;
        c5)
                run bench_c5 600 python bench.py --total-stripes 1048576 --steps 2 --warmup 1
                cp "$OUT/bench_c5.log" "$OUT/bench_c5.json"
                ;;
        c1)
                run bench_c1 120 python bench.py --workload c1
                ;;
        zc)
                run zc_probe 300 python tools/zc_probe.py
                ;;
        calltrace)
                run calltrace 300 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d "$OUT/calltrace" -o t -- python3 tools/host_call_trace.py
                ;;
        chunks)
                run chunk_sweep 300 python tools/chunk_sweep.py
                ;;
        route)
                run route_crossover 300 python tools/route_crossover.py
                run latency_probe 120 python tools/latency_probe.py
                ;;
        crcbench)
                for wl in encode-crc encode-crc64 crc crc64; do
                        run bench_$wl 300 python bench.py --workload $wl --no-cpu-baseline
                done
                ;;
        ttsweep)
                for tt in ${TT_LIST:-8 16 32 64}; do
                        for wl in encode-crc64 encode-crc crc64; do
                                ISAL_HIP_CRC_TILES=$tt run bench_${wl}_tt$tt 300 python bench.py --workload $wl --no-cpu-baseline
                        done
                done
                ;;
        e2etrace)
                for dp in 2 6; do
                        run e2etrace_d$dp 300 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d "$OUT/e2etrace_d$dp" -o t -- python3 bench.py --workload e2e-encode --steps 100 --warmup 10 --depth $dp
                done
                ;;
        e2ering)
                for dr in 2:4 2:12 6:6 6:12 3:3; do
                        run bench_e2e_encode_d${dr%:*}_r${dr#*:} 300 python bench.py --workload e2e-encode --steps 200 --warmup 10 --depth ${dr%:*} --ring ${dr#*:}
                done
                ;;
        e2esweep)
                for dp in ${E2E_DEPTHS:-2 3 4 6}; do
                        run bench_e2e_encode_d$dp 300 python bench.py --workload e2e-encode --steps 200 --warmup 10 --depth $dp
                done
                ;;
        *)
                echo "unknown step $s"
                exit 2
                ;;
        esac
done
echo "[$(date +%T)] session $TAG done"
