#!/usr/bin/env python3
"""Where the drop-in call's CPU route stops paying (GPU box diagnostic).

Times one synchronous ec_encode_data call on HOST-resident shards (k=10, p=4,
plain pageable numpy buffers — what a storage daemon hands the reference) at
shard lengths from 1 KiB to 16 MiB, forced onto the CPU route
(ISAL_HIP_BACKEND=cpu, up to 4 MiB) and onto the GPU (=gpu), and prints the per-call times
and the byte count (k + p) * len where the GPU starts to win. That count is
DEFAULT_CPU_MAX_BYTES in isal_hip_shim.c. Also times hipPointerGetAttributes,
the per-pointer classification cost every routed call pays. From 1 MiB shards on
it also times the chunked GPU route one chunk at a time
(ISAL_HIP_PIPE_CHUNKS=0, the round-2 behaviour) and with page-locked buffers.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch's)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "isa-l_amd"))
import isal_amd  # noqa: E402


def per_call(k, p, n, backend, budget=0.5, piped="1", pinned=False):
    os.environ["ISAL_HIP_BACKEND"] = backend
    os.environ["ISAL_HIP_PIPE_CHUNKS"] = piped
    isal_amd.reload_config()
    rng = np.random.default_rng(n)
    if pinned:  # page-locked host buffers (torch pin_memory = hipHostMalloc)
        src = [torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).pin_memory().numpy() for _ in range(k)]
        dst = [torch.zeros(n, dtype=torch.uint8).pin_memory().numpy() for _ in range(p)]
    else:
        src = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
        dst = [np.zeros(n, np.uint8) for _ in range(p)]
    a = isal_amd.gf_gen_rs_matrix(k + p, k)
    tbls = isal_amd.ec_init_tables(k, p, a[k * k:])
    L = isal_amd.lib()
    sp, dp = isal_amd._pp(src), isal_amd._pp(dst)
    tp = isal_amd._p(tbls)
    L.ec_encode_data(n, k, p, tp, sp, dp)  # warm (staging buffers, streams)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget or reps < 3:
        L.ec_encode_data(n, k, p, tp, sp, dp)
        reps += 1
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    k, p = 10, 4
    rows = []
    crossover = pinned_crossover = None
    for n in [1 << e for e in range(10, 25)]:
        cpu = per_call(k, p, n, "cpu") if n <= 1 << 22 else None
        gpu = per_call(k, p, n, "gpu")
        row = {"len": n, "bytes": (k + p) * n, "cpu_us": cpu and round(cpu, 1), "gpu_us": round(gpu, 1)}
        # page-locked buffers: the kernels use them in place (no staging copy)
        row["gpu_pinned_us"] = round(per_call(k, p, n, "gpu", pinned=True), 1)
        row["gpu_pinned_gb_s"] = round((k + p) * n / row["gpu_pinned_us"] / 1e3, 2)
        if n >= 1 << 20:  # the chunked route: pipelined (default) vs one chunk at a time
            row["gpu_unpipelined_us"] = round(per_call(k, p, n, "gpu", piped="0"), 1)
            os.environ["ISAL_HIP_PAR_COPY"] = "0"  # one thread issues every copy (round-2 behaviour)
            row["gpu_one_thread_us"] = round(per_call(k, p, n, "gpu", piped="0"), 1)
            os.environ["ISAL_HIP_PAR_COPY"] = ""
            row["gpu_gb_s"] = round((k + p) * n / gpu / 1e3, 2)
        if pinned_crossover is None and cpu is not None and row["gpu_pinned_us"] < cpu:
            pinned_crossover = (k + p) * n
        rows.append(row)
        print(json.dumps(rows[-1]), flush=True)
        if crossover is None and cpu is not None and gpu < cpu:
            crossover = (k + p) * n
    hip = ctypes.CDLL("libamdhip64.so")
    attr = ctypes.create_string_buffer(64)
    buf = np.zeros(4096, np.uint8)
    t0 = time.perf_counter()
    for _ in range(20000):
        hip.hipPointerGetAttributes(attr, ctypes.c_void_p(buf.ctypes.data))
    cls = (time.perf_counter() - t0) / 20000 * 1e6
    print(json.dumps({"first_len_where_gpu_wins_bytes": crossover,
                      "first_len_where_gpu_wins_pinned_bytes": pinned_crossover,
                      "hipPointerGetAttributes_host_us": round(cls, 2)}), flush=True)


if __name__ == "__main__":
    main()
