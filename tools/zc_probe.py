#!/usr/bin/env python3
"""Zero-copy encode of host-resident stripes (GPU box diagnostic).

The encode kernel reads its k sources from, and writes its p parity rows to,
page-locked host memory directly over PCIe (no staging copies): reads and
writes use the two directions of the link at once. Times one k=10 p=4
stripe per launch for 1-16 MiB shards on
  * hipHostMalloc'd buffers (torch pin_memory),
  * pageable numpy buffers registered per call with hipHostRegister (and
    unregistered after it: what a drop-in call on a caller's pageable
    buffers would have to do), and the registration cost alone,
and prints GB/s of (k + p) * len.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "isa-l_amd"))
import isal_amd  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]


def timed(fn, budget=0.3):
    fn()
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget or n < 3:
        fn()
        n += 1
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    k, p = 10, 4
    a = isal_amd.gf_gen_rs_matrix(k + p, k)
    tbls = isal_amd.ec_init_tables(k, p, a[k * k:])
    torch.cuda.init()
    h = torch.cuda.current_stream().cuda_stream
    for n in (1 << 20, 2 << 20, 4 << 20, 16 << 20):
        src = [torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory() for _ in range(k)]
        dst = [torch.zeros(n, dtype=torch.uint8).pin_memory() for _ in range(p)]
        dev = []
        for x in src + dst:  # the device's view of each page-locked buffer
            d = ctypes.c_void_p()
            assert hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(int(x.data_ptr())), 0) == 0
            dev.append(d.value)
        b = isal_amd.Batch(n, k, p, tbls, 1, dev[:k], dev[k:])

        def run():
            b.encode(h)
            torch.cuda.current_stream().synchronize()

        us = timed(run)
        want = [np.zeros(n, np.uint8) for _ in range(p)]
        isal_amd.ec_encode_data(n, k, p, tbls, [x.numpy() for x in src], want)  # engine, staged path
        ok = all(np.array_equal(dst[l].numpy(), want[l]) for l in range(p))
        b.close()
        row = {"len": n, "pinned_zc_us": round(us, 1), "pinned_zc_gb_s": round((k + p) * n / us / 1e3, 2),
               "parity_ok": ok}
        # pageable buffers registered for the call
        psrc = [x.numpy().copy() for x in src]  # pageable copies
        pdst = [np.zeros(n, np.uint8) for _ in range(p)]
        bufs = psrc + pdst

        def reg_call():
            devs = []
            for x in bufs:
                assert hip.hipHostRegister(x.ctypes.data, n, 2) == 0  # hipHostRegisterMapped
                d = ctypes.c_void_p()
                assert hip.hipHostGetDevicePointer(ctypes.byref(d), x.ctypes.data, 0) == 0
                devs.append(d.value)
            bb = isal_amd.Batch(n, k, p, tbls, 1, devs[:k], devs[k:])
            bb.encode(h)
            torch.cuda.current_stream().synchronize()
            bb.close()
            for x in bufs:
                hip.hipHostUnregister(x.ctypes.data)

        def reg_only():
            for x in bufs:
                hip.hipHostRegister(x.ctypes.data, n, 2)
            for x in bufs:
                hip.hipHostUnregister(x.ctypes.data)

        us2 = timed(reg_call)
        ok2 = all(np.array_equal(pdst[l], want[l]) for l in range(p))
        fresh = [np.ones(n, np.uint8) for _ in range(k + p)]  # never registered before
        t0 = time.perf_counter()
        for x in fresh:
            hip.hipHostRegister(x.ctypes.data, n, 2)
        t_fresh = (time.perf_counter() - t0) * 1e6
        for x in fresh:
            hip.hipHostUnregister(x.ctypes.data)
        row.update({"registered_zc_us": round(us2, 1), "registered_zc_gb_s": round((k + p) * n / us2 / 1e3, 2),
                    "registered_parity_ok": ok2, "register_unregister_us": round(timed(reg_only), 1),
                    "register_fresh_us": round(t_fresh, 1)})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
