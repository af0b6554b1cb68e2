#!/usr/bin/env python3
"""Single-thread throughput of the library's checksum entry points on host
buffers (the CPU route of crc_cpu.c): crc64_ecma_refl, crc64_ecma_norm and
crc32_iscsi over one buffer of each size, repeated, GB/s per call.

usage: ISAL_HIP_BACKEND=cpu tools/crc_host_speed.py [SIZE ...]
       (ISAL_HIP_CPU_SIMD=0: the slicing-by-8 tables alone)"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lib = ctypes.CDLL(os.path.join(REPO, "isa-l_amd", "lib", "libisal_hip.so"))
    for f in ("crc64_ecma_refl", "crc64_ecma_norm"):
        getattr(lib, f).restype = ctypes.c_uint64
        getattr(lib, f).argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
    lib.crc32_iscsi.restype = ctypes.c_uint32
    lib.crc32_iscsi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]
    sizes = [int(s) for s in sys.argv[1:]] or [4096, 65536, 1 << 20, 64 << 20]
    for size in sizes:
        buf = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8)
        p = buf.ctypes.data
        calls = {"crc64_ecma_refl": lambda: lib.crc64_ecma_refl(0, p, size),
                 "crc64_ecma_norm": lambda: lib.crc64_ecma_norm(0, p, size),
                 "crc32_iscsi": lambda: lib.crc32_iscsi(p, size, 0)}
        for name, f in calls.items():
            f()
            n = max(5, (256 << 20) // size)
            t = time.perf_counter()
            for _ in range(n):
                f()
            dt = (time.perf_counter() - t) / n
            print(json.dumps({"call": name, "bytes": size, "gb_s": round(size / dt / 1e9, 2),
                              "simd": os.environ.get("ISAL_HIP_CPU_SIMD", "default")}))


if __name__ == "__main__":
    main()
