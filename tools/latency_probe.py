"""Per-call latency of the synchronous drop-in path (GPU box diagnostic)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch's)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "isa-l_amd"))
import isal_amd  # noqa: E402

L = isal_amd.lib()
hip = ctypes.CDLL("libamdhip64.so")
vects, n, reps = 17, 1024, 2000
bufs = [np.random.default_rng(j).integers(0, 256, n, dtype=np.uint8) for j in range(vects)]
arr = (ctypes.c_void_p * vects)(*[b.ctypes.data for b in bufs])
f = L.xor_gen
f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
g = L.xor_check
g.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
f(vects, n, arr)
for name, fn in (("xor_gen", f), ("xor_check", g)):
    t = time.perf_counter()
    for _ in range(reps):
        fn(vects, n, arr)
    print(f"{name} host 17x1KiB: {(time.perf_counter() - t) / reps * 1e6:.1f} us/call", flush=True)
attr = ctypes.create_string_buffer(64)
t = time.perf_counter()
for _ in range(reps * 17):
    hip.hipPointerGetAttributes(attr, ctypes.c_void_p(bufs[0].ctypes.data))
print(f"hipPointerGetAttributes(host): {(time.perf_counter() - t) / (reps * 17) * 1e6:.2f} us", flush=True)
d = torch.empty(n, dtype=torch.uint8, device="cuda")
t = time.perf_counter()
for _ in range(reps * 17):
    hip.hipPointerGetAttributes(attr, ctypes.c_void_p(d.data_ptr()))
print(f"hipPointerGetAttributes(device): {(time.perf_counter() - t) / (reps * 17) * 1e6:.2f} us", flush=True)
dev = [torch.from_numpy(b).cuda() for b in bufs]
darr = (ctypes.c_void_p * vects)(*[x.data_ptr() for x in dev])
t = time.perf_counter()
for _ in range(reps):
    g(vects, n, darr)
print(f"xor_check device 17x1KiB: {(time.perf_counter() - t) / reps * 1e6:.1f} us/call", flush=True)
s = torch.cuda.Stream()
t = time.perf_counter()
for _ in range(reps):
    torch.cuda.synchronize()
print(f"torch.cuda.synchronize: {(time.perf_counter() - t) / reps * 1e6:.1f} us", flush=True)
