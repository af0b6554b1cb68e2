"""isal_amd — Python mirror of the reference erasure-code API over libisal_hip.so.

The product is the C-ABI library ``isa-l_amd/lib/libisal_hip.so`` (headers in
``include/``). This module binds it with ctypes, keeping the reference's
function names, argument order and meaning (reference include/erasure_code.h,
include/gf_vect_mul.h), so tests and the benchmark read like the reference's
own C tests. Buffers may be numpy uint8 arrays (host memory), torch tensors
(host or device; their storage address is passed), or raw integer addresses.

There is no Python fallback: every data-path call goes through the library
(a missing library raises immediately). The library itself routes each
drop-in call (include/isal_hip.h "routing"): device-resident shards and large
host calls to the GPU kernels, small host calls to its CPU route;
ISAL_HIP_BACKEND=gpu forces the kernels.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

__all__ = [
    "LIB_PATH", "lib", "gf_mul", "gf_inv", "gf_gen_rs_matrix", "gf_gen_cauchy1_matrix",
    "gf_invert_matrix", "gf_vect_mul_init", "ec_init_tables", "ec_encode_data",
    "ec_encode_data_base", "ec_encode_data_update", "ec_encode_data_update_base",
    "gf_vect_dot_prod", "gf_vect_dot_prod_base", "gf_vect_mad", "gf_vect_mad_base",
    "gf_vect_mul", "gf_vect_mul_base", "Batch", "Pipe", "kernel_launches", "max_rows_per_pass",
    "version", "addr", "cpu_calls", "fallbacks", "reload_config", "Multi", "partition",
    "route_device", "contexts_created", "selftest_kernels", "crc32_iscsi", "crc64", "CRC64_VARIANTS", "slow_waits",
]

LIB_PATH = os.environ.get(
    "ISAL_HIP_LIB",
    os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, "lib", "libisal_hip.so"),
)

_u8p = ctypes.POINTER(ctypes.c_ubyte)
_u8pp = ctypes.POINTER(_u8p)
_lib = None


# Variant numbers of isal_hip_batch_crc64 (ISAL_HIP_CRC64_*): the crc64_*
# functions of the reference's include/crc64.h, in its order.
CRC64_VARIANTS = ("ecma_refl", "ecma_norm", "iso_refl", "iso_norm",
                  "jones_refl", "jones_norm", "rocksoft_refl", "rocksoft_norm")


def _one_hip_runtime() -> None:
    """A process must hold exactly ONE HIP runtime. PyTorch-ROCm ships its own
    libamdhip64.so.7; if libisal_hip.so were loaded first it would bind
    /opt/rocm's copy, torch would then load a second one, and whichever
    initialises second sees no device. Loading torch first makes the engine's
    NEEDED libamdhip64.so.7 resolve to the runtime torch already holds (same
    SONAME), so device pointers and streams are shared. Set ISAL_AMD_NO_TORCH=1
    in processes that never use torch."""
    if os.environ.get("ISAL_AMD_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> ctypes.CDLL:
    """Load libisal_hip.so (raises if it has not been built: no silent fallback)."""
    global _lib
    if _lib is None:
        path = os.path.abspath(LIB_PATH)
        if not os.path.exists(path):
            raise RuntimeError(f"libisal_hip.so not built at {path}: run `make -C isa-l_amd`")
        _one_hip_runtime()
        L = ctypes.CDLL(path)
        i, v = ctypes.c_int, None
        sig = {
            "gf_mul": (ctypes.c_ubyte, [ctypes.c_ubyte, ctypes.c_ubyte]),
            "gf_inv": (ctypes.c_ubyte, [ctypes.c_ubyte]),
            "gf_gen_rs_matrix": (v, [_u8p, i, i]),
            "gf_gen_cauchy1_matrix": (v, [_u8p, i, i]),
            "gf_invert_matrix": (i, [_u8p, _u8p, i]),
            "gf_vect_mul_init": (v, [ctypes.c_ubyte, _u8p]),
            "gf_vect_mul_init_base": (v, [ctypes.c_ubyte, _u8p]),
            "ec_init_tables": (v, [i, i, _u8p, _u8p]),
            "ec_init_tables_base": (v, [i, i, _u8p, _u8p]),
            "ec_encode_data": (v, [i, i, i, _u8p, _u8pp, _u8pp]),
            "ec_encode_data_base": (v, [i, i, i, _u8p, _u8pp, _u8pp]),
            "ec_encode_data_update": (v, [i, i, i, i, _u8p, _u8p, _u8pp]),
            "ec_encode_data_update_base": (v, [i, i, i, i, _u8p, _u8p, _u8pp]),
            "gf_vect_dot_prod": (v, [i, i, _u8p, _u8pp, _u8p]),
            "gf_vect_dot_prod_base": (v, [i, i, _u8p, _u8pp, _u8p]),
            "gf_vect_mad": (v, [i, i, i, _u8p, _u8p, _u8p]),
            "gf_vect_mad_base": (v, [i, i, i, _u8p, _u8p, _u8p]),
            "gf_vect_mul": (i, [i, _u8p, ctypes.c_void_p, ctypes.c_void_p]),
            "gf_vect_mul_base": (i, [i, _u8p, _u8p, _u8p]),
            "isal_get_version": (ctypes.c_uint, []),
            "isal_get_version_str": (ctypes.c_char_p, []),
            "isal_hip_batch_create": (i, [ctypes.POINTER(ctypes.c_void_p), i, i, i, _u8p, i, _u8pp, _u8pp]),
            "isal_hip_batch_set_tables": (i, [ctypes.c_void_p, _u8p]),
            "isal_hip_batch_encode": (i, [ctypes.c_void_p, ctypes.c_void_p]),
            "isal_hip_batch_update": (i, [ctypes.c_void_p, i, ctypes.c_void_p]),
            "isal_hip_batch_destroy": (i, [ctypes.c_void_p]),
            "isal_hip_batch_encode_crc": (i, [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]),
            "isal_hip_batch_crc": (i, [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]),
            "isal_hip_batch_crc64": (i, [ctypes.c_void_p, i, ctypes.c_ulonglong, ctypes.c_void_p, ctypes.c_void_p]),
            "isal_hip_batch_encode_crc64": (i, [ctypes.c_void_p, i, ctypes.c_ulonglong, ctypes.c_void_p,
                                                ctypes.c_void_p]),
            "isal_hip_pipe_create": (i, [ctypes.POINTER(ctypes.c_void_p), i, i, i, _u8p, i, i]),
            "isal_hip_pipe_submit": (i, [ctypes.c_void_p, _u8pp, _u8pp]),
            "isal_hip_pipe_flush": (i, [ctypes.c_void_p]),
            "isal_hip_pipe_destroy": (i, [ctypes.c_void_p]),
            "isal_hip_kernel_launches": (ctypes.c_ulonglong, []),
            "isal_hip_cpu_calls": (ctypes.c_ulonglong, []),
            "isal_hip_multi_create": (i, [ctypes.POINTER(ctypes.c_void_p), i, i, i, i, _u8p, i]),
            "isal_hip_multi_ndev": (i, [ctypes.c_void_p]),
            "isal_hip_multi_encode": (i, [ctypes.c_void_p, ctypes.c_longlong, _u8pp, _u8pp]),
            "isal_hip_multi_destroy": (i, [ctypes.c_void_p]),
            "isal_hip_multi_partition": (None, [ctypes.c_longlong, i, i, ctypes.POINTER(ctypes.c_longlong),
                                                ctypes.POINTER(ctypes.c_longlong)]),
            "isal_hip_multi_numa_node": (i, [ctypes.c_void_p, i]),
            "isal_hip_multi_worker_cpus": (i, [ctypes.c_void_p, i]),
            "isal_hip_pci_numa_node": (i, [ctypes.c_char_p, ctypes.c_char_p]),
            "isal_hip_numa_node_cpus": (i, [ctypes.c_char_p, i, ctypes.POINTER(ctypes.c_int), i]),
            "isal_hip_fallbacks": (ctypes.c_ulonglong, []),
            "isal_hip_config_reload": (None, []),
            "isal_hip_max_rows_per_pass": (i, []),
            "isal_hip_target": (ctypes.c_char_p, []),
            "isal_hip_route_device": (i, [i, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), i,
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
            "isal_hip_contexts_created": (ctypes.c_ulonglong, []),
            "isal_hip_slow_waits": (ctypes.c_ulonglong, []),
            "isal_hip_selftest_kernels": (i, [ctypes.POINTER(ctypes.c_int)]),
            "crc32_iscsi": (ctypes.c_uint, [ctypes.c_void_p, i, ctypes.c_uint]),
            "crc32_iscsi_base": (ctypes.c_uint, [ctypes.c_void_p, i, ctypes.c_uint]),
        }
        for v in CRC64_VARIANTS:
            for suffix in ("", "_base"):
                sig[f"crc64_{v}{suffix}"] = (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64])
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


# ---------------------------------------------------------------------------
# buffer plumbing
# ---------------------------------------------------------------------------

def addr(buf) -> int:
    """Address of a byte buffer: numpy array, torch tensor, ctypes buffer or int."""
    if isinstance(buf, int):
        return buf
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            raise ValueError("buffer must be C-contiguous")
        return buf.ctypes.data
    if hasattr(buf, "data_ptr"):  # torch.Tensor
        if not buf.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return int(buf.data_ptr())
    if isinstance(buf, (ctypes.Array, bytearray)):
        return ctypes.addressof(ctypes.c_char.from_buffer(buf))
    raise TypeError(f"unsupported buffer type {type(buf)!r}")


def _p(buf) -> _u8p:
    return ctypes.cast(ctypes.c_void_p(addr(buf)), _u8p)


def _pp(bufs: Sequence) -> ctypes.Array:
    arr = (_u8p * max(1, len(bufs)))()
    for j, b in enumerate(bufs):
        arr[j] = _p(b)
    return arr


def _u8(a) -> np.ndarray:
    a = np.ascontiguousarray(np.frombuffer(bytes(a), dtype=np.uint8) if isinstance(a, (bytes, bytearray)) else a,
                             dtype=np.uint8)
    return a


# ---------------------------------------------------------------------------
# host-side GF math (reference ec_base.c:37-280 semantics)
# ---------------------------------------------------------------------------

def gf_mul(a: int, b: int) -> int:
    return int(lib().gf_mul(a & 0xFF, b & 0xFF))


def gf_inv(a: int) -> int:
    return int(lib().gf_inv(a & 0xFF))


def gf_gen_rs_matrix(m: int, k: int) -> np.ndarray:
    a = np.zeros(m * k, dtype=np.uint8)
    lib().gf_gen_rs_matrix(_p(a), m, k)
    return a


def gf_gen_cauchy1_matrix(m: int, k: int) -> np.ndarray:
    a = np.zeros(m * k, dtype=np.uint8)
    lib().gf_gen_cauchy1_matrix(_p(a), m, k)
    return a


def gf_invert_matrix(mat, n: int):
    """Returns (ret, inverse, destroyed_input) like the C call (input is copied first)."""
    inp = _u8(mat).copy()
    out = np.zeros(n * n, dtype=np.uint8)
    ret = lib().gf_invert_matrix(_p(inp), _p(out), n)
    return int(ret), out, inp


def gf_vect_mul_init(c: int) -> np.ndarray:
    t = np.zeros(32, dtype=np.uint8)
    lib().gf_vect_mul_init(c & 0xFF, _p(t))
    return t


def ec_init_tables(k: int, rows: int, a) -> np.ndarray:
    a = _u8(a)
    t = np.zeros(max(1, 32 * k * rows), dtype=np.uint8)
    lib().ec_init_tables(k, rows, _p(a), _p(t))
    return t


# ---------------------------------------------------------------------------
# data path (GPU) — same argument order as the C API
# ---------------------------------------------------------------------------

def ec_encode_data(len_: int, k: int, rows: int, gftbls, data: Sequence, coding: Sequence) -> None:
    lib().ec_encode_data(len_, k, rows, _p(gftbls), _pp(data), _pp(coding))


def ec_encode_data_base(len_: int, k: int, rows: int, gftbls, data: Sequence, coding: Sequence) -> None:
    lib().ec_encode_data_base(len_, k, rows, _p(gftbls), _pp(data), _pp(coding))


def ec_encode_data_update(len_: int, k: int, rows: int, vec_i: int, gftbls, data, coding: Sequence) -> None:
    lib().ec_encode_data_update(len_, k, rows, vec_i, _p(gftbls), _p(data), _pp(coding))


def ec_encode_data_update_base(len_: int, k: int, rows: int, vec_i: int, gftbls, data, coding: Sequence) -> None:
    lib().ec_encode_data_update_base(len_, k, rows, vec_i, _p(gftbls), _p(data), _pp(coding))


def gf_vect_dot_prod(len_: int, vlen: int, gftbls, src: Sequence, dest) -> None:
    lib().gf_vect_dot_prod(len_, vlen, _p(gftbls), _pp(src), _p(dest))


def gf_vect_dot_prod_base(len_: int, vlen: int, gftbls, src: Sequence, dest) -> None:
    lib().gf_vect_dot_prod_base(len_, vlen, _p(gftbls), _pp(src), _p(dest))


def gf_vect_mad(len_: int, vec: int, vec_i: int, gftbls, src, dest) -> None:
    lib().gf_vect_mad(len_, vec, vec_i, _p(gftbls), _p(src), _p(dest))


def gf_vect_mad_base(len_: int, vec: int, vec_i: int, gftbls, src, dest) -> None:
    lib().gf_vect_mad_base(len_, vec, vec_i, _p(gftbls), _p(src), _p(dest))


def gf_vect_mul(len_: int, gftbl, src, dest) -> int:
    return int(lib().gf_vect_mul(len_, _p(gftbl), ctypes.c_void_p(addr(src)), ctypes.c_void_p(addr(dest))))


def gf_vect_mul_base(len_: int, gftbl, src, dest) -> int:
    return int(lib().gf_vect_mul_base(len_, _p(gftbl), _p(src), _p(dest)))


# ---------------------------------------------------------------------------
# batched extension (include/isal_hip.h)
# ---------------------------------------------------------------------------

class Batch:
    """nstripes stripes sharing one coefficient matrix; shards are device buffers.

    data[s*k + j] / coding[s*rows + l] are addresses (or tensors) of stripe s.
    encode()/update() only enqueue on `stream` (a hipStream_t as int; 0 = default).
    """

    def __init__(self, len_: int, k: int, rows: int, gftbls, nstripes: int,
                 data: Sequence, coding: Sequence):
        self.len, self.k, self.rows, self.nstripes = len_, k, rows, nstripes
        if len(data) != nstripes * k or len(coding) != nstripes * rows:
            raise ValueError("pointer lists must hold nstripes*k and nstripes*rows entries")
        h = ctypes.c_void_p()
        rc = lib().isal_hip_batch_create(ctypes.byref(h), len_, k, rows, _p(gftbls), nstripes,
                                         _pp(data), _pp(coding))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_create failed ({rc})")
        self._h = h

    def set_tables(self, gftbls) -> None:
        rc = lib().isal_hip_batch_set_tables(self._h, _p(gftbls))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_set_tables failed ({rc})")

    def encode(self, stream: int = 0) -> None:
        rc = lib().isal_hip_batch_encode(self._h, ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_encode failed ({rc})")

    def update(self, vec_i: int, stream: int = 0) -> None:
        rc = lib().isal_hip_batch_update(self._h, vec_i, ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_update failed ({rc})")

    def check(self, bad, stream: int = 0) -> None:
        """Verify every stripe (isal_hip_batch_check): the DEVICE buffer bad
        (nstripes uint64) gets ~0 for a consistent stripe, else its first
        mismatch as column << 8 | row."""
        rc = lib().isal_hip_batch_check(self._h, ctypes.c_void_p(addr(bad)), ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_check failed ({rc})")

    def encode_crc(self, init: int, crc, stream: int = 0) -> None:
        """encode() plus crc32_iscsi(shard, len, init) of every source and parity
        shard into the DEVICE buffer crc (nstripes*(k+rows) uint32, stripe-major,
        sources then parity)."""
        rc = lib().isal_hip_batch_encode_crc(self._h, init & 0xFFFFFFFF, ctypes.c_void_p(addr(crc)),
                                             ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_encode_crc failed ({rc})")

    def crc(self, init: int, crc, stream: int = 0) -> None:
        """crc32_iscsi of every shard (no encoding), layout as encode_crc()."""
        rc = lib().isal_hip_batch_crc(self._h, init & 0xFFFFFFFF, ctypes.c_void_p(addr(crc)),
                                      ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_crc failed ({rc})")

    def crc64(self, variant: int, init: int, crc, stream: int = 0) -> None:
        """crc64_<variant>(init, shard, len) of every shard into the DEVICE buffer
        crc (nstripes*(k+rows) 64-bit words, layout as encode_crc()); variant =
        CRC64_VARIANTS.index(name), the order of the reference's crc64.h."""
        rc = lib().isal_hip_batch_crc64(self._h, variant, init & 0xFFFFFFFFFFFFFFFF,
                                        ctypes.c_void_p(addr(crc)), ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_crc64 failed ({rc})")

    def encode_crc64(self, variant: int, init: int, crc, stream: int = 0) -> None:
        """encode() plus crc64_<variant>(init, shard, len) of every source and
        parity shard, layout as crc64(); one pass over HBM where the shape allows."""
        rc = lib().isal_hip_batch_encode_crc64(self._h, variant, init & 0xFFFFFFFFFFFFFFFF,
                                               ctypes.c_void_p(addr(crc)), ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"isal_hip_batch_encode_crc64 failed ({rc})")

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().isal_hip_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Pipe:
    """Streaming encoder for host-resident stripes (include/isal_hip.h pipeline).

    mode "update": sources folded into parity as they land (ec_encode_data_update);
    mode "encode": one ec_encode_data per stripe once all sources landed.
    Host buffers must stay alive until flush() returns."""

    MODES = {"update": 0, "encode": 1}

    def __init__(self, len_: int, k: int, rows: int, gftbls, depth: int = 3, mode: str = "update"):
        self.len, self.k, self.rows = len_, k, rows
        h = ctypes.c_void_p()
        rc = lib().isal_hip_pipe_create(ctypes.byref(h), len_, k, rows, _p(gftbls), depth,
                                        self.MODES[mode])
        if rc != 0:
            raise RuntimeError(f"isal_hip_pipe_create failed ({rc})")
        self._h = h
        self._keep = []

    def submit(self, data: Sequence, coding: Sequence) -> None:
        d, c = _pp(data), _pp(coding)
        self._keep.append((d, c))  # pointer arrays are read at submit; keep refs cheap anyway
        rc = lib().isal_hip_pipe_submit(self._h, d, c)
        if rc != 0:
            raise RuntimeError(f"isal_hip_pipe_submit failed ({rc})")

    def flush(self) -> None:
        rc = lib().isal_hip_pipe_flush(self._h)
        self._keep.clear()
        if rc != 0:
            raise RuntimeError(f"isal_hip_pipe_flush failed ({rc})")

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().isal_hip_pipe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """Host-resident stripes encoded on several GPUs of this process
    (include/isal_hip.h multi-device): contiguous stripe ranges per GPU, one
    pipeline and host thread each. ndev = 0: every visible GPU."""

    def __init__(self, len_: int, k: int, rows: int, gftbls, ndev: int = 0, depth: int = 3):
        self.len, self.k, self.rows = len_, k, rows
        h = ctypes.c_void_p()
        rc = lib().isal_hip_multi_create(ctypes.byref(h), ndev, len_, k, rows, _p(gftbls), depth)
        if rc != 0:
            raise RuntimeError(f"isal_hip_multi_create failed ({rc})")
        self._h = h

    @property
    def ndev(self) -> int:
        return int(lib().isal_hip_multi_ndev(self._h))

    def numa_node(self, dev: int) -> int:
        """NUMA node of device dev's PCIe root (-1 unknown)."""
        return int(lib().isal_hip_multi_numa_node(self._h, dev))

    def worker_cpus(self, dev: int) -> int:
        """How many CPUs device dev's worker thread is pinned to (0: not pinned)."""
        return int(lib().isal_hip_multi_worker_cpus(self._h, dev))

    def encode(self, nstripes: int, data: Sequence, coding: Sequence) -> None:
        """data[s*k + j], coding[s*rows + l]: host buffers of stripe s."""
        if len(data) != nstripes * self.k or len(coding) != nstripes * self.rows:
            raise ValueError("pointer lists must hold nstripes*k and nstripes*rows entries")
        rc = lib().isal_hip_multi_encode(self._h, nstripes, _pp(data), _pp(coding))
        if rc != 0:
            raise RuntimeError(f"isal_hip_multi_encode failed ({rc})")

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().isal_hip_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def partition(nstripes: int, ndev: int, dev: int) -> tuple[int, int]:
    """(first, count) of device/rank `dev`'s contiguous stripe range
    (isal_hip_multi_partition; no GPU needed)."""
    first, count = ctypes.c_longlong(), ctypes.c_longlong()
    lib().isal_hip_multi_partition(nstripes, ndev, dev, ctypes.byref(first), ctypes.byref(count))
    return int(first.value), int(count.value)


def pci_numa_node(pci_bus_id: str, sysfs_root: str | None = None) -> int:
    """NUMA node of a PCI device from sysfs (-1 unknown); no GPU needed."""
    return int(lib().isal_hip_pci_numa_node(sysfs_root.encode() if sysfs_root else None, pci_bus_id.encode()))


def numa_node_cpus(node: int, sysfs_root: str | None = None) -> list[int] | None:
    """CPUs of a NUMA node from its sysfs cpulist (None when unreadable)."""
    buf = (ctypes.c_int * 4096)()
    n = lib().isal_hip_numa_node_cpus(sysfs_root.encode() if sysfs_root else None, node, buf, 4096)
    return None if n < 0 else list(buf[:min(n, 4096)])


def crc32_iscsi(buf, len_: int, init_crc: int, base: bool = False) -> int:
    """crc.h crc32_iscsi(buffer, len, init_crc) (reference include/crc.h:136-150):
    host buffers on the library's CPU route, device buffers on the GPU."""
    f = lib().crc32_iscsi_base if base else lib().crc32_iscsi
    return int(f(ctypes.c_void_p(addr(buf) if buf is not None else 0), len_, init_crc & 0xFFFFFFFF))


def crc64(variant, init_crc: int, buf, len_: int, base: bool = False) -> int:
    """crc64.h crc64_<variant>(init_crc, buf, len) (reference include/crc64.h:54-163);
    variant: a CRC64_VARIANTS name or its index (ISAL_HIP_CRC64_*)."""
    name = variant if isinstance(variant, str) else CRC64_VARIANTS[variant]
    f = getattr(lib(), f"crc64_{name}{'_base' if base else ''}")
    return int(f(init_crc & 0xFFFFFFFFFFFFFFFF, ctypes.c_void_p(addr(buf) if buf is not None else 0), len_))


MEM_PAGEABLE, MEM_DEVICE, MEM_MANAGED, MEM_PINNED = 0, 1, 2, 3


def route_device(kinds: Sequence[int], devs: Sequence[int], cur: int) -> tuple[int, int, list[int]]:
    """isal_hip_route_device: the device a drop-in call with these shards runs
    on (-2: device shards on two GPUs), the first shard on a second GPU (-1:
    none) and the per-shard in-place flags. Pure logic, no GPU needed."""
    n = len(kinds)
    K = (ctypes.c_int * max(n, 1))(*kinds)
    D = (ctypes.c_int * max(n, 1))(*devs)
    P = (ctypes.c_int * max(n, 1))()
    bad = ctypes.c_int(0)
    dev = lib().isal_hip_route_device(n, K, D, cur, ctypes.byref(bad), P)
    return dev, bad.value, list(P[:n])


def selftest_kernels() -> tuple[int, int]:
    """isal_hip_selftest_kernels: (kernels without usable device code, kernels checked)."""
    n = ctypes.c_int(0)
    bad = lib().isal_hip_selftest_kernels(ctypes.byref(n))
    return int(bad), int(n.value)


def slow_waits() -> int:
    """Kernel-argument calls completed by hipStreamSynchronize after the spin expired."""
    return int(lib().isal_hip_slow_waits())


def contexts_created() -> int:
    """Per-thread, per-device contexts the drop-in calls have created."""
    return int(lib().isal_hip_contexts_created())


def kernel_launches() -> int:
    return int(lib().isal_hip_kernel_launches())


def cpu_calls() -> int:
    """Drop-in calls the library served on its CPU route (small host calls,
    ISAL_HIP_BACKEND=cpu, no GPU, HIP-failure fallbacks)."""
    return int(lib().isal_hip_cpu_calls())


def fallbacks() -> int:
    """Drop-in calls that hit a HIP failure and finished on the CPU route."""
    return int(lib().isal_hip_fallbacks())


def reload_config() -> None:
    """Re-read the ISAL_HIP_* environment knobs (read once otherwise)."""
    lib().isal_hip_config_reload()


def max_rows_per_pass() -> int:
    return int(lib().isal_hip_max_rows_per_pass())


def version() -> str:
    return lib().isal_get_version_str().decode()
