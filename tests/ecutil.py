"""Shared test helpers: repo paths, the seeded byte stream, and the oracle.

The oracle (oracle/liboracle.so, a CPU restatement of the reference's
erasure_code/ec_base.c) is test infrastructure: it is only ever the CHECKER
here, never the code under test.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys
from functools import lru_cache

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")
ENGINE_DIR = os.path.join(REPO, "isa-l_amd")
ENGINE_LIB = os.path.join(ENGINE_DIR, "lib", "libisal_hip.so")
GOLDEN = os.path.join(REPO, "tests", "golden", "ec_base_golden.json")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")

if ENGINE_DIR not in sys.path:
    sys.path.insert(0, ENGINE_DIR)

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def fill_bytes(n: int, seed: int) -> np.ndarray:
    """Counter-based splitmix64 stream (same bytes as oracle_fill_bytes in C)."""
    nw = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (np.arange(1, nw + 1, dtype=np.uint64) * _G)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


@lru_cache(maxsize=1)
def golden() -> dict:
    with open(GOLDEN) as f:
        return json.load(f)


def build_oracle() -> None:
    if not os.path.exists(ORACLE_LIB):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)


def build_engine() -> None:
    if not os.path.exists(ENGINE_LIB):
        subprocess.run(["make", "-s", "-C", ENGINE_DIR], check=True)


_u8p = ctypes.POINTER(ctypes.c_ubyte)


def _p(a: np.ndarray):
    return ctypes.cast(ctypes.c_void_p(a.ctypes.data), _u8p)


def _pp(arrs):
    arr = (_u8p * max(1, len(arrs)))()
    for j, a in enumerate(arrs):
        arr[j] = _p(a)
    return arr


class Oracle:
    """ctypes view of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY)."""

    def __init__(self):
        build_oracle()
        L = ctypes.CDLL(ORACLE_LIB)
        L.oracle_gf_mul.restype = ctypes.c_ubyte
        L.oracle_gf_mul.argtypes = [ctypes.c_ubyte, ctypes.c_ubyte]
        L.oracle_gf_inv.restype = ctypes.c_ubyte
        L.oracle_gf_inv.argtypes = [ctypes.c_ubyte]
        L.oracle_gf_invert_matrix.restype = ctypes.c_int
        L.oracle_gf_vect_mul.restype = ctypes.c_int
        L.oracle_fnv1a32.restype = ctypes.c_uint
        L.oracle_fnv1a32.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
        L.oracle_crc32_iscsi.restype = ctypes.c_uint
        L.oracle_crc32_iscsi.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_uint]
        L.oracle_crc64.restype = ctypes.c_ulonglong
        L.oracle_crc64.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_ulonglong]
        self.L = L

    def gf_mul(self, a, b):
        return int(self.L.oracle_gf_mul(a, b))

    def gf_inv(self, a):
        return int(self.L.oracle_gf_inv(a))

    def gf_gen_rs_matrix(self, m, k):
        a = np.zeros(m * k, np.uint8)
        self.L.oracle_gf_gen_rs_matrix(_p(a), m, k)
        return a

    def gf_gen_cauchy1_matrix(self, m, k):
        a = np.zeros(m * k, np.uint8)
        self.L.oracle_gf_gen_cauchy1_matrix(_p(a), m, k)
        return a

    def gf_invert_matrix(self, mat, n):
        inp = np.array(mat, dtype=np.uint8).copy()
        out = np.zeros(n * n, np.uint8)
        ret = self.L.oracle_gf_invert_matrix(_p(inp), _p(out), n)
        return int(ret), out, inp

    def gf_vect_mul_init(self, c):
        t = np.zeros(32, np.uint8)
        self.L.oracle_gf_vect_mul_init(ctypes.c_ubyte(c), _p(t))
        return t

    def ec_init_tables(self, k, rows, a):
        a = np.ascontiguousarray(a, dtype=np.uint8)
        t = np.zeros(max(1, 32 * k * rows), np.uint8)
        self.L.oracle_ec_init_tables(k, rows, _p(a), _p(t))
        return t

    def ec_encode_data(self, length, k, rows, tbls, src, dst):
        self.L.oracle_ec_encode_data(length, k, rows, _p(tbls), _pp(src), _pp(dst))

    def ec_encode_data_update(self, length, k, rows, vec_i, tbls, data, dst):
        self.L.oracle_ec_encode_data_update(length, k, rows, vec_i, _p(tbls), _p(data), _pp(dst))

    def gf_vect_dot_prod(self, length, vlen, tbls, src, dest):
        self.L.oracle_gf_vect_dot_prod(length, vlen, _p(tbls), _pp(src), _p(dest))

    def gf_vect_mad(self, length, vec, vec_i, tbls, src, dest):
        self.L.oracle_gf_vect_mad(length, vec, vec_i, _p(tbls), _p(src), _p(dest))

    def gf_vect_mul(self, length, tbl, src, dest):
        return int(self.L.oracle_gf_vect_mul(length, _p(tbl), _p(src), _p(dest)))

    def raid(self, name, vects, length, arrs):
        """oracle_{xor_gen,xor_check,pq_gen,pq_check} over numpy vectors (in place)."""
        f = getattr(self.L, "oracle_" + name)
        f.restype = ctypes.c_int
        return int(f(vects, length, _pp(arrs)))

    def crc32_iscsi(self, a: np.ndarray, init: int) -> int:
        """crc_base.c crc32_iscsi_base(buf, len, init) (oracle restatement)."""
        a = np.ascontiguousarray(a, dtype=np.uint8)
        return int(self.L.oracle_crc32_iscsi(ctypes.c_void_p(a.ctypes.data), a.size, init & 0xFFFFFFFF))

    def crc64(self, variant: int, a: np.ndarray, init: int) -> int:
        """crc64_base.c crc64_<variant>_base(init, buf, len) (oracle restatement);
        variant order of include/crc64.h (ecma/iso/jones/rocksoft x refl/norm)."""
        a = np.ascontiguousarray(a, dtype=np.uint8)
        return int(self.L.oracle_crc64(variant, ctypes.c_void_p(a.ctypes.data), a.size,
                                       init & 0xFFFFFFFFFFFFFFFF))

    def fnv(self, a: np.ndarray) -> int:
        return int(self.L.oracle_fnv1a32(ctypes.c_void_p(a.ctypes.data), a.size))

    # convenience: encode fresh parity for a list of source arrays
    def encode(self, coef: np.ndarray, k: int, rows: int, src):
        n = len(src[0]) if k else 0
        tbls = self.ec_init_tables(k, rows, coef)
        dst = [np.zeros(n, np.uint8) for _ in range(rows)]
        self.ec_encode_data(n, k, rows, tbls, src, dst)
        return dst


@lru_cache(maxsize=1)
def oracle() -> Oracle:
    return Oracle()


def coeffs(gen: str, k: int, rows: int, seed: int, o: Oracle | None = None) -> np.ndarray:
    """Parity-row coefficients as gen_golden.c:make_coeffs builds them."""
    o = o or oracle()
    if gen == "rs":
        return o.gf_gen_rs_matrix(k + rows, k)[k * k:].copy()
    if gen == "cauchy":
        return o.gf_gen_cauchy1_matrix(k + rows, k)[k * k:].copy()
    return fill_bytes(k * rows, seed ^ 0xC0EFF1C1E47)


def crc_fixture_bytes(entry: dict) -> np.ndarray:
    """Input buffer of one tests/golden crc32_iscsi / crc64 entry (gen_golden.c)."""
    n = entry["len"]
    if entry["fill"] == "zero":
        return np.zeros(n, np.uint8)
    if entry["fill"] == "8a":
        return np.full(n, 0x8A, np.uint8)
    return fill_bytes(n, entry["seed"])


def decode_matrix(a: np.ndarray, k: int, errs, o: Oracle | None = None):
    """Recovery rows for erased fragments `errs` (erasure_code_perf.c:134-168).

    Returns (ret, c, survivors) — c is len(errs) x k; survivors the k fragment
    indices the rows apply to."""
    o = o or oracle()
    in_err = set(errs)
    surv = [i for i in range(len(a) // k) if i not in in_err][:k]
    b = np.concatenate([a[r * k:(r + 1) * k] for r in surv])
    ret, d, _ = o.gf_invert_matrix(b, k)
    c = np.zeros(len(errs) * k, np.uint8)
    if ret == 0:
        for i, s in enumerate(errs):
            for j in range(k):
                acc = 0
                for r in range(k):
                    acc ^= o.gf_mul(int(d[k * r + j]), int(a[k * s + r]))
                c[k * i + j] = acc
    return ret, c, surv
