"""CPU tier: the library's CPU route (isa-l_amd/csrc/ec_cpu.c) — the route the
drop-in calls take for small host-resident calls, for ISAL_HIP_BACKEND=cpu,
on hosts without a GPU, and as the fallback when a HIP call fails.

Checked like the GPU path: against the reference's own outputs
(tests/golden, generated from /root/reference ec_base.c / raid_base.c), the
oracle on random shapes, the reference's contracts (padding untouched,
update == encode, RAID check positions) and the reference's own test
programs linked against libisal_hip.so. The GFNI (AVX-512), AVX2 and per-byte
variants all run. No GPU needed: ISAL_HIP_BACKEND=cpu pins the route either way.
"""
import os
import subprocess

import numpy as np
import pytest

import ecutil
from ecutil import coeffs, fill_bytes, golden


@pytest.fixture(params=["gfni", "avx2", "scalar"])
def cpu_engine(engine, request, monkeypatch):
    """The CPU route at each width (capped by ISAL_HIP_CPU_SIMD; a CPU without
    GFNI / AVX2 runs the next narrower path, still checked)."""
    monkeypatch.setenv("ISAL_HIP_BACKEND", "cpu")
    monkeypatch.setenv("ISAL_HIP_CPU_SIMD", {"gfni": "2", "avx2": "1", "scalar": "0"}[request.param])
    engine.reload_config()
    launches, calls = engine.kernel_launches(), engine.cpu_calls()
    yield engine
    assert engine.kernel_launches() == launches, "CPU route launched GPU kernels"
    assert engine.cpu_calls() > calls, "calls did not take the CPU route"
    monkeypatch.undo()
    engine.reload_config()


def _h(s):
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


def test_golden_encode_update_decode(cpu_engine, oracle):
    e = cpu_engine
    for case in golden()["encode"]:
        k, rows, n = case["k"], case["rows"], case["len"]
        tbls = e.ec_init_tables(k, rows, _h(case["coef"]))
        src = [fill_bytes(n, case["seed"] + j) for j in range(k)]
        dst = [np.full(n, 0xA5, np.uint8) for _ in range(rows)]
        e.ec_encode_data(n, k, rows, tbls, src, dst)
        assert [oracle.fnv(d) for d in dst] == case["fnv"], (k, rows, n)
        if "parity" in case:
            assert [d.tobytes().hex() for d in dst] == case["parity"]
    for case in golden()["update"]:
        k, rows, n = case["k"], case["rows"], case["len"]
        tbls = e.ec_init_tables(k, rows, coeffs(case["gen"], k, rows, case["seed"]))
        src = [fill_bytes(n, case["seed"] + j) for j in range(k)]
        dst = [np.zeros(n, np.uint8) for _ in range(rows)]
        for v in (range(k - 1, -1, -1) if case["reverse"] else range(k)):
            e.ec_encode_data_update(n, k, rows, v, tbls, src[v], dst)
        assert [oracle.fnv(d) for d in dst] == case["fnv"]
    for case in golden()["decode"]:
        k, p, n, errs = case["k"], case["p"], case["len"], case["errs"]
        gen = e.gf_gen_rs_matrix if case["gen"] == "rs" else e.gf_gen_cauchy1_matrix
        a = gen(k + p, k)
        ret, c, surv = ecutil.decode_matrix(a, k, errs)
        frag = [fill_bytes(n, case["seed"] + j) for j in range(k)] + [np.zeros(n, np.uint8) for _ in range(p)]
        e.ec_encode_data(n, k, p, e.ec_init_tables(k, p, a[k * k:]), frag[:k], frag[k:])
        rec = [np.zeros(n, np.uint8) for _ in errs]
        e.ec_encode_data(n, k, len(errs), e.ec_init_tables(k, len(errs), c), [frag[s] for s in surv], rec)
        assert [oracle.fnv(r) for r in rec] == case["fnv"]


def test_golden_single_output_primitives(cpu_engine):
    e, g = cpu_engine, golden()
    for case in g["dot_prod"]:
        vlen, n = case["vlen"], case["len"]
        tbls = np.concatenate([e.gf_vect_mul_init(int(c)) for c in fill_bytes(vlen, case["coef_seed"])])
        src = [fill_bytes(n, case["src_seed"] + j) for j in range(vlen)]
        for f in (e.gf_vect_dot_prod, e.gf_vect_dot_prod_base):
            d = np.zeros(n, np.uint8)
            f(n, vlen, tbls, src, d)
            assert d.tobytes().hex() == case["dest"]
    for case in g["mad"]:
        vec, n = case["vec"], case["len"]
        tbls = np.concatenate([e.gf_vect_mul_init(int(c)) for c in fill_bytes(vec, case["coef_seed"])])
        for f in (e.gf_vect_mad, e.gf_vect_mad_base):
            d = fill_bytes(n, case["dest_seed"])
            f(n, vec, case["vec_i"], tbls, fill_bytes(n, case["src_seed"]), d)
            assert d.tobytes().hex() == case["dest"]
    for case in g["vect_mul"]:
        n = case["len"]
        for f in (e.gf_vect_mul, e.gf_vect_mul_base):
            d = np.zeros(n, np.uint8)
            assert f(n, e.gf_vect_mul_init(case["c"]), fill_bytes(n, case["src_seed"]), d) == case["ret"]
            assert d.tobytes().hex() == case["dest"]


def test_random_shapes_vs_oracle(cpu_engine, oracle):
    """k up to 64, rows up to 20 (several 4-row groups), ragged lengths across
    the 32-column SIMD step and the 4 KiB block."""
    rng = np.random.default_rng(11)
    lens = [0, 1, 2, 15, 31, 32, 33, 63, 255, 4095, 4096, 4097, 8191, 12345]
    for it in range(40):
        k = int(rng.integers(1, 65)) if it % 4 else int(rng.integers(1, 8))
        rows = int(rng.integers(1, 21))
        n = lens[it % len(lens)]
        coef = fill_bytes(k * rows, 1000 + it)
        src = [fill_bytes(n, 5000 + 97 * it + j) for j in range(k)]
        got = [np.zeros(n, np.uint8) for _ in range(rows)]
        cpu_engine.ec_encode_data(n, k, rows, cpu_engine.ec_init_tables(k, rows, coef), src, got)
        want = oracle.encode(coef, k, rows, src)
        for l in range(rows):
            assert np.array_equal(got[l], want[l]), (it, k, rows, n, l)


def test_misaligned_pointers_and_padding_untouched(cpu_engine, oracle):
    """erasure_code_test.c:583-709: offsets 0..31; bytes outside [ptr, ptr+len) untouched."""
    rng = np.random.default_rng(7)
    pad, canary = 64, np.uint8(0x5C)
    for it in range(24):
        k, rows = int(rng.integers(1, 17)), int(rng.integers(1, 11))
        n = int(rng.integers(16, 3000))
        coef = fill_bytes(k * rows, 77 + it)
        offs = [int(rng.integers(0, 32)) for _ in range(k + rows)]
        src = [fill_bytes(n, 900 + 31 * it + j) for j in range(k)]
        bufs = [np.full(n + 2 * pad, canary, np.uint8) for _ in range(k + rows)]
        for j in range(k):
            bufs[j][pad + offs[j]:pad + offs[j] + n] = src[j]
        views = [bufs[j][pad + offs[j]:pad + offs[j] + n] for j in range(k + rows)]
        cpu_engine.ec_encode_data(n, k, rows, cpu_engine.ec_init_tables(k, rows, coef), views[:k], views[k:])
        want = oracle.encode(coef, k, rows, src)
        for l in range(rows):
            b, o = bufs[k + l], offs[k + l]
            assert np.array_equal(b[pad + o:pad + o + n], want[l]), (it, l)
            assert (b[:pad + o] == canary).all() and (b[pad + o + n:] == canary).all(), (it, l)


def test_update_equals_encode_and_mad_tails(cpu_engine):
    """erasure_code_update_test.c:320-333 + lengths 0..256 (:596-624)."""
    rng = np.random.default_rng(3)
    e = cpu_engine
    for n in list(range(0, 257, 7)) + [4096, 4111, 70000]:
        k, rows = int(rng.integers(1, 20)), int(rng.integers(1, 12))
        tbls = e.ec_init_tables(k, rows, fill_bytes(k * rows, n + 1))
        src = [fill_bytes(n, 3 * n + j) for j in range(k)]
        want = [np.zeros(n, np.uint8) for _ in range(rows)]
        e.ec_encode_data(n, k, rows, tbls, src, want)
        got = [np.zeros(n, np.uint8) for _ in range(rows)]
        for v in rng.permutation(k):
            e.ec_encode_data_update(n, k, rows, int(v), tbls, src[int(v)], got)
        for l in range(rows):
            assert np.array_equal(got[l], want[l]), (n, k, rows, l)


def _raid(engine, name):
    import ctypes

    f = getattr(engine.lib(), name)
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    return f


def _vp(bufs):
    import ctypes

    arr = (ctypes.c_void_p * len(bufs))()
    for i, b in enumerate(bufs):
        arr[i] = b.ctypes.data
    return arr


def test_raid_vs_reference_fixtures(cpu_engine, oracle):
    """xor/pq gen + check (the verify op) against raid_base.c outputs, including
    the reference's corruption-position return codes (raid_base.c:96-99)."""
    e = cpu_engine
    xg, xc = _raid(e, "xor_gen"), _raid(e, "xor_check")
    pgb, pc = _raid(e, "pq_gen_base"), _raid(e, "pq_check")
    for case in golden()["raid"]:
        v, n = case["vects"], case["len"]
        bx = [fill_bytes(n, case["seed"] + j) for j in range(v)]
        bp = [fill_bytes(n, case["seed"] + j) for j in range(v)]
        assert xg(v, n, _vp(bx)) == case["xor_ret"]
        assert pgb(v, n, _vp(bp)) == case["pq_ret"]
        assert xc(v, n, _vp(bx)) == case["xor_check"]
        assert pc(v, n & ~7, _vp(bp)) == case["pq_check"]
        assert oracle.fnv(bx[v - 1]) == case["xor_fnv"]
        if v >= 4:
            assert oracle.fnv(bp[v - 2]) == case["p_fnv"] and oracle.fnv(bp[v - 1]) == case["q_fnv"]
    for case in golden()["raid"]:
        v, n = case["vects"], case["len"]
        if n < 8:
            continue
        li = [0, 1, 13, 31, 32, 101, 1024, 4096 + 7].index(n)
        at, vi = (n & ~7) - 2 - (li % 3), (li + v) % (v - 2 if v > 3 else 1)
        bx = [fill_bytes(n, case["seed"] + j) for j in range(v)]
        xg(v, n, _vp(bx))
        bx[vi][at] ^= 0x20
        assert xc(v, n, _vp(bx)) == case["xor_check_corrupt"]
        if v >= 4:
            bp = [fill_bytes(n, case["seed"] + j) for j in range(v)]
            pgb(v, n, _vp(bp))
            bp[vi][at] ^= 0x20
            assert pc(v, n & ~7, _vp(bp)) == case["pq_check_corrupt"], (v, n, vi, at)


def test_pq_check_every_corruption_position(cpu_engine, oracle):
    pg, pc = _raid(cpu_engine, "pq_gen"), _raid(cpu_engine, "pq_check")
    v, n = 12, 1 << 16
    bufs = [fill_bytes(n, 77 + j) for j in range(v)]
    assert pg(v, n, _vp(bufs)) == 0
    assert pc(v, n, _vp(bufs)) == 0
    rng = np.random.default_rng(5)
    for _ in range(40):
        j, i = int(rng.integers(0, v)), int(rng.integers(0, n))
        bufs[j][i] ^= 0x41
        want = [x.copy() for x in bufs]
        assert pc(v, n, _vp(bufs)) == oracle.raid("pq_check", v, n, want), (j, i)
        bufs[j][i] ^= 0x41


CONFORMANCE = ["gf_inverse_test", "gf_vect_mul_test", "gf_vect_mul_base_test",
               "gf_vect_dot_prod_base_test", "gf_vect_dot_prod_test", "gf_vect_mad_test",
               "erasure_code_base_test", "erasure_code_test", "erasure_code_update_test",
               "xor_gen_test", "pq_gen_test", "xor_check_test", "pq_check_test", "crc64_funcs_test"]


def run_programs(directory, names, env, timeout=600):
    """Run the reference's test programs concurrently (one per host core);
    returns {name: (rc, output tail)}, skipping programs that are not built."""
    from concurrent.futures import ThreadPoolExecutor

    def one(name):
        exe = os.path.join(directory, name)
        if not os.path.exists(exe):
            return name, None
        r = subprocess.run([exe], capture_output=True, text=True, timeout=timeout, env=env)
        return name, (r.returncode, (r.stdout + r.stderr)[-2000:])

    with ThreadPoolExecutor(max_workers=max(1, min(8, os.cpu_count() or 1))) as ex:
        return dict(ex.map(one, names))


def test_reference_test_programs_on_cpu_route():
    """The reference's own EC / RAID test programs, unmodified, linked against
    libisal_hip.so, with every call on the CPU route."""
    res = run_programs(os.path.join(ecutil.REF_DIR, "conformance"), CONFORMANCE,
                       dict(os.environ, ISAL_HIP_BACKEND="cpu"))
    if all(v is None for v in res.values()):
        pytest.skip("not built (make -C oracle conformance needs /root/reference)")
    for name, v in res.items():
        assert v is not None, f"{name} not built"
        rc, out = v
        assert rc == 0 and "pass" in out.lower(), (name, out)


def test_bench_c1_cpu_plumbing():
    """BASELINE configs[0] (C1, k=4 p=2 Cauchy, one 64 KiB stripe on the CPU):
    `bench.py --workload c1` times the drop-in call (engine CPU route) and the
    reference's ec_encode_data_base, both == the fixture's parity."""
    import json
    import subprocess
    import sys

    r = subprocess.run([sys.executable, os.path.join(ecutil.REPO, "bench.py"), "--workload", "c1",
                        "--cpu-seconds", "0.2"], capture_output=True, text=True, timeout=300, cwd=ecutil.REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["parity_matches_fixture"] is True and out["value"] > 0
    if out["cpu_baseline"] is not None:
        assert out["cpu_baseline"]["parity_matches_fixture"] is True


# --------------------------------------------------------------------------
# checksum entry points (crc.h / crc64.h) on host buffers: the CPU route
# --------------------------------------------------------------------------

def _crc_lengths():
    return list(range(0, 301)) + [511, 4095, 4096, 4097, 65536 + 7, 1 << 20]


@pytest.mark.parametrize("simd", ["1", "0"])
def test_crc32_iscsi_host_route_vs_oracle(engine, oracle, monkeypatch, simd):
    """crc32_iscsi / _base (reference include/crc.h:136-150) on host buffers:
    == the oracle's restatement of crc_base.c:205-219 at lengths 0..300 and
    beyond (every 128-byte fold count with ragged tails from 256 on: the
    PCLMULQDQ folding, then SSE4.2), misaligned starts, random inits; and
    (CPU_SIMD=0) the slicing-by-8 tables; the committed reference fixtures."""
    monkeypatch.setenv("ISAL_HIP_CPU_SIMD", simd)
    engine.reload_config()
    rng = np.random.default_rng(5)
    big = fill_bytes((1 << 20) + 64, 77)
    for n in _crc_lengths() + list(range(301, 1400, 13)) + [(1 << 20) - 1, (1 << 20) - 129]:
        off = int(rng.integers(0, 16))
        a = np.ascontiguousarray(big[off: off + n])
        init = int(rng.integers(0, 1 << 32))
        want = oracle.crc32_iscsi(a, init)
        assert engine.crc32_iscsi(a, n, init) == want, (n, off)
        assert engine.crc32_iscsi(a, n, init, base=True) == want, (n, off)
    assert engine.crc32_iscsi(None, 0, 0x1234) == 0x1234
    assert engine.crc32_iscsi(big, -5, 0x1234) == 0x1234  # no byte runs for len <= 0
    for case in golden().get("crc32_iscsi", []):
        a = ecutil.crc_fixture_bytes(case)
        assert engine.crc32_iscsi(a, a.size, case["init"]) == case["crc"], case.get("len")
    monkeypatch.undo()
    engine.reload_config()


@pytest.mark.parametrize("simd", ["1", "0"])
@pytest.mark.parametrize("variant", range(8))
def test_crc64_host_route_vs_oracle(engine, oracle, monkeypatch, variant, simd):
    """crc64_<flavour> / _base (reference include/crc64.h:54-163) on host
    buffers: == the oracle's restatement of crc64_base.c at lengths 0..300
    and beyond — every 128-byte fold count with ragged tails from 256 on
    (the PCLMULQDQ path) — misaligned starts, random inits; (CPU_SIMD=0) the
    slicing-by-8 tables alone; chaining crc(crc(init, A), B) ==
    crc(init, A || B); the reference fixtures."""
    monkeypatch.setenv("ISAL_HIP_CPU_SIMD", simd)
    engine.reload_config()
    rng = np.random.default_rng(100 + variant)
    big = fill_bytes((1 << 20) + 64, 88)
    for n in _crc_lengths() + list(range(301, 1400, 13)) + [(1 << 20) - 1, (1 << 20) - 129]:
        off = int(rng.integers(0, 16))
        a = np.ascontiguousarray(big[off: off + n])
        init = int(rng.integers(0, 1 << 63)) * 2 + int(rng.integers(0, 2))
        want = oracle.crc64(variant, a, init)
        assert engine.crc64(variant, init, a, n) == want, (variant, n, off)
        assert engine.crc64(variant, init, a, n, base=True) == want, (variant, n, off)
    a = big[:100000]
    cut = 31337
    assert engine.crc64(variant, engine.crc64(variant, 7, a[:cut], cut), np.ascontiguousarray(a[cut:]),
                        a.size - cut) == engine.crc64(variant, 7, a, a.size)
    assert engine.crc64(variant, 0, None, 0) == 0
    for case in golden().get("crc64", []):
        if case["variant"] == variant:
            b = ecutil.crc_fixture_bytes(case)
            assert engine.crc64(variant, int(case["init"]), b, b.size) == int(case["crc"]), case.get("len")
    monkeypatch.undo()
    engine.reload_config()
