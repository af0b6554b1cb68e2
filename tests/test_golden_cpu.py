"""CPU tier: pin the oracle to the reference, and the engine's host math to both.

tests/golden/ec_base_golden.json was produced by oracle/gen_golden.c linked
against the reference's own erasure_code/ec_base.c (see the fixture's
"generator" field). Nothing here needs a GPU.
"""
import numpy as np
import pytest

import ecutil
from ecutil import coeffs, fill_bytes, golden


def _h(s):
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


# --------------------------------------------------------------------------
# oracle == reference (the oracle is trusted only because of these)
# --------------------------------------------------------------------------

def test_oracle_gf_mul_full_table(oracle):
    want = _h(golden()["gf_mul_table"]).reshape(256, 256)
    got = np.array([[oracle.gf_mul(a, b) for b in range(256)] for a in range(256)], np.uint8)
    assert np.array_equal(got, want)


def test_oracle_gf_inv_and_tables(oracle):
    assert bytes(oracle.gf_inv(a) for a in range(256)) == bytes.fromhex(golden()["gf_inv_table"])
    tbl = np.concatenate([oracle.gf_vect_mul_init(c) for c in range(256)])
    assert np.array_equal(tbl, _h(golden()["mul_init_tables"]))


@pytest.mark.parametrize("kind", ["rs", "cauchy"])
def test_oracle_matrices(oracle, kind):
    for m in golden()[f"{kind}_matrices"]:
        gen = oracle.gf_gen_rs_matrix if kind == "rs" else oracle.gf_gen_cauchy1_matrix
        assert np.array_equal(gen(m["m"], m["k"]), _h(m["a"])), (m["m"], m["k"])


def test_oracle_invert(oracle):
    for case in golden()["invert"]:
        n = case["n"]
        ret, out, after = oracle.gf_invert_matrix(_h(case["in"]), n)
        assert ret == case["ret"]
        assert np.array_equal(out, _h(case["out"]))
        assert np.array_equal(after, _h(case["in_after"]))


def _encode_oracle(oracle, case):
    k, rows, n = case["k"], case["rows"], case["len"]
    coef = _h(case["coef"])
    assert np.array_equal(coef, coeffs(case["gen"], k, rows, case["seed"], oracle))
    src = [fill_bytes(n, case["seed"] + j) for j in range(k)]
    return oracle.encode(coef, k, rows, src)


def test_oracle_encode(oracle):
    for case in golden()["encode"]:
        dst = _encode_oracle(oracle, case)
        assert [oracle.fnv(d) for d in dst] == case["fnv"], (case["k"], case["rows"], case["len"])
        if "parity" in case:
            assert [d.tobytes().hex() for d in dst] == case["parity"]
        else:
            assert [d[:16].tobytes().hex() for d in dst] == case["head"]
            assert [d[-16:].tobytes().hex() for d in dst] == case["tail"]


def test_oracle_update(oracle):
    for case in golden()["update"]:
        k, rows, n = case["k"], case["rows"], case["len"]
        coef = coeffs(case["gen"], k, rows, case["seed"], oracle)
        tbls = oracle.ec_init_tables(k, rows, coef)
        src = [fill_bytes(n, case["seed"] + j) for j in range(k)]
        dst = [np.zeros(n, np.uint8) for _ in range(rows)]
        order = range(k - 1, -1, -1) if case["reverse"] else range(k)
        for v in order:
            oracle.ec_encode_data_update(n, k, rows, v, tbls, src[v], dst)
        assert [oracle.fnv(d) for d in dst] == case["fnv"]


def test_oracle_decode(oracle):
    for case in golden()["decode"]:
        k, p, n, errs = case["k"], case["p"], case["len"], case["errs"]
        gen = oracle.gf_gen_rs_matrix if case["gen"] == "rs" else oracle.gf_gen_cauchy1_matrix
        a = gen(k + p, k)
        ret, c, surv = ecutil.decode_matrix(a, k, errs, oracle)
        assert ret == case["invert_ret"]
        assert c.tobytes().hex() == case["decode_matrix"]
        assert case["recovered_ok"] == 1
        frag = [fill_bytes(n, case["seed"] + j) for j in range(k)]
        frag += oracle.encode(a[k * k:], k, p, frag)
        rec = oracle.encode(c, k, len(errs), [frag[s] for s in surv])
        for i, e in enumerate(errs):
            assert np.array_equal(rec[i], frag[e])
            assert oracle.fnv(rec[i]) == case["fnv"][i]


def test_oracle_single_output_primitives(oracle):
    g = golden()
    for case in g["dot_prod"]:
        vlen, n = case["vlen"], case["len"]
        coef = fill_bytes(vlen, case["coef_seed"])
        tbls = np.concatenate([oracle.gf_vect_mul_init(int(c)) for c in coef])
        src = [fill_bytes(n, case["src_seed"] + j) for j in range(vlen)]
        d = np.zeros(n, np.uint8)
        oracle.gf_vect_dot_prod(n, vlen, tbls, src, d)
        assert d.tobytes().hex() == case["dest"]
    for case in g["mad"]:
        vec, n = case["vec"], case["len"]
        coef = fill_bytes(vec, case["coef_seed"])
        tbls = np.concatenate([oracle.gf_vect_mul_init(int(c)) for c in coef])
        s = fill_bytes(n, case["src_seed"])
        d = fill_bytes(n, case["dest_seed"])
        oracle.gf_vect_mad(n, vec, case["vec_i"], tbls, s, d)
        assert d.tobytes().hex() == case["dest"]
    for case in g["vect_mul"]:
        n = case["len"]
        s = fill_bytes(n, case["src_seed"])
        d = np.zeros(n, np.uint8)
        assert oracle.gf_vect_mul(n, oracle.gf_vect_mul_init(case["c"]), s, d) == case["ret"]
        assert d.tobytes().hex() == case["dest"]


def test_fill_bytes_matches_c(oracle):
    import ctypes

    for n, seed in [(0, 1), (1, 2), (13, 3), (4096, 77), (1001, 2**63 + 5)]:
        c = np.zeros(max(n, 1), np.uint8)
        oracle.L.oracle_fill_bytes(ctypes.c_void_p(c.ctypes.data), ctypes.c_longlong(n),
                                   ctypes.c_ulonglong(seed))
        assert np.array_equal(c[:n], fill_bytes(n, seed))


# --------------------------------------------------------------------------
# engine host-side math (libisal_hip.so, no GPU involved) == reference
# --------------------------------------------------------------------------

def test_engine_gf_scalar(engine):
    want = _h(golden()["gf_mul_table"]).reshape(256, 256)
    for a in range(0, 256, 3):
        assert bytes(engine.gf_mul(a, b) for b in range(256)) == want[a].tobytes()
    assert bytes(engine.gf_inv(a) for a in range(256)) == bytes.fromhex(golden()["gf_inv_table"])


def test_engine_tables_and_matrices(engine):
    tbl = np.concatenate([engine.gf_vect_mul_init(c) for c in range(256)])
    assert np.array_equal(tbl, _h(golden()["mul_init_tables"]))
    for m in golden()["rs_matrices"]:
        assert np.array_equal(engine.gf_gen_rs_matrix(m["m"], m["k"]), _h(m["a"]))
    for m in golden()["cauchy_matrices"]:
        assert np.array_equal(engine.gf_gen_cauchy1_matrix(m["m"], m["k"]), _h(m["a"]))
    # ec_init_tables emits the portable base format (byte 1 = coefficient)
    coef = fill_bytes(40, 9)
    assert np.array_equal(engine.ec_init_tables(10, 4, coef), ecutil.oracle().ec_init_tables(10, 4, coef))


def test_engine_invert(engine):
    for case in golden()["invert"]:
        ret, out, after = engine.gf_invert_matrix(_h(case["in"]), case["n"])
        assert ret == case["ret"]
        assert np.array_equal(out, _h(case["out"]))
        assert np.array_equal(after, _h(case["in_after"]))


def test_engine_invert_reference_fixed_matrices(engine):
    """The fixed matrices of the reference's gf_inverse_test.c:132-174."""
    ret, _, _ = engine.gf_invert_matrix([0, 0, 0, 0, 1, 0, 0, 0, 1], 3)  # singular
    assert ret != 0
    for n, m in [(3, [1, 0, 0, 0, 1, 0, 0, 0, 1]), (4, [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17])]:
        ret, inv, _ = engine.gf_invert_matrix(m, n)
        if ret:
            continue
        for i in range(n):
            for j in range(n):
                s = 0
                for t in range(n):
                    s ^= engine.gf_mul(m[i * n + t], int(inv[t * n + j]))
                assert s == (1 if i == j else 0)


def test_engine_version(engine):
    assert engine.version() == "2.32.1"
    assert engine.lib().isal_get_version() == (2 << 16) | (32 << 8) | 1
    assert engine.max_rows_per_pass() >= 6


def test_gf_vect_mul_rejects_bad_length_without_gpu(engine):
    """Reference contract (gf_vect_mul_test.c:179-187): len % 32 != 0 -> non-zero, nothing touched."""
    s = fill_bytes(100, 1)
    d = np.zeros(100, np.uint8)
    t = engine.gf_vect_mul_init(7)
    for n in (1, 31, 33, 63, 99):
        assert engine.gf_vect_mul(n, t, s, d) != 0
        assert engine.gf_vect_mul_base(n, t, s, d) != 0
    assert not d.any()


def test_gfni_port_matches_oracle(oracle):
    """The CPU SIMD baseline (port of the reference's AVX-512+GFNI kernels) is bit-exact."""
    import ctypes
    import os

    path = os.path.join(ecutil.ORACLE_DIR, "libgfni_port.so")
    if not os.path.exists(path):
        import subprocess

        subprocess.run(["make", "-s", "-C", ecutil.ORACLE_DIR, "libgfni_port.so"], check=True)
    G = ctypes.CDLL(path)
    if not G.gfni_port_available():
        pytest.skip("host CPU lacks AVX-512BW + GFNI")
    from ecutil import _p, _pp

    for k, rows, n in [(10, 4, 65536), (20, 6, 4096 + 13), (3, 7, 63), (1, 1, 1), (64, 16, 1000), (10, 4, 0)]:
        coef = fill_bytes(k * rows, k * 100 + rows)
        t = oracle.ec_init_tables(k, rows, coef)
        src = [fill_bytes(n, 7 * j + k) for j in range(k)]
        want = oracle.encode(coef, k, rows, src)
        got = [np.zeros(n, np.uint8) for _ in range(rows)]
        G.gfni_port_ec_encode_data(n, k, rows, _p(t), _pp(src), _pp(got))
        assert all(np.array_equal(a, b) for a, b in zip(got, want)), (k, rows, n)


def _raid_case_arrays(case):
    v, n = case["vects"], case["len"]
    return [fill_bytes(n, case["seed"] + j) for j in range(v)]


def test_oracle_raid(oracle):
    """oracle restatement of raid_base.c == the reference's raid_base.c outputs."""
    for case in golden()["raid"]:
        v, n = case["vects"], case["len"]
        bx, bp = _raid_case_arrays(case), _raid_case_arrays(case)
        assert oracle.raid("xor_gen", v, n, bx) == case["xor_ret"]
        assert oracle.raid("pq_gen", v, n, bp) == case["pq_ret"]
        assert oracle.raid("xor_check", v, n, bx) == case["xor_check"]
        assert oracle.raid("pq_check", v, n & ~7, bp) == case["pq_check"]
        assert oracle.fnv(bx[v - 1]) == case["xor_fnv"]
        if v >= 4:
            assert oracle.fnv(bp[v - 2]) == case["p_fnv"] and oracle.fnv(bp[v - 1]) == case["q_fnv"]


def test_oracle_crc32_iscsi(oracle):
    """oracle restatement of crc_base.c crc32_iscsi_base == the reference's outputs
    (tests/golden crc32_iscsi section), plus the standard CRC32C check value."""
    from ecutil import crc_fixture_bytes

    cases = golden()["crc32_iscsi"]
    assert len(cases) >= 50
    for case in cases:
        assert oracle.crc32_iscsi(crc_fixture_bytes(case), case["init"]) == case["crc"], case
    # CRC-32C check value (RFC 3720 convention: init ~0, final ~): 0xE3069283
    msg = np.frombuffer(b"123456789", np.uint8)
    assert oracle.crc32_iscsi(msg, 0xFFFFFFFF) ^ 0xFFFFFFFF == 0xE3069283


def test_oracle_crc64(oracle):
    """oracle restatement of crc64_base.c (all eight crc64_*_base flavours) ==
    the reference's outputs (tests/golden crc64 section), plus the published
    check values of the two ECMA-182 conventions."""
    from ecutil import crc_fixture_bytes

    cases = golden()["crc64"]
    assert {c["variant"] for c in cases} == set(range(8)) and len(cases) >= 100
    for case in cases:
        got = oracle.crc64(case["variant"], crc_fixture_bytes(case), int(case["init"]))
        assert got == int(case["crc"]), case
    msg = np.frombuffer(b"123456789", np.uint8)
    assert oracle.crc64(0, msg, 0) == 0x995DC9BBDF1939FA  # CRC-64/XZ = crc64_ecma_refl(0, .)
    assert oracle.crc64(1, msg, 0) == 0x62EC59E3F1A4F00A  # CRC-64/WE = crc64_ecma_norm(0, .)


def test_simd_port_crc32_iscsi_matches_oracle(oracle):
    """The SSE4.2 crc32 baseline (oracle/ec_gfni_port.c) == oracle crc32_iscsi."""
    import ctypes
    import os

    path = os.path.join(ecutil.ORACLE_DIR, "libgfni_port.so")
    if not os.path.exists(path):
        pytest.skip("libgfni_port.so not built")
    G = ctypes.CDLL(path)
    G.gfni_port_crc32_iscsi.restype = ctypes.c_uint
    G.gfni_port_crc32_iscsi.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_uint]
    for n in (0, 1, 7, 8, 23, 24, 25, 4096, 65536 + 5):
        a = fill_bytes(n, n + 11)
        init = (n * 2654435761) & 0xFFFFFFFF
        assert G.gfni_port_crc32_iscsi(a.ctypes.data, n, init) == oracle.crc32_iscsi(a, init), n
