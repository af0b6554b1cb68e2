"""GPU tier: the HIP path (through the C ABI of libisal_hip.so) vs the oracle.

Bar: bit-exact. Sizes where the oracle finishes in seconds are compared byte
for byte with the oracle and with the committed reference fixtures; the
BASELINE.json full sizes are checked through size-independent properties
(decode round trips, the all-ones Vandermonde row == XOR of sources, and
oracle spot checks of sampled stripes).
"""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import ecutil
from ecutil import coeffs, fill_bytes, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _force_gpu_route(engine):
    """Every drop-in call in this module runs the GPU kernels, whatever its size
    (the library's default would send small host calls to its CPU route)."""
    with pytest.MonkeyPatch.context() as mp:
        mp.setenv("ISAL_HIP_BACKEND", "gpu")
        engine.reload_config()
        yield
    engine.reload_config()


@pytest.fixture(autouse=True)
def _reload_knobs_after(engine):
    """Knobs are read once by the library: tests that change one re-read them
    (_setenv), and every test leaves the library re-synced with os.environ."""
    yield
    engine.reload_config()


def _setenv(monkeypatch, name, value):
    import isal_amd

    if value is None:  # back to the library's default
        monkeypatch.delenv(name, raising=False)
    else:
        monkeypatch.setenv(name, value)
    isal_amd.reload_config()


def _h(s):
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


def _dev(torch, a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _host(t):
    return t.cpu().numpy()


# --------------------------------------------------------------------------
# golden fixtures through the drop-in API (host and device buffers)
# --------------------------------------------------------------------------

@pytest.mark.parametrize("where", ["host", "device"])
def test_golden_encode(engine, oracle, gpu, where):
    import torch

    launches0 = engine.kernel_launches()
    for case in golden()["encode"]:
        k, rows, n = case["k"], case["rows"], case["len"]
        coef = _h(case["coef"])
        tbls = engine.ec_init_tables(k, rows, coef)
        src = [fill_bytes(n, case["seed"] + j) for j in range(k)]
        if where == "host":
            dst = [np.full(n, 0xA5, np.uint8) for _ in range(rows)]
            engine.ec_encode_data(n, k, rows, tbls, src, dst)
        else:
            dsrc = [_dev(torch, s, gpu) for s in src]
            ddst = [torch.full((n,), 0xA5, dtype=torch.uint8, device=gpu) for _ in range(rows)]
            engine.ec_encode_data(n, k, rows, tbls, dsrc, ddst)
            dst = [_host(d) for d in ddst]
        assert [oracle.fnv(d) for d in dst] == case["fnv"], (k, rows, n, where)
        if "parity" in case:
            assert [d.tobytes().hex() for d in dst] == case["parity"]
    assert engine.kernel_launches() > launches0  # the GPU path really ran


def test_golden_update_and_decode(engine, oracle, gpu):
    for case in golden()["update"]:
        k, rows, n = case["k"], case["rows"], case["len"]
        tbls = engine.ec_init_tables(k, rows, coeffs(case["gen"], k, rows, case["seed"]))
        src = [fill_bytes(n, case["seed"] + j) for j in range(k)]
        dst = [np.zeros(n, np.uint8) for _ in range(rows)]
        for v in (range(k - 1, -1, -1) if case["reverse"] else range(k)):
            engine.ec_encode_data_update(n, k, rows, v, tbls, src[v], dst)
        assert [oracle.fnv(d) for d in dst] == case["fnv"]
    for case in golden()["decode"]:
        k, p, n, errs = case["k"], case["p"], case["len"], case["errs"]
        gen = engine.gf_gen_rs_matrix if case["gen"] == "rs" else engine.gf_gen_cauchy1_matrix
        a = gen(k + p, k)
        ret, c, surv = ecutil.decode_matrix(a, k, errs)
        assert c.tobytes().hex() == case["decode_matrix"]
        frag = [fill_bytes(n, case["seed"] + j) for j in range(k)] + [np.zeros(n, np.uint8) for _ in range(p)]
        engine.ec_encode_data(n, k, p, engine.ec_init_tables(k, p, a[k * k:]), frag[:k], frag[k:])
        rec = [np.zeros(n, np.uint8) for _ in errs]
        engine.ec_encode_data(n, k, len(errs), engine.ec_init_tables(k, len(errs), c),
                              [frag[s] for s in surv], rec)
        assert [oracle.fnv(r) for r in rec] == case["fnv"]
        for i, e in enumerate(errs):
            assert np.array_equal(rec[i], frag[e])


def test_golden_single_output_primitives(engine, gpu):
    g = golden()
    for case in g["dot_prod"]:
        vlen, n = case["vlen"], case["len"]
        tbls = np.concatenate([engine.gf_vect_mul_init(int(c)) for c in fill_bytes(vlen, case["coef_seed"])])
        src = [fill_bytes(n, case["src_seed"] + j) for j in range(vlen)]
        for f in (engine.gf_vect_dot_prod, engine.gf_vect_dot_prod_base):
            d = np.zeros(n, np.uint8)
            f(n, vlen, tbls, src, d)
            assert d.tobytes().hex() == case["dest"]
    for case in g["mad"]:
        vec, n = case["vec"], case["len"]
        tbls = np.concatenate([engine.gf_vect_mul_init(int(c)) for c in fill_bytes(vec, case["coef_seed"])])
        for f in (engine.gf_vect_mad, engine.gf_vect_mad_base):
            d = fill_bytes(n, case["dest_seed"])
            f(n, vec, case["vec_i"], tbls, fill_bytes(n, case["src_seed"]), d)
            assert d.tobytes().hex() == case["dest"]
    for case in g["vect_mul"]:
        n = case["len"]
        for f in (engine.gf_vect_mul, engine.gf_vect_mul_base):
            d = np.zeros(n, np.uint8)
            assert f(n, engine.gf_vect_mul_init(case["c"]), fill_bytes(n, case["src_seed"]), d) == case["ret"]
            assert d.tobytes().hex() == case["dest"]


# --------------------------------------------------------------------------
# randomized differential sweeps vs the oracle
# --------------------------------------------------------------------------

def test_random_shapes_vs_oracle(engine, oracle, gpu):
    """k up to 64, rows up to 20 (> one kernel pass), ragged lengths incl. 0..17."""
    rng = np.random.default_rng(11)
    lens = [0, 1, 2, 15, 16, 17, 31, 33, 255, 4095, 4096, 4097, 8191, 12345, 65536 + 3]
    for it in range(60):
        k = int(rng.integers(1, 65)) if it % 4 else int(rng.integers(1, 8))
        rows = int(rng.integers(1, 21))
        n = lens[it % len(lens)]
        coef = fill_bytes(k * rows, 1000 + it)
        tbls = engine.ec_init_tables(k, rows, coef)
        src = [fill_bytes(n, 5000 + 97 * it + j) for j in range(k)]
        want = oracle.encode(coef, k, rows, src)
        got = [np.zeros(n, np.uint8) for _ in range(rows)]
        engine.ec_encode_data(n, k, rows, tbls, src, got)
        for l in range(rows):
            assert np.array_equal(got[l], want[l]), (it, k, rows, n, l)


def test_gf_vect_mul_every_constant(engine, oracle, gpu):
    """gf_vect_mul_test.c:92-110 shape: every constant 0..254 over a 128 KiB vector."""
    import torch

    n = 128 * 1024
    s = fill_bytes(n, 42)
    ds = _dev(torch, s, gpu)
    dd = torch.empty(n, dtype=torch.uint8, device=gpu)
    table = np.array([[oracle.gf_mul(c, x) for x in range(256)] for c in range(256)], np.uint8)
    for c in range(255):
        assert engine.gf_vect_mul(n, engine.gf_vect_mul_init(c), ds, dd) == 0
        assert np.array_equal(_host(dd), table[c][s]), c


@pytest.mark.parametrize("where", ["host", "device"])
def test_misaligned_pointers_and_padding_untouched(engine, oracle, gpu, where):
    """erasure_code_test.c:583-709: random offsets 0..31 per shard; bytes outside
    [ptr, ptr+len) must stay untouched."""
    import torch

    rng = np.random.default_rng(7)
    pad = 64
    for it in range(24):
        k, rows = int(rng.integers(1, 17)), int(rng.integers(1, 11))
        n = int(rng.integers(16, 3000))
        coef = fill_bytes(k * rows, 77 + it)
        tbls = engine.ec_init_tables(k, rows, coef)
        offs = [int(rng.integers(0, 32)) for _ in range(k + rows)]
        src_np = [fill_bytes(n, 900 + 31 * it + j) for j in range(k)]
        want = oracle.encode(coef, k, rows, src_np)
        canary = np.uint8(0x5C)
        bufs = []
        for j in range(k + rows):
            b = np.full(n + 2 * pad, canary, np.uint8)
            if j < k:
                b[pad + offs[j]:pad + offs[j] + n] = src_np[j]
            bufs.append(b)
        if where == "device":
            dbufs = [_dev(torch, b, gpu) for b in bufs]
            views = [dbufs[j][pad + offs[j]:pad + offs[j] + n] for j in range(k + rows)]
            engine.ec_encode_data(n, k, rows, tbls, views[:k], views[k:])
            bufs = [_host(b) for b in dbufs]
        else:
            views = [bufs[j][pad + offs[j]:pad + offs[j] + n] for j in range(k + rows)]
            engine.ec_encode_data(n, k, rows, tbls, views[:k], views[k:])
        for l in range(rows):
            b, o = bufs[k + l], offs[k + l]
            assert np.array_equal(b[pad + o:pad + o + n], want[l]), (it, l)
            assert (b[:pad + o] == canary).all() and (b[pad + o + n:] == canary).all(), (it, l)


def test_update_equals_encode_and_mad_tails(engine, oracle, gpu):
    """erasure_code_update_test.c:320-333 + lengths 0..256 (:596-624)."""
    rng = np.random.default_rng(3)
    for n in list(range(0, 257, 7)) + [4096, 4111, 70000]:
        k, rows = int(rng.integers(1, 20)), int(rng.integers(1, 12))
        coef = fill_bytes(k * rows, n + 1)
        tbls = engine.ec_init_tables(k, rows, coef)
        src = [fill_bytes(n, 3 * n + j) for j in range(k)]
        want = [np.zeros(n, np.uint8) for _ in range(rows)]
        engine.ec_encode_data(n, k, rows, tbls, src, want)
        got = [np.zeros(n, np.uint8) for _ in range(rows)]
        for v in rng.permutation(k):
            engine.ec_encode_data_update(n, k, rows, int(v), tbls, src[int(v)], got)
        for l in range(rows):
            assert np.array_equal(got[l], want[l]), (n, k, rows, l)
        assert all(np.array_equal(g, w) for g, w in zip(want, oracle.encode(coef, k, rows, src)))


def test_concurrent_callers(engine, oracle, gpu):
    """The boundary is reentrant: per-thread streams/staging (SURVEY.md §8b threading)."""
    errors = []

    def worker(t):
        try:
            for it in range(6):
                k, rows, n = 5 + t, 3, 10000 + 17 * it
                coef = fill_bytes(k * rows, 100 * t + it)
                src = [fill_bytes(n, 7 * t + 13 * it + j) for j in range(k)]
                got = [np.zeros(n, np.uint8) for _ in range(rows)]
                engine.ec_encode_data(n, k, rows, engine.ec_init_tables(k, rows, coef), src, got)
                want = oracle.encode(coef, k, rows, src)
                if not all(np.array_equal(a, b) for a, b in zip(got, want)):
                    errors.append((t, it))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors, errors


def test_concurrent_large_host_callers(engine, oracle, gpu, monkeypatch):
    """Large host calls from four threads at once, each thread with its own
    staging sets, streams and copy-out worker: pipelined pageable calls
    (several 64 KiB chunks), page-locked in-place calls and updates, every
    result == oracle; the threads' workers are joined when the threads exit."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "gpu")
    _setenv(monkeypatch, "ISAL_HIP_CHUNK_KB", "64")
    _setenv(monkeypatch, "ISAL_HIP_STAGE_MB", "8")
    errors = []

    def worker(t):
        try:
            for it in range(3):
                k, rows, n = 4 + t, 2 + it, 800000 + 4096 * t + 16 * it  # > 4 MiB staged: chunked
                coef = fill_bytes(k * rows, 1000 * t + it)
                tbls = engine.ec_init_tables(k, rows, coef)
                src = [fill_bytes(n, 70 * t + 11 * it + j) for j in range(k)]
                if (t + it) % 2:  # page-locked sources and outputs: used in place
                    src = [torch.from_numpy(x).pin_memory().numpy() for x in src]
                    got = [torch.zeros(n, dtype=torch.uint8).pin_memory().numpy() for _ in range(rows)]
                else:
                    got = [np.zeros(n, np.uint8) for _ in range(rows)]
                engine.ec_encode_data(n, k, rows, tbls, src, got)
                want = oracle.encode(coef, k, rows, src)
                if not all(np.array_equal(a, b) for a, b in zip(got, want)):
                    errors.append(("encode", t, it))
                upd = [np.zeros(n, np.uint8) for _ in range(rows)]
                for v in range(k):
                    engine.ec_encode_data_update(n, k, rows, v, tbls, src[v], upd)
                if not all(np.array_equal(a, b) for a, b in zip(upd, want)):
                    errors.append(("update", t, it))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors, errors


# --------------------------------------------------------------------------
# batched extension + BASELINE.json configurations
# --------------------------------------------------------------------------

def _stripes(torch, gpu, nstripes, k, rows, n, seed):
    data = torch.empty((nstripes, k, n), dtype=torch.uint8, device=gpu)
    data.random_(generator=torch.Generator(device=gpu).manual_seed(seed))  # uniform 0..255
    coding = torch.zeros((nstripes, rows, n), dtype=torch.uint8, device=gpu)
    dptr = [int(data[s, j].data_ptr()) for s in range(nstripes) for j in range(k)]
    cptr = [int(coding[s, l].data_ptr()) for s in range(nstripes) for l in range(rows)]
    return data, coding, dptr, cptr


def test_batch_encode_update_vs_oracle(engine, oracle, gpu):
    import torch

    k, rows, n, ns = 10, 4, 65536 + 48, 37
    a = engine.gf_gen_rs_matrix(k + rows, k)
    tbls = engine.ec_init_tables(k, rows, a[k * k:])
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 5)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    h_data, h_cod = _host(data), _host(coding)
    for s in (0, 1, 17, ns - 1):
        want = oracle.encode(a[k * k:], k, rows, [h_data[s, j] for j in range(k)])
        for l in range(rows):
            assert np.array_equal(h_cod[s, l], want[l]), (s, l)
    coding.zero_()
    for v in range(k):
        b.update(v, 0)
    torch.cuda.synchronize()
    assert np.array_equal(_host(coding), h_cod)
    b.close()


@pytest.mark.parametrize("k,rows,n,ns", [(10, 4, 65536 + 48, 37), (10, 4, 1 << 20, 16), (7, 3, 4096 * 3, 5)])
def test_batch_encode_xcd_order_vs_oracle(engine, oracle, gpu, k, rows, n, ns):
    """The XCD-contiguous work order (EncOrder<2>, the library's) covers every
    (stripe, tile) exactly once: item counts divisible by 8 and not (the
    identity order then), ragged tiles, == oracle on every stripe."""
    import torch

    a = engine.gf_gen_rs_matrix(k + rows, k)
    tbls = engine.ec_init_tables(k, rows, a[k * k:])
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 77)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    h_data, h_cod = _host(data), _host(coding)
    want = _oracle_encode_all(oracle, a[k * k:], k, rows, [[h_data[s, j] for j in range(k)] for s in range(ns)])
    for s in range(ns):
        for l in range(rows):
            assert np.array_equal(h_cod[s, l], want[s][l]), (s, l)
    b.close()


def _coef_01(rng, k, rows, kind):
    """Coefficient matrices for the encode's 0/1 fast path (isal_hip_encmask):
    'mask' = random bytes with row 0 and column 0 random 0/1 (the masks
    matter, not only all-ones), 'rowonly' = row 0 is 0/1 but column 0 is not
    (the pass falls back to lookups), 'big' = no 0/1 structure at all."""
    c = rng.integers(2, 256, (rows, k), dtype=np.uint8)
    if kind in ("mask", "rowonly"):
        c[0] = rng.integers(0, 2, k, dtype=np.uint8)
    if kind == "mask":
        c[:, 0] = rng.integers(0, 2, rows, dtype=np.uint8)
    return c.reshape(-1)


@pytest.mark.parametrize("xor,lds,glds,ldsx", [("1", "1", "1", "0"), ("0", "1", "1", "0"), ("1", "1", "0", "0"),
                                               ("0", "1", "0", "0"), ("1", "0", "0", "0"), ("0", "0", "0", "0"),
                                               ("1", "1", "1", "1"), ("0", "0", "0", "1")])
@pytest.mark.parametrize("k,rows,n,ns,gen", [
    (10, 4, 65536 + 48, 9, "rs"),       # C2 shape class, pairs of sources
    (10, 6, 65536, 8, "rs"),            # P = 6: no pairs
    (10, 8, 32768 + 16, 5, "rs"),       # P = 8
    (20, 6, 65536, 4, "rs"),            # two load groups of 10: source 10 starts no sum
    (12, 9, 16384, 3, "rs"),            # a second pass (row 8): its row 0 is not 0/1
    (7, 5, 4096 * 3 + 32, 6, "rs"),     # U = 4 with a remainder pair and single
    (3, 3, 8192, 4, "rs"),              # k < U: every source in the remainder loop
    (5, 5, 8192, 4, "rs"),              # U = 5 = k
    (64, 4, 4096, 2, "rs"),             # widest k with masks
    (65, 3, 4096, 2, "rs"),             # k > 64: no masks, lookups
    (10, 4, 65536, 5, "mask"), (20, 6, 16384, 3, "mask"), (10, 8, 8192, 3, "mask"),
    (10, 5, 8192, 3, "rowonly"), (10, 4, 8192, 3, "big"),
])
def test_encode_xor_fast_path_vs_oracle(engine, oracle, gpu, monkeypatch, xor, lds, glds, ldsx, k, rows, n, ns, gen):
    """Rows and columns of 0/1 coefficients (gf_gen_rs_matrix row 0 and column
    0, RAID P) take XORs instead of v_perm lookups (ISAL_HIP_ENC_XOR), the low
    table halves come from LDS (ISAL_HIP_ENC_LDS) and passes of 5-8 rows stage
    their sources through the LDS-DMA ring (ISAL_HIP_ENC_GLDS, which always
    takes the LDS halves) — or, for batches over k <= 64 sources, look their
    products up in LDS product tables (ISAL_HIP_ENC_LDSX=1 forces them for
    every such pass): batch and drop-in encode == oracle with each on and off."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_ENC_XOR", xor)
    _setenv(monkeypatch, "ISAL_HIP_ENC_LDS", lds)
    _setenv(monkeypatch, "ISAL_HIP_ENC_GLDS", glds)
    _setenv(monkeypatch, "ISAL_HIP_ENC_LDSX", ldsx)
    if gen == "rs":
        coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    else:
        coef = _coef_01(np.random.default_rng(k * 131 + rows), k, rows, gen)
    tbls = engine.ec_init_tables(k, rows, coef)
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 1000 + k + rows)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    h_data, h_cod = _host(data), _host(coding)
    want = _oracle_encode_all(oracle, coef, k, rows, [[h_data[s, j] for j in range(k)] for s in range(ns)])
    for s in range(ns):
        for l in range(rows):
            assert np.array_equal(h_cod[s, l], want[s][l]), (s, l)
    b.close()
    # the drop-in call on device shards of the last stripe
    out = [torch.zeros(n, dtype=torch.uint8, device=gpu) for _ in range(rows)]
    engine.ec_encode_data(n, k, rows, tbls, [data[ns - 1, j] for j in range(k)], out)
    for l in range(rows):
        assert np.array_equal(out[l].cpu().numpy(), want[ns - 1][l]), l


@pytest.mark.parametrize("k,rows,n,ns,gen", [
    (20, 6, 65536 + 48, 5, "rs"),       # two groups of 10, XOR + LDS variant, ragged tail
    (16, 4, 4096 * 3 + 16, 7, "rs"),    # two groups of 8, one-vector tail
    (24, 8, 32768, 3, "rs"),            # two groups of 12, P = 8
    (40, 3, 8192 + 4000, 4, "rs"),      # four groups of 10
    (30, 1, 16384, 9, "rs"),            # three groups of 10 (odd), P = 1
    (32, 5, 8192, 8, "big"),            # four groups of 8, no 0/1 structure
    (20, 7, 4096, 2, "mask"),           # masks, a group that does not start at source 0
    (36, 12, 8192, 3, "rs"),            # two passes (8 + 4 rows) of three groups of 12
    (13, 6, 4096 * 5, 3, "rs"),         # odd k: the LDS-DMA ring's single last source
    (9, 7, 4096 * 4 + 16, 3, "mask"),   # ring of 4 over k = 9: a partial last round
])
@pytest.mark.parametrize("glds,ldsx", [("1", "0"), ("0", "0"), ("1", "1"), (None, None)])
def test_encode_load_groups_vs_oracle(engine, oracle, gpu, monkeypatch, glds, ldsx, k, rows, n, ns, gen):
    """Stripes of two or more load groups (enc_group: k a multiple of 8, 10 or
    12 above it): batch encode == oracle with ragged tails, odd group counts
    and two passes; passes of 5-8 rows through the LDS product tables
    (ISAL_HIP_ENC_LDSX=1), the LDS-DMA ring (ISAL_HIP_ENC_LDSX=0), through
    registers (ISAL_HIP_ENC_GLDS=0) and as the library picks by default."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_ENC_GLDS", glds)
    _setenv(monkeypatch, "ISAL_HIP_ENC_LDSX", ldsx)

    if gen == "rs":
        coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    else:
        coef = _coef_01(np.random.default_rng(k * 7 + rows), k, rows, gen)
    tbls = engine.ec_init_tables(k, rows, coef)
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 2000 + k + rows)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    h_data, h_cod = _host(data), _host(coding)
    want = _oracle_encode_all(oracle, coef, k, rows, [[h_data[s, j] for j in range(k)] for s in range(ns)])
    for s in range(ns):
        for l in range(rows):
            assert np.array_equal(h_cod[s, l], want[s][l]), (s, l)
    b.close()


_KARG_SHAPES = [
    (10, 4, 1 << 20),      # C2 stripe
    (10, 4, 16),           # shortest kernel-argument call: one lane
    (10, 4, 4096 * 3 + 7), # ragged tail: 3 bytes past the last full lane dword
    (13, 5, 8192 + 12),    # k % 8: the remainder loop
    (29, 3, 4096),         # k + rows = 32 pointers (the kernel-argument limit)
    (10, 8, 4096 + 4),     # 8 rows
    (1, 1, 64),
    (14, 6, 20000),        # 5 * k * rows = 420 of the 448 table dwords
    (11, 8, 8192 + 100),   # 8 rows on the LDS product tables, k at the table limit, ragged
    (2, 7, 48),            # product tables, k below the load pair, three lanes
    (9, 7, 4096 + 16),     # product tables, odd k, one lane into the second tile
]


@pytest.mark.parametrize("seed", range(8))
def test_batch_encode_random_shapes_vs_oracle(engine, oracle, gpu, seed):
    """Randomized shapes through the batch encode, whatever kernel the
    library's dispatch picks for each pass (v16 at 128 or 256 lanes, the
    LDS-DMA ring, the LDS product tables, byte lanes for ragged tails): k in
    1..64, rows in 1..16 (several passes), any len up to ~40 KiB, random,
    0/1-structured or Vandermonde coefficients; every parity byte == oracle."""
    import torch

    rng = np.random.default_rng(7000 + seed)
    for _ in range(12):
        k = int(rng.integers(1, 65))
        rows = int(rng.integers(1, 17))
        n = int(rng.choice([int(rng.integers(1, 4096)), int(rng.integers(4096, 40960)),
                            4096 * int(rng.integers(1, 10))]))
        ns = int(rng.integers(1, 4))
        kind = str(rng.choice(["rs", "mask", "big"]))
        if kind == "rs" and k + rows <= 255:
            coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
        else:
            coef = _coef_01(rng, k, rows, "mask" if kind == "mask" else "big")
        tbls = engine.ec_init_tables(k, rows, coef)
        data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, int(rng.integers(1, 1 << 30)))
        b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
        b.encode(0)
        torch.cuda.synchronize()
        h_data, h_cod = _host(data), _host(coding)
        want = _oracle_encode_all(oracle, coef, k, rows, [[h_data[s, j] for j in range(k)] for s in range(ns)])
        for s in range(ns):
            for l in range(rows):
                assert np.array_equal(h_cod[s, l], want[s][l]), (k, rows, n, ns, kind, s, l)
        b.close()


@pytest.mark.parametrize("narrow,k,rows,n", [(w,) + s for w in ("1", "0") for s in _KARG_SHAPES] + [
    ("", 10, 4, 1 << 20),         # default threshold: the last 4-byte-lane size
    ("", 10, 4, (1 << 20) + 16),  # one lane past it: the 16-byte-lane kernel
])
def test_dropin_kernel_args_vs_oracle(engine, oracle, gpu, monkeypatch, capfd, narrow, k, rows, n):
    """The drop-in call on 16-byte-aligned device shards passes its pointers and
    tables as kernel arguments; its kernel takes 16 bytes per lane or, with
    ISAL_HIP_KARG_NARROW (default for shards up to 1 MiB while at least 12
    such calls are in flight), 4 bytes per lane: both == oracle, tails
    included, and the route log names the route and the kernel. narrow "" is
    the default: a lone call takes the 16-byte-lane kernel at 1 MiB and at
    1 MiB + 16 (test_dropin_lane_width_follows_concurrency covers the
    concurrent side)."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "gpu")
    _setenv(monkeypatch, "ISAL_HIP_KARG_NARROW", narrow or None)
    _setenv(monkeypatch, "ISAL_HIP_LOG", "2")
    coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:] if rows > 1 else np.full(k, 3, dtype=np.uint8)
    tbls = engine.ec_init_tables(k, rows, coef)
    stride = (n + 15) // 16 * 16 + 256
    buf = torch.empty((k + rows) * stride, dtype=torch.uint8, device=gpu)
    buf.random_(generator=torch.Generator(device=gpu).manual_seed(k * 1000 + n))
    shard = lambda i: buf[i * stride: i * stride + n]  # noqa: E731
    h = _host(buf)
    src = [h[j * stride: j * stride + n] for j in range(k)]
    canary = h[k * stride: (k + rows) * stride].copy()
    want = oracle.encode(coef, k, rows, src)
    capfd.readouterr()
    engine.ec_encode_data(n, k, rows, tbls, [shard(j) for j in range(k)], [shard(k + l) for l in range(rows)])
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    assert "kernel-args" in err
    four = narrow == "1"  # default, one call in flight: 16-byte lanes
    # 16-byte lanes over 7-8 rows take the LDS product tables (isal_hip_karg_ldsx)
    name = "ec_encode_karg4" if four else "ec_encode_karg_ldsx" if rows >= 7 and k <= 12 else "ec_encode_karg"
    assert f"kernel {name}<{rows}>" in err, err
    out = _host(buf)
    for l in range(rows):
        base = (k + l) * stride
        assert np.array_equal(out[base: base + n], want[l]), l
        assert np.array_equal(out[base + n: base + stride], canary[l * stride + n: (l + 1) * stride]), l


@pytest.mark.parametrize("site,step", [("1", "ensure_done"), ("3", "encode launch (kernel arguments)")])
def test_device_resident_failure_aborts_naming_the_call(gpu, site, step):
    """DESIGN §2 'Failures': a call with device-resident shards cannot fall back
    to the CPU route, so a failing HIP step aborts the process with the step
    named. A child process makes one kernel-argument call with a fault
    injected at the allocation site (ISAL_HIP_FAULT=1) or at the launch
    (=3): both fire before anything is launched, so no GPU work is in flight
    when it aborts."""
    code = (
        "import sys; sys.path.insert(0, 'isa-l_amd'); import torch, isal_amd as e\n"
        "k, r, n = 4, 2, 65536\n"
        "a = e.gf_gen_rs_matrix(k + r, k); t = e.ec_init_tables(k, r, a[k * k:])\n"
        "b = torch.zeros((k + r, n), dtype=torch.uint8, device='cuda')\n"
        "e.ec_encode_data(n, k, r, t, [b[j] for j in range(k)], [b[k + l] for l in range(r)])\n"
        "print('returned')\n")
    env = {x: v for x, v in os.environ.items() if not x.startswith("ISAL_HIP_")}
    env["ISAL_HIP_FAULT"] = site
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=ecutil.REPO,
                       timeout=300)
    assert p.returncode != 0 and "returned" not in p.stdout, (p.returncode, p.stdout, p.stderr[-2000:])
    assert step in p.stderr and "device-resident shards" in p.stderr and "aborting" in p.stderr, \
        p.stderr[-2000:]


def test_dropin_lane_width_follows_concurrency(gpu):
    """Default lane width of the drop-in encode (ec_kernels.hip karg_narrow):
    16-byte lanes while fewer than 12 kernel-argument calls are in flight,
    4-byte lanes from 12 on. tools/dropin_bench (C threads, no GIL between
    calls) runs 16 threads of 200 calls each with the kernel log on: both
    kernels must appear, the first (warm-up, one thread) call must be the
    16-byte one, and the run's own parity self-check must pass."""
    exe = os.path.join(ecutil.REPO, "tools", "dropin_bench")
    if not os.path.exists(exe):
        pytest.fail("tools/dropin_bench not built (make -C isa-l_amd tools)")
    env = {k: v for k, v in os.environ.items() if not k.startswith("ISAL_HIP_")}
    env["ISAL_HIP_LOG"] = "2"
    r = subprocess.run([exe, "10", "4", "65536", "64", "16", "0", "200"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert '"self_check": true' in r.stdout, r.stdout
    kern = [l.split("kernel ", 1)[1] for l in r.stderr.splitlines() if l.startswith("isal_hip: kernel ec_encode_karg")]
    assert kern and kern[0] == "ec_encode_karg<4>", kern[:4]
    assert "ec_encode_karg4<4>" in kern, "16 concurrent callers never took the 4-byte-lane kernel"


def test_config_c1_cauchy_k4_p2_64k(engine, gpu):
    case = golden()["encode"][0]
    assert (case["k"], case["rows"], case["len"], case["gen"]) == (4, 2, 65536, "cauchy")
    src = [fill_bytes(65536, case["seed"] + j) for j in range(4)]
    a = engine.gf_gen_cauchy1_matrix(6, 4)
    dst = [np.zeros(65536, np.uint8) for _ in range(2)]
    engine.ec_encode_data(65536, 4, 2, engine.ec_init_tables(4, 2, a[16:]), src, dst)
    assert [ecutil.oracle().fnv(d) for d in dst] == case["fnv"]


def _oracle_encode_all(oracle, coef, k, rows, srcs, threads=16, out=None):
    """Oracle parity of many stripes at once: srcs[s] = list of k host arrays;
    returns (or fills) out[s, row]. ctypes releases the GIL inside the oracle,
    so the stripes run in parallel on the host cores (the oracle is the
    checker, never the code under test). The outputs are one block allocated
    here, not per worker thread: 1 MiB arrays allocated in worker threads and
    freed in this one stayed resident in glibc's per-thread arenas (the GPU
    suite's peak RSS reached 12 GiB, profiles/r05/r05_rss_probe.txt)."""
    from concurrent.futures import ThreadPoolExecutor

    tbls = oracle.ec_init_tables(k, rows, coef)
    n = len(srcs[0][0])
    if out is None:
        out = np.empty((len(srcs), rows, n), np.uint8)

    def one(i):
        oracle.ec_encode_data(n, k, rows, tbls, srcs[i], [out[i, l] for l in range(rows)])

    with ThreadPoolExecutor(max_workers=min(threads, os.cpu_count() or 1)) as ex:
        list(ex.map(one, range(len(srcs))))
    return out


def _check_stripes_vs_oracle(oracle, coef, k, rows, srcs_of, out, ns, chunk=64):
    """out[s] (device, rows x n) == the oracle's encode of srcs_of(s) (a list
    of k device shards) for every stripe s, `chunk` stripes at a time through
    three host blocks allocated once (sources, oracle parity, device parity),
    so the host holds ~chunk x (k + 2 rows) shards, not the whole batch."""
    import torch

    n = int(out.shape[-1])
    c = min(chunk, ns)
    src = np.empty((c, k, n), np.uint8)
    want = np.empty((c, rows, n), np.uint8)
    got = np.empty((c, rows, n), np.uint8)
    for s0 in range(0, ns, chunk):
        s1 = min(ns, s0 + chunk)
        for i, s in enumerate(range(s0, s1)):
            for j, x in enumerate(srcs_of(s)):
                torch.from_numpy(src[i, j]).copy_(x)
        torch.from_numpy(got[:s1 - s0]).copy_(out[s0:s1])
        _oracle_encode_all(oracle, coef, k, rows, [[src[i, j] for j in range(k)] for i in range(s1 - s0)],
                           out=want)
        for i in range(s1 - s0):
            for l in range(rows):
                assert np.array_equal(got[i, l], want[i, l]), (s0 + i, l)


def test_config_c2_c3_full_size(engine, oracle, gpu):
    """C2: k=10 p=4, 1 MiB shards x 1024 stripes in one launch; C3: recover 3
    erased data shards {4,6,7} of every stripe. Full size and byte for byte:
    all 1024 x 4 parity shards == the oracle, all 1024 x 3 recovered shards ==
    the oracle's decode of the same survivors, and == the erased data."""
    import torch

    k, p, n, ns = 10, 4, 1 << 20, 1024
    a = engine.gf_gen_rs_matrix(k + p, k)
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, p, n, 2024)
    enc = engine.Batch(n, k, p, engine.ec_init_tables(k, p, a[k * k:]), ns, dptr, cptr)
    enc.encode(0)
    torch.cuda.synchronize()
    _check_stripes_vs_oracle(oracle, a[k * k:], k, p, lambda s: [data[s, j] for j in range(k)], coding, ns)
    errs = [4, 6, 7]
    ret, c, surv = ecutil.decode_matrix(a, k, errs)
    assert ret == 0
    frag = lambda s, i: data[s, i] if i < k else coding[s, i - k]  # noqa: E731
    rec = torch.zeros((ns, len(errs), n), dtype=torch.uint8, device=gpu)
    sptr = [int(frag(s, i).data_ptr()) for s in range(ns) for i in surv]
    rptr = [int(rec[s, i].data_ptr()) for s in range(ns) for i in range(len(errs))]
    dec = engine.Batch(n, k, len(errs), engine.ec_init_tables(k, len(errs), c), ns, sptr, rptr)
    dec.encode(0)
    torch.cuda.synchronize()
    _check_stripes_vs_oracle(oracle, c, k, len(errs), lambda s: [frag(s, i) for i in surv], rec, ns)
    # and the recovered shards are the erased data, every byte (on the device)
    assert bool(torch.equal(rec, data[:, errs]))
    enc.close()
    dec.close()


@pytest.mark.parametrize("k,rows", [(223, 32), (250, 5), (128, 127), (1, 254)])
def test_maximum_stripe_width_vs_oracle(engine, oracle, gpu, k, rows):
    """The widest stripes GF(2^8) allows (k + rows <= 255; the reference's
    erasure_code_test.c runs up to 127 sources, gf_vect_dot_prod_base_test.c
    250): device shards through the drop-in call (several kernel passes of
    rows, every source in each), ragged length, byte for byte vs the oracle."""
    import torch

    n = 4096 * 3 + 13
    coef = fill_bytes(k * rows, 77 + k)
    tbls = engine.ec_init_tables(k, rows, coef)
    src = [fill_bytes(n, 900 + j) for j in range(k)]
    want = oracle.encode(coef, k, rows, src)
    dsrc = [_dev(torch, s, gpu) for s in src]
    dout = [torch.zeros(n, dtype=torch.uint8, device=gpu) for _ in range(rows)]
    launches = engine.kernel_launches()
    engine.ec_encode_data(n, k, rows, tbls, dsrc, dout)
    assert engine.kernel_launches() > launches
    for l in range(rows):
        assert np.array_equal(_host(dout[l]), want[l]), l
    # update path at the same width: fold the sources in one at a time
    for d in dout:
        d.zero_()
    for v in range(k):
        engine.ec_encode_data_update(n, k, rows, v, tbls, dsrc[v], dout)
    for l in range(rows):
        assert np.array_equal(_host(dout[l]), want[l]), ("update", l)


def test_maximum_shard_length(engine, gpu):
    """len = INT_MAX (2^31 - 1 bytes, the largest `int len` the API takes):
    32-bit buffer offsets and the ragged last tile at the top of the range.
    Checked through size-independent properties: row 0 of the Vandermonde
    matrix is all ones, so parity 0 == XOR of the sources (torch, exact);
    row 1 at 2^20 sampled byte positions plus the first and last 64 KiB ==
    the GF(2^8) product table (built from gf_mul); the 65 guard bytes after
    every shard stay untouched."""
    import torch

    if torch.cuda.get_device_properties(gpu).total_memory < 64 << 30:
        pytest.skip("needs a large-HBM GPU")
    k, rows, n, guard = 2, 2, (1 << 31) - 1, 65  # rows start 16-byte aligned
    a = engine.gf_gen_rs_matrix(k + rows, k)
    tbls = engine.ec_init_tables(k, rows, a[k * k:])
    g = torch.Generator(device=gpu).manual_seed(31)
    src = torch.empty((k, n + guard), dtype=torch.uint8, device=gpu)
    src.random_(generator=g)
    out = torch.full((rows, n + guard), 0xA5, dtype=torch.uint8, device=gpu)
    engine.ec_encode_data(n, k, rows, tbls, [src[j] for j in range(k)], [out[l] for l in range(rows)])
    torch.cuda.synchronize()
    assert torch.equal(out[0, :n], src[0, :n] ^ src[1, :n])
    assert bool((out[:, n:] == 0xA5).all())
    mul = torch.tensor([[engine.gf_mul(c, x) for x in range(256)] for c in range(256)],
                       dtype=torch.uint8, device=gpu)
    c0, c1 = int(a[(k + 1) * k]), int(a[(k + 1) * k + 1])
    pos = torch.cat([torch.arange(0, 1 << 16, device=gpu), torch.arange(n - (1 << 16), n, device=gpu),
                     torch.randint(0, n, (1 << 20,), generator=g, device=gpu)])
    s0, s1 = src[0, pos].long(), src[1, pos].long()
    assert torch.equal(out[1, pos], mul[c0][s0] ^ mul[c1][s1])


@pytest.mark.parametrize("site", [1, 2, 3, 4, 5])
def test_hip_failure_falls_back_to_cpu_route(engine, oracle, gpu, monkeypatch, site):
    """SURVEY §5 'never fail where the reference succeeds': ISAL_HIP_FAULT makes
    every GPU-routed host call fail at one site (allocation, H2D, launch, D2H
    of output row 1, final sync). The call must still return the oracle's
    bytes — from the CPU route, for the columns not yet final — and count a
    fallback; an update that failed after some parity rows were copied back
    must not fold them twice. Zero-copy, packed and column-chunked calls."""
    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    _setenv(monkeypatch, "ISAL_HIP_CPU_MAX_BYTES", "0")  # host calls go to the GPU first
    _setenv(monkeypatch, "ISAL_HIP_STAGE_MB", "1")       # several column chunks
    _setenv(monkeypatch, "ISAL_HIP_FAULT", str(site))
    rng = np.random.default_rng(site)
    for n in (4096, 65536 + 48, 300000):                 # zero-copy, packed, chunked
        k, rows = 6, 5
        coef = fill_bytes(k * rows, n + site)
        tbls = engine.ec_init_tables(k, rows, coef)
        src = [fill_bytes(n, 17 * site + j) for j in range(k)]
        want = oracle.encode(coef, k, rows, src)
        before = engine.fallbacks()
        got = [np.zeros(n, np.uint8) for _ in range(rows)]
        engine.ec_encode_data(n, k, rows, tbls, src, got)
        assert all(np.array_equal(a, b) for a, b in zip(got, want)), ("encode", site, n)
        upd = [np.zeros(n, np.uint8) for _ in range(rows)]
        for v in rng.permutation(k):
            engine.ec_encode_data_update(n, k, rows, int(v), tbls, src[int(v)], upd)
        assert all(np.array_equal(a, b) for a, b in zip(upd, want)), ("update", site, n)
        zero_copy = n == 4096  # the kernel reads/writes pinned memory: no H2D / D2H copies
        if not (zero_copy and site in (2, 4)):
            assert engine.fallbacks() > before, (site, n)


@pytest.mark.parametrize("piped", ["1", "0", "seq"])
@pytest.mark.parametrize("site", [2, 3, 4, 5])
def test_hip_failure_in_a_later_chunk_resumes_on_cpu(engine, oracle, gpu, monkeypatch, site, piped):
    """A HIP failure in column chunk 3 of a call (ISAL_HIP_FAULT_CHUNK): chunks
    0-2 already went through the GPU, so the CPU route resumes at a column
    > 0; an update that failed while copying chunk 3's parity back must not
    fold the rows already copied a second time; RAID checks (the verify
    kernel) must still find the first mismatch. Pipelined chunks
    (ISAL_HIP_PIPE_CHUNKS=1, H2D / kernel / D2H of neighbouring chunks in
    flight at once) and one-chunk-at-a-time (=0). Every result == oracle."""
    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    _setenv(monkeypatch, "ISAL_HIP_CPU_MAX_BYTES", "0")
    _setenv(monkeypatch, "ISAL_HIP_STAGE_MB", "1")
    _setenv(monkeypatch, "ISAL_HIP_CHUNK_KB", "64")
    # "1": pipelined chunks; "0": one chunk at a time, copies shared with the
    # helper thread; "seq": one chunk at a time, one issuing thread
    _setenv(monkeypatch, "ISAL_HIP_PIPE_CHUNKS", "1" if piped == "1" else "0")
    _setenv(monkeypatch, "ISAL_HIP_PAR_COPY", "0" if piped == "seq" else "1")
    _setenv(monkeypatch, "ISAL_HIP_FAULT", str(site))
    _setenv(monkeypatch, "ISAL_HIP_FAULT_CHUNK", "3")
    rng = np.random.default_rng(site)
    k, rows, n = 6, 5, 600000 + 16 * site  # 11 staged shards x n > 4 MiB: the chunked routes
    coef = fill_bytes(k * rows, n)
    tbls = engine.ec_init_tables(k, rows, coef)
    src = [fill_bytes(n, 31 * site + j) for j in range(k)]
    want = oracle.encode(coef, k, rows, src)
    before = engine.fallbacks()
    got = [np.zeros(n, np.uint8) for _ in range(rows)]
    engine.ec_encode_data(n, k, rows, tbls, src, got)
    assert all(np.array_equal(a, b) for a, b in zip(got, want)), ("encode", site)
    assert engine.fallbacks() > before, site
    upd = [np.zeros(n, np.uint8) for _ in range(rows)]
    for v in rng.permutation(k):
        engine.ec_encode_data_update(n, k, rows, int(v), tbls, src[int(v)], upd)
    assert all(np.array_equal(a, b) for a, b in zip(upd, want)), ("update", site)
    # verify (xor_check / pq_check) with a corrupted byte in chunk 4
    xc, pc = _raid_fn(engine, "xor_check"), _raid_fn(engine, "pq_check")
    vec = [fill_bytes(n, 7 * site + j) for j in range(6)]
    assert oracle.raid("pq_gen", 6, n, vec) == 0
    pos = 4 * 28672 + 123 + site
    vec[1][pos] ^= 0x5A
    assert pc(6, n, _vp(vec)) == oracle.raid("pq_check", 6, n, [x.copy() for x in vec])
    xv = [fill_bytes(n, 3 * site + j) for j in range(5)]
    assert oracle.raid("xor_gen", 5, n, xv) == 0
    xv[2][pos] ^= 1
    assert xc(5, n, _vp(xv)) == oracle.raid("xor_check", 5, n, [x.copy() for x in xv])


@pytest.mark.parametrize("direct", ["1", "0"])
def test_pinned_host_shards_read_in_place(engine, oracle, gpu, monkeypatch, capfd, direct):
    """Page-locked host shards (hipHostMalloc via torch pin_memory, the NIC /
    disk-buffer case) are read and written by the kernels in place over PCIe
    (ISAL_HIP_PINNED_DIRECT=1, default) instead of being staged; byte offsets
    into the allocations, pinned + pageable mixes, encode / update / RAID
    verify == oracle either way. An update's parity is staged even when
    pinned (route log), so a failed kernel can never fold a row twice."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    _setenv(monkeypatch, "ISAL_HIP_PINNED_DIRECT", direct)
    _setenv(monkeypatch, "ISAL_HIP_LOG", "1")
    k, rows, n = 6, 3, (3 << 20) + 40
    coef = fill_bytes(k * rows, 77)
    tbls = engine.ec_init_tables(k, rows, coef)
    pool = torch.empty((k + rows) * (n + 64), dtype=torch.uint8).pin_memory().numpy()
    shard = lambda i: pool[i * (n + 64) + 1 + i: i * (n + 64) + 1 + i + n]  # noqa: E731  (odd offsets)
    src = [shard(j) for j in range(k)]
    for j in range(k):
        src[j][:] = fill_bytes(n, 500 + j)
    want = oracle.encode(coef, k, rows, src)
    out = [shard(k + l) for l in range(rows)]
    for mixed in (False, True):
        if mixed:
            src[2] = src[2].copy()  # one pageable source among the pinned ones
        for o in out:
            o[:] = 0x5A
        capfd.readouterr()
        engine.ec_encode_data(n, k, rows, tbls, src, out)
        err = capfd.readouterr().err
        if not mixed:  # every shard page-locked: one launch, no copies at all
            assert ("gpu direct" in err) == (direct == "1"), err
        for l in range(rows):
            assert np.array_equal(out[l], want[l]), (mixed, l)
    upd = [shard(k + l) for l in range(rows)]
    for u in upd:
        u[:] = 0
    for v in range(k):
        engine.ec_encode_data_update(n, k, rows, v, tbls, src[v], upd)
    for l in range(rows):
        assert np.array_equal(upd[l], want[l]), ("update", l)
    pc = _raid_fn(engine, "pq_check")
    vec = [shard(i) for i in range(6)]
    for i in range(4):
        vec[i][:] = fill_bytes(n, 70 + i)
    assert oracle.raid("pq_gen", 6, n - 40, vec) == 0
    vec[3][12345] ^= 0x11
    assert pc(6, n - 40, _vp(vec)) == oracle.raid("pq_check", 6, n - 40, [x.copy() for x in vec])


def test_partly_registered_host_shard_is_staged(engine, oracle, gpu, monkeypatch, capfd):
    """A shard whose first bytes lie in a hipHostRegister'ed range but whose
    tail runs past it must not be read in place (the kernel would touch
    unmapped memory): the engine checks the shard's last byte and stages it.
    Shards wholly inside the registration are still used in place."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    _setenv(monkeypatch, "ISAL_HIP_LOG", "1")
    _setenv(monkeypatch, "ISAL_HIP_CPU_MAX_BYTES", "0")  # every host call to the GPU
    page, k, rows, n = 4096, 4, 2, 1 << 20
    raw = np.zeros((k + rows) * n + 2 * page, np.uint8)
    off = (-raw.ctypes.data) % page
    buf = raw[off:off + (k + rows) * n]
    shard = [buf[i * n:(i + 1) * n] for i in range(k + rows)]
    for j in range(k):
        shard[j][:] = fill_bytes(n, 900 + j)
    coef = fill_bytes(k * rows, 901)
    tbls = engine.ec_init_tables(k, rows, coef)
    want = oracle.encode(coef, k, rows, shard[:k])
    cudart = torch.cuda.cudart()
    for reg in ((k + rows) * n - n // 2, (k + rows) * n):  # last shard half registered, all registered
        assert int(cudart.cudaHostRegister(buf.ctypes.data, reg, 0)) == 0
        try:
            for l in range(rows):
                shard[k + l][:] = 0x5A
            capfd.readouterr()
            engine.ec_encode_data(n, k, rows, tbls, shard[:k], shard[k:])
            err = capfd.readouterr().err
            for l in range(rows):
                assert np.array_equal(shard[k + l], want[l]), (reg, l)
            # partly registered: the tail shard is staged; wholly registered: in place
            assert ("gpu direct" in err) == (reg == (k + rows) * n), err
        finally:
            assert int(cudart.cudaHostUnregister(buf.ctypes.data)) == 0


def test_copy_helper_cap(engine, oracle, gpu, monkeypatch):
    """ISAL_HIP_MAX_HELPERS caps the per-thread copy-out helpers of large staged
    host calls: past the cap a thread issues its copies alone. Results ==
    oracle with no helper at all and with one helper shared by three threads'
    worth of calls."""
    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    k, rows, n = 6, 5, (9 << 20) + 48  # pageable, several 4 MiB chunks: the pipelined route
    coef = fill_bytes(k * rows, 4242)
    tbls = engine.ec_init_tables(k, rows, coef)
    src = [fill_bytes(n, 4300 + j) for j in range(k)]
    want = oracle.encode(coef, k, rows, src)
    for cap in ("0", "1"):
        _setenv(monkeypatch, "ISAL_HIP_MAX_HELPERS", cap)
        outs = [[np.zeros(n, np.uint8) for _ in range(rows)] for _ in range(3)]
        ths = [threading.Thread(target=engine.ec_encode_data, args=(n, k, rows, tbls, src, outs[t]))
               for t in range(3)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        for t in range(3):
            for l in range(rows):
                assert np.array_equal(outs[t][l], want[l]), (cap, t, l)


def test_pinned_calls_take_the_gpu_earlier(engine, oracle, gpu, monkeypatch, capfd):
    """Routing under ISAL_HIP_BACKEND=auto: a 3.7 MB k=10 p=4 call stays on the
    CPU route from pageable buffers (the staged GPU route loses below ~29 MB)
    but goes to the GPU when every shard is page-locked (used in place, the
    GPU wins from ~1.8 MB); both == oracle."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    _setenv(monkeypatch, "ISAL_HIP_LOG", "1")
    k, p, n = 10, 4, 262144
    coef = engine.gf_gen_rs_matrix(k + p, k)[k * k:]
    tbls = engine.ec_init_tables(k, p, coef)
    src = [fill_bytes(n, 40 + j) for j in range(k)]
    want = oracle.encode(coef, k, p, src)
    for pinned in (False, True):
        if pinned:
            s = [torch.from_numpy(x).pin_memory().numpy() for x in src]
            out = [torch.zeros(n, dtype=torch.uint8).pin_memory().numpy() for _ in range(p)]
        else:
            s, out = src, [np.zeros(n, np.uint8) for _ in range(p)]
        capfd.readouterr()
        engine.ec_encode_data(n, k, p, tbls, s, out)
        err = capfd.readouterr().err
        assert ("-> gpu" in err) == pinned and ("-> cpu" in err) == (not pinned), err
        for l in range(p):
            assert np.array_equal(out[l], want[l]), (pinned, l)


def test_large_host_call_pipelined_vs_oracle(engine, oracle, gpu, monkeypatch):
    """A 64 MiB-per-shard synchronous call on pageable host buffers goes
    through the pipelined column chunks (H2D / kernel / D2H of neighbouring
    chunks overlapped); encode and a full update sequence == oracle."""
    _setenv(monkeypatch, "ISAL_HIP_BACKEND", "auto")
    _setenv(monkeypatch, "ISAL_HIP_LOG", "0")
    k, rows, n = 4, 2, 64 << 20
    coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    tbls = engine.ec_init_tables(k, rows, coef)
    src = [fill_bytes(n, 900 + j) for j in range(k)]
    want = oracle.encode(coef, k, rows, src)
    launches = engine.kernel_launches()
    got = [np.zeros(n, np.uint8) for _ in range(rows)]
    engine.ec_encode_data(n, k, rows, tbls, src, got)
    assert engine.kernel_launches() >= launches + 16  # 4 MiB chunks: one launch each
    for l in range(rows):
        assert np.array_equal(got[l], want[l]), l
    upd = [np.zeros(n, np.uint8) for _ in range(rows)]
    for v in range(k):
        engine.ec_encode_data_update(n, k, rows, v, tbls, src[v], upd)
    for l in range(rows):
        assert np.array_equal(upd[l], want[l]), ("update", l)


def test_dropin_call_ordered_after_default_stream_work(engine, oracle, gpu):
    """A synchronous drop-in call on device shards sees work the caller queued
    on the legacy default stream just before it (torch writes the sources and
    clears the outputs, asynchronously) — the engine's stream is blocking."""
    import torch

    k, rows, n = 10, 4, 8 << 20
    coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    tbls = engine.ec_init_tables(k, rows, coef)
    src = torch.zeros((k, n), dtype=torch.uint8, device=gpu)
    out = torch.full((rows, n), 0x77, dtype=torch.uint8, device=gpu)
    for it in range(3):
        # long default-stream kernels right before the call
        src.random_(generator=torch.Generator(device=gpu).manual_seed(it))
        src.bitwise_xor_(torch.full_like(src, 0x5A))
        out.fill_(0x33)
        engine.ec_encode_data(n, k, rows, tbls, [src[j] for j in range(k)], [out[l] for l in range(rows)])
        h = _host(src)
        win = slice(n - 65536, n)  # the last columns: written last by torch
        want = oracle.encode(coef, k, rows, [h[j, win] for j in range(k)])
        got = _host(out[:, win])
        for l in range(rows):
            assert np.array_equal(got[l], want[l]), (it, l)


# --------------------------------------------------------------------------
# fused fragment checksums (CRC32C = reference crc32_iscsi) — SURVEY §8(f)
# --------------------------------------------------------------------------

def test_crc_golden_fixtures(engine, oracle, gpu):
    """isal_hip_batch_crc of one shard == the reference's crc32_iscsi_base outputs
    (tests/golden crc32_iscsi: zero / 0x8a / random buffers, lengths across the
    16-byte lane and 4 KiB tile boundaries, three init values)."""
    import torch

    from ecutil import crc_fixture_bytes

    tbls = engine.ec_init_tables(1, 1, np.array([1], np.uint8))
    out = torch.zeros(2, dtype=torch.int32, device=gpu)
    for case in golden()["crc32_iscsi"]:
        n = case["len"]
        src = _dev(torch, crc_fixture_bytes(case), gpu) if n else torch.zeros(16, dtype=torch.uint8, device=gpu)
        dst = torch.zeros(max(n, 16), dtype=torch.uint8, device=gpu)
        b = engine.Batch(n, 1, 1, tbls, 1, [int(src.data_ptr())], [int(dst.data_ptr())])
        b.crc(case["init"], out, 0)
        torch.cuda.synchronize()
        assert int(out[0].item()) & 0xFFFFFFFF == case["crc"], case
        b.encode_crc(case["init"], out, 0)  # parity = 1 * src: both CRCs equal
        torch.cuda.synchronize()
        got = [int(v) & 0xFFFFFFFF for v in out.tolist()]
        assert got == [case["crc"], case["crc"]], case
        b.close()


def _crc64_words(t):
    return [int(v) & 0xFFFFFFFFFFFFFFFF for v in t.tolist()]


def test_crc64_golden_fixtures(engine, oracle, gpu):
    """isal_hip_batch_crc64 of one shard == the reference's crc64_*_base outputs
    for all eight flavours (tests/golden crc64: lengths across the 16-byte lane,
    4 KiB tile and tail boundaries, three init values)."""
    import torch

    from ecutil import crc_fixture_bytes

    tbls = engine.ec_init_tables(1, 1, np.array([1], np.uint8))
    out = torch.zeros(2, dtype=torch.int64, device=gpu)
    for case in golden()["crc64"]:
        n = case["len"]
        src = _dev(torch, crc_fixture_bytes(case), gpu) if n else torch.zeros(16, dtype=torch.uint8, device=gpu)
        dst = torch.zeros(max(n, 16), dtype=torch.uint8, device=gpu)
        dst[:n] = src[:n]
        b = engine.Batch(n, 1, 1, tbls, 1, [int(src.data_ptr())], [int(dst.data_ptr())])
        b.crc64(case["variant"], int(case["init"]), out, 0)
        torch.cuda.synchronize()
        assert _crc64_words(out) == [int(case["crc"])] * 2, case
        b.close()


CRC64_SHAPES = [
    # k, rows, len, nstripes, byte offset of every shard (0: 16-B aligned), tiles/workgroup
    (10, 4, 65536, 3, 0, None),
    (4, 2, 4096 * 23 + 2048, 2, 0, 3),   # partial last block, tail of whole chunks
    (3, 2, 4096 * 5 + 4095, 2, 0, 2),    # tail with 15 loose bytes
    (2, 1, 4095, 3, 0, None),            # no full tile
    (3, 3, 4096 * 9 + 77, 2, 3, 4),      # unaligned shards: byte-load kernel
    (1, 1, 1, 2, 0, None),
    (5, 2, 4096 * 40, 2, 0, 16),         # several blocks of 16 tiles
]


@pytest.mark.parametrize("variant", range(8))
@pytest.mark.parametrize("k,rows,n,ns,skew,tt", CRC64_SHAPES)
def test_crc64_vs_oracle(engine, oracle, gpu, monkeypatch, variant, k, rows, n, ns, skew, tt):
    """crc64_<variant> of every shard of a batch == the oracle, over ragged
    lengths, unaligned shards and tile-per-workgroup choices; a second variant
    on the same batch re-uploads the tables."""
    import torch

    if tt:
        _setenv(monkeypatch, "ISAL_HIP_CRC_TILES", str(tt))
    a = oracle.gf_gen_rs_matrix(k + rows, k)
    tbls = engine.ec_init_tables(k, rows, a[k * k:].copy())
    bufs = [fill_bytes(n, 7919 * s + j + variant) for s in range(ns) for j in range(k + rows)]
    store = [torch.zeros(n + 32, dtype=torch.uint8, device=gpu) for _ in bufs]
    for t, h in zip(store, bufs):
        t[skew:skew + n] = _dev(torch, h, gpu)
    ptr = [int(t.data_ptr()) + skew for t in store]
    dptr = [ptr[s * (k + rows) + j] for s in range(ns) for j in range(k)]
    cptr = [ptr[s * (k + rows) + k + l] for s in range(ns) for l in range(rows)]
    out = torch.zeros(ns * (k + rows), dtype=torch.int64, device=gpu)
    init = [0, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF][variant % 3]
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.crc64(variant, init, out, 0)
    torch.cuda.synchronize()
    got = _crc64_words(out)
    assert got == [oracle.crc64(variant, h, init) for h in bufs]
    other = (variant + 3) % 8
    b.crc64(other, init, out, 0)
    torch.cuda.synchronize()
    assert _crc64_words(out) == [oracle.crc64(other, h, init) for h in bufs]
    b.close()


CRC_SHAPES = [
    # k, rows, len, nstripes, byte offset of every shard (0: 16-B aligned)
    (10, 4, 65536, 9, 0),             # C2 shape, fused path, tt halving
    (10, 4, 4096 * 37 + 2048, 5, 0),  # ragged last tile, 16-B multiple
    (4, 2, 65536 + 4000, 3, 0),       # fused, ragged tile
    (6, 3, 1000, 4, 0),               # single partial tile
    (3, 2, 4096 * 3 + 13, 3, 0),      # len % 16 != 0 -> encode + CRC pass
    (5, 5, 20000, 2, 1),              # unaligned shards -> byte-load CRC kernel
    (4, 10, 4096 * 5, 2, 0),          # rows > 8: two fused passes
    (64, 4, 4096 * 3 + 32, 2, 0),     # k = 64: the largest fused k (most LDS source chains)
    (70, 3, 4096 * 2 + 32, 2, 0),     # k > 64: encode + CRC pass
    (1, 1, 16, 3, 0),
]


@pytest.mark.parametrize("k,rows,n,ns,skew", CRC_SHAPES)
def test_encode_crc_vs_oracle(engine, oracle, gpu, k, rows, n, ns, skew):
    """Fused encode + CRC: parity == oracle encode, every shard's CRC == oracle
    crc32_iscsi; the checksum-only pass agrees."""
    import torch

    rng = np.random.default_rng(k * 1000 + n)
    a = oracle.gf_gen_rs_matrix(k + rows, k) if k + rows <= 32 else rng.integers(0, 256, (k + rows) * k, dtype=np.uint8)
    coef = a[k * k:].copy()
    tbls = engine.ec_init_tables(k, rows, coef)
    stride = n + 64
    pool = torch.zeros(ns * (k + rows) * stride + 64, dtype=torch.uint8, device=gpu)
    h_data = [[fill_bytes(n, 7 * s + j + n) for j in range(k)] for s in range(ns)]

    def at(s, i):
        return (s * (k + rows) + i) * stride + skew

    for s in range(ns):
        for j in range(k):
            pool[at(s, j):at(s, j) + n] = _dev(torch, h_data[s][j], gpu)
    base = int(pool.data_ptr())
    dptr = [base + at(s, j) for s in range(ns) for j in range(k)]
    cptr = [base + at(s, k + l) for s in range(ns) for l in range(rows)]
    init = 0x9E3779B9 ^ n
    crc = torch.zeros(ns * (k + rows), dtype=torch.int32, device=gpu)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode_crc(init, crc, 0)
    torch.cuda.synchronize()
    h_pool, got = _host(pool), [int(v) & 0xFFFFFFFF for v in crc.tolist()]
    for s in range(ns):
        want = oracle.encode(coef, k, rows, h_data[s])
        shards = h_data[s] + want
        for l in range(rows):
            assert np.array_equal(h_pool[at(s, k + l):at(s, k + l) + n], want[l]), (s, l)
        for i, buf in enumerate(shards):
            assert got[s * (k + rows) + i] == oracle.crc32_iscsi(buf, init), (s, i)
    crc2 = torch.zeros_like(crc)
    b.crc(init, crc2, 0)
    torch.cuda.synchronize()
    assert torch.equal(crc, crc2)
    b.close()


@pytest.mark.parametrize("tt", [1, 2, 3, 5, 8, 16])
@pytest.mark.parametrize("k,rows", [(10, 4), (7, 3)])
def test_encode_crc_tiles_per_workgroup(engine, oracle, gpu, monkeypatch, k, rows, tt):
    """Every tiles-per-workgroup choice (ISAL_HIP_CRC_TILES) gives the oracle's
    CRCs: covers the 8-tile batches and their double buffering in the
    checksum-only kernel (tt >= 8), the one-tile prefetch of the fused kernel,
    partial last blocks (23 full tiles % tt) and the ragged tile."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_CRC_TILES", str(tt))
    n, ns = 4096 * 23 + 2048, 3
    a = oracle.gf_gen_rs_matrix(k + rows, k)
    coef = a[k * k:].copy()
    tbls = engine.ec_init_tables(k, rows, coef)
    h_data = [[fill_bytes(n, 31 * s + j + tt) for j in range(k)] for s in range(ns)]
    data = torch.stack([torch.stack([_dev(torch, h_data[s][j], gpu) for j in range(k)]) for s in range(ns)])
    coding = torch.zeros((ns, rows, n), dtype=torch.uint8, device=gpu)
    dptr = [int(data[s, j].data_ptr()) for s in range(ns) for j in range(k)]
    cptr = [int(coding[s, l].data_ptr()) for s in range(ns) for l in range(rows)]
    crc = torch.zeros(ns * (k + rows), dtype=torch.int32, device=gpu)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode_crc(0xFFFFFFFF, crc, 0)
    torch.cuda.synchronize()
    got = [int(v) & 0xFFFFFFFF for v in crc.tolist()]
    for s in range(ns):
        want = oracle.encode(coef, k, rows, h_data[s])
        for l in range(rows):
            assert np.array_equal(_host(coding[s, l]), want[l]), (s, l)
        for i, buf in enumerate(h_data[s] + want):
            assert got[s * (k + rows) + i] == oracle.crc32_iscsi(buf, 0xFFFFFFFF), (s, i)
    crc2 = torch.zeros_like(crc)
    b.crc(0xFFFFFFFF, crc2, 0)
    torch.cuda.synchronize()
    assert torch.equal(crc, crc2)
    b.close()


@pytest.mark.parametrize("xrows", ["1", "0"])
@pytest.mark.parametrize("k,n,tt", [(10, 4096 * 37 + 2048, 4), (7, 65536, None), (10, 65536, None),
                                    (8, 4096 * 21, 2)])
def test_fused_crc_derived_xor_rows(engine, oracle, gpu, monkeypatch, xrows, k, n, tt):
    """A parity row 0 whose coefficients are all 0/1 gets its CRC32C / CRC64
    chains from the sources' chains instead of being checksummed
    (ISAL_HIP_CRC_XROWS=1, default; other 0/1 rows, an all-zero row and a
    general row are checksummed); both ways every CRC == the oracle, full and
    ragged tiles; k = 8 takes the CRC64 byte-table path after each pair (two
    lane groups per workgroup), k = 10 the path pipelined into the rows."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_CRC_XROWS", xrows)
    if tt:
        _setenv(monkeypatch, "ISAL_HIP_CRC_TILES", str(tt))
    rows, ns = 5, 3
    coef = np.concatenate([np.ones(k, np.uint8),                              # all ones
                           (np.arange(k) % 2).astype(np.uint8),               # 0/1 mix
                           fill_bytes(k, 5),                                  # general
                           np.zeros(k, np.uint8),                             # all zero
                           (np.arange(k) % 3 == 0).astype(np.uint8)])         # sparse 0/1
    tbls = engine.ec_init_tables(k, rows, coef)
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 31 + k)
    h = _host(data)
    want = _oracle_encode_all(oracle, coef, k, rows, [[h[s, j] for j in range(k)] for s in range(ns)])
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    c32 = torch.zeros(ns * (k + rows), dtype=torch.int32, device=gpu)
    b.encode_crc(0x1234567, c32, 0)
    torch.cuda.synchronize()
    hc = _host(coding)
    g32 = [int(v) & 0xFFFFFFFF for v in c32.tolist()]
    coding.zero_()
    c64 = torch.zeros(ns * (k + rows), dtype=torch.int64, device=gpu)
    b.encode_crc64(6, 0xABCDEF, c64, 0)
    torch.cuda.synchronize()
    g64 = [int(v) & 0xFFFFFFFFFFFFFFFF for v in c64.tolist()]
    assert np.array_equal(_host(coding), hc)
    for s in range(ns):
        shards = [h[s, j] for j in range(k)] + list(want[s])
        for l in range(rows):
            assert np.array_equal(hc[s, l], want[s][l]), (s, l)
        for i, buf in enumerate(shards):
            assert g32[s * (k + rows) + i] == oracle.crc32_iscsi(buf, 0x1234567), (s, i, "crc32c")
            assert g64[s * (k + rows) + i] == oracle.crc64(6, buf, 0xABCDEF), (s, i, "crc64")
    b.close()


def test_encode_crc_c2_full_size(engine, oracle, gpu):
    """C2 at full size through the fused path: parity identical to the plain
    encode kernel's, CRCs == oracle on sampled stripes and == the standalone
    checksum pass on all 14336 shards."""
    import torch

    k, p, n, ns = 10, 4, 1 << 20, 1024
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, p, n, 77)
    b = engine.Batch(n, k, p, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    ref = coding.clone()
    coding.zero_()
    crc = torch.zeros(ns * (k + p), dtype=torch.int32, device=gpu)
    b.encode_crc(0xFFFFFFFF, crc, 0)
    torch.cuda.synchronize()
    assert torch.equal(coding, ref)
    del ref
    got = crc.view(ns, k + p)
    for s in (0, 1, 333, 1023):
        for i in range(k + p):
            buf = _host(data[s, i]) if i < k else _host(coding[s, i - k])
            assert int(got[s, i].item()) & 0xFFFFFFFF == oracle.crc32_iscsi(buf, 0xFFFFFFFF), (s, i)
    crc2 = torch.zeros_like(crc)
    b.crc(0xFFFFFFFF, crc2, 0)
    torch.cuda.synchronize()
    assert torch.equal(crc, crc2)
    b.close()


def test_crc64_c2_full_size(engine, oracle, gpu):
    """CRC64 at the C2 size (1024 stripes x 14 x 1 MiB): sampled stripes ==
    oracle for a refl and a norm flavour; on all 14336 shards the affine
    identity crc(P0) = XOR_j crc(d_j) ^ crc(0^n) (k = 10 sources, parity row 0
    = their XOR) holds."""
    import torch

    k, p, n, ns = 10, 4, 1 << 20, 1024
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, p, n, 91)
    b = engine.Batch(n, k, p, tbls, ns, dptr, cptr)
    b.encode(0)
    crc = torch.zeros(ns * (k + p), dtype=torch.int64, device=gpu)
    for variant in (0, 5):
        b.crc64(variant, 0, crc, 0)
        torch.cuda.synchronize()
        got = crc.view(ns, k + p)
        for s in (0, 517, 1023):
            for i in range(k + p):
                buf = _host(data[s, i]) if i < k else _host(coding[s, i - k])
                assert int(got[s, i].item()) & 0xFFFFFFFFFFFFFFFF == oracle.crc64(variant, buf, 0), (variant, s, i)
        c0 = oracle.crc64(variant, np.zeros(n, np.uint8), 0)
        x = got[:, 0].clone()
        for j in range(1, k):
            x ^= got[:, j]
        x ^= c0 if c0 < (1 << 63) else c0 - (1 << 64)
        assert torch.equal(x, got[:, k])
    b.close()


ENCODE_CRC64_SHAPES = [
    # k, rows, len, nstripes, byte offset of every shard, tiles/workgroup, variant
    (10, 4, 65536, 5, 0, None, 0),        # C2 shape: source chains in registers
    (10, 4, 4096 * 37 + 2048, 3, 0, 4, 1),  # ragged tile encoded by the last block
    (7, 3, 4096 * 20, 2, 0, 3, 2),        # k % U != 0: LDS source chains
    (12, 8, 4096 * 9 + 160, 2, 0, 2, 5),  # rows = 8, one group of 12
    (20, 6, 4096 * 6, 2, 0, None, 7),     # k > U: two load groups, LDS chains
    (4, 10, 4096 * 3, 2, 0, None, 4),     # rows > 8 -> encode, then CRC64
    (3, 2, 4096 * 2 + 13, 2, 0, None, 3), # len % 16 != 0 -> encode, then CRC64
    (5, 2, 3000, 3, 0, None, 6),          # no full tile -> encode, then CRC64
    (4, 3, 4096 * 4, 2, 5, None, 0),      # unaligned shards -> encode, then CRC64
    (32, 4, 4096 * 5 + 64, 2, 0, None, 1),  # k = 32: the largest fused k (most LDS source chains)
    (33, 2, 4096 * 2, 2, 0, None, 2),     # k > 32 -> encode, then CRC64
]


@pytest.mark.parametrize("k,rows,n,ns,skew,tt,variant", ENCODE_CRC64_SHAPES)
def test_encode_crc64_vs_oracle(engine, oracle, gpu, monkeypatch, k, rows, n, ns, skew, tt, variant):
    """Fused encode + CRC64 (isal_hip_batch_encode_crc64): parity == oracle
    encode, every shard's crc64_<variant> == oracle; the fallback shapes agree
    through encode-then-CRC64."""
    import torch

    if tt:
        _setenv(monkeypatch, "ISAL_HIP_CRC_TILES", str(tt))
    a = oracle.gf_gen_rs_matrix(k + rows, k)
    coef = a[k * k:].copy()
    tbls = engine.ec_init_tables(k, rows, coef)
    stride = n + 64
    pool = torch.zeros(ns * (k + rows) * stride + 64, dtype=torch.uint8, device=gpu)
    h_data = [[fill_bytes(n, 13 * s + j + n + variant) for j in range(k)] for s in range(ns)]

    def at(s, i):
        return (s * (k + rows) + i) * stride + skew

    for s in range(ns):
        for j in range(k):
            pool[at(s, j):at(s, j) + n] = _dev(torch, h_data[s][j], gpu)
    base = int(pool.data_ptr())
    dptr = [base + at(s, j) for s in range(ns) for j in range(k)]
    cptr = [base + at(s, k + l) for s in range(ns) for l in range(rows)]
    init = [0, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF][variant % 3]
    out = torch.zeros(ns * (k + rows), dtype=torch.int64, device=gpu)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode_crc64(variant, init, out, 0)
    torch.cuda.synchronize()
    h_pool, got = _host(pool), _crc64_words(out)
    for s in range(ns):
        want = oracle.encode(coef, k, rows, h_data[s])
        for l in range(rows):
            assert np.array_equal(h_pool[at(s, k + l):at(s, k + l) + n], want[l]), (s, l)
        for i, buf in enumerate(h_data[s] + want):
            assert got[s * (k + rows) + i] == oracle.crc64(variant, buf, init), (s, i)
    b.close()


@pytest.mark.parametrize("variant", range(8))
def test_encode_crc64_every_flavour(engine, oracle, gpu, monkeypatch, variant):
    """All eight crc64.h flavours through the fused kernel's two chunk paths
    (the u-domain byte-swaps the norm flavours' chains): pipelined into the
    rows for load group 10 (k = 10), after each pair elsewhere (k = 7)."""
    test_encode_crc64_vs_oracle(engine, oracle, gpu, monkeypatch, 10, 4, 4096 * 37 + 2048, 3, 0, 4,
                                variant)
    test_encode_crc64_vs_oracle(engine, oracle, gpu, monkeypatch, 7, 3, 4096 * 20, 2, 0, 3, variant)


@pytest.mark.parametrize("xrows", ["1", "0"])
@pytest.mark.parametrize("k,rows,n,tt,variant", [
    (10, 1, 4096 * 9, None, 0), (10, 2, 4096 * 11 + 1024, 3, 1), (10, 3, 4096 * 8, 2, 2),
    (10, 4, 4096 * 37 + 2048, 4, 5), (20, 3, 4096 * 6 + 512, None, 7), (20, 4, 4096 * 5, 1, 3)])
def test_encode_crc64_pipelined_rows(engine, oracle, gpu, monkeypatch, xrows, k, rows, n, tt, variant):
    """The chain steps pipelined into the GF rows (load group 10, 1-4 rows):
    every row count it serves (rows split over its three stages, one or none
    of them empty), one and two load groups of 10, row 0 derived or computed
    == oracle."""
    _setenv(monkeypatch, "ISAL_HIP_CRC_XROWS", xrows)
    test_encode_crc64_vs_oracle(engine, oracle, gpu, monkeypatch, k, rows, n, 3, 0, tt, variant)


def test_encode_crc64_c2_full_size(engine, oracle, gpu):
    """C2 at full size through the fused encode + CRC64 pass: parity identical
    to the plain encode kernel's, CRC64s == the standalone CRC64 pass on all
    14336 shards and == oracle on sampled stripes."""
    import torch

    k, p, n, ns = 10, 4, 1 << 20, 1024
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, p, n, 53)
    b = engine.Batch(n, k, p, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    ref = coding.clone()
    coding.zero_()
    crc = torch.zeros(ns * (k + p), dtype=torch.int64, device=gpu)
    b.encode_crc64(0, 0, crc, 0)
    torch.cuda.synchronize()
    assert torch.equal(coding, ref)
    del ref
    crc2 = torch.zeros_like(crc)
    b.crc64(0, 0, crc2, 0)
    torch.cuda.synchronize()
    assert torch.equal(crc, crc2)
    got = crc.view(ns, k + p)
    for s in (0, 700, 1023):
        for i in range(k + p):
            buf = _host(data[s, i]) if i < k else _host(coding[s, i - k])
            assert int(got[s, i].item()) & 0xFFFFFFFFFFFFFFFF == oracle.crc64(0, buf, 0), (s, i)
    b.close()


def test_config_c4_streaming_update_k20_p6(engine, oracle, gpu):
    """C4: k=20 p=6, 4 MiB shards, 20 ec_encode_data_update calls into pre-zeroed
    parity == ec_encode_data, and == oracle on a sampled window."""
    import torch

    k, p, n = 20, 6, 4 << 20
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    data, coding, dptr, cptr = _stripes(torch, gpu, 1, k, p, n, 44)
    full = torch.zeros_like(coding)
    engine.ec_encode_data(n, k, p, tbls, [data[0, j] for j in range(k)], [full[0, l] for l in range(p)])
    for v in range(k):
        engine.ec_encode_data_update(n, k, p, v, tbls, data[0, v], [coding[0, l] for l in range(p)])
    assert torch.equal(coding, full)
    lo, hi = 12345, 12345 + 8192
    want = oracle.encode(a[k * k:], k, p, [_host(data[0, j, lo:hi]) for j in range(k)])
    for l in range(p):
        assert np.array_equal(_host(coding[0, l, lo:hi]), want[l])


def test_config_c4_pipeline_full_shape_vs_oracle(engine, oracle, gpu):
    """C4 through the host-memory pipeline at its real shape: k=20 p=6, 4 MiB
    pinned host shards, 4 stripes, update mode (each source folded as it lands)
    with H2D / compute / D2H overlapped — every parity byte == the oracle
    (erasure_code_update_test.c:320-333: update must equal ec_encode_data)."""
    import torch

    k, p, n, ns = 20, 6, 4 << 20, 4
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    src = torch.empty((ns, k, n), dtype=torch.uint8).pin_memory()
    src.random_(generator=torch.Generator().manual_seed(404))
    par = torch.full((ns, p, n), 0xEE, dtype=torch.uint8).pin_memory()
    pipe = engine.Pipe(n, k, p, tbls, depth=3, mode="update")
    for s in range(ns):
        pipe.submit([src[s, j] for j in range(k)], [par[s, l] for l in range(p)])
    pipe.flush()
    pipe.close()
    h = src.numpy()
    want = _oracle_encode_all(oracle, a[k * k:], k, p, [[h[s, j] for j in range(k)] for s in range(ns)])
    for s in range(ns):
        for l in range(p):
            assert np.array_equal(par[s, l].numpy(), want[s][l]), (s, l)


# --------------------------------------------------------------------------
# the reference's own test programs, linked against libisal_hip.so
# --------------------------------------------------------------------------

CONFORMANCE = ["gf_inverse_test", "gf_vect_mul_test", "gf_vect_mul_base_test",
               "gf_vect_dot_prod_base_test", "gf_vect_dot_prod_test", "gf_vect_mad_test",
               "erasure_code_base_test", "erasure_code_test", "erasure_code_update_test",
               "xor_gen_test", "pq_gen_test", "xor_check_test", "pq_check_test", "crc64_funcs_test"]


# xor_check_test / pq_check_test sweep every (length, error position, vector)
# with 1.65e7 / 1.20e7 small synchronous calls (counted from ISAL_HIP_LOG=1
# route lines): forced onto the GPU a 17-buffer 1 KiB call costs 22 us
# (xor_check) / 34 us (pq_check) on pageable memory
# (profiles/r05/r05_raid_small_calls.txt), ~6-7 minutes apiece, so under
# ISAL_HIP_BACKEND=gpu they run only with ISAL_SLOW_CONFORMANCE=1 (logs:
# profiles/r05/r05_slow_conformance.txt, r01/r01_slow_conformance_*.log). Under
# the library's default routing (auto: small host calls on the CPU route, the
# rest on the GPU) all thirteen run.
SLOW_CONFORMANCE = {"xor_check_test", "pq_check_test"}


def _run_streaming(exe, timeout, env=None):
    """Run a test program, echoing a heartbeat so long runs visibly progress."""
    import time

    p = subprocess.Popen([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    t0 = time.time()
    out = []
    while True:
        try:
            o, _ = p.communicate(timeout=60)
            out.append(o)
            break
        except subprocess.TimeoutExpired:
            print(f"[{os.path.basename(exe)}: running {time.time() - t0:.0f} s]", flush=True)
            if time.time() - t0 > timeout:
                p.kill()
                o, _ = p.communicate()
                out.append(o)
                break
    return p.returncode, "".join(out)


@pytest.mark.parametrize("backend", ["gpu", "auto"])
@pytest.mark.parametrize("name", CONFORMANCE)
def test_reference_test_programs(name, backend, gpu):
    if backend == "gpu" and name in SLOW_CONFORMANCE and not os.environ.get("ISAL_SLOW_CONFORMANCE"):
        pytest.skip("~1.6e7 synchronous GPU round trips; set ISAL_SLOW_CONFORMANCE=1 (auto runs it)")
    exe = os.path.join(ecutil.REF_DIR, "conformance", name)
    if not os.path.exists(exe):
        pytest.skip(f"{name} not built (make -C oracle conformance needs /root/reference)")
    rc, out = _run_streaming(exe, timeout=1500, env=dict(os.environ, ISAL_HIP_BACKEND=backend))
    assert rc == 0, out[-3000:]
    assert "Pass" in out or "pass" in out.lower()


# --------------------------------------------------------------------------
# host-memory streaming pipeline (isal_hip_pipe_*)
# --------------------------------------------------------------------------

@pytest.mark.parametrize("mode", ["update", "encode"])
@pytest.mark.parametrize("pinned", [True, False])
def test_pipe_host_stripes_vs_oracle(engine, oracle, gpu, mode, pinned):
    import torch

    k, p, n, ns = 20, 6, 256 * 1024 + 48, 7
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    src = torch.from_numpy(np.stack([np.stack([fill_bytes(n, 1000 * s + j) for j in range(k)]) for s in range(ns)]))
    par = torch.full((ns, p, n), 0xEE, dtype=torch.uint8)
    if pinned:
        src, par = src.pin_memory(), par.pin_memory()
    pipe = engine.Pipe(n, k, p, tbls, depth=3, mode=mode)
    for s in range(ns):
        pipe.submit([src[s, j] for j in range(k)], [par[s, l] for l in range(p)])
    pipe.flush()
    pipe.close()
    for s in range(ns):
        want = oracle.encode(a[k * k:], k, p, [src[s, j].numpy() for j in range(k)])
        for l in range(p):
            assert np.array_equal(par[s, l].numpy(), want[l]), (mode, pinned, s, l)


# --------------------------------------------------------------------------
# deprecated per-ISA aliases (reference erasure_code.h:249-1050)
# --------------------------------------------------------------------------

def test_deprecated_per_isa_aliases(engine, oracle, gpu):
    import ctypes

    L = engine.lib()
    u8p = ctypes.POINTER(ctypes.c_ubyte)

    def pp(arrs):
        a = (u8p * len(arrs))()
        for i, x in enumerate(arrs):
            a[i] = x.ctypes.data_as(u8p)
        return a

    n, k = 1000 + 3, 7
    src = [fill_bytes(n, 40 + j) for j in range(k)]
    for isa in ("sse", "avx", "avx2"):
        for N in range(1, 7):
            coef = fill_bytes(k * N, 10 * N + len(isa))
            t = oracle.ec_init_tables(k, N, coef)
            want = oracle.encode(coef, k, N, src)
            got = [np.zeros(n, np.uint8) for _ in range(N)]
            if N == 1:
                getattr(L, f"gf_vect_dot_prod_{isa}")(n, k, t.ctypes.data_as(u8p), pp(src),
                                                     got[0].ctypes.data_as(u8p))
            else:
                getattr(L, f"gf_{N}vect_dot_prod_{isa}")(n, k, t.ctypes.data_as(u8p), pp(src), pp(got))
            assert all(np.array_equal(a, b) for a, b in zip(got, want)), (isa, N, "dot")
            # mad: accumulate every source -> the same parity
            acc = [np.zeros(n, np.uint8) for _ in range(N)]
            for v in range(k):
                if N == 1:
                    getattr(L, f"gf_vect_mad_{isa}")(n, k, v, t.ctypes.data_as(u8p),
                                                    src[v].ctypes.data_as(u8p), acc[0].ctypes.data_as(u8p))
                else:
                    getattr(L, f"gf_{N}vect_mad_{isa}")(n, k, v, t.ctypes.data_as(u8p),
                                                       src[v].ctypes.data_as(u8p), pp(acc))
            assert all(np.array_equal(a, b) for a, b in zip(acc, want)), (isa, N, "mad")
        coef = fill_bytes(k * 4, 99)
        t = oracle.ec_init_tables(k, 4, coef)
        got = [np.zeros(n, np.uint8) for _ in range(4)]
        getattr(L, f"ec_encode_data_{isa}")(n, k, 4, t.ctypes.data_as(u8p), pp(src), pp(got))
        assert all(np.array_equal(a, b) for a, b in zip(got, oracle.encode(coef, k, 4, src)))
        upd = [np.zeros(n, np.uint8) for _ in range(4)]
        for v in range(k):
            getattr(L, f"ec_encode_data_update_{isa}")(n, k, 4, v, t.ctypes.data_as(u8p),
                                                       src[v].ctypes.data_as(u8p), pp(upd))
        assert all(np.array_equal(a, b) for a, b in zip(upd, got))
    for isa in ("sse", "avx"):
        f = getattr(L, f"gf_vect_mul_{isa}")
        f.restype = ctypes.c_int
        d = np.zeros(96, np.uint8)
        s = fill_bytes(96, 5)
        assert f(96, oracle.gf_vect_mul_init(0x53).ctypes.data_as(u8p), ctypes.c_void_p(s.ctypes.data),
                 ctypes.c_void_p(d.ctypes.data)) == 0
        assert bytes(d) == bytes(oracle.gf_mul(0x53, int(x)) for x in s)
        assert f(95, oracle.gf_vect_mul_init(0x53).ctypes.data_as(u8p), ctypes.c_void_p(s.ctypes.data),
                 ctypes.c_void_p(d.ctypes.data)) != 0



# --------------------------------------------------------------------------
# RAID P+Q (include/raid.h) on the erasure-code kernels
# --------------------------------------------------------------------------

def _raid_fn(engine, name):
    import ctypes

    f = getattr(engine.lib(), name)
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    return f


def _vp(bufs):
    import ctypes

    arr = (ctypes.c_void_p * len(bufs))()
    for i, b in enumerate(bufs):
        arr[i] = engine_addr(b)
    return arr


def engine_addr(b):
    import isal_amd

    return isal_amd.addr(b)


@pytest.mark.parametrize("where", ["host", "device"])
def test_raid_vs_reference_fixtures(engine, oracle, gpu, where):
    import torch

    xg, xc = _raid_fn(engine, "xor_gen"), _raid_fn(engine, "xor_check")
    pg, pgb, pc = _raid_fn(engine, "pq_gen"), _raid_fn(engine, "pq_gen_base"), _raid_fn(engine, "pq_check")
    for case in golden()["raid"]:
        v, n = case["vects"], case["len"]
        mk = lambda: [fill_bytes(n, case["seed"] + j) for j in range(v)]  # noqa: E731
        bx, bp = mk(), mk()
        if where == "device":
            bx = [torch.from_numpy(b).to(gpu) for b in bx]
            bp = [torch.from_numpy(b).to(gpu) for b in bp]
        assert xg(v, n, _vp(bx)) == case["xor_ret"], (v, n)
        assert pgb(v, n, _vp(bp)) == case["pq_ret"], (v, n)  # base semantics: len & ~7 bytes
        assert xc(v, n, _vp(bx)) == case["xor_check"]
        assert pc(v, n & ~7, _vp(bp)) == case["pq_check"]
        hx = [b.cpu().numpy() if where == "device" else b for b in bx]
        hp = [b.cpu().numpy() if where == "device" else b for b in bp]
        assert oracle.fnv(hx[v - 1]) == case["xor_fnv"], (v, n)
        if v >= 4:
            assert oracle.fnv(hp[v - 2]) == case["p_fnv"] and oracle.fnv(hp[v - 1]) == case["q_fnv"], (v, n)
        # dispatched pq_gen: the x86 kernels' contract, len % 32 != 0 -> 1, untouched
        if v >= 4:
            again = mk()
            if where == "device":
                again = [torch.from_numpy(b).to(gpu) for b in again]
            r = pg(v, n, _vp(again))
            if n == 0 or n % 32 == 0:
                assert r == 0
            else:
                assert r == 1
    # corruption results: positions exactly as gen_golden.c chose them
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


def test_raid_pq_large_and_every_corruption_position(engine, oracle, gpu):
    """pq_check localises corruption like raid_base.c:96-99 at any byte of any vector."""
    import torch

    pg, pc = _raid_fn(engine, "pq_gen"), _raid_fn(engine, "pq_check")
    v, n = 12, 1 << 20
    bufs = [torch.from_numpy(fill_bytes(n, 77 + j)).to(gpu) for j in range(v)]
    assert pg(v, n, _vp(bufs)) == 0
    h = [b.cpu().numpy() for b in bufs]
    ref = [x.copy() for x in h]
    assert oracle.raid("pq_gen", v, n, ref) == 0
    assert all(np.array_equal(a, b) for a, b in zip(h, ref))
    assert pc(v, n, _vp(bufs)) == 0
    rng = np.random.default_rng(5)
    for _ in range(12):
        j, i = int(rng.integers(0, v)), int(rng.integers(0, n))
        old = int(bufs[j][i])
        bufs[j][i] = old ^ 0x41
        want = [x.copy() for x in h]
        want[j][i] ^= 0x41
        assert pc(v, n, _vp(bufs)) == oracle.raid("pq_check", v, n, want), (j, i)
        bufs[j][i] = old


# --------------------------------------------------------------------------
# the N>1 bench path with real GPU work (two ranks share GPU 0 over gloo;
# RCCL itself needs one GPU per rank and is exercised by the 8-GPU driver run)
# --------------------------------------------------------------------------

def test_bench_two_ranks_on_one_gpu(gpu):
    import json
    import socket
    import sys

    # the driver's own form: `bench.py --gpus 2` with no torchrun, bench.py starts
    # both ranks itself (gloo lets them share this box's one GPU)
    env = {a: b for a, b in os.environ.items() if a not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ecutil.REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--stripes", "64", "--len", "65536", "--steps", "4", "--warmup", "1"]
    for workload in ("encode", "decode"):
        r = subprocess.run(cmd + ["--workload", workload], capture_output=True, text=True,
                           timeout=600, cwd=ecutil.REPO, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, r.stdout
        out = json.loads(lines[0])
        assert out["n_gpus"] == 2 and out["value"] > 0 and out["self_check"] is True, out
        assert [d["rank"] for d in out["rank_devices"]] == [0, 1] and out["dist_backend"] == "gloo"
    # under torchrun the same flags must agree with WORLD_SIZE
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + cmd[1:]
    # C5 mode: 300 stripes split over the two ranks, batches of 64 (4 full + 1 ragged
    # launch per rank), every stripe counted once per step
    r = subprocess.run(cmd + ["--total-stripes", "300"], capture_output=True, text=True, timeout=600,
                       cwd=ecutil.REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["config"]["stripe_ranges"] == [[0, 150], [150, 300]], out
    assert out["stripes_encoded"] == 300 * 4 and out["self_check"] is True, out
    assert out["scaling"] == "strong" and out["value"] > 0


def test_c5_full_workload_eight_ranks(gpu):
    """BASELINE configs[4] (C5) at its real size: 1,048,576 stripes of k=10
    m=4 1 MiB shards split over 8 ranks — the driver's `bench.py --gpus 8`
    form with gloo so all eight share this box's one GPU (RCCL needs a GPU
    per rank; the 8-GPU node runs the same code over it). Every rank encodes
    its contiguous 131,072-stripe range from resident 256-stripe batches and
    self-checks three stripes with a decode round trip through every parity
    row; every stripe-encode is counted."""
    import json
    import sys

    env = {a: b for a, b in os.environ.items() if a not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    T, W, steps = 1 << 20, 8, 1
    r = subprocess.run([sys.executable, os.path.join(ecutil.REPO, "bench.py"), "--gpus", str(W),
                        "--dist-backend", "gloo", "--total-stripes", str(T), "--len", str(1 << 20),
                        "--stripes", "256", "--steps", str(steps), "--warmup", "1"],
                       capture_output=True, text=True, timeout=900, cwd=ecutil.REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    print(json.dumps({a: out[a] for a in ("value", "ms_per_step", "n_gpus", "stripes_encoded", "self_check")}))
    assert out["n_gpus"] == W and out["scaling"] == "strong"
    assert out["config"]["stripe_ranges"] == [[q * (T // W), (q + 1) * (T // W)] for q in range(W)], out
    assert out["config"]["total_stripes"] == T and out["config"]["batch_stripes"] == 256
    assert out["stripes_encoded"] == T * steps == out["stripes_expected"], out
    assert out["self_check"] is True and "decode round trip" in out["self_check_method"], out
    assert out["value"] > 0 and out["shard_crc32c_digest"] > 0


FUZZ_RSS_LIMIT_MB = 2048


def test_differential_fuzz_on_the_kernels(gpu, tmp_path):
    """tests/fuzz/ec_diff_fuzz.c against the shipped libisal_hip.so with every
    call forced onto the kernels: encode / update / dot / mad / mul / RAID
    gen + check with len in [0, 16384], k and rows up to 16, raw table bytes,
    misaligned shards, each output and canary compared with the oracle
    (the reference's own fuzz harness only looks for crashes,
    tests/fuzz/ec_fuzz_test.c:322-348)."""
    import sys

    exe = os.path.join(ecutil.ENGINE_DIR, "build", "fuzzgpu", "ec_diff_fuzz_gpu")
    assert os.path.exists(exe), "build() makes it: make -C tests/fuzz gpu"
    corpus = tmp_path / "corpus"
    subprocess.run([sys.executable, os.path.join(ecutil.REPO, "tests", "fuzz", "seeds.py"), "diff", str(corpus)],
                   check=True, capture_output=True)
    env = dict(os.environ, ISAL_HIP_BACKEND="gpu")
    # libFuzzer's own memory bounds, explicit: the process's RSS (HIP runtime
    # and code objects included) and any single malloc stay under 2 GiB.
    # libFuzzer reads its RSS as getrusage(RUSAGE_SELF).ru_maxrss, which Linux
    # carries across execve from the launching process's memory image: started
    # straight from this pytest process (which holds GBs of full-size C2/C3
    # arrays by now) the target began at ru_maxrss ~23 GB and was stopped as
    # out of memory before its first input — the round-3 failure. A forking
    # shell in between gives the target a fresh high-water mark.
    r = subprocess.run(["/bin/sh", "-c", '"$@"; exit $?', "sh", exe, "-max_total_time=45", "-max_len=300000",
                        "-print_final_stats=1", f"-rss_limit_mb={FUZZ_RSS_LIMIT_MB}",
                        f"-malloc_limit_mb={FUZZ_RSS_LIMIT_MB}", f"-artifact_prefix={tmp_path}/", str(corpus)],
                       capture_output=True, text=True, timeout=240, env=env, cwd=tmp_path)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    stat = {l.split(":")[-2]: int(l.split(":")[-1]) for l in out.splitlines()
            if l.startswith("stat::") and l.split(":")[-1].strip().isdigit()}
    assert stat.get("number_of_executed_units", 0) >= 200, out[-2000:]
    assert 0 < stat["peak_rss_mb"] < FUZZ_RSS_LIMIT_MB, stat


def test_bench_refuses_more_rccl_ranks_than_gpus(gpu):
    """`bench.py --gpus N` over RCCL with fewer than N GPUs visible must fail
    loudly instead of stacking ranks on one GPU (or running one rank)."""
    import sys
    import torch

    n = torch.cuda.device_count() + 1
    env = {a: b for a, b in os.environ.items() if a not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ecutil.REPO, "bench.py"), "--gpus", str(n),
                        "--stripes", "8", "--len", "65536", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, cwd=ecutil.REPO, env=env)
    assert r.returncode != 0
    assert "has no GPU of its own" in r.stderr and "rank(s) failed" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_rccl_control_plane_single_rank(gpu):
    """The nccl (= RCCL) branch of bench.py's Dist on this one-GPU box: a
    world-size-1 process group over RCCL carries the matrix broadcast, the
    barriers, the max of the timings and the sums of counts / digests / ranges,
    in both the C2 (weak) and the C5 (--total-stripes) modes."""
    import json
    import socket
    import sys

    for extra in ([], ["--total-stripes", "100"]):
        sock = socket.socket()
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
        sock.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(port),
               os.path.join(ecutil.REPO, "bench.py"), "--dist-always", "--dist-backend", "nccl",
               "--stripes", "32", "--len", "65536", "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline"] + extra
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ecutil.REPO)
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert out["n_gpus"] == 1 and out["self_check"] is True and out["value"] > 0, out
        assert out["shard_crc32c_digest"] > 0
        assert out["rccl_world_size"] == 1 and out["rank_devices"][0]["pci"], out


@pytest.mark.parametrize("args,env", [
    (["--k", "10", "--p", "4"], {}),                                  # C2 shape: XOR path, groups of 10
    (["--k", "10", "--p", "8"], {}),                                  # 8 rows: LDS product tables
    (["--k", "20", "--p", "7", "--len", "262144", "--stripes", "8"], {}),  # 7 rows: product tables
    (["--k", "20", "--p", "6", "--len", "262144", "--stripes", "8"], {}),  # 6 rows over k >= 16: product tables
    (["--k", "13", "--p", "6", "--len", "262144", "--stripes", "8"], {}),  # 6 rows over k < 16: the LDS-DMA ring
    (["--k", "7", "--p", "5"], {"ISAL_HIP_ENC_LDSX": "1"}),           # product tables forced, odd k
    (["--k", "10", "--p", "4"], {"ISAL_HIP_ENC_LDSX": "1"}),          # product tables forced on 4 rows
    (["--k", "10", "--p", "8"], {"ISAL_HIP_ENC_LDSX": "0"}),          # 8 rows: the LDS-DMA ring
    (["--k", "10", "--p", "6"], {"ISAL_HIP_ENC_WIDE5": "0", "ISAL_HIP_ENC_GLDS": "0", "ISAL_HIP_ENC_LDSX": "0"}),
    (["--k", "10", "--p", "6"], {"ISAL_HIP_ENC_LDS": "0", "ISAL_HIP_ENC_XOR": "0", "ISAL_HIP_ENC_GLDS": "0",
                                 "ISAL_HIP_ENC_LDSX": "0"}),
    (["--k", "12", "--p", "5"], {"ISAL_HIP_ENC_GROUP": "4", "ISAL_HIP_ENC_GLDS": "0", "ISAL_HIP_ENC_LDSX": "0"}),
    (["--k", "10", "--p", "8"], {"ISAL_HIP_ENC_GLDS": "0", "ISAL_HIP_ENC_LDSX": "0"}),  # 8 rows through registers
    (["--k", "7", "--p", "5"], {"ISAL_HIP_ENC_XOR": "0", "ISAL_HIP_ENC_LDSX": "0"}),     # LDS-DMA ring, lookups only
    (["--workload", "decode"], {}),
    (["--k", "10", "--p", "2"], {}),                                  # 2 rows: 128-lane workgroups
    (["--k", "12", "--p", "1"], {"ISAL_HIP_ENC_XOR": "0"}),           # 1 row, lookups: 128 lanes
    (["--workload", "pq_gen"], {}),
    (["--workload", "xor_gen"], {}),
])
def test_bench_kernel_label_matches_launch(gpu, args, env):
    """bench.py's roofline.kernel (the name its PMC / steady-state profile files
    are looked up by) is the instantiation the library launched, as the library
    itself names it under ISAL_HIP_LOG=2."""
    import json
    import sys

    base = ["--len", "65536", "--stripes", "16"] if "--len" not in args else []
    cmd = [sys.executable, os.path.join(ecutil.REPO, "bench.py"), "--workload", "encode", "--steps", "1",
           "--warmup", "1", "--no-cpu-baseline"] + base + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ecutil.REPO,
                       env={**os.environ, "ISAL_HIP_LOG": "2", **env})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    launched = {l.split("kernel ", 1)[1] for l in r.stderr.splitlines() if l.startswith("isal_hip: kernel ")}
    assert out["roofline"]["kernel"] in launched, (out["roofline"]["kernel"], launched)


def test_multi_device_encode_host_stripes_vs_oracle(engine, oracle, gpu):
    """isal_hip_multi_*: host stripes over every visible GPU (here: one), each
    GPU its contiguous range through its own pipeline; == oracle."""
    import torch

    k, p, n, ns = 10, 4, 65536 + 32, 9
    a = engine.gf_gen_rs_matrix(k + p, k)
    tbls = engine.ec_init_tables(k, p, a[k * k:])
    src = torch.empty((ns, k, n), dtype=torch.uint8).pin_memory()
    src.random_(generator=torch.Generator().manual_seed(9))
    par = torch.full((ns, p, n), 0xEE, dtype=torch.uint8).pin_memory()
    m = engine.Multi(n, k, p, tbls, ndev=0, depth=2)
    assert m.ndev == torch.cuda.device_count()
    for d in range(m.ndev):
        # the device's NUMA node from sysfs, and its worker pinned within our affinity
        bus = torch.cuda.get_device_properties(d)
        want = engine.pci_numa_node("%04x:%02x:%02x.0" % (bus.pci_domain_id, bus.pci_bus_id, bus.pci_device_id))
        assert m.numa_node(d) == want
        assert 0 <= m.worker_cpus(d) <= len(os.sched_getaffinity(0))
        assert (m.worker_cpus(d) > 0) == (want >= 0 and bool(
            set(engine.numa_node_cpus(want) or []) & os.sched_getaffinity(0)))
    launches = engine.kernel_launches()
    m.encode(ns, [src[s, j] for s in range(ns) for j in range(k)], [par[s, l] for s in range(ns) for l in range(p)])
    assert engine.kernel_launches() >= launches + ns
    h = src.numpy()
    want = _oracle_encode_all(oracle, a[k * k:], k, p, [[h[s, j] for j in range(k)] for s in range(ns)])
    for s in range(ns):
        for l in range(p):
            assert np.array_equal(par[s, l].numpy(), want[s][l]), (s, l)
    m.encode(0, [], [])
    m.close()
    with pytest.raises(RuntimeError):
        engine.Multi(n, k, p, tbls, ndev=torch.cuda.device_count() + 1)


@pytest.mark.parametrize("backend", ["gpu", "auto"])
def test_k0_empty_sum_on_a_fresh_thread(engine, gpu, monkeypatch, backend):
    """k = 0 is the empty sum: every parity row becomes zero (ec_base.c:309-325
    with no sources). Run as a thread's FIRST GPU-route call, on device parity:
    the per-thread table cache starts empty there and k * rows = 0 tables must
    still be a valid (non-NULL) table."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_BACKEND", backend)
    rows, n = 3, 4096 + 16
    out = {}

    def call():
        try:
            par = [torch.full((n,), 0x5A, dtype=torch.uint8, device=gpu) for _ in range(rows)]
            engine.ec_encode_data(n, 0, rows, np.zeros(32, np.uint8), [], par)
            torch.cuda.synchronize()
            out["par"] = [_host(p) for p in par]
        except BaseException as e:  # noqa: BLE001 - surfaced below
            out["err"] = e

    launches, fb = engine.kernel_launches(), engine.fallbacks()
    t = threading.Thread(target=call)
    t.start()
    t.join()
    assert "err" not in out, out.get("err")
    assert all(not p.any() for p in out["par"])
    assert engine.kernel_launches() > launches and engine.fallbacks() == fb


def test_dropin_result_visible_to_other_streams(engine, oracle, gpu):
    """A kernel-argument call returns when its kernel's last workgroup has
    written the host mailbox (isal_hip_kdone), before the runtime has seen the
    kernel end: the parity must already be visible to work the caller issues
    right away on a NON-blocking stream (no implicit ordering with the
    engine's stream, no synchronize in between) — a copy to the host and a
    kernel reading it. Encode and update, at a 16-byte multiple and at a ragged
    length (whose per-byte tail takes the one agent-scope writeback)."""
    import torch

    k, rows = 10, 4
    coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    tbls = engine.ec_init_tables(k, rows, coef)
    side = torch.cuda.Stream(device=gpu)  # torch creates it non-blocking
    for n in (256 << 10, (256 << 10) + 5, 4096 * 3 + 13):
        src = torch.empty((k, n), dtype=torch.uint8, device=gpu)
        out = torch.zeros((rows, n), dtype=torch.uint8, device=gpu)
        pin = torch.empty((rows, n), dtype=torch.uint8).pin_memory()
        for it in range(12):
            src.random_(generator=torch.Generator(device=gpu).manual_seed(100 + it + n))
            h = _host(src)
            want = oracle.encode(coef, k, rows, [h[j] for j in range(k)])
            torch.cuda.synchronize()
            if it % 2 == 0:
                engine.ec_encode_data(n, k, rows, tbls, [src[j] for j in range(k)], [out[l] for l in range(rows)])
            else:
                out.zero_()
                torch.cuda.synchronize()
                for v in range(k):
                    engine.ec_encode_data_update(n, k, rows, v, tbls, src[v], [out[l] for l in range(rows)])
            with torch.cuda.stream(side):
                pin.copy_(out, non_blocking=True)
                x = out[rows - 1].clone()  # a kernel on the side stream reading the last row
            side.synchronize()
            for l in range(rows):
                assert np.array_equal(pin[l].numpy(), want[l]), (n, it, l)
            assert np.array_equal(_host(x), want[rows - 1]), (n, it)


@pytest.mark.parametrize("done", ["1", "0"])
def test_dropin_completion_paths_vs_oracle(engine, oracle, gpu, monkeypatch, done):
    """Encode, update and verify on device shards through the kernel-argument
    route with the host mailbox (default) and with ISAL_HIP_KARG_DONE=0
    (hipStreamSynchronize; a verify then takes the generic route): == oracle,
    many calls in a row (the counter and result words reset themselves) and
    from four threads at once (one mailbox per thread)."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_KARG_DONE", done)
    pc = _raid_fn(engine, "pq_check")
    errors = []

    def worker(t):
        try:
            k, rows, n = 6 + t, 2 + t % 3, 4096 * (3 + t) + 16 * t
            coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
            tbls = engine.ec_init_tables(k, rows, coef)
            g = torch.Generator(device=gpu).manual_seed(t)
            for it in range(20):
                src = torch.empty((k, n), dtype=torch.uint8, device=gpu)
                src.random_(generator=g)
                out = torch.full((rows, n), 0xAB, dtype=torch.uint8, device=gpu)
                torch.cuda.synchronize()
                engine.ec_encode_data(n, k, rows, tbls, [src[j] for j in range(k)], [out[l] for l in range(rows)])
                h = _host(src)
                want = oracle.encode(coef, k, rows, [h[j] for j in range(k)])
                if not all(np.array_equal(_host(out[l]), want[l]) for l in range(rows)):
                    errors.append(("encode", t, it))
                upd = torch.zeros((rows, n), dtype=torch.uint8, device=gpu)
                for v in range(k):
                    engine.ec_encode_data_update(n, k, rows, v, tbls, src[v], [upd[l] for l in range(rows)])
                if not torch.equal(upd, out):
                    errors.append(("update", t, it))
            # verify (pq_check) on device shards, consistent then corrupted
            v, n2 = 4 + t, 8192 + 32 * t
            bufs = [torch.from_numpy(fill_bytes(n2, 500 + 10 * t + j)).to(gpu) for j in range(v)]
            if _raid_fn(engine, "pq_gen")(v, n2, _vp(bufs)) != 0 or pc(v, n2, _vp(bufs)) != 0:
                errors.append(("pq_check clean", t))
            for it in range(6):
                j, i = (t + it) % v, (977 * it + 13 * t) % n2
                old = int(bufs[j][i])
                bufs[j][i] = old ^ 0x04
                want = [b.cpu().numpy() for b in bufs]
                got = pc(v, n2, _vp(bufs))
                bufs[j][i] = old
                want[j][i] = old
                ref = [w.copy() for w in want]
                ref[j][i] ^= 0x04
                if got != oracle.raid("pq_check", v, n2, ref):
                    errors.append(("pq_check", t, it, got))
                if pc(v, n2, _vp(bufs)) != 0:
                    errors.append(("pq_check after", t, it))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors, errors


@pytest.mark.parametrize("xor", ["1", "0"])
@pytest.mark.parametrize("karg", ["1", "0"])
@pytest.mark.parametrize("v", [3, 4, 6, 8, 12, 18, 22, 32])
def test_raid_check_routes_vs_oracle(engine, oracle, gpu, monkeypatch, xor, karg, v):
    """xor_check / pq_check on device shards: the kernel-argument verify
    (default; source counts hitting every load group 10/8/6/4 and the
    remainder path) and the generic verify (ISAL_HIP_KARG=0), with the 0/1
    XOR path on and off; every result == the oracle's (raid_base.c:96-99
    encoding), corruption in sources, P and Q, near the tail and the start."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_ENC_XOR", xor)
    _setenv(monkeypatch, "ISAL_HIP_KARG", karg)
    xc, pc, pg, xg = (_raid_fn(engine, f) for f in ("xor_check", "pq_check", "pq_gen", "xor_gen"))
    n = 4096 * 2 + 96
    h = [fill_bytes(n, 40 * v + j) for j in range(v)]
    hx = [a.copy() for a in h]
    assert oracle.raid("pq_gen", v, n, h) == 0 if v >= 4 else True
    assert oracle.raid("xor_gen", v, n, hx) == 0
    bp = [torch.from_numpy(a).to(gpu) for a in h]
    bx = [torch.from_numpy(a).to(gpu) for a in hx]
    if v >= 4:
        assert pc(v, n, _vp(bp)) == 0
    assert xc(v, n, _vp(bx)) == 0
    for j, i in [(0, 0), (v - 1, n - 1), (v // 2, n // 2), (1, 4095), (v - 2, 17)]:
        for bufs, host, f, name in ((bp, h, pc, "pq_check"), (bx, hx, xc, "xor_check")):
            if name == "pq_check" and v < 4:
                continue
            old = int(bufs[j][i])
            bufs[j][i] = old ^ 0x80
            ref = [a.copy() for a in host]
            ref[j][i] ^= 0x80
            got = f(v, n, _vp(bufs))
            bufs[j][i] = old
            assert got == oracle.raid(name, v, n, ref), (name, j, i, got)


def test_raid6_batch_full_size_vs_oracle(engine, oracle, gpu):
    """The bench's pq_gen / pq_check shape at full size (10 sources, 1 MiB x
    1024 stripes, raid_base.c:44-140 coefficients: P all ones, Q = 2^j): every
    P and Q byte == the oracle's (chunked), the batch check finds every stripe
    consistent, then one flipped byte in a source / P / Q of three stripes is
    reported at its column and the first mismatching row (a source byte
    breaks P first), the rest stay consistent."""
    import torch

    k, rows, n, ns = 10, 2, 1 << 20, 1024
    coef = np.ones(k * rows, np.uint8)
    q = 1
    for j in range(k):
        coef[k + j] = q
        q = engine.gf_mul(q, 2)
    tbls = engine.ec_init_tables(k, rows, coef)
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 4242)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode(0)
    torch.cuda.synchronize()
    _check_stripes_vs_oracle(oracle, coef, k, rows, lambda s: [data[s, j] for j in range(k)], coding, ns,
                             chunk=16)
    bad = torch.zeros(ns, dtype=torch.int64, device=gpu)
    b.check(bad, 0)
    torch.cuda.synchronize()
    assert bool((bad == -1).all())
    flips = {0: (3, 12345, 0), ns // 2: (k, n - 1, 0), ns - 1: (k + 1, 777777, 1)}  # stripe: (shard, col, row)
    for s, (which, col, _) in flips.items():
        t = data[s, which] if which < k else coding[s, which - k]
        t[col] ^= 0x10
    b.check(bad, 0)
    torch.cuda.synchronize()
    got = _host(bad)
    for s in range(ns):
        if s in flips:
            _, col, row = flips[s]
            assert int(got[s]) == (col << 8) | row, (s, hex(int(got[s])))
        else:
            assert got[s] == -1, s
    b.close()


@pytest.mark.parametrize("xor", ["1", "0"])
@pytest.mark.parametrize("k,rows,n,ns", [
    (10, 2, 65536, 24),      # RAID-6 shape: XOR path, group 10
    (8, 1, 4096 * 5, 16),    # RAID-5
    (10, 4, 4096 * 3 + 48, 9),  # RS rows, ragged tail
    (7, 3, 8192, 8),         # k % 4 remainder
    (12, 12, 4096 * 2, 5),   # two passes (rows > 8)
    (24, 6, 4096 * 4, 8),    # group 8... (24 % 10 != 0)
])
def test_batch_check_vs_oracle(engine, oracle, gpu, monkeypatch, xor, k, rows, n, ns):
    """isal_hip_batch_check: bad[s] = ~0 for consistent stripes, else the first
    mismatch (smallest column, then row) — computed here from the oracle's
    parity — for corruption in sources and in any parity row, two passes."""
    import torch

    _setenv(monkeypatch, "ISAL_HIP_ENC_XOR", xor)
    if rows <= 2:  # RAID P (+ Q = 2^j): raid_base.c:44-68
        coef = np.ones(k * rows, np.uint8)
        q = 1
        for j in range(k * (rows - 1)):
            coef[k + j] = q
            q = engine.gf_mul(q, 2)
    else:
        coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:] if k + rows <= 32 else fill_bytes(k * rows, k + rows)
    tbls = engine.ec_init_tables(k, rows, coef)
    data, coding, dptr, cptr = _stripes(torch, gpu, ns, k, rows, n, 17 + k)
    b = engine.Batch(n, k, rows, tbls, ns, dptr, cptr)
    b.encode(0)
    bad = torch.zeros(ns, dtype=torch.int64, device=gpu)
    b.check(bad, 0)
    torch.cuda.synchronize()
    assert bool((bad == -1).all())
    rng = np.random.default_rng(k * rows)
    flips = {}
    for s in range(0, ns, 2):
        which = int(rng.integers(0, k + rows))
        col = int(rng.integers(0, n))
        flips[s] = (which, col)
        t = data[s, which] if which < k else coding[s, which - k]
        t[col] ^= 0x40
    b.check(bad, 0)
    torch.cuda.synchronize()
    h_data, h_cod = _host(data), _host(coding)
    want = _oracle_encode_all(oracle, coef, k, rows, [[h_data[s, j] for j in range(k)] for s in range(ns)])
    got = _host(bad)
    for s in range(ns):
        mism = np.stack([h_cod[s, l] != want[s][l] for l in range(rows)])
        if not mism.any():
            assert got[s] == -1, s
            continue
        col = int(np.nonzero(mism.any(axis=0))[0][0])
        row = int(np.nonzero(mism[:, col])[0][0])
        assert int(got[s]) == (col << 8) | row, (s, flips.get(s), hex(int(got[s])), col, row)
    b.close()


def test_one_context_per_thread_and_device(engine, oracle, gpu):
    """A thread keeps one context (stream, buffers, mailbox) per GPU it calls
    on: 1,000 drop-in calls from a fresh thread that calls hipSetDevice(0)
    between them create exactly one (isal_hip_contexts_created), every result
    matches the oracle, and the thread's current device is unchanged after
    each call (isal_hip.h "Several GPUs")."""
    import ctypes

    import torch

    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already holds (same SONAME)
    dev = torch.device(gpu).index or 0
    k, rows, n = 10, 4, 64 << 10
    coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    tbls = engine.ec_init_tables(k, rows, coef)
    src = torch.empty((k, n), dtype=torch.uint8, device=gpu).random_(generator=torch.Generator(device=gpu).manual_seed(9))
    h = _host(src)
    want = oracle.encode(coef, k, rows, [h[j] for j in range(k)])
    res = {}

    def worker():
        try:
            out = torch.zeros((rows, n), dtype=torch.uint8, device=gpu)
            torch.cuda.synchronize()
            before = engine.contexts_created()
            cur = ctypes.c_int(-1)
            moved = 0
            for it in range(1000):
                assert hip.hipSetDevice(dev) == 0
                engine.ec_encode_data(n, k, rows, tbls, [src[j] for j in range(k)], [out[l] for l in range(rows)])
                hip.hipGetDevice(ctypes.byref(cur))
                moved += cur.value != dev
            res["delta"] = engine.contexts_created() - before
            res["moved"] = moved
            res["ok"] = all(np.array_equal(_host(out[l]), want[l]) for l in range(rows))
        except Exception as e:  # pragma: no cover - reported below
            res["err"] = repr(e)

    t = threading.Thread(target=worker)
    t.start()
    t.join()
    assert "err" not in res, res
    assert res["delta"] == 1, res
    assert res["moved"] == 0 and res["ok"], res


def test_batch_rejects_memory_no_kernel_of_its_device_can_reach(engine, gpu):
    """isal_hip_batch_create accepts only shards its device's kernels reach:
    hipMalloc memory of its device (and managed / page-locked host memory);
    pageable host memory is ISAL_HIP_EINVAL, checked before anything is
    allocated (memory of another GPU, ISAL_HIP_EDEVICE, needs a second GPU)."""
    import ctypes

    import torch

    L = engine.lib()
    k, rows, n, ns = 4, 2, 4096, 3
    tbls = engine.ec_init_tables(k, rows, engine.gf_gen_rs_matrix(k + rows, k)[k * k:])
    dev = torch.zeros((ns * (k + rows), n), dtype=torch.uint8, device=gpu)
    pinned = torch.zeros((ns * (k + rows), n), dtype=torch.uint8).pin_memory()
    pageable = np.zeros((ns * (k + rows), n), np.uint8)
    u8p = ctypes.POINTER(ctypes.c_ubyte)

    def create(rows_of):
        data = (u8p * (ns * k))(*[ctypes.cast(rows_of(s * (k + rows) + j), u8p) for s in range(ns) for j in range(k)])
        coding = (u8p * (ns * rows))(*[ctypes.cast(rows_of(s * (k + rows) + k + l), u8p)
                                       for s in range(ns) for l in range(rows)])
        h = ctypes.c_void_p()
        rc = L.isal_hip_batch_create(ctypes.byref(h), n, k, rows, ctypes.cast(tbls.ctypes.data, u8p), ns, data, coding)
        if rc == 0:
            L.isal_hip_batch_destroy(h)
        return rc

    assert create(lambda i: dev[i].data_ptr()) == 0
    assert create(lambda i: pinned[i].data_ptr()) == 0
    assert create(lambda i: pageable[i].ctypes.data) == -1
    # one pageable shard among device ones
    assert create(lambda i: pageable[i].ctypes.data if i == 7 else dev[i].data_ptr()) == -1


def test_selftest_every_launchable_kernel_resolves(engine, gpu):
    """isal_hip_selftest_kernels: the HIP runtime resolves every kernel the
    launchers can select (encode, LDS-DMA, verify, update, kernel-argument,
    CRC32C, CRC64, fused) — a missing one is a test failure here instead of
    an abort in a caller's launch (DESIGN.md §3 "Kernel registry")."""
    bad, n = engine.selftest_kernels()
    assert n > 800, n
    assert bad == 0, f"{bad} of {n} kernels have no usable device code (named on stderr)"


# --------------------------------------------------------------------------
# checksum entry points (crc.h / crc64.h) on device buffers
# --------------------------------------------------------------------------

_CRC_DEV_LENGTHS = list(range(0, 301)) + [4095, 4096, 4097, 65536 + 7, 1 << 20, (1 << 20) + 3]


def test_crc_entry_points_device_buffers_vs_oracle(engine, oracle, gpu):
    """crc32_iscsi / crc64_* and their _base twins (reference include/crc.h:
    136-150, include/crc64.h:54-163) on DEVICE buffers run the GPU checksum
    kernels: == the oracle at lengths 0..300, around a tile and at 1 MiB, from
    misaligned starts, with random inits, all eight CRC64 flavours."""
    import torch

    rng = np.random.default_rng(2024)
    host = fill_bytes((1 << 20) + 64, 4242)
    dev = torch.from_numpy(host).to(gpu)
    launches = engine.kernel_launches()
    for n in _CRC_DEV_LENGTHS:
        off = int(rng.integers(0, 16))
        a = host[off: off + n]
        p = dev.data_ptr() + off
        i32 = int(rng.integers(0, 1 << 32))
        want = oracle.crc32_iscsi(a, i32)
        assert engine.crc32_iscsi(p, n, i32) == want, ("crc32_iscsi", n, off)
        assert engine.crc32_iscsi(p, n, i32, base=True) == want, ("crc32_iscsi_base", n, off)
        for v in range(8):
            i64 = int(rng.integers(0, 1 << 62)) * 4 + v
            want = oracle.crc64(v, a, i64)
            assert engine.crc64(v, i64, p, n) == want, (engine.CRC64_VARIANTS[v], n, off)
            if n % 7 == 0:
                assert engine.crc64(v, i64, p, n, base=True) == want, (v, n, off)
    assert engine.kernel_launches() > launches, "the GPU checksum kernels did not run"


def test_crc_entry_points_host_buffers_staged_under_gpu_backend(engine, oracle, gpu):
    """Under ISAL_HIP_BACKEND=gpu (this module's setting) host buffers are staged
    into HBM and checksummed by the kernels too: == the oracle."""
    rng = np.random.default_rng(7)
    launches = engine.kernel_launches()
    for n in (1, 15, 16, 17, 4096 + 5, 300000):
        a = fill_bytes(n, n)
        assert engine.crc32_iscsi(a, n, 0x5A5A5A5A) == oracle.crc32_iscsi(a, 0x5A5A5A5A), n
        for v in range(8):
            init = int(rng.integers(0, 1 << 63))
            assert engine.crc64(v, init, a, n) == oracle.crc64(v, a, init), (v, n)
    assert engine.kernel_launches() > launches


def test_crc64_device_buffer_beyond_one_gib(engine, oracle, gpu):
    """A device buffer longer than the kernels' int length is checksummed in
    1 GiB pieces chained through the register: == the oracle."""
    import torch

    n = (1 << 30) + 4096 * 3 + 5
    t = torch.empty(n, dtype=torch.uint8, device=gpu)
    t.random_(generator=torch.Generator(device=gpu).manual_seed(11))
    h = t.cpu().numpy()
    assert engine.crc64(0, 0x1234, t.data_ptr(), n) == oracle.crc64(0, h, 0x1234)
    assert engine.crc32_iscsi(t.data_ptr(), (1 << 30) + 17, 9) == oracle.crc32_iscsi(h[:(1 << 30) + 17], 9)


def test_dropin_waits_out_a_slow_stream(engine, oracle, gpu):
    """The mailbox wait (isal_hip_shim.c wait_done) spins 20 ms, then lets
    hipStreamSynchronize finish the call. Here > 30 ms of torch work queued on
    the legacy default stream — ending with the writes of the very source
    shards — holds the engine's blocking stream back: a drop-in encode and a
    pq_check on device shards must take that branch (isal_hip_slow_waits) and
    still return the oracle's results."""
    import torch

    k, rows, n = 10, 4, 256 << 10
    coef = engine.gf_gen_rs_matrix(k + rows, k)[k * k:]
    tbls = engine.ec_init_tables(k, rows, coef)
    want_src = torch.empty((k, n), dtype=torch.uint8, device=gpu)
    want_src.random_(generator=torch.Generator(device=gpu).manual_seed(31))
    h = _host(want_src)
    want = oracle.encode(coef, k, rows, [h[j] for j in range(k)])
    x = torch.randn((4096, 4096), device=gpu)
    torch.cuda.synchronize()

    def slow_then(fill):
        y = x
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(100):  # ~0.14 TFLOP each: ~1 ms apiece
            y = (y @ x) * 1e-3
        fill()
        t1.record()
        return y, t0, t1

    slow0 = engine.slow_waits()
    src = torch.zeros((k, n), dtype=torch.uint8, device=gpu)
    out = torch.zeros((rows, n), dtype=torch.uint8, device=gpu)
    y, t0, t1 = slow_then(lambda: src.copy_(want_src))
    engine.ec_encode_data(n, k, rows, tbls, [src[j] for j in range(k)], [out[l] for l in range(rows)])
    torch.cuda.synchronize()
    assert t0.elapsed_time(t1) > 30.0, f"queued work too short to outlast the spin: {t0.elapsed_time(t1):.1f} ms"
    for l in range(rows):
        assert np.array_equal(_host(out[l]), want[l]), l
    # pq_check (a verify: its result travels in the mailbox too)
    v, n2 = 8, 65536
    bufs = torch.from_numpy(np.stack([fill_bytes(n2, 900 + j) for j in range(v)])).to(gpu)
    assert _raid_fn(engine, "pq_gen")(v, n2, _vp([bufs[j] for j in range(v)])) == 0
    ref = [b.cpu().numpy().copy() for b in bufs]
    ref[3][1234] ^= 0x10
    bad = torch.from_numpy(np.stack(ref)).to(gpu)
    chk = torch.zeros_like(bad)
    torch.cuda.synchronize()
    y, t0, t1 = slow_then(lambda: chk.copy_(bad))
    got = _raid_fn(engine, "pq_check")(v, n2, _vp([chk[j] for j in range(v)]))
    assert got == oracle.raid("pq_check", v, n2, ref), got
    assert engine.slow_waits() >= slow0 + 2, (slow0, engine.slow_waits())
    del y
