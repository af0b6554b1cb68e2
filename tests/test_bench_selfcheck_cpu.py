"""bench.py's self-check logic on the host (no GPU: the drop-in calls it makes
run on the engine's CPU route here, the kernels on the GPU box).

The N>1 / C5 bench lines print `self_check`; it must catch a wrong byte in
ANY parity row, not only row 0 (which is the XOR of the sources). The check is
a decode round trip: erase data shards, recover them from the survivors —
which include every parity row — and compare (erasure_code_test.c:273-339
pins the reference's encode the same way)."""
import os
import sys

import numpy as np
import pytest

import ecutil

sys.path.insert(0, ecutil.REPO)
import bench  # noqa: E402


def _stripe(engine, k, p, n, gen, seed):
    a = gen(k + p, k)
    data = [ecutil.fill_bytes(n, seed + j) for j in range(k)]
    parity = [np.zeros(n, np.uint8) for _ in range(p)]
    engine.ec_encode_data(n, k, p, engine.ec_init_tables(k, p, a[k * k:]), data, parity)
    return a, data, parity


@pytest.mark.parametrize("k,p,gen", [(10, 4, "rs"), (4, 2, "cauchy"), (20, 6, "rs"), (4, 4, "cauchy")])
def test_roundtrip_catches_a_wrong_byte_in_every_parity_row(engine, k, p, gen):
    fn = engine.gf_gen_rs_matrix if gen == "rs" else engine.gf_gen_cauchy1_matrix
    n = 4096 + 48
    a, data, parity = _stripe(engine, k, p, n, fn, 31 * k + p)
    for s in range(3):
        assert bench.decode_roundtrip(k, p, n, a, data, parity, s), s
    rng = np.random.default_rng(k * p)
    for row in range(p):
        col = int(rng.integers(0, n))
        for s in range(3):
            parity[row][col] ^= 0x5A
            # p <= k: every parity row is a survivor of every erasure set
            bad = not bench.decode_roundtrip(k, p, n, a, data, parity, s)
            parity[row][col] ^= 0x5A
            assert bad, (row, col, s, bench.erasure_set(k, p, s))
    # and a wrong source byte is caught too (the recovered shard differs or a survivor is wrong)
    data[k - 1][7] ^= 1
    assert not all(bench.decode_roundtrip(k, p, n, a, data, parity, s) for s in range(3))


def test_erasure_sets_rotate_and_stay_in_range():
    k, p = 10, 4
    seen = set()
    for s in range(10):
        e = bench.erasure_set(k, p, s)
        assert len(e) == p and all(0 <= x < k for x in e)
        seen.update(e)
    assert seen == set(range(k))
    assert bench.erasure_set(3, 5, 0) == [0, 1, 2]


def test_cpu_baseline_cores_spread_over_l3_domains(monkeypatch):
    """The CPU baseline pins one thread per physical core, round-robin over
    the L3 domains (tools/cpu_ref_baseline.py _physical_cpus): on a host of
    two CCDs x 4 cores with SMT siblings, 4 cores are two per CCD, never a
    sibling of another chosen CPU; the usable count is capped by the cgroup
    quota."""
    sys.path.insert(0, os.path.join(ecutil.REPO, "tools"))
    import cpu_ref_baseline as crb

    # CPUs 0-7: CCD 0 cores 0-3 and CCD 1 cores 4-7; CPUs 8-15 their siblings
    def fake_read(path):
        cpu = int(path.split("/cpu/cpu")[1].split("/")[0])
        core = cpu % 8
        if path.endswith("thread_siblings_list"):
            return f"{core},{core + 8}"
        if path.endswith("index3/shared_cpu_list"):
            return "0-3,8-11" if core < 4 else "4-7,12-15"
        return None

    monkeypatch.setattr(crb, "_read", fake_read)
    monkeypatch.setattr(crb.os, "sched_getaffinity", lambda pid: set(range(16)))
    assert crb._physical_cpus(4) == [0, 4, 1, 5]
    assert sorted(crb._physical_cpus(0)) == list(range(8))
    monkeypatch.setattr(crb, "cgroup_cpu_quota", lambda: 3.0)
    assert crb.usable_cores() == 3
    monkeypatch.setattr(crb, "cgroup_cpu_quota", lambda: None)
    assert crb.usable_cores() == 8
