"""CPU tier: the N>1 path of bench.py (one process per GPU, stripes partitioned,
control plane only: broadcast of the generator matrix, barrier, max-reduce of
wall times, sums of stripe counts) exercised with the gloo backend at
world_size 2 and 8, including the C5 partition of 1,048,576 stripes."""
import pytest
import json
import os
import socket
import subprocess
import sys

import ecutil


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_harness_two_ranks_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ecutil.REPO, "bench.py"), "--dry-run", "--gpus", "2", "--steps", "4", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ecutil.REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["stripes"] == 2048.0
    # max over ranks: rank 1 sleeps 4 ms per step, so the max wall >= 4 steps x 4 ms
    assert out["wall"] >= 4 * 0.004
    # the broadcast matrix is rank 0's gf_gen_rs_matrix(14, 10)
    assert out["matrix_fnv"] == int(ecutil.oracle().gf_gen_rs_matrix(14, 10).sum())


@pytest.mark.parametrize("world", [2, 8])
def test_c5_partition_of_1m_stripes_gloo(world):
    """BASELINE configs[4] (C5): 1,048,576 stripes split into contiguous,
    covering, balanced ranges over the ranks; every stripe counted once per
    step after the all-reduce; batches of 1024 -> 1024 launches per step in all."""
    T, steps = 1 << 20, 3
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ecutil.REPO, "bench.py"), "--dry-run", "--steps", str(steps), "--warmup", "1",
           "--total-stripes", str(T)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ecutil.REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    rng = out["stripe_ranges"]
    assert out["n_gpus"] == world and len(rng) == world
    assert rng[0][0] == 0 and rng[-1][1] == T
    assert all(rng[i][1] == rng[i + 1][0] for i in range(world - 1))  # contiguous, no overlap
    sizes = [b - a for a, b in rng]
    assert max(sizes) - min(sizes) <= 1 and sizes == [T // world] * world
    assert out["stripes_encoded"] == out["stripes_expected"] == T * steps
    assert out["launches_per_step"] == T // 1024


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    return subprocess.run([sys.executable, os.path.join(ecutil.REPO, "bench.py")] + args,
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ecutil.REPO)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_gpus_flag_launches_ranks_itself(world):
    """The driver's form `python bench.py --gpus N` (no torchrun): bench.py
    starts the N ranks itself, every rank sees WORLD_SIZE == N, and the parent
    relays exactly rank 0's JSON line with n_gpus == N and contiguous ranges,
    in both the weak (C2) and the strong (C5 --total-stripes) modes."""
    for extra in ([], ["--total-stripes", str(1 << 20)]):
        r = _bench(["--dry-run", "--gpus", str(world), "--steps", "3", "--warmup", "1"] + extra)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, r.stdout
        out = json.loads(lines[0])
        assert out["n_gpus"] == world and out["dist_backend"] == "gloo"
        assert [x["rank"] for x in out["rank_devices"]] == list(range(world))
        rng = out["stripe_ranges"]
        assert len(rng) == world and rng[0][0] == 0
        assert all(rng[i][1] == rng[i + 1][0] for i in range(world - 1))
        if extra:
            assert rng[-1][1] == 1 << 20 and out["stripes_encoded"] == 3 << 20
        else:
            assert rng[-1][1] == 1024 * world and out["stripes"] == 1024.0 * world


def test_bench_gpus_flag_fails_when_a_rank_fails():
    """One rank dies before the first collective: the launcher stops the
    peers blocked in it and exits non-zero (no hang, no JSON line)."""
    r = _bench(["--dry-run", "--gpus", "3", "--steps", "2", "--warmup", "0"],
               {"ISAL_BENCH_DRY_FAIL_RANK": "1"}, timeout=200)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "rank(s) failed" in r.stderr


def test_bench_gpus_flag_must_match_torchrun_world():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ecutil.REPO, "bench.py"), "--dry-run", "--gpus", "3", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ecutil.REPO)
    assert r.returncode != 0 and "--gpus 3 but this launch has WORLD_SIZE=2" in r.stderr


def test_partition_is_balanced_for_ragged_counts():
    import isal_amd

    for T in (0, 1, 7, 1000003, (1 << 20) + 5):
        for W in (1, 2, 3, 8):
            parts = [isal_amd.partition(T, W, r) for r in range(W)]
            assert parts[0][0] == 0 and sum(c for _, c in parts) == T
            assert all(parts[r][0] + parts[r][1] == parts[r + 1][0] for r in range(W - 1))
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    assert isal_amd.partition(10, 0, 0) == (0, 0) and isal_amd.partition(10, 3, 3) == (0, 0)
