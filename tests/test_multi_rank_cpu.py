"""CPU tier: the N>1 path of bench.py (one process per GPU, stripes partitioned,
control plane only: broadcast of the generator matrix, barrier, max-reduce of
wall times) exercised with the gloo backend at world_size 2."""
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
           os.path.join(ecutil.REPO, "bench.py"), "--dry-run", "--steps", "4", "--warmup", "1"]
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
