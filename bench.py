#!/usr/bin/env python3
"""bench.py — ec_encode_data throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): Reed-Solomon encode, k=10 sources,
p=4 parity (ISA-L rows=4, m=14), Vandermonde matrix from gf_gen_rs_matrix,
1 MiB shards, 1024 stripes per GPU, shards resident in HBM before timing.
One step = one batched launch that encodes all 1024 stripes
(isal_hip_batch_encode -> ec_encode_v16<4>).

value = (k+p) * shard_bytes * stripes * steps * n_gpus / wall seconds, GiB/s
        (the reference's perf_print byte convention, erasure_code_perf.c:304).

Multi-GPU: one process per GPU, stripes partitioned across ranks (weak
scaling: every rank encodes its own 1024 stripes from its own HBM); RCCL
carries only the control plane (broadcast of the coefficient matrix, barrier,
max-reduce of timings). There is no data-path collective. Ranks come either
from torchrun's environment (RANK / WORLD_SIZE / LOCAL_RANK) or, for
`bench.py --gpus N` started without one, from this script itself: the parent
starts N rank processes as fresh children before it touches the GPU, relays
rank 0's JSON line and exits non-zero when any rank fails. Every rank checks
that the process group has exactly --gpus ranks, each on its own GPU.

Extra JSON fields:
  roofline      dominant kernel's algorithmic bytes per launch / its average
                launch duration (HIP events on the launch stream) vs 8 TB/s;
  cpu_baseline  the reference's own CPU path (oracle/_ref/libisal_ref.so =
                /root/reference erasure_code/ec_base.c built for this box's
                host; nasm is absent so the AVX-512/GFNI kernels cannot be
                assembled) on a bounded sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "isa-l_amd"))

METRIC = "ec_encode_data GiB/s device-resident, k=10 m=4 1 MiB shards; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
GIB = float(1 << 30)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU). Without a torchrun environment and N > 1 this script "
                         "starts the N rank processes itself; under torchrun it must equal WORLD_SIZE. "
                         "Default: WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--len", type=int, default=1 << 20, help="shard bytes")
    ap.add_argument("--stripes", type=int, default=1024, help="stripes per GPU per step")
    ap.add_argument("--workload", choices=["encode", "decode", "update", "encode-crc", "crc", "crc64", "encode-crc64",
                                           "e2e-update", "e2e-encode", "c1", "dropin", "pq_gen", "xor_gen",
                                           "pq_check"],
                    default="encode",
                    help="e2e-*: host-resident (pinned) stripes streamed through the pipeline; pq_gen / "
                         "xor_gen / pq_check: RAID-6 / RAID-5 parity over --k sources (raid.h; p is 2 / 1)")
    ap.add_argument("--depth", type=int, default=3, help="e2e pipeline depth (stripes in flight)")
    ap.add_argument("--ring", type=int, default=0,
                    help="e2e: distinct pinned host stripes cycled through (0 = max(2*depth, 4))")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads / pinned processes for the CPU baselines; 0 = one per physical "
                         "core this process may use: its affinity set capped by its cgroup CPU quota "
                         "(SURVEY.md §8(d))")
    ap.add_argument("--cold-ring", type=int, default=8,
                    help="distinct stripes each thread of the cold-cache SIMD-port baseline cycles over")
    ap.add_argument("--total-stripes", type=int, default=0,
                    help="C5 mode: this many stripes in total, split into contiguous ranges over the "
                         "ranks (isal_hip_multi_partition); a step encodes every rank's range as a loop "
                         "of device-resident --stripes batches (strong scaling). 0 = C2 weak scaling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N>1 control-plane backend (nccl = RCCL over xGMI; gloo lets several "
                         "ranks share one GPU for testing)")
    ap.add_argument("--dist-always", action="store_true",
                    help="initialise the process group even at world size 1 (exercises the RCCL "
                         "control plane on a one-GPU box)")
    ap.add_argument("--dropin-threads", default="1,4,16",
                    help="dropin: calling threads per run (tools/dropin_bench), comma-separated")
    ap.add_argument("--dropin-seconds", type=float, default=3.0, help="dropin: seconds per thread count")
    ap.add_argument("--dropin-op", default="encode", choices=["encode", "pq_gen", "xor_gen", "pq_check", "xor_check"],
                    help="dropin: the synchronous call driven per stripe (ec_encode_data or a raid.h call)")
    ap.add_argument("--dry-run", action="store_true",
                    help="exercise the distributed harness without a GPU (gloo, dummy step)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# distributed harness (shared by the real and the dry-run path)
# ---------------------------------------------------------------------------

class Dist:
    def __init__(self, dry: bool, backend: str = "nccl", always: bool = False, want: int | None = None):
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        if want is not None and want != self.world:
            raise SystemExit(f"bench.py: --gpus {want} but this launch has WORLD_SIZE={self.world}")
        self.gpu = self.local_rank
        self.dist = None
        self.backend = None
        self.shared_gpu = False
        if not dry:
            import torch

            # one process per GPU (device_count() does not initialise HIP here).
            # Only the gloo test mode may put several ranks on one GPU.
            ndev = max(1, torch.cuda.device_count())
            if self.local_rank >= ndev:
                if backend != "gloo":
                    raise SystemExit(f"bench.py: local rank {self.local_rank} has no GPU of its own "
                                     f"({ndev} visible); one rank per GPU")
                self.shared_gpu = True
            self.gpu = self.local_rank % ndev
        if self.world > 1 or always:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", str(self.rank))
            os.environ.setdefault("WORLD_SIZE", str(self.world))

            self.backend = "gloo" if dry else backend  # nccl == RCCL on ROCm
            if self.backend == "gloo":
                dist.init_process_group(self.backend)
            else:
                import torch

                # bind this rank's GPU first so RCCL builds its communicator on it
                torch.cuda.set_device(self.gpu)
                dist.init_process_group(self.backend, device_id=torch.device("cuda", self.gpu))
            self.dist = dist
            if dist.get_world_size() != self.world or dist.get_rank() != self.rank:
                raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks "
                                 f"(this is {dist.get_rank()}), launch said {self.world} ({self.rank})")

    def topology(self, dry: bool):
        """Every rank's (GPU index, PCI domain:bus:device) gathered over the
        control plane; with nccl (RCCL) each rank must sit on a distinct GPU."""
        if dry:
            ident = [self.gpu, -1]
        else:
            import torch

            pr = torch.cuda.get_device_properties(self.gpu)
            ident = [self.gpu, (pr.pci_domain_id << 16) | (pr.pci_bus_id << 8) | pr.pci_device_id]
        flat = [0] * (2 * self.world)
        flat[2 * self.rank], flat[2 * self.rank + 1] = ident[0] + 1, ident[1] + 1
        red = self.sum_i64(flat)
        self.devs = devs = [{"rank": r, "gpu": red[2 * r] - 1,
                 "pci": None if red[2 * r + 1] <= 0 else "%04x:%02x:%02x" % (
                     (red[2 * r + 1] - 1) >> 16, ((red[2 * r + 1] - 1) >> 8) & 0xFF, (red[2 * r + 1] - 1) & 0xFF)}
                for r in range(self.world)]
        if not dry and self.backend != "gloo":
            seen = [(x["gpu"], x["pci"]) for x in devs]
            if len(set(seen)) != len(seen):
                raise SystemExit(f"bench.py: two ranks share a GPU: {devs}")
        return devs

    def info(self):
        return {"dist_backend": self.backend or "none",
                "rccl_world_size": self.dist.get_world_size() if self.dist and self.backend == "nccl" else None,
                "rank_devices": self.devs}

    def _dev(self):
        import torch

        return torch.device("cpu") if self.backend == "gloo" else torch.device("cuda", self.gpu)

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def broadcast_bytes(self, data: bytes) -> bytes:
        """Control plane: rank 0's bytes to every rank (RCCL broadcast)."""
        if not self.dist:
            return data
        import torch

        t = torch.tensor(list(data), dtype=torch.uint8, device=self._dev())
        self.dist.broadcast(t, src=0)
        return bytes(t.cpu().tolist())

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64, device=self._dev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if not self.dist:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64, device=self._dev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def sum_i64(self, xs):
        """Element-wise SUM over ranks of a list of int64 (RCCL all-reduce)."""
        if not self.dist:
            return [int(x) for x in xs]
        import torch

        t = torch.tensor([int(x) for x in xs], dtype=torch.int64, device=self._dev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return [int(v) for v in t.cpu().tolist()]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def timed_steps(d: Dist, step, sync, steps: int, warmup: int):
    """W untimed steps, then exactly K steps between barrier+sync brackets.
    Returns the max over ranks of the wall time of the K steps."""
    for _ in range(warmup):
        step()
    sync()
    d.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    t1 = time.perf_counter()
    d.barrier()
    return d.max(t1 - t0)


def enc_kernel(rows: int, k: int, coef) -> str:
    """The vector encode kernel the library launches for one pass of `rows`
    (<= 8) outputs with coefficient matrix coef (rows x k): variant bit 0 the
    XOR path for 0/1 rows and columns (isal_hip_enc_masks: row 0 and column 0
    hold only 0/1, k <= 64; ISAL_HIP_ENC_XOR=0 off), bit 1 low table halves
    from LDS (more than 4 looked-up rows in passes of up to 6 rows, or of 7-8
    rows loading in groups of 5; ISAL_HIP_ENC_LDS=1 always, =0 never); passes
    of 5-8 rows stage their sources through the LDS-DMA ring (ec_encode_glds,
    4 slots per wave, table halves from LDS; ISAL_HIP_ENC_GLDS=0 off) unless
    they look their products up in LDS product tables (ec_encode_ldsx: 7-8
    rows, or 5-6 rows over k >= 16, k <= 64; ISAL_HIP_ENC_LDSX=1 every 4-8
    row pass, =0 off). Passes of 1-2 rows run 128-lane workgroups. The library
    names the same instantiation on stderr with ISAL_HIP_LOG=2."""
    import numpy as np

    c = np.asarray(coef, dtype=np.uint8).reshape(rows, k)
    ldsx = os.environ.get("ISAL_HIP_ENC_LDSX")
    if rows >= 4 and k <= 64 and ldsx != "0" and (ldsx == "1" or rows >= 7 or (rows >= 5 and k >= 16)):
        # LDS product tables (ec_kernels.hip enc_ldsx, kLdsxGroup); batches and pipelines upload them
        return f"ec_encode_ldsx<{rows}, 2>"
    fl = 0
    if os.environ.get("ISAL_HIP_ENC_XOR") != "0" and k <= 64 and int(c[0].max()) <= 1 and int(c[:, 0].max()) <= 1:
        fl |= 1
    if rows >= 5 and os.environ.get("ISAL_HIP_ENC_GLDS") != "0":
        return f"ec_encode_glds<{rows}, 4, {fl | 2}>"  # ec_kernels.hip enc_glds
    lds = os.environ.get("ISAL_HIP_ENC_LDS")
    wide5 = os.environ.get("ISAL_HIP_ENC_WIDE5") != "0"
    if lds == "1" or (lds != "0" and rows - (fl & 1) > 4
                      and (rows <= 6 or (enc_group(k, rows) == 5 and wide5))):  # ec_kernels.hip enc_lds
        fl |= 2
    # rocprofv3 prints every template argument, defaults included: the
    # variant's 0 and the lanes per workgroup (128 for passes of 1-2 rows,
    # ec_kernels.hip enc_block, else 256)
    lanes = 128 if rows <= 2 else 256
    return f"ec_encode_v16<{rows}, EncPol<{enc_group(k, rows)}, 2, 2, 2>, {fl}, {lanes}>"


def copy_ceiling(dev, nbytes: int = 2 << 30, reps: int = 10) -> dict:
    """Achievable HBM rate on this GPU: tools/copy_probe.hip,
    the encode's memory skeleton without arithmetic (16 B per lane, nt buffer
    loads and stores, XCD-contiguous 4 KiB tiles), copying `nbytes` `reps`
    times, HIP events on its stream, read + write bytes counted. Falls back to
    torch's device copy (named as such) when the probe is not built."""
    import ctypes

    import torch

    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    src.fill_(0x5A)
    torch.cuda.synchronize(dev)
    so = os.path.join(REPO, "tools", "libcopy_probe.so")
    if os.path.exists(so):
        lib = ctypes.CDLL(so)
        lib.copy_probe_gbs.restype = ctypes.c_double
        lib.copy_probe_gbs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int]
        gbs = lib.copy_probe_gbs(dst.data_ptr(), src.data_ptr(), nbytes, reps)
        if gbs <= 0:
            raise RuntimeError(f"copy probe failed ({gbs})")
        ok = bool(torch.equal(dst[:1 << 20], src[:1 << 20]) and torch.equal(dst[-(1 << 20):], src[-(1 << 20):]))
        name = "copy_tiles (tools/copy_probe.hip: 16 B/lane nt buffer load+store, 4 KiB tiles), 2 GiB"
    else:
        for _ in range(3):
            dst.copy_(src)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize(dev)
        gbs = 2 * nbytes / (e0.elapsed_time(e1) / 1e3 / reps) / 1e9
        ok = True
        name = "device-to-device copy (torch Tensor.copy_; tools/libcopy_probe.so not built), 2 GiB"
    del src, dst
    return {"kernel": name, "gb_s": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4), "copy_ok": ok}


def enc_group(k: int, rows: int = 0) -> int:
    """Sources per load group the engine launches with for a pass of `rows`
    outputs (ec_kernels.hip:enc_group, enc_wide5)."""
    force = os.environ.get("ISAL_HIP_ENC_GROUP", "")
    if force in ("12", "10", "8", "6", "5", "4"):
        return int(force)
    if rows >= 6 and k >= 10 and k % 5 == 0 and os.environ.get("ISAL_HIP_ENC_WIDE5") != "0":
        return 5
    return next((u for u in (12, 10, 8, 6, 5, 4) if k >= u and k % u == 0), 4)


SELF_CHECK_METHOD = {
    w: ("3 stripes per rank: parity row 0 == XOR of the sources, and a decode round trip (min(p,k) data "
        "shards erased, recovered from the survivors incl. every parity row with gf_invert_matrix + the "
        "engine, == the originals)" + extra)
    for w, extra in (("encode", ""), ("encode-crc", "; fused CRC32C == the checksum-only kernel"),
                     ("encode-crc64", "; fused CRC64 == the checksum-only kernel, crc(P0) == XOR of crc(D_j)"))}
SELF_CHECK_METHOD.update({
    "decode": "every recovered shard of every stripe == the erased original",
    "crc": "checksum-only CRC32C == the fused kernel's",
    "crc64": "crc(P0) == XOR of the sources' CRC64 (linearity) on 3 stripes"})


SELF_CHECK_METHOD.update({
    "pq_gen": "3 stripes: P == XOR of the sources, Q == sum of 2^j * D_j (host gf_mul of the sources' bytes "
              "at 4096 sampled columns), and the batch verify finds every stripe consistent",
    "xor_gen": "3 stripes: P == XOR of the sources, and the batch verify finds every stripe consistent",
    "pq_check": "every stripe consistent after the timed checks; then one byte flipped in a source of one stripe "
                "and in Q of another: exactly those two stripes flagged, at the flipped column (row 0 for a "
                "source byte, row 1 for Q)"})

# raid.h workloads: parity rows
RAID_ROWS = {"pq_gen": 2, "xor_gen": 1, "pq_check": 2}


def raid_coef(k: int, p: int):
    """Coefficient rows of RAID P (all ones) and Q (2^j for source j): the
    matrix pq_gen / xor_gen compute (raid_base.c:44-68,100-118)."""
    import numpy as np

    import isal_amd

    c = np.ones((p, k), np.uint8)
    if p == 2:
        q = 1
        for j in range(k):
            c[1, j] = q
            q = isal_amd.gf_mul(q, 2)
    return c.reshape(-1)


def verify_kernel(rows: int, k: int, coef) -> str:
    """The batch verify kernel the library launches (ec_kernels.hip
    isal_hip_launch_verify_batch: load group verify_group(k), tile order with
    the XCD mapping of a batch, bit 0 = the 0/1 XOR path)."""
    import numpy as np

    c = np.asarray(coef, dtype=np.uint8).reshape(rows, k)
    fl = 1 if (os.environ.get("ISAL_HIP_ENC_XOR") != "0" and k <= 64 and int(c[0].max()) <= 1
               and int(c[:, 0].max()) <= 1) else 0
    u = next((g for g in (10, 8, 6, 4) if k >= g and k % g == 0), 4)
    return f"ec_verify_v16<{rows}, EncPol<{u}, 2, 2, 0>, {fl}>"


def raid_self_check(workload, batch, data, out, k, p, n, S, h, dev) -> bool:
    """No oracle: P and Q recomputed on the host from the sources' bytes at
    sampled columns with the library's gf_mul (itself pinned by the reference
    fixtures), and the engine's batch verify as a second opinion (pq_check: it
    must also localise injected corruption)."""
    import numpy as np
    import torch

    import isal_amd

    ok = True
    bad = torch.empty(S, dtype=torch.int64, device=dev)
    batch.check(bad, h)
    torch.cuda.synchronize(dev)
    ok &= bool((bad == -1).all())
    cols = np.unique(np.concatenate([np.arange(64), np.arange(n - 64, n),
                                     np.random.default_rng(3).integers(0, n, 4096)]))
    mul = np.array([[isal_amd.gf_mul(a, b) for b in range(256)] for a in range(256)], np.uint8)
    tcols = torch.as_tensor(cols, device=dev)
    for s_ in sorted({0, S // 2, S - 1}):
        src = data[s_][:, tcols].cpu().numpy()
        par = out[s_][:, tcols].cpu().numpy()
        ok &= bool(np.array_equal(np.bitwise_xor.reduce(src, axis=0), par[0]))
        if p == 2:
            q, g = np.zeros(len(cols), np.uint8), 1
            for j in range(k):
                q ^= mul[g][src[j]]
                g = isal_amd.gf_mul(g, 2)
            ok &= bool(np.array_equal(q, par[1]))
    if workload == "pq_check" and S >= 2:
        s1, s2, c1, c2 = 0, S - 1, n // 3, n - 5
        data[s1, 3, c1] ^= 0x10
        out[s2, 1, c2] ^= 0x01
        batch.check(bad, h)
        torch.cuda.synchronize(dev)
        want = torch.full((S,), -1, dtype=torch.int64, device=dev)
        want[s1], want[s2] = c1 << 8, (c2 << 8) | 1
        ok &= bool(torch.equal(bad, want))
        data[s1, 3, c1] ^= 0x10
        out[s2, 1, c2] ^= 0x01
    return ok


def erasure_set(k: int, p: int, s: int) -> list[int]:
    """The data shards a self-check erases in sampled stripe s: min(p, k)
    distinct indices, rotating with s so different samples lose different
    shards."""
    return sorted({(3 * s + i) % k for i in range(min(p, k))})


def decode_roundtrip(k, p, n, a, data, parity, s=0):
    """Self-check of one encoded stripe with no oracle: erase min(p, k) of its
    data shards, recover them with the engine's own decode — gf_invert_matrix
    of the k surviving generator rows, then ec_encode_data with the erased
    shards' rows of that inverse (erasure_code_test.c:273-339 pins encode the
    same way) — and compare with the originals.

    For p <= k the survivors are the other data shards and EVERY parity shard,
    so a wrong byte in any parity row changes a recovered shard (an MDS code
    cannot recover p erasures from p - 1 parity rows); for p > k the first k
    parity rows. data / parity: the stripe's
    shard buffers (torch tensors on the GPU, where the call runs the kernels;
    numpy arrays on a host without one, where it runs the CPU route)."""
    import numpy as np

    import isal_amd

    errs = erasure_set(k, p, s)
    surv = [i for i in range(k + p) if i not in errs][:k]
    b = np.concatenate([np.asarray(a[r * k:(r + 1) * k], dtype=np.uint8) for r in surv])
    ret, inv, _ = isal_amd.gf_invert_matrix(b, k)
    if ret != 0:
        return False
    c = np.concatenate([inv[e * k:(e + 1) * k] for e in errs])
    frag = [data[i] if i < k else parity[i - k] for i in surv]
    if hasattr(data[0], "data_ptr"):  # torch
        import torch

        out = [torch.empty_like(data[0]) for _ in errs]
        same = torch.equal
    else:
        out = [np.empty_like(data[0]) for _ in errs]
        same = np.array_equal
    isal_amd.ec_encode_data(n, k, len(errs), isal_amd.ec_init_tables(k, len(errs), c), frag, out)
    return all(bool(same(out[i], data[e])) for i, e in enumerate(errs))


def control_plane_matrix(d: Dist, k: int, p: int) -> bytes:
    """Rank 0 generates the m x k generator (gf_gen_rs_matrix) and broadcasts it."""
    import isal_amd

    a = isal_amd.gf_gen_rs_matrix(k + p, k).tobytes() if d.rank == 0 else bytes((k + p) * k)
    return d.broadcast_bytes(a)


# ---------------------------------------------------------------------------
# HBM traffic of the dominant kernel from the committed rocprofv3 PMC passes
# ---------------------------------------------------------------------------

def pmc_traffic(workload, k, p, n, S, kernel):
    """HBM bytes per launch measured by `rocprofv3 --pmc FETCH_SIZE` and
    `--pmc WRITE_SIZE` (separate passes) of this same bench configuration,
    committed under profiles/*_pmc_*.csv. gfx950 correction: FETCH_SIZE counts
    half of a wide streaming read, so bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB.
    Returns (bytes, source) for the newest matching file, or None."""
    import glob
    import statistics

    want = {"workload": workload, "k": str(k), "p": str(p), "len": str(n), "stripes": str(S)}
    def norm(x):  # rocprof prints "void " before template kernels only
        x = x.replace("(anonymous namespace)::", "").replace(" ", "")
        return x[4:] if x.startswith("void") else x

    name = norm(kernel)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "**", "*_pmc_*.csv"), recursive=True),
                       key=os.path.basename, reverse=True):  # newest round first (rNN_ prefix)
        with open(path) as f:
            lines = f.read().splitlines()
        cfg = next((l for l in lines if l.startswith("# config:")), "")
        kv = dict(t.split("=", 1) for t in cfg[len("# config:"):].split(";")[0].split() if "=" in t)
        if any(kv.get(a) != b for a, b in want.items()):
            continue
        vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
        for l in lines:
            parts = l.split(",", 3)
            if len(parts) == 4 and parts[0] in vals and norm(parts[3]).split("(")[0] == name:
                vals[parts[0]].append(float(parts[2]))
        if vals["FETCH_SIZE"] and vals["WRITE_SIZE"]:
            kib = 2 * statistics.median(vals["FETCH_SIZE"]) + statistics.median(vals["WRITE_SIZE"])
            return int(kib * 1024), os.path.relpath(path, REPO)
    return None


def kernel_stats(workload, k, p, n, S, kernel):
    """Steady-state rocprofv3 kernel-trace summary of this configuration's
    dominant kernel, committed under profiles/*_kernel_steady.csv by
    tools/kernel_stats.py (the first --warmup dispatches dropped, the K timed
    ones averaged — what the HIP events here measure). Returns
    (avg launch ms, source) for the newest matching file, or None."""
    import glob

    want = {"workload": workload, "k": str(k), "p": str(p), "len": str(n), "stripes": str(S)}
    name = kernel.replace(" ", "")
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "**", "*_kernel_steady.csv"), recursive=True),
                       key=os.path.basename, reverse=True):
        with open(path) as f:
            rows = [l.rstrip("\n") for l in f]
        cfg = next((l for l in rows if l.startswith("# config:")), "")
        kv = dict(t.split("=", 1) for t in cfg[len("# config:"):].split() if "=" in t)
        if any(kv.get(a) != b for a, b in want.items()):
            continue
        fields = dict(l.split(",", 1) for l in rows if "," in l and not l.startswith("#"))
        kname = fields.get("kernel", "").strip('"').replace("(anonymous namespace)::", "").replace(" ", "")
        if name not in kname or "avg_ns" not in fields:
            continue
        return float(fields["avg_ns"]) / 1e6, os.path.relpath(path, REPO)
    return None


# ---------------------------------------------------------------------------
# CPU baseline: the reference's own ec_encode_data on this host
# ---------------------------------------------------------------------------

def cpu_baseline(k, p, n, seconds, threads, check=None, impl="reference", crc=False, encode=True, ring=1):
    """Times the reference ec_encode_data (oracle/_ref/libisal_ref.so: ec_base.c +
    ec_base_aliases.c compiled from /root/reference) on `threads` host threads,
    each encoding its own k x n stripe repeatedly for ~`seconds`.

    check = (data_host[k][n], parity_gpu[p][n]): parity of that stripe recomputed
    by the reference on the CPU must equal the GPU's bytes."""
    import numpy as np

    if impl == "gfni":
        # port of the reference's AVX-512+GFNI kernels (oracle/ec_gfni_port.c);
        # tables and matrix from the oracle restatement of ec_base.c
        lib_path, kind = os.path.join(REPO, "oracle", "libgfni_port.so"), "port"
        if not (os.path.exists(lib_path) and os.path.exists(os.path.join(REPO, "oracle", "liboracle.so"))):
            return None
        G = ctypes.CDLL(lib_path)
        if not G.gfni_port_available():
            return None
        L = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        enc = G.gfni_port_ec_encode_data
        init, gen = L.oracle_ec_init_tables, L.oracle_gf_gen_rs_matrix
        what = "AVX-512+GFNI port of gf_Nvect_dot_prod_avx512_gfni (oracle/ec_gfni_port.c)"
    else:
        ref = os.path.join(REPO, "oracle", "_ref", "libisal_ref.so")
        kind = "reference"
        if not os.path.exists(ref):
            ref, kind = os.path.join(REPO, "oracle", "liboracle.so"), "port"
        if not os.path.exists(ref):
            return None
        L = ctypes.CDLL(ref)
        prefix = "" if kind == "reference" else "oracle_"
        enc = getattr(L, prefix + "ec_encode_data")
        init = getattr(L, prefix + "ec_init_tables")
        gen = getattr(L, prefix + "gf_gen_rs_matrix")
        what = ("reference ec_base.c (noarch build; no nasm for the AVX-512/GFNI kernels)"
                if kind == "reference" else "oracle port of ec_base.c")
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    enc.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.POINTER(u8p), ctypes.POINTER(u8p)]
    enc.restype = None
    crc_fn = None
    if crc == "crc64":
        # crc64_ecma_refl of every shard: the reference's crc64_base.c when built
        cref = os.path.join(REPO, "oracle", "_ref", "libisal_ref_crc.so")
        if kind == "reference" and os.path.exists(cref):
            crc_fn = ctypes.CDLL(cref).crc64_ecma_refl_base
        else:
            raw = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so")).oracle_crc64
            raw.argtypes = [ctypes.c_int, u8p, ctypes.c_longlong, ctypes.c_ulonglong]
            raw.restype = ctypes.c_ulonglong
            crc_fn = lambda init, buf, n_: raw(0, buf, n_, init)  # noqa: E731
        if hasattr(crc_fn, "argtypes"):
            crc_fn.argtypes = [ctypes.c_ulonglong, u8p, ctypes.c_ulonglong]
            crc_fn.restype = ctypes.c_ulonglong
        crc_what = "crc64_ecma_refl of all k+p shards (crc64_base.c)"
        what = f"ec_encode_data from {what} + {crc_what}" if encode else crc_what
    elif crc:
        # + crc32_iscsi of every shard: the reference's crc_base.c when built
        # (oracle/_ref/libisal_ref_crc.so), else the oracle restatement of it
        cref = os.path.join(REPO, "oracle", "_ref", "libisal_ref_crc.so")
        if impl == "gfni":  # SSE4.2 crc32q, 3 streams (as crc32_iscsi_01.asm)
            crc_fn = G.gfni_port_crc32_iscsi
            crc_fn.argtypes = [u8p, ctypes.c_longlong, ctypes.c_uint]
        elif kind == "reference" and os.path.exists(cref):
            crc_fn = ctypes.CDLL(cref).crc32_iscsi_base
            crc_fn.argtypes = [u8p, ctypes.c_int, ctypes.c_uint]
        else:
            crc_fn = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so")).oracle_crc32_iscsi
            crc_fn.argtypes = [u8p, ctypes.c_longlong, ctypes.c_uint]
        crc_fn.restype = ctypes.c_uint
        crc_what = ("crc32_iscsi of all k+p shards (" +
                    ("SSE4.2 port of crc32_iscsi_01" if impl == "gfni" else "crc_base.c") + ")")
        what = f"ec_encode_data from {what} + {crc_what}" if encode else crc_what
    else:
        what = f"ec_encode_data from {what}"

    a = np.zeros((k + p) * k, np.uint8)
    gen(a.ctypes.data_as(u8p), k + p, k)
    tbls = np.zeros(32 * k * p, np.uint8)
    init(k, p, a[k * k:].ctypes.data_as(u8p), tbls.ctypes.data_as(u8p))

    def ptrs(bufs):
        arr = (u8p * len(bufs))()
        for i, b in enumerate(bufs):
            arr[i] = b.ctypes.data_as(u8p)
        return arr

    parity_ok = None
    if check is not None:
        data_h, parity_gpu = check
        out = [np.zeros(n, np.uint8) for _ in range(p)]
        enc(n, k, p, tbls.ctypes.data_as(u8p), ptrs(list(data_h)), ptrs(out))
        parity_ok = all(np.array_equal(out[l], parity_gpu[l]) for l in range(p))

    counts = [0] * threads
    rng = np.random.default_rng(1)
    # ring > 1: each thread cycles over `ring` distinct stripes (cold caches);
    # one random stripe copied into every buffer (distinct memory, same bytes)
    proto = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    bufs = [[([x.copy() for x in proto], [np.zeros(n, np.uint8) for _ in range(p)]) for _ in range(ring)]
            for _ in range(threads)]
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import cpu_ref_baseline as crb

    cpus = crb.physical_cpus(threads)  # one thread pinned per physical core
    deadline = time.perf_counter() + seconds

    def worker(i):
        if i < len(cpus):
            os.sched_setaffinity(0, {cpus[i]})  # pid 0 = this thread
        srcs = [ptrs(b[0]) for b in bufs[i]]
        dsts = [ptrs(b[1]) for b in bufs[i]]
        t = tbls.ctypes.data_as(u8p)
        shards = [b.ctypes.data_as(u8p) for b in bufs[i][0][0] + bufs[i][0][1]]
        while time.perf_counter() < deadline:
            r = counts[i] % ring
            src, dst = srcs[r], dsts[r]
            if encode:
                enc(n, k, p, t, src, dst)  # ctypes drops the GIL for the call
            if crc == "crc64":
                for sh in shards:
                    crc_fn(0, sh, n)
            elif crc_fn is not None:
                for sh in shards:
                    crc_fn(sh, n, 0xFFFFFFFF)
            counts[i] += 1

    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    wall = time.perf_counter() - t0
    stripes = sum(counts)
    return {
        "value": round(stripes * (k + p) * n / wall / GIB, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": kind,
        "sample": f"{stripes} stripes of k={k} p={p} x {n} B, {what}, "
                  f"{threads} threads x {wall:.1f} s ({min(threads, len(cpus))} pinned one per physical core)"
                  + (f", each thread cycling over {ring} distinct stripes (cold caches)" if ring > 1
                     else ", each thread re-encoding one cache-warm stripe"),
        "parity_stripe_match": parity_ok,
    }


def ref_harness_baseline(workload, k, p, n, procs):
    """The reference's OWN perf harness on this host's cores
    (tools/cpu_ref_baseline.py): erasure_code_perf.c (C2 encode / C3 decode,
    -k 10 -p 4 -e 3 -s 1M) or erasure_code_update_perf.c at the C4 shape, built
    from /root/reference by `make -C oracle ref` on its portable ec_base.c (the
    image has no nasm for the AVX-512/GFNI kernels). Single-threaded by design,
    so it runs once on one core and once as `procs` pinned processes at once,
    MB/s summed. None when the shape is not one the harness takes."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import cpu_ref_baseline as crb

    if workload in ("encode", "decode") and (k, p, n) == (10, 4, 1 << 20):
        which, phase, factor = "encode", workload, 1.0
        conv = ""
    elif workload == "update" and (k, p, n) == (20, 6, 4 << 20):
        # the harness counts (p+1)*len per single-source update call
        # (erasure_code_update_perf.c:348); this bench counts the (1+2p)*len
        # read-modify-write bytes of the same call
        which, phase, factor = "update", "update_single_src", (1 + 2 * p) / (p + 1)
        conv = f", converted from its (p+1)*len to this bench's (1+2p)*len bytes per call"
    else:
        return None
    one, many = crb.run(which, 1), crb.run(which, procs or 0)
    if "error" in one or "error" in many or phase not in many or phase not in one:
        return {"error": one.get("error") or many.get("error") or "phase missing"}
    host = crb.host_info()
    gib = lambda mb: round(mb * 1e6 * factor / GIB, 3)  # noqa: E731
    per_core = one[phase]["mb_s_sum"]
    res = {
        "value": gib(many[phase]["mb_s_sum"]),
        "unit": "GiB/s",
        "cores": many["procs"],
        "kind": "reference",
        "sample": f"{many['command']} ({phase} phase): {many['procs']} pinned processes x ~3 s "
                  f"(BENCHMARK_TIME), MB/s summed{conv}; reference ec_base.c path (no nasm: the "
                  f"AVX-512/GFNI kernels cannot be assembled)",
        "single_core_gib_s": gib(per_core),
        "host": {a: host.get(a) for a in ("model", "sockets", "physical_cores", "affinity_physical_cores",
                                          "cgroup_cpu_quota", "usable_cores", "cpus", "isa", "nasm")},
    }
    return res


def ref_parity_check(k, rows, n, coef, src_host, parity_gpu):
    """The reference's own ec_encode_data (oracle/_ref/libisal_ref.so) on one
    stripe must give the GPU's bytes. None when the reference build is absent."""
    import numpy as np

    path = os.path.join(REPO, "oracle", "_ref", "libisal_ref.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    tbls = np.zeros(32 * k * rows, np.uint8)
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    L.ec_init_tables(k, rows, coef.ctypes.data_as(u8p), tbls.ctypes.data_as(u8p))
    out = [np.zeros(n, np.uint8) for _ in range(rows)]
    src = [np.ascontiguousarray(s) for s in src_host]

    def pp(bufs):
        arr = (u8p * len(bufs))()
        for i, b in enumerate(bufs):
            arr[i] = b.ctypes.data_as(u8p)
        return arr

    L.ec_encode_data(n, k, rows, tbls.ctypes.data_as(u8p), pp(src), pp(out))
    return all(np.array_equal(out[l], parity_gpu[l]) for l in range(rows))


def total_stripes_run(args, d: Dist, a, k, p, n):
    """C5 (BASELINE configs[4]): args.total_stripes stripes in all, rank r owns
    the contiguous range isal_hip_multi_partition(T, W, r) and encodes it from
    its own HBM as a loop of device-resident batches of args.stripes stripes
    (the reference perf apps' re-encode-resident-buffers convention,
    erasure_code_perf.c:126-132; every stripe-encode is counted). One step =
    every rank encodes its whole range once. RCCL carries only the control
    plane: matrix broadcast, barrier, max of the timings, sums of the stripe
    counts and of a CRC32C digest of every rank's shards, and the ranges."""
    import torch

    import isal_amd

    T, W = args.total_stripes, d.world
    first, count = isal_amd.partition(T, W, d.rank)
    B = max(1, min(args.stripes, count))
    dev = torch.device("cuda", d.gpu)
    data = torch.empty((B, k, n), dtype=torch.uint8, device=dev)
    data.random_(generator=torch.Generator(device=dev).manual_seed(1234 + d.rank))
    out = torch.zeros((B, p, n), dtype=torch.uint8, device=dev)
    tbls = isal_amd.ec_init_tables(k, p, a[k * k:])
    dptr = [int(data[s, j].data_ptr()) for s in range(B) for j in range(k)]
    cptr = [int(out[s, l].data_ptr()) for s in range(B) for l in range(p)]
    full, rem = divmod(count, B)
    batch = isal_amd.Batch(n, k, p, tbls, B, dptr, cptr)
    rem_batch = isal_amd.Batch(n, k, p, tbls, rem, dptr[:rem * k], cptr[:rem * p]) if rem else None
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    launches = full + (1 if rem else 0)

    def step():
        for _ in range(full):
            batch.encode(h)
        if rem_batch is not None:
            rem_batch.encode(h)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    d.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    d.barrier()
    wall = d.max(t1 - t0)
    step_s = ev0.elapsed_time(ev1) / 1e3 / args.steps

    # self-check (all-ones Vandermonde row) and a digest of this rank's shards:
    # CRC32C of every source and parity shard of the resident batch, summed
    # (a rank whose range is empty — fewer stripes than ranks — encoded nothing
    # and has nothing to check or digest)
    ok, digest = True, 0
    if count:
        for s_ in sorted({0, B // 2, B - 1}):
            x = data[s_, 0].clone()
            for j in range(1, k):
                x ^= data[s_, j]
            ok &= bool(torch.equal(x, out[s_, 0]))
            # every parity row: erase data shards, decode, compare
            ok &= decode_roundtrip(k, p, n, a, [data[s_, j] for j in range(k)], [out[s_, l] for l in range(p)],
                                   s_ + first)
        crc = torch.zeros(B * (k + p), dtype=torch.int32, device=dev)
        batch.crc(0xFFFFFFFF, crc, h)
        torch.cuda.synchronize(dev)
        digest = int((crc.to(torch.int64) & 0xFFFFFFFF).sum().item())
    ranges = [0] * (2 * W)
    ranges[2 * d.rank], ranges[2 * d.rank + 1] = first, count
    red = d.sum_i64([count * args.steps, digest, 0 if ok else 1] + ranges)
    encoded, digest_all, bad = red[0], red[1], red[2]
    rng = [(red[3 + 2 * r], red[3 + 2 * r + 1]) for r in range(W)]
    step_bytes = (k + p) * n * T
    value = step_bytes * args.steps / wall / GIB
    bytes_per_launch = (k + p) * n * count / launches if launches else 0
    achieved = (k + p) * n * count / step_s / 1e9 if count else 0.0
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": W,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch RNG on device); each rank re-encodes its "
                "resident batch for every stripe of its range",
        "config": {
            "workload": f"C5 encode: {T} stripes of k={k} p={p} Vandermonde RS, {n} B shards, split "
                        f"over {W} GPU(s) in contiguous ranges, device-resident batches of {B}",
            "k": k, "p": p, "shard_bytes": n, "total_stripes": T, "batch_stripes": B,
            "stripe_ranges": [[f, f + c] for f, c in rng],
            "parallelism": f"stripe ranges over {W} GPU(s), no data-path collective",
        },
        "per_gpu_gib_s": round(value / W, 2),
        "stripes_encoded": encoded,
        "stripes_expected": T * args.steps,
        "shard_crc32c_digest": digest_all,
        "self_check": bad == 0 and encoded == T * args.steps,
        "self_check_method": "3 stripes per rank: parity row 0 == XOR of the sources, and a decode round trip "
                             "(min(p,k) data shards erased, recovered from the survivors incl. every parity row "
                             "with gf_invert_matrix + the engine, == the originals)",
        "roofline": {
            "bound": "hbm",
            "kernel": enc_kernel(p, k, a[k * k:]),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "launch_ms": round(step_s / max(1, launches) * 1e3, 4),
            "bytes_per_launch": int(bytes_per_launch),
        },
        "cpu_baseline": None,
        **d.info(),
    }
    if d.rank == 0:
        print(json.dumps(result), flush=True)
    batch.close()
    if rem_batch is not None:
        rem_batch.close()
    d.close()
    return 0


# ---------------------------------------------------------------------------
# main
# ---------------------------------------------------------------------------

def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` (N > 1) with no torchrun environment: start the N
    rank processes ourselves, one per GPU, as fresh children (this process has
    not touched the GPU and never execs). Each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* as torchrun would set them and re-checks them against
    --gpus. Rank 0's stdout (its JSON line) is relayed to ours, other ranks'
    stdout goes to stderr. When a rank fails the others would wait in a
    collective forever, so they are stopped; the exit code is non-zero then."""
    import signal
    import socket
    import subprocess

    n = args.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, relays = [], []

    def relay(pipe, out):
        for line in pipe:
            out.write(line)
            out.flush()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                             stdout=subprocess.PIPE, text=True)
        t = threading.Thread(target=relay, args=(p.stdout, sys.stdout if r == 0 else sys.stderr), daemon=True)
        t.start()
        procs.append(p)
        relays.append(t)

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    old = {sig: signal.signal(sig, lambda *a: (stop(), sys.exit(143))) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        while True:
            rcs = [p.poll() for p in procs]
            if all(rc is not None for rc in rcs):
                break
            if any(rc not in (None, 0) for rc in rcs):
                time.sleep(2)  # let the failing rank's peers report their own error first
                stop()
                rcs = [p.poll() for p in procs]
                break
            time.sleep(0.1)
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
    for t in relays:
        t.join(timeout=5)
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        print(f"bench.py: rank(s) failed (rank, exit code): {bad}", file=sys.stderr, flush=True)
        return 1
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if (args.gpus or 1) > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    if args.workload == "c1":
        return c1_cpu(args)
    if args.workload == "dropin":
        return dropin(args)
    d = Dist(args.dry_run, args.dist_backend, args.dist_always, args.gpus)
    d.topology(args.dry_run)
    if args.dry_run:
        return dry_run(args, d)

    import numpy as np
    import torch

    import isal_amd

    torch.cuda.set_device(d.gpu)
    dev = torch.device("cuda", d.gpu)
    k, p, n, S = args.k, args.p, args.len, args.stripes
    # the BASELINE.json shape (configs[1]): only it is labelled "C2"
    c2 = "C2 " if (k, p, n, S) == (10, 4, 1 << 20, 1024) else ""
    if args.workload in RAID_ROWS:
        p = RAID_ROWS[args.workload]
    a = np.frombuffer(control_plane_matrix(d, k, p), dtype=np.uint8)
    if args.workload.startswith("e2e"):
        return e2e(args, d, a, k, p, n)
    if args.total_stripes:
        if args.workload != "encode":
            raise SystemExit("--total-stripes is the C5 encode configuration")
        return total_stripes_run(args, d, a, k, p, n)

    # shards resident in HBM: data[s][j], coding[s][l]
    data = torch.empty((S, k, n), dtype=torch.uint8, device=dev)
    data.random_(generator=torch.Generator(device=dev).manual_seed(1234 + d.rank))
    dptr = [int(data[s, j].data_ptr()) for s in range(S) for j in range(k)]

    if args.workload == "decode":
        # C3: recover data shards {4,6,7} of every stripe from the k survivors
        errs = [4, 6, 7]
        rows = len(errs)
        in_err = set(errs)
        surv = [i for i in range(k + p) if i not in in_err][:k]
        b = np.concatenate([a[r * k:(r + 1) * k] for r in surv])
        ret, dinv, _ = isal_amd.gf_invert_matrix(b, k)
        assert ret == 0
        c = np.zeros(rows * k, np.uint8)
        for i, e in enumerate(errs):
            for j in range(k):
                acc = 0
                for r in range(k):
                    acc ^= isal_amd.gf_mul(int(dinv[k * r + j]), int(a[k * e + r]))
                c[k * i + j] = acc
        coding = torch.empty((S, p, n), dtype=torch.uint8, device=dev)
        enc = isal_amd.Batch(n, k, p, isal_amd.ec_init_tables(k, p, a[k * k:]), S, dptr,
                             [int(coding[s, l].data_ptr()) for s in range(S) for l in range(p)])
        enc.encode(torch.cuda.current_stream().cuda_stream)
        frag = lambda s, i: data[s, i] if i < k else coding[s, i - k]  # noqa: E731
        out = torch.empty((S, rows, n), dtype=torch.uint8, device=dev)
        batch = isal_amd.Batch(n, k, rows, isal_amd.ec_init_tables(k, rows, c), S,
                               [int(frag(s, i).data_ptr()) for s in range(S) for i in surv],
                               [int(out[s, i].data_ptr()) for s in range(S) for i in range(rows)])
        bytes_per_launch = (k + rows) * n * S
        kernel = enc_kernel(rows, k, c)
        workload = f"C3 decode: recover data shards {errs} of k={k} p={p} RS, {n} B shards x {S} stripes/GPU"
    else:
        rows = p
        out = torch.zeros((S, p, n), dtype=torch.uint8, device=dev)
        batch = isal_amd.Batch(n, k, p, isal_amd.ec_init_tables(k, p, a[k * k:]), S, dptr,
                               [int(out[s, l].data_ptr()) for s in range(S) for l in range(p)])
        if args.workload == "encode":
            bytes_per_launch = (k + p) * n * S
            kernel = enc_kernel(p, k, a[k * k:])
            workload = f"{c2}encode: k={k} p={p} Vandermonde RS, {n} B shards x {S} stripes/GPU"
        elif args.workload in ("encode-crc", "crc"):
            # fragment checksums: crc32_iscsi of all k+p shards,
            # fused into the encode pass or as a checksum-only pass
            crc_out = torch.zeros(S * (k + p), dtype=torch.int32, device=dev)
            bytes_per_launch = (k + p) * n * S
            if args.workload == "encode-crc":
                u = next((g for g in (12, 10, 8, 6, 5, 4) if k >= g and k % g == 0), 4)  # enc_group_crc
                # lane groups per workgroup: the launcher's rule (crc_kernels.hip fused_nv32)
                tabs_b, la_b, cap = 32 * 256 * 4, k * 256 * 4, 160 * 1024
                nv = 1 if tabs_b + 2 * la_b >= cap else (2 if 2 * (cap // (tabs_b + 2 * la_b)) > cap // (tabs_b + la_b)
                                                         else 1)
                # <P, FusedPol<U>, REG, SRC, X0 (Vandermonde row 0 derived), NB (byte tables), NV>
                kernel = f"ec_encode_crc_v16<{p}, EncPol<{u}, 1, 1, 0>, false, true, true, 4, {nv}>"
                workload = (f"{c2}encode + CRC32C (crc32_iscsi) of all k+p shards in one pass: k={k} "
                            f"p={p} Vandermonde RS, {n} B shards x {S} stripes/GPU")
            else:
                batch.encode(torch.cuda.current_stream(dev).cuda_stream)
                kernel = "crc32c_shards_pre"  # pre-shifted chains, field tables
                workload = (f"CRC32C (crc32_iscsi) of all k+p={k + p} shards, {n} B x {S} "
                            f"stripes/GPU, device-resident")
        elif args.workload == "encode-crc64":
            # encode + CRC64 (crc64_ecma_refl) of all k+p shards in one pass
            crc_out = torch.zeros(S * (k + p), dtype=torch.int64, device=dev)
            bytes_per_launch = (k + p) * n * S
            u = next((g for g in (12, 10, 8, 6, 5, 4) if k >= g and k % g == 0), 4)  # group_u
            # chunk path: 3 = byte tables pipelined into the GF rows (load group 10,
            # p <= 4, one lane group), else 1 = byte tables after each pair, lane
            # groups by the launcher's rule (crc64_kernels.hip fused_nv)
            if u == 10 and p <= 4:
                sl, nv = 3, 1
            else:
                tabs_b, la_b, cap = 4096 * 8, k * 256 * 8, 160 * 1024
                sl = 1
                nv = 1 if tabs_b + 2 * la_b >= cap else (2 if 2 * (cap // (tabs_b + 2 * la_b)) > cap // (tabs_b + la_b)
                                                         else 1)
            kernel = f"ec_encode_crc64_v16<{p}, {u}, true, {sl}, {nv}>"  # <P, U, X0 (row 0 derived), SL, NV>
            workload = (f"{c2}encode + CRC64 (crc64_ecma_refl) of all k+p shards in one pass: k={k} "
                        f"p={p} Vandermonde RS, {n} B shards x {S} stripes/GPU")
        elif args.workload == "crc64":
            # CRC64 (crc64_ecma_refl, include/crc64.h:55) of all k+p shards
            crc_out = torch.zeros(S * (k + p), dtype=torch.int64, device=dev)
            bytes_per_launch = (k + p) * n * S
            batch.encode(torch.cuda.current_stream(dev).cuda_stream)
            kernel = "crc64_shards_pre"  # pre-shifted chains, field tables
            workload = (f"CRC64 (crc64_ecma_refl) of all k+p={k + p} shards, {n} B x {S} "
                        f"stripes/GPU, device-resident")
        elif args.workload in RAID_ROWS:
            # RAID-6 P+Q / RAID-5 P over k sources (raid.h pq_gen / xor_gen /
            # pq_check; raid_base.c:44-140): the encode kernels with rows {1,..,1}
            # and {2^0, 2^1, ..} (the Horner loop q = D_j ^ 2q is sum 2^j D_j),
            # the verify kernel for the check. Bytes: (k+p)*len per stripe, the
            # reference harness's (sources+2)*len (raid/pq_gen_perf.c:79)
            coef = raid_coef(k, p)
            batch.set_tables(isal_amd.ec_init_tables(k, p, coef))
            bytes_per_launch = (k + p) * n * S
            if args.workload == "pq_check":
                batch.encode(torch.cuda.current_stream(dev).cuda_stream)
                bad = torch.empty(S, dtype=torch.int64, device=dev)
                kernel = verify_kernel(p, k, coef)
            else:
                kernel = enc_kernel(p, k, coef)
            workload = (f"{args.workload}: RAID-{5 if p == 1 else 6} parity over {k} sources "
                        f"({'P' if p == 1 else 'P+Q'}), {n} B shards x {S} stripes/GPU, device-resident")
        else:
            bytes_per_launch = (1 + 2 * p) * n * S
            kernel = f"ec_update_v16<{p}, 128>"  # ec_kernels.hip kUpdBlock
            workload = (f"ec_encode_data_update: fold one source into p={p} parity (k={k}), "
                        f"{n} B shards x {S} stripes/GPU, device-resident")

    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    vec = [0]

    def step():
        if args.workload == "update":
            batch.update(vec[0] % k, h)
            vec[0] += 1
        elif args.workload == "encode-crc":
            batch.encode_crc(0xFFFFFFFF, crc_out, h)
        elif args.workload == "crc":
            batch.crc(0xFFFFFFFF, crc_out, h)
        elif args.workload == "crc64":
            batch.crc64(0, 0, crc_out, h)
        elif args.workload == "encode-crc64":
            batch.encode_crc64(0, 0, crc_out, h)
        elif args.workload == "pq_check":
            batch.check(bad, h)
        else:
            batch.encode(h)

    # HIP events on the launch stream bracket exactly the K timed launches
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    d.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    d.barrier()
    wall = d.max(t1 - t0)
    launch_s = ev0.elapsed_time(ev1) / 1e3 / args.steps

    # Self-check on this rank's own batch (no oracle): Vandermonde parity row 0
    # is all ones, so it must equal the XOR of the sources; decode must return
    # exactly the erased shards. Reduced with MIN over ranks.
    ok = True
    if args.workload in ("encode-crc", "crc"):
        # the fused kernel and the checksum-only kernel must agree on every shard
        crc_ref = torch.zeros_like(crc_out)
        if args.workload == "encode-crc":
            batch.crc(0xFFFFFFFF, crc_ref, h)
        else:
            batch.encode_crc(0xFFFFFFFF, crc_ref, h)
        torch.cuda.synchronize(dev)
        ok &= bool(torch.equal(crc_ref, crc_out))
    if args.workload == "encode-crc64":
        # the fused kernel and the standalone CRC64 pass must agree on every shard
        crc_ref = torch.zeros_like(crc_out)
        batch.crc64(0, 0, crc_ref, h)
        torch.cuda.synchronize(dev)
        ok &= bool(torch.equal(crc_ref, crc_out))
    if args.workload in ("crc64", "encode-crc64"):
        # CRC64 is affine in the data: crc(x) = L(x) ^ crc(0^n). Parity row 0 is
        # the XOR of the k sources, so crc(P0) = XOR_j crc(d_j) ^ ((k+1)&1)*crc(0^n).
        zero = torch.zeros((2, n), dtype=torch.uint8, device=dev)
        zb = isal_amd.Batch(n, 1, 1, isal_amd.ec_init_tables(1, 1, [1]), 1,
                            [int(zero[0].data_ptr())], [int(zero[1].data_ptr())])
        c0 = torch.zeros(2, dtype=torch.int64, device=dev)
        zb.crc64(0, 0, c0, h)
        torch.cuda.synchronize(dev)
        zb.close()
        got = crc_out.view(S, k + p)
        for s_ in sorted({0, S // 2, S - 1}):
            x = int(c0[0]) if (k + 1) & 1 else 0
            for j in range(k):
                x ^= int(got[s_, j])
            ok &= x == int(got[s_, k])
    if args.workload in ("encode", "encode-crc", "encode-crc64"):
        for s_ in sorted({0, S // 2, S - 1}):
            x = data[s_, 0].clone()
            for j in range(1, k):
                x ^= data[s_, j]
            ok &= bool(torch.equal(x, out[s_, 0]))
            # every parity row: erase data shards, decode with the engine, compare
            ok &= decode_roundtrip(k, p, n, a, [data[s_, j] for j in range(k)], [out[s_, l] for l in range(p)],
                                   s_ + d.rank * S)
    elif args.workload == "decode":
        for i, e in enumerate(errs):
            ok &= bool(torch.equal(out[:, i], data[:, e]))
    elif args.workload in RAID_ROWS:
        ok &= raid_self_check(args.workload, batch, data, out, k, p, n, S, h, dev)
    self_check = None if args.workload == "update" else bool(d.max(0.0 if ok else 1.0) == 0.0)
    digest = None
    if args.workload in ("encode", "decode"):
        # control-plane digest of every rank's shards: CRC32C of all sources and
        # parity of the batch, summed on each rank and all-reduced (RCCL)
        dg = torch.zeros(S * (batch.k + batch.rows), dtype=torch.int32, device=dev)
        batch.crc(0xFFFFFFFF, dg, h)
        torch.cuda.synchronize(dev)
        digest = d.sum_i64([int((dg.to(torch.int64) & 0xFFFFFFFF).sum().item())])[0]
        del dg

    if args.workload == "update":
        step_bytes = (1 + 2 * p) * n * S
    elif args.workload == "decode":
        step_bytes = (k + rows) * n * S  # erasure_code_perf.c:324 convention
    else:
        step_bytes = (k + p) * n * S  # erasure_code_perf.c:304 convention
    total = step_bytes * args.steps * d.world
    value = total / wall / GIB
    achieved = bytes_per_launch / launch_s / 1e9

    result = {
        # BASELINE.json's metric names the C2 shape: other shapes say their own
        "metric": (METRIC if args.workload == "encode" and c2
                   else f"ec_encode_data GiB/s device-resident, k={k} m={p} {n} B shards" if args.workload == "encode"
                   else f"{args.workload} GiB/s device-resident, k={k} m={p} {n} B shards"),
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch RNG on device)",
        "config": {
            "workload": workload,
            "k": k, "p": p, "shard_bytes": n, "stripes_per_gpu": S,
            "stripe_ranges": [[r * S, (r + 1) * S] for r in range(d.world)],
            "parallelism": f"stripes sharded over {d.world} GPU(s), no data-path collective",
        },
        "payload_gib_s": round(k * n * S * args.steps * d.world / wall / GIB, 2),
        "self_check": self_check,
        "self_check_method": SELF_CHECK_METHOD.get(args.workload),
        "shard_crc32c_digest": digest,
        "roofline": {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "launch_ms": round(launch_s * 1e3, 4),
            "bytes_per_launch": bytes_per_launch,
        },
        **d.info(),
    }
    traffic = pmc_traffic(args.workload, k, p, n, S, kernel)
    if traffic:
        result["roofline"]["traffic"] = traffic[0]
        result["roofline"]["traffic_source"] = traffic[1]
    prof = kernel_stats(args.workload, k, p, n, S, kernel)
    if prof:
        # the committed rocprofv3 steady-state average of the same kernel and
        # configuration (another run, possibly another box): the cross-check
        result["roofline"]["profile_launch_ms"] = round(prof[0], 4)
        result["roofline"]["profile_frac"] = round(bytes_per_launch / (prof[0] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
        result["roofline"]["kernel_stats_source"] = prof[1]
    if d.world == 1:
        # the achievable peak, measured live with a device copy
        cc = copy_ceiling(dev)
        result["roofline"]["copy_ceiling"] = cc
        result["roofline"]["frac_of_copy_ceiling"] = round(achieved / cc["gb_s"], 4)

    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import cpu_ref_baseline as crb

        # one pinned process (or thread) per physical core
        # this process may use (its affinity set, capped by its cgroup CPU
        # quota); the count is recorded in each baseline
        threads = args.cpu_threads or crb.usable_cores()
        if args.workload in ("encode", "decode", "update"):
            # the reference's own perf harness (erasure_code_perf.c /
            # erasure_code_update_perf.c) on this host's cores
            result["cpu_baseline"] = ref_harness_baseline(args.workload, k, p, n, threads)
            if args.workload == "encode":
                result["cpu_parity_stripe_match"] = ref_parity_check(
                    k, p, n, a[k * k:], data[0].cpu().numpy(), out[0].cpu().numpy())
            elif args.workload == "decode":
                result["cpu_parity_stripe_match"] = ref_parity_check(
                    k, rows, n, c, [frag(0, i).cpu().numpy() for i in surv], out[0].cpu().numpy())
            if args.workload in ("encode", "decode"):
                # the reference's fast x86 path (AVX-512+GFNI, gf_Nvect_dot_prod_avx512_gfni)
                # restated in C intrinsics: cache-warm like the reference harness, and
                # cold (each thread cycling over distinct stripes, HBM-like streaming)
                # encode: the port's parity of stripe 0 is compared with the GPU's
                # (decode would need the decode matrix, which the port does not take)
                port_check = (data[0].cpu().numpy(), out[0].cpu().numpy()) if args.workload == "encode" else None
                for key, ring in (("cpu_baseline_simd_port", 1), ("cpu_baseline_simd_port_cold", args.cold_ring)):
                    result[key] = cpu_baseline(k, rows, n, min(args.cpu_seconds, 5.0), threads,
                                               port_check, impl="gfni", ring=ring)
        else:
            check = None
            if args.workload in ("encode-crc", "encode-crc64"):
                check = (data[0].cpu().numpy(), out[0].cpu().numpy())
            with_crc = "crc64" if args.workload in ("crc64", "encode-crc64") else args.workload in ("encode-crc", "crc")
            only_crc = args.workload in ("crc", "crc64")
            result["cpu_baseline"] = cpu_baseline(k, p, n, args.cpu_seconds, threads, check, crc=with_crc,
                                                  encode=not only_crc)
            if args.workload not in ("crc64", "encode-crc64"):  # no SIMD port of the crc64 kernels
                result["cpu_baseline_simd_port"] = cpu_baseline(k, p, n, args.cpu_seconds, threads, check,
                                                                impl="gfni", crc=with_crc, encode=not only_crc)
    else:
        result["cpu_baseline"] = None
    if d.rank == 0:
        print(json.dumps(result), flush=True)
    d.close()
    return 0


def c1_cpu(args):
    """BASELINE configs[0] (C1): k=4 p=2 Cauchy RS, one 64 KiB-shard stripe on
    the CPU — the bit-exact plumbing case. Times the engine's drop-in
    ec_encode_data on host buffers (a 384 KiB call: the engine's CPU route)
    beside the reference's ec_encode_data_base (oracle/_ref/libisal_ref.so,
    erasure_code/ec_base.c built from /root/reference; the same loop
    erasure_code_base_perf.c times), both single-threaded, and checks that
    both give the reference fixture's parity (FNV-1a of each row)."""
    import numpy as np

    import isal_amd

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import ecutil

    k, p, n = 4, 2, 65536
    case = ecutil.golden()["encode"][0]
    assert (case["k"], case["rows"], case["len"], case["gen"]) == (k, p, n, "cauchy")
    src = [ecutil.fill_bytes(n, case["seed"] + j) for j in range(k)]
    a = isal_amd.gf_gen_cauchy1_matrix(k + p, k)
    tbls = isal_amd.ec_init_tables(k, p, a[k * k:])
    L = isal_amd.lib()
    dst = [np.zeros(n, np.uint8) for _ in range(p)]
    sp, dp, tp = isal_amd._pp(src), isal_amd._pp(dst), isal_amd._p(tbls)

    def rate(fn):
        fn()
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(args.cpu_seconds, 2.0) or reps < 10:
            fn()
            reps += 1
        return (time.perf_counter() - t0) / reps

    t_eng = rate(lambda: L.ec_encode_data(n, k, p, tp, sp, dp))
    fnv = ecutil.oracle().fnv
    ok_eng = [fnv(x) for x in dst] == case["fnv"]
    ref = None
    path = os.path.join(REPO, "oracle", "_ref", "libisal_ref.so")
    if os.path.exists(path):
        R = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_ubyte)
        rt = np.zeros(32 * k * p, np.uint8)
        R.ec_init_tables_base(k, p, a[k * k:].ctypes.data_as(u8p), rt.ctypes.data_as(u8p))
        rdst = [np.zeros(n, np.uint8) for _ in range(p)]
        rs, rd = isal_amd._pp(src), isal_amd._pp(rdst)
        t_ref = rate(lambda: R.ec_encode_data_base(n, k, p, rt.ctypes.data_as(u8p), rs, rd))
        ref = {"value": round((k + p) * n / t_ref / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "reference",
               "sample": "ec_encode_data_base of the C1 stripe, erasure_code/ec_base.c built from /root/reference, "
                         f"1 thread, {min(args.cpu_seconds, 2.0):.0f} s",
               "parity_matches_fixture": [fnv(x) for x in rdst] == case["fnv"]}
    result = {
        "metric": "C1 ec_encode_data GiB/s on the host CPU (bit-exact plumbing, no GPU)",
        "value": round((k + p) * n / t_eng / GIB, 4),
        "unit": "GiB/s",
        "n_gpus": 0,
        "steps": None,
        "warmup": 1,
        "ms_per_step": round(t_eng * 1e3, 5),
        "higher_is_better": True,
        "scaling": "none",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "the reference fixture's C1 stripe (tests/golden/ec_base_golden.json encode[0])",
        "config": {"workload": "C1: k=4 p=2 Cauchy RS (gf_gen_cauchy1_matrix), one stripe of 64 KiB shards, "
                               "drop-in ec_encode_data on host buffers (engine CPU route)",
                   "k": k, "p": p, "shard_bytes": n},
        "parity_matches_fixture": ok_eng,
        "cpu_baseline": ref,
    }
    print(json.dumps(result), flush=True)
    return 0 if ok_eng else 1


def dropin(args):
    """The drop-in API as a storage caller drives it: one synchronous
    ec_encode_data per stripe on device-resident shards
    (erasure_code_perf.c:126-132 calls it in a loop the same way), from
    1 / 4 / 16 host threads (tools/dropin_bench, a C program linked against
    libisal_hip.so — no Python in the timed loop; started as a child process
    before this one touches the GPU). value = GiB/s of (k+p)*len per call at
    the largest thread count; every run self-checks two stripes' parity
    against the library's host GF math."""
    import subprocess

    exe = os.path.join(REPO, "tools", "dropin_bench")
    if not os.path.exists(exe):
        raise SystemExit("bench.py: tools/dropin_bench not built (make -C isa-l_amd tools)")
    k, p, n = args.k, args.p, args.len
    op = args.dropin_op
    if op != "encode":
        p = 2 if op.startswith("pq") else 1
    stripes = min(args.stripes, 64)
    runs = []
    for t in [int(x) for x in args.dropin_threads.split(",") if x]:
        r = subprocess.run([exe, str(k), str(p), str(n), str(stripes), str(t), str(args.dropin_seconds), "0",
                            args.dropin_op],
                           capture_output=True, text=True, timeout=120 + 2 * args.dropin_seconds)
        if r.returncode != 0:
            raise SystemExit(f"bench.py: dropin_bench failed ({r.returncode}): {r.stderr[-2000:]}")
        runs.append(json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1]))
    top = runs[-1]
    result = {
        "metric": (f"{'ec_encode_data' if op == 'encode' else op} drop-in GiB/s device-resident, one synchronous "
                   "call per stripe"),
        "value": round(top["gib_s"], 2),
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": top["calls"],
        "warmup": 2 * top["threads"],
        "ms_per_step": round(top["us_per_call"] / 1e3, 5),
        "higher_is_better": True,
        "scaling": "none",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (xorshift bytes copied into HBM; 64 resident stripes cycled)",
        "config": {"workload": (f"drop-in ec_encode_data(len={n}, k={k}, rows={p})" if op == "encode" else
                                f"drop-in {op}(vects={k + p}, len={n})") +
                               f" per stripe on hipMalloc'ed shards, {stripes} stripes, from {top['threads']} "
                               "host threads",
                   "k": k, "p": p, "shard_bytes": n},
        "threads": [{a: r[a] for a in ("threads", "calls", "us_per_call", "calls_per_s", "gib_s", "self_check")}
                    for r in runs],
        "self_check": all(r["self_check"] for r in runs),
        "roofline": None,
        "cpu_baseline": None,
    }
    print(json.dumps(result), flush=True)
    return 0 if result["self_check"] else 1


def e2e(args, d: Dist, a, k, p, n):
    """Host-memory end-to-end rate: pinned host stripes -> H2D (copy stream) ->
    GF work (compute stream) -> D2H parity (second copy stream), overlapped
    across stripes by isal_hip_pipe (depth stripes in flight). One step = one
    stripe. Bytes counted: (k+p)*len per stripe (erasure_code_update_perf.c:342
    convention); the PCIe traffic is the same k*len H2D + p*len D2H."""
    import torch

    import isal_amd

    mode = "update" if args.workload == "e2e-update" else "encode"
    ring = args.ring or max(2 * args.depth, 4)
    src = torch.empty((ring, k, n), dtype=torch.uint8).pin_memory()
    src.random_(generator=torch.Generator().manual_seed(5 + d.rank))
    par = torch.empty((ring, p, n), dtype=torch.uint8).pin_memory()
    pipe = isal_amd.Pipe(n, k, p, isal_amd.ec_init_tables(k, p, a[k * k:]), depth=args.depth, mode=mode)
    sptr = [[int(src[r, j].data_ptr()) for j in range(k)] for r in range(ring)]
    cptr = [[int(par[r, l].data_ptr()) for l in range(p)] for r in range(ring)]
    i = [0]

    def step():
        r = i[0] % ring
        pipe.submit(sptr[r], cptr[r])
        i[0] += 1

    wall = timed_steps(d, step, pipe.flush, args.steps, args.warmup)
    total = (k + p) * n * args.steps * d.world
    # spot check: the last stripe's parity equals a device-resident re-encode
    r = (i[0] - 1) % ring
    dsrc = src[r].to(dev := torch.device("cuda", d.gpu))
    dpar = torch.empty((p, n), dtype=torch.uint8, device=dev)
    isal_amd.ec_encode_data(n, k, p, isal_amd.ec_init_tables(k, p, a[k * k:]),
                            [dsrc[j] for j in range(k)], [dpar[l] for l in range(p)])
    ok = bool(torch.equal(dpar.cpu(), par[r]))
    result = {
        "metric": f"{args.workload} GiB/s host-resident (pinned) end-to-end incl. H2D/D2H",
        "value": round(total / wall / GIB, 3),
        "unit": "GiB/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, pinned host memory)",
        "config": {"workload": f"{mode} pipeline, k={k} p={p}, {n} B shards, depth {args.depth}, "
                               f"{ring} pinned host stripes cycled",
                   "k": k, "p": p, "shard_bytes": n},
        "pcie": {"h2d_gb_s": round(k * n * args.steps / wall / 1e9, 2),
                 "d2h_gb_s": round(p * n * args.steps / wall / 1e9, 2),
                 "peak_gb_s_per_direction": 63.0},
        "parity_check_last_stripe": ok,
        "cpu_baseline": None,
        **d.info(),
    }
    if d.rank == 0:
        print(json.dumps(result), flush=True)
    pipe.close()
    d.close()
    return 0


def dry_run(args, d: Dist):
    """Harness only (CPU, gloo): control-plane broadcast, barrier, max-over-ranks,
    and — with --total-stripes — the C5 partition of the stripes over the
    ranks (isal_hip_multi_partition, the library's pure host function) with
    the SUM all-reduce of counts and ranges that the GPU run performs."""
    import numpy as np

    k, p = args.k, args.p
    if os.environ.get("ISAL_BENCH_DRY_FAIL_RANK") == str(d.rank):
        # harness test hook: this rank dies before the first collective, so the
        # launcher must stop its peers (blocked in the broadcast) and fail
        raise SystemExit(f"bench.py: dry-run rank {d.rank} failing on request")
    a = control_plane_matrix(d, k, p) if d.rank == 0 or d.world > 1 else b""
    sleep = 0.002 * (1 + d.rank)
    wall = timed_steps(d, lambda: time.sleep(sleep), lambda: None, args.steps, args.warmup)
    total_stripes = d.sum(float(args.stripes))
    out = {"metric": METRIC, "dry_run": True, "n_gpus": d.world, "wall": wall, "stripes": total_stripes,
           "matrix_fnv": int(np.frombuffer(a, np.uint8).sum()),
           "stripe_ranges": [[r * args.stripes, (r + 1) * args.stripes] for r in range(d.world)],
           **d.info()}
    if args.total_stripes:
        import isal_amd

        first, count = isal_amd.partition(args.total_stripes, d.world, d.rank)
        B = max(1, min(args.stripes, count))
        launches = count // B + (1 if count % B else 0)
        ranges = [0] * (2 * d.world)
        ranges[2 * d.rank], ranges[2 * d.rank + 1] = first, count
        red = d.sum_i64([count * args.steps, launches] + ranges)
        out.update({"stripes_encoded": red[0], "stripes_expected": args.total_stripes * args.steps,
                    "launches_per_step": red[1],
                    "stripe_ranges": [[red[2 + 2 * r], red[2 + 2 * r] + red[3 + 2 * r]] for r in range(d.world)]})
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
