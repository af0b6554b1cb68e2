#!/usr/bin/env python3
"""CPU baseline from the reference's OWN perf harnesses (bench infrastructure).

Runs the binaries `make -C oracle ref` builds from /root/reference sources
(never shipped in the product):
  oracle/_ref/erasure_code_perf            erasure_code/erasure_code_perf.c
  oracle/_ref/erasure_code_update_perf_c4  erasure_code/erasure_code_update_perf.c
                                           with TEST_CUSTOM, 4 MiB shards
linked against the reference's portable ec_base.c (the image has no nasm, so
the AVX-512/GFNI kernels cannot be assembled — see DESIGN.md §6).

Each harness is single-threaded (reference include/test.h BENCHMARK macros),
so the host rate is measured as the reference's own README suggests for
throughput: one process per core, pinned with sched_setaffinity, run
concurrently, MB/s summed. The line names printed by the harness
(`erasure_code_encode_cold: ... = X MB/s`) are parsed; MB = 1e6 B
(test.h:384-397).

usage: tools/cpu_ref_baseline.py [--procs N] [--which encode|update] [--json]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref")
LINE = re.compile(r"^(\S+): runtime = .*= ([0-9.]+) MB/s")

HARNESS = {
    # C2 / C3 shape: k=10 p=4, 1 MiB shards, 3 erasures (the perf app's own
    # srand(0x1234) choice; erasure_code_perf.c:257-270)
    "encode": (["erasure_code_perf", "-k", "10", "-p", "4", "-e", "3", "-s", "1M"],
               {"erasure_code_encode_cold": "encode", "erasure_code_decode_cold": "decode",
                "erasure_code_encode_warm": "encode", "erasure_code_decode_warm": "decode",
                "erasure_code_encode_cus": "encode", "erasure_code_decode_cus": "decode"}),
    # C4 shape: k=20 p=6, 4 MiB shards (update harness, TEST_CUSTOM build)
    "update": (["erasure_code_update_perf_c4", "-k", "20", "-p", "6", "-e", "3"],
               {"ec_encode_data_update_cus": "update_stripe",
                "ec_encode_data_update_single_src_cus": "update_single_src",
                "ec_encode_data_update_decode_cus": "update_decode"}),
}


def host_info() -> dict:
    """CPU model and core counts of this host (lscpu), plus this process's affinity."""
    info = {"affinity_cpus": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "affinity_physical_cores": len(_physical_cpus(0)), "cgroup_cpu_quota": cgroup_cpu_quota(),
            "usable_cores": usable_cores()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                a, b = line.split(":", 1)
                kv[a.strip()] = b.strip()
        info["model"] = kv.get("Model name")
        for key, name in (("Socket(s)", "sockets"), ("Core(s) per socket", "cores_per_socket"),
                          ("Thread(s) per core", "threads_per_core"), ("CPU(s)", "cpus")):
            if kv.get(key, "").isdigit():
                info[name] = int(kv[key])
        if "sockets" in info and "cores_per_socket" in info:
            info["physical_cores"] = info["sockets"] * info["cores_per_socket"]
        flags = kv.get("Flags", "").split()
        info["isa"] = [f for f in ("avx2", "avx512f", "avx512bw", "gfni", "vpclmulqdq") if f in flags]
    except (OSError, subprocess.TimeoutExpired):
        pass
    try:
        v = subprocess.run(["nasm", "-v"], capture_output=True, text=True, timeout=10)
        info["nasm"] = v.stdout.strip() or v.stderr.strip()
    except OSError:
        info["nasm"] = None  # absent: the reference's x86 SIMD kernels cannot be assembled
    return info


def cgroup_cpu_quota() -> float | None:
    """CPUs' worth of time this process's cgroup may use (cgroup v2 cpu.max,
    v1 cfs quota/period), None when unlimited or unknown: a quota below the
    core count caps what any number of pinned processes can measure."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def physical_cpus(n: int = 0) -> list[int]:
    """n (0 = all) CPUs of this process's affinity set, one per physical core
    where the topology says which logical CPUs are hyperthread siblings."""
    return _physical_cpus(n)


def usable_cores() -> int:
    """Physical cores this process may use at once: one per physical core of
    its affinity set, capped by its cgroup CPU quota. (The GPU box grants 16
    CPUs of quota on a 2 x 64-core host: 128 pinned processes there measured
    the reference harness at 7.02 GiB/s — what 16 cores give — and the GFNI
    port at 68 GiB/s against 384 with 16 threads, every thread throttled in
    turn; profiles/r05/r05_bench_c2_allcores_quota16.json.)"""
    n = len(_physical_cpus(0))
    q = cgroup_cpu_quota()
    return max(1, min(n, int(q))) if q else n


def _physical_cpus(n: int) -> list[int]:
    """n (0 = all) CPUs of this process's affinity set, one per physical core where the
    topology says which logical CPUs are hyperthread siblings, taken round-robin
    over the L3 domains (CCDs) so that n cores spread over the host's caches and
    memory links. Taking the first n cores put 16 threads on two CCDs of the GPU
    box's EPYC 9575F: the GFNI port measured 109 GiB/s there against 384-423
    with the same 16 threads placed by the scheduler
    (profiles/r05/r05_bench_c2_pinned_first16.json, r04_bench_c2.json)."""
    cpus = sorted(os.sched_getaffinity(0))
    domains, seen = {}, set()
    for c in cpus:
        sib = _read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") or str(c)
        if sib in seen:
            continue
        seen.add(sib)
        l3 = (_read(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list")
              or _read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") or "0")
        domains.setdefault(l3, []).append(c)
    groups = list(domains.values())
    chosen = []
    for i in range(max((len(g) for g in groups), default=0)):
        chosen.extend(g[i] for g in groups if i < len(g))
    return chosen[:n] if n else chosen


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def run(which: str, procs: int, timeout: float = 180.0) -> dict:
    """Run `procs` (0 = usable_cores(): one per physical core this process may use)
    pinned copies of the harness at once (plus nothing else) and sum their
    per-phase MB/s. Returns {phase: {"mb_s_sum", "mb_s_per_proc"}, ...}."""
    argv, names = HARNESS[which]
    exe = os.path.join(REF, argv[0])
    if not os.path.exists(exe):
        return {"error": f"{exe} not built (make -C oracle ref needs /root/reference)"}
    cpus = _physical_cpus(procs or usable_cores())

    def pin(c):
        return lambda: os.sched_setaffinity(0, {c})

    t0 = time.time()
    ps = [subprocess.Popen([exe] + argv[1:], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True, preexec_fn=pin(c)) for c in cpus]
    outs = []
    for p in ps:
        o, _ = p.communicate(timeout=timeout)
        outs.append((p.returncode, o))
    wall = time.time() - t0
    phases: dict = {}
    for rc, o in outs:
        if rc != 0 or "Pass" not in o:
            return {"error": f"harness failed rc={rc}: {o[-500:]}"}
        for line in o.splitlines():
            m = LINE.match(line.strip())
            if m and m.group(1) in names:
                phases.setdefault(names[m.group(1)], []).append(float(m.group(2)))
    res = {"procs": len(cpus), "cpus": cpus, "wall_s": round(wall, 1),
           "command": " ".join(["oracle/_ref/" + argv[0]] + argv[1:])}
    for ph, v in phases.items():
        res[ph] = {"mb_s_sum": round(sum(v), 2), "mb_s_per_proc": [round(x, 2) for x in v]}
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=-1,
                    help="-1 = 1 and usable_cores() (one per physical core of the affinity set, capped "
                         "by the cgroup CPU quota); 0 = the latter only")
    ap.add_argument("--which", choices=sorted(HARNESS), default="encode")
    a = ap.parse_args(argv)
    out = {"host": host_info()}
    counts = [a.procs] if a.procs >= 0 else [1, 0]
    for n in counts:
        out[f"procs_{n}"] = run(a.which, n)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
