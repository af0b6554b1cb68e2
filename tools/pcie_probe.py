#!/usr/bin/env python3
"""PCIe copy-engine behaviour behind the host-memory pipeline (GPU box diagnostic).

Mimics isal_hip_pipe's stream structure with plain torch copies (no engine
code): stripe i's 10 MiB of sources go host->device on stream A, its 4 MiB of
parity device->host on stream B after an event, and slot i % depth is reused
only once its parity left (host waits on an event). Prints GB/s per direction
for depth 1..8, and for H2D-only / D2H-only streams, to tell whether the rate
drop of the pipeline at depth >= 4 is the copy engines' or the pipeline's.
"""
import json
import time

import torch


def run(depth, steps=200, h2d=True, d2h=True, src_mb=10, par_mb=4):
    dev = torch.device("cuda", 0)
    ring = max(depth, 4)
    hs = torch.empty((ring, src_mb << 20), dtype=torch.uint8).pin_memory()
    hp = torch.empty((ring, par_mb << 20), dtype=torch.uint8).pin_memory()
    ds = torch.empty((depth, src_mb << 20), dtype=torch.uint8, device=dev)
    dp = torch.empty((depth, par_mb << 20), dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    free = [None] * depth

    def step(i):
        s, r = i % depth, i % ring
        if free[s] is not None:
            free[s].synchronize()
        ev = torch.cuda.Event()
        if h2d:
            with torch.cuda.stream(sa):
                ds[s].copy_(hs[r], non_blocking=True)
                ev.record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(ev)
            if d2h:
                hp[r].copy_(dp[s], non_blocking=True)
            f = torch.cuda.Event()
            f.record(sb)
        free[s] = f

    for i in range(10):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(10 + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"depth": depth, "h2d": h2d, "d2h": d2h,
            "h2d_gb_s": round(src_mb * 2**20 * steps / dt / 1e9, 2) if h2d else None,
            "d2h_gb_s": round(par_mb * 2**20 * steps / dt / 1e9, 2) if d2h else None,
            "ms_per_stripe": round(dt / steps * 1e3, 4)}


def main():
    for depth in (1, 2, 3, 4, 6, 8):
        print(json.dumps(run(depth)), flush=True)
    for depth in (2, 6):
        print(json.dumps(run(depth, d2h=False)), flush=True)
        print(json.dumps(run(depth, h2d=False)), flush=True)


if __name__ == "__main__":
    main()
