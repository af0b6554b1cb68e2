#!/usr/bin/env python3
"""Timeline of large synchronous host-resident calls (GPU box diagnostic).

Run under `rocprofv3 --memory-copy-trace --kernel-trace` to see how the
column-chunked route overlaps its copies: a k=10 p=4 ec_encode_data of 2 MiB
(or --len) shards, several times per configuration, with a 20 ms gap between
configurations so they separate on the timeline. Prints one JSON line per
configuration with the per-call wall time; the copy/kernel records come from
the profiler's CSVs (tools/trace_summary.py).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "isa-l_amd"))
import isal_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=2 << 20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    k, p, n = 10, 4, args.len
    a = isal_amd.gf_gen_rs_matrix(k + p, k)
    tbls = isal_amd.ec_init_tables(k, p, a[k * k:])
    rng = np.random.default_rng(1)
    pageable = ([rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)],
                [np.zeros(n, np.uint8) for _ in range(p)])
    pinned = ([torch.from_numpy(x).pin_memory().numpy() for x in pageable[0]],
              [torch.zeros(n, dtype=torch.uint8).pin_memory().numpy() for _ in range(p)])
    L = isal_amd.lib()
    configs = [("pageable", "0", ""), ("pageable", "1", "1024"), ("pageable", "1", "4096"),
               ("pinned", "0", ""), ("pinned", "1", "512"), ("pinned", "1", "1024"), ("pinned", "1", "2048")]
    for mem, piped, kb in configs:
        os.environ.update(ISAL_HIP_BACKEND="gpu", ISAL_HIP_PIPE_CHUNKS=piped, ISAL_HIP_CHUNK_KB=kb)
        isal_amd.reload_config()
        src, dst = pageable if mem == "pageable" else pinned
        sp, dp, tp = isal_amd._pp(src), isal_amd._pp(dst), isal_amd._p(tbls)
        L.ec_encode_data(n, k, p, tp, sp, dp)  # warm
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            L.ec_encode_data(n, k, p, tp, sp, dp)
            ts.append((time.perf_counter() - t0) * 1e6)
        print(json.dumps({"mem": mem, "piped": piped, "chunk_kb": kb or "default", "len": n,
                          "us": [round(t, 1) for t in ts], "best_us": round(min(ts), 1)}), flush=True)
        time.sleep(0.02)


if __name__ == "__main__":
    main()
