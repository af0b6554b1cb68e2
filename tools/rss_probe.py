"""Which host-allocation pattern of the full-size GPU tests keeps anonymous
memory resident after it is freed (tests/test_gpu_parity.py
_check_stripes_vs_oracle: 1 MiB device shards copied to numpy, the oracle's
outputs allocated in 16 worker threads, 4 MiB x 64 output slabs copied back).
Prints RssAnon (MiB) after each phase. Usage: python tools/rss_probe.py PHASE..."""
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def anon():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("RssAnon"):
                return int(line.split()[1]) // 1024
    return -1


def main():
    dev = torch.device("cuda:0")
    k, rows, n, ns, chunk = 10, 4, 1 << 20, 1024, 64
    data = torch.zeros((ns, k, n), dtype=torch.uint8, device=dev)
    out = torch.zeros((ns, rows, n), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    print("start", anon(), flush=True)
    for phase in sys.argv[1:]:
        for s0 in range(0, ns, chunk):
            if phase == "shards":      # 1 MiB device views -> numpy, freed per chunk
                keep = [[data[s, j].cpu().numpy() for j in range(k)] for s in range(s0, s0 + chunk)]
            elif phase == "threads":   # worker-thread numpy allocations, freed per chunk
                with ThreadPoolExecutor(16) as ex:
                    keep = list(ex.map(lambda s: [np.ones(n, np.uint8) for _ in range(rows)], range(chunk)))
            elif phase == "slab":      # one 256 MiB device slab -> numpy
                keep = out[s0:s0 + chunk].cpu().numpy()
            else:
                raise SystemExit(f"unknown phase {phase}")
            del keep
        print(phase, anon(), flush=True)


if __name__ == "__main__":
    main()
