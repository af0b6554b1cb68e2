#!/usr/bin/env python3
"""Column-chunk size of the pipelined host-call route (GPU box diagnostic).

Times a synchronous k=10 p=4 ec_encode_data on pageable host shards of 2, 4
and 16 MiB through the pipelined chunks at several ISAL_HIP_CHUNK_KB values,
plus the one-chunk-at-a-time route (ISAL_HIP_PIPE_CHUNKS=0). One JSON line per
(len, chunk); GB/s counts the (k + p) * len bytes crossing PCIe.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import route_crossover as rc  # noqa: E402


def main():
    k, p = 10, 4
    for n in (2 << 20, 4 << 20, 16 << 20):
        for kb in (0, 256, 512, 1024, 2048, 4096):
            os.environ["ISAL_HIP_CHUNK_KB"] = str(kb) if kb else ""
            us = rc.per_call(k, p, n, "gpu", budget=0.4)
            print(json.dumps({"len": n, "chunk_kb": kb or "default", "us": round(us, 1),
                              "gb_s": round((k + p) * n / us / 1e3, 2)}), flush=True)
        os.environ["ISAL_HIP_CHUNK_KB"] = ""
        us = rc.per_call(k, p, n, "gpu", budget=0.4, piped="0")
        print(json.dumps({"len": n, "chunk_kb": "unpipelined", "us": round(us, 1),
                          "gb_s": round((k + p) * n / us / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
