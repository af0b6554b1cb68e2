#!/usr/bin/env python3
"""The memory skeleton of each encode shape as its own ceiling (DESIGN.md §3,
"What bounds each encode shape"): tools/copy_probe.hip:skel_tiles reads K
source shards and writes P output shards per stripe exactly as the encode
does (16 B per lane, 4 KiB column tiles, XCD-contiguous items, nt buffer
loads/stores) with the GF arithmetic replaced by one XOR fold. Prints one JSON
line per (shape, LDS cap): GB/s of (K+P)*len*S per pass and the fraction of
8 TB/s. `pointer_table`: the shard addresses are read from a device pointer
table as the batch encode does, instead of computed from the layout.
`tiles_per_wg` (TILES=1,2,4 in the environment; the xor_gen / pq_gen / C2
shapes only above 1): consecutive 4 KiB tiles per workgroup. `threads_per_wg`
(BLOCKS=256,128,512,1024; xor_gen and C2 only besides 256): a tile is
threads x 16 bytes. `shard_pad` (PAD=0,256,4096,... in the environment,
pointer table only): bytes between consecutive shards beyond len.
Run on the GPU box: python3 tools/skel_probe.py [REPS [SHAPE]]
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MiB = 1 << 20
SHAPES = [  # (label, k, p, len, stripes)
    ("copy 1:1", 1, 1, MiB, 4096),
    ("C2 encode k10p4", 10, 4, MiB, 1024),
    ("C3 decode k10 -> 3", 10, 3, MiB, 1024),
    ("pq_gen k10p2", 10, 2, MiB, 1024),
    ("xor_gen k10p1", 10, 1, MiB, 1024),
    ("k10p6", 10, 6, MiB, 1024),
    ("k10p8", 10, 8, MiB, 1024),
    ("k20p6", 20, 6, 4 * MiB, 64),
    ("k20p8", 20, 8, 4 * MiB, 64),
    ("C4 update k20p6 (7 read, 6 written)", 7, 6, 4 * MiB, 64),
    ("read-only k10", 10, 0, MiB, 1024),
    ("read-only k12 (pq_check)", 12, 0, MiB, 1024),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2] if len(sys.argv) > 2 else None  # shape-label substring
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libcopy_probe.so"))
    lib.skel_probe_gbs.restype = ctypes.c_double
    lib.skel_probe_gbs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_uint, ctypes.c_int, ctypes.c_uint, ctypes.c_int]
    data = torch.empty(12 << 30, dtype=torch.uint8, device="cuda")
    data.view(torch.int32).random_()
    coding = torch.empty(8 << 30, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for label, k, p, n, s in SHAPES:
        if only and only not in label:
            continue
        assert k * n * s <= data.numel() and p * n * s <= coding.numel()
        for blk in [int(b) for b in os.environ.get("BLOCKS", "256").split(",")]:
         for tpi in [int(t) for t in os.environ.get("TILES", "1").split(",")]:
          pads = [int(x) for x in os.environ.get("PAD", "").split(",") if x]
          combos = [(32768, 1, pad) for pad in pads] if pads else [(0, 0, 0), (32768, 0, 0), (32768, 1, 0)]
          for lds, ptrs, pad in combos:
            if pads:
                if k * (n + pad) * s > data.numel() or p * (n + pad) * s > coding.numel():
                    continue
                lib.skel_probe_set_pad(ctypes.c_ulonglong(pad))
            code = ptrs | (tpi << 8) | ((blk if blk != 256 else 0) << 16)
            g = lib.skel_probe_gbs(data.data_ptr(), coding.data_ptr(), n, k, p, s, reps, lds, code)
            print(json.dumps({"shape": label, "k": k, "p": p, "len": n, "stripes": s, "lds_bytes": lds,
                              "pointer_table": bool(ptrs), "shard_pad": pad, "tiles_per_wg": tpi,
                              "threads_per_wg": blk,
                              "reps": reps, "gb_s": round(g, 1), "frac_of_8tbs": round(g / 8000.0, 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
