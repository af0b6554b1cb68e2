#!/usr/bin/env python3
"""Resource model of the fused encode + checksum kernels (DESIGN.md §3,
"Fragment checksums: what bounds them"): from committed files only, no GPU.

For each kernel it reads the SQ counters of one launch (rocprofv3 --pmc, the
rNN_pmc_sq_fused*.txt files this tool's caller commits) and its steady-state
launch time (rNN_*_kernel_steady.csv), and sets three times side by side:

  valu   SQ_INSTS_VALU wave-instructions / CUs / the chip's measured issue
         rate for this instruction mix at 3-4 waves per SIMD
         (profiles/r03/r03_valu_probe.jsonl: v_perm_b32 and the other ops
         the kernels use, harmonic mean — an optimistic rate for the fused
         kernels, which also issue SDWA shifts and 64-bit folds);
  lds    SQ_LDS_IDX_ACTIVE cycles / CUs at the shader clock, and the same
         without SQ_LDS_BANK_CONFLICT — the LDS time a conflict-free table
         layout with the SAME instruction count would take;
  hbm    algorithmic bytes at the kernel's own memory skeleton (DESIGN §3,
         "the memory skeleton"): a read-only pass (the checksum-only kernels)
         at the read-only skeleton, 0.9236 of 8 TB/s; a pass that reads k
         shards and writes p (the fused kernels) at the C2 encode skeleton,
         0.7807 of 8 TB/s. (Round 5 priced every kernel at the 1:1 copy
         ceiling, 6.29 TB/s, which made a read-only kernel look closer to its
         bound than it is.)

The kernel cannot run faster than max(valu, lds, hbm); `overlap` is that
bound over the measured time. A formulation is worth building when the bound
it implies (fewer VALU, conflict-free LDS) is below the target.

  python3 tools/fused_model.py profiles/r05/r05_pmc_sq_fused.txt --steady SUB=CSV ... \
      --compose LABEL=SUB*W+SUB*W > profiles/r05/r05_fused_model.txt
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = lambda *a: os.path.join(ROOT, "profiles", *a)  # noqa: E731
CUS = 256
CLOCK_GHZ = 2.4          # MI355X shader clock (MI355X_MICROARCH.md)
COPY_CEILING = 6.29e12   # B/s, nt float4 copy (MI355X_MICROARCH.md; bench.py copy probe 6.29-6.48)
# per-kernel HBM ceilings: the memory skeletons (profiles/r05/r05_skel_probe_m.jsonl)
READ_ONLY_SKELETON = 0.9236 * 8e12   # pq_check-shaped read-only pass
ENCODE_SKELETON = 0.7807 * 8e12      # C2 k10p4: 10 shards read, 4 written
READ_ONLY_KERNELS = ("crc64_shards_pre", "crc32c_shards_pre", "crc64_pre_", "ec_verify")


def hbm_ceiling(label):
    """B/s the kernel's memory pattern reaches with no arithmetic."""
    return READ_ONLY_SKELETON if any(k in label for k in READ_ONLY_KERNELS) else ENCODE_SKELETON
TARGET_MS = 2.9          # encode + CRC64 at C2 <= 2.9 ms (0.648 of 8 TB/s)


def rates():
    r = {}
    for line in open(P("r03", "r03_valu_probe.jsonl")):
        d = json.loads(line)
        if d.get("waves_per_simd") == 4:
            r[d["op"]] = d["wave_instr_per_cu_ns"]
    others = ["v_bitop3_b32", "v_and_b32", "v_lshrrev_b32", "v_xor_b32", "v_add_u32"]
    return len(others) / sum(1.0 / r[o] for o in others)


def sections(path):
    """{kernel: {counter: value}} from a `rocprofv3 --pmc` summary written as
    a kernel line followed by indented `COUNTER value` lines."""
    out, cur = {}, None
    for line in open(path):
        if line.startswith("#") or not line.strip():
            continue
        m = re.match(r"\s+([A-Z0-9_]+)\s+([0-9.e+]+)", line)
        if m and cur is not None:
            out[cur][m.group(1)] = float(m.group(2))
        elif not line.startswith(" "):
            cur = line.strip().replace("void ", "")
            out.setdefault(cur, {})
    return out


def steady_ms(path, kernel):
    kv = {}
    for l in open(path):
        if "," in l and not l.startswith("#"):
            a, b = l.rstrip("\n").split(",", 1)
            kv[a] = b
    return float(kv["avg_ns"]) / 1e6, int(kv["bytes_per_launch"])


def find(counters, sub):
    hits = [k for k in counters if sub in k]
    if len(hits) != 1:
        raise SystemExit(f"fused_model: {sub!r} matches {hits}")
    return hits[0]


def row(label, c, meas_ms, nbytes, rate):
    valu_ms = c.get("SQ_INSTS_VALU", 0) / CUS / rate / 1e6
    act = c.get("SQ_LDS_IDX_ACTIVE", 0)
    conf = c.get("SQ_LDS_BANK_CONFLICT", 0)
    lds_ms = act / CUS / CLOCK_GHZ / 1e6
    lds_cf_ms = (act - conf) / CUS / CLOCK_GHZ / 1e6
    hbm_ms = nbytes / hbm_ceiling(label) * 1e3
    bound = max(valu_ms, lds_ms, hbm_ms)
    bound_cf = max(valu_ms, lds_cf_ms, hbm_ms)
    ov = f"{bound / meas_ms:.3f}" if meas_ms == meas_ms else ""
    meas = f"{meas_ms:.4f}" if meas_ms == meas_ms else ""
    print(f"{label},{valu_ms:.3f},{lds_ms:.3f},{lds_cf_ms:.3f},{hbm_ms:.3f},{bound:.3f},{bound_cf:.3f},"
          f"{meas},{ov},{conf / act if act else 0:.3f}")


def main(argv):
    """argv: COUNTERS.txt [--steady SUB=CSV ...] [--compose LABEL=SUB*W+SUB*W ...]"""
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("counters")
    ap.add_argument("--steady", action="append", default=[], help="kernel substring=steady-state csv")
    ap.add_argument("--compose", action="append", default=[],
                    help="LABEL=SUB*W+SUB*W: a formulation not built yet, its counters as a weighted sum "
                         "of measured kernels' (e.g. the GF half of the encode plus 13/14 of a checksum pass)")
    ap.add_argument("--bytes", type=float, default=15032385536.0, help="algorithmic bytes per launch")
    a = ap.parse_args(argv[1:])
    rate = rates()  # wave-instructions per CU per ns
    counters = sections(a.counters)
    print(f"# fused-kernel resource model: tools/fused_model.py {' '.join(argv[1:])}")
    print(f"# VALU issue rate {rate:.3f} wave-instr/CU/ns (profiles/r03/r03_valu_probe.jsonl, 4 waves/SIMD); "
          f"{CUS} CUs at {CLOCK_GHZ} GHz; HBM at each kernel's memory skeleton (read-only "
          f"{READ_ONLY_SKELETON / 1e12:.2f} TB/s, encode {ENCODE_SKELETON / 1e12:.2f} TB/s); "
          f"{a.bytes / 1e9:.3f} GB per launch")
    print("kernel,valu_ms,lds_ms,lds_conflict_free_ms,hbm_ms,bound_ms,bound_conflict_free_ms,measured_ms,"
          "bound_over_measured,conflict_share")
    for spec in a.steady:
        sub, f = spec.split("=", 1)
        k = find(counters, sub)
        meas, nbytes = steady_ms(f, k)
        row(k, counters[k], meas, nbytes, rate)
    for spec in a.compose:
        label, expr = spec.split("=", 1)
        c = {}
        for term in expr.split("+"):
            sub, w = term.rsplit("*", 1)
            for name, v in counters[find(counters, sub)].items():
                c[name] = c.get(name, 0.0) + float(w) * v
        row(label + " (composed)", c, float("nan"), a.bytes, rate)
    print(f"# target {TARGET_MS} ms (VERDICT r04). bound = max(valu, lds, hbm): no schedule beats it; "
          "bound_over_measured is the overlap the kernel achieves. A composed formulation is worth "
          "building when its bound, at the measured kernels' overlap, lands below the target.")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
