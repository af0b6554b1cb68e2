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
  hbm    algorithmic bytes at the copy ceiling (a plain nt 16-B-per-lane copy,
         MI355X_MICROARCH.md / bench.py copy_ceiling: 6.29-6.48 TB/s).

The kernel cannot run faster than max(valu, lds, hbm); `overlap` is that
bound over the measured time. A formulation is worth building when the bound
it implies (fewer VALU, conflict-free LDS) is below the target.

  python3 tools/fused_model.py profiles/r05_pmc_sq_fused.txt > profiles/r05_fused_model.txt
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


def main(argv):
    if len(argv) < 2:
        print(__doc__)
        return 2
    rate = rates()  # wave-instructions per CU per ns
    counters = sections(argv[1])
    steady = {}
    for spec in argv[2:]:  # kernel=steady.csv
        k, f = spec.split("=", 1)
        steady[k] = f
    print(f"# fused-kernel resource model, tools/fused_model.py {' '.join(os.path.relpath(a, ROOT) for a in argv[1:])}")
    print(f"# VALU issue rate {rate:.3f} wave-instr/CU/ns (r03_valu_probe, 4 waves/SIMD); "
          f"{CUS} CUs at {CLOCK_GHZ} GHz; HBM at the copy ceiling {COPY_CEILING / 1e12:.2f} TB/s")
    print("kernel,valu_ms,lds_ms,lds_conflict_free_ms,hbm_ms,bound_ms,bound_conflict_free_ms,measured_ms,"
          "overlap,conflict_share")
    for kern, c in counters.items():
        valu_ms = c.get("SQ_INSTS_VALU", 0) / CUS / rate / 1e6
        act = c.get("SQ_LDS_IDX_ACTIVE", 0)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0)
        lds_ms = act / CUS / CLOCK_GHZ / 1e6
        lds_cf_ms = (act - conf) / CUS / CLOCK_GHZ / 1e6
        meas, nbytes = steady_ms(steady[kern], kern) if kern in steady else (float("nan"), 15032385536)
        hbm_ms = nbytes / COPY_CEILING * 1e3
        bound = max(valu_ms, lds_ms, hbm_ms)
        bound_cf = max(valu_ms, lds_cf_ms, hbm_ms)
        print(f"{kern},{valu_ms:.3f},{lds_ms:.3f},{lds_cf_ms:.3f},{hbm_ms:.3f},{bound:.3f},{bound_cf:.3f},"
              f"{meas:.4f},{bound / meas:.3f},{conf / act if act else 0:.3f}")
    print(f"# target {TARGET_MS} ms (VERDICT r04); a layout is worth building when its bound, with the "
          "overlap the current kernel achieves, lands below it")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
