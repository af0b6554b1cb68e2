#!/usr/bin/env python3
"""VALU-issue model of the encode kernels ("What bounds the wide
stripes"): from committed files only, no GPU.

For each shape: the kernel's VALU wave-instructions per launch (SQ_INSTS_VALU,
rocprofv3 --pmc, profiles/r04_pmc_sq_*.txt), split into v_perm_b32 (3 per
looked-up GF product and 16-byte lane dword, counted from the coefficient
structure: with the 0/1 fast path, row 0 and source 0 take no lookups) and
the rest; each part timed at its measured chip-wide issue rate
(profiles/r03/r03_valu_probe.jsonl, 4 waves per SIMD); compared with the
steady-state launch time (profiles/r04_*_kernel_steady.csv) and with the HBM
time at the copy ceiling (MI355X_MICROARCH.md: float4 copy 6.29 TB/s).

  python3 tools/valu_model.py > profiles/r04_valu_model.txt
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = lambda *a: os.path.join(ROOT, "profiles", *a)
CUS = 256
COPY_CEILING = 6.29e12  # B/s, float4 copy (MI355X_MICROARCH.md)

# label, SQ file, section header (None = first kernel line matching), kernel, k, p, len, stripes, xor, steady csv
SHAPES = [
    ("C2 k10p4", "r04_pmc_sq_c2.txt", None, "ec_encode_v16<4, EncPol<10, 2, 2, 2>, 1>", 10, 4, 1 << 20, 1024, True,
     "r04_c2_encode_kernel_steady.csv"),
    ("k10p6", "r04_pmc_sq_wide.txt", "## k10p6", "ec_encode_v16<6, EncPol<5, 2, 2, 2>, 3>", 10, 6, 1 << 20, 1024, True,
     "r04_k10p6_encode_kernel_steady.csv"),
    ("k10p8", "r04_pmc_sq_wide.txt", "## k10p8", "ec_encode_v16<8, EncPol<5, 2, 2, 2>, 3>", 10, 8, 1 << 20, 1024, True,
     "r04_k10p8_encode_kernel_steady.csv"),
    ("k20p6", "r04_pmc_sq_wide.txt", "## k20p6", "ec_encode_v16<6, EncPol<5, 2, 2, 2>, 3>", 20, 6, 4 << 20, 64, True,
     "r04_k20p6_encode_kernel_steady.csv"),
    # the same shapes with groups of 10 (ISAL_HIP_ENC_WIDE5=0; another box)
    ("k10p6 g10", "r04_pmc_sq_wide_g10.txt", "## k10p6", "ec_encode_v16<6, EncPol<10, 2, 2, 2>, 3>", 10, 6, 1 << 20,
     1024, True, "r04_k10p6_encode_g10_kernel_steady.csv"),
    ("k10p8 g10", "r04_pmc_sq_wide_g10.txt", "## k10p8", "ec_encode_v16<8, EncPol<10, 2, 2, 2>, 1>", 10, 8, 1 << 20,
     1024, True, "r04_k10p8_encode_g10_kernel_steady.csv"),
    ("k20p6 g10", "r04_pmc_sq_wide_g10.txt", "## k20p6", "ec_encode_v16<6, EncPol<10, 2, 2, 2>, 3>", 20, 6, 4 << 20,
     64, True, "r04_k20p6_encode_g10_kernel_steady.csv"),
]


def rates():
    """Chip-wide wave-instructions per CU per ns at 4 waves per SIMD."""
    r = {}
    for line in open(P("r03", "r03_valu_probe.jsonl")):
        d = json.loads(line)
        if d.get("waves_per_simd") == 4:
            r[d["op"]] = d["wave_instr_per_cu_ns"]
    others = ["v_bitop3_b32", "v_and_b32", "v_lshrrev_b32", "v_xor_b32", "v_add_u32"]
    other = len(others) / sum(1.0 / r[o] for o in others)  # harmonic mean: equal counts of each
    return r["v_perm_b32"], other


def valu_count(fname, header, kernel):
    lines = open(P(fname)).read().splitlines()
    i = 0
    if header:
        i = next(n for n, l in enumerate(lines) if l.startswith(header))
    j = next(n for n in range(i, len(lines)) if lines[n].strip() == "void " + kernel or lines[n].strip() == kernel)
    for l in lines[j + 1:j + 12]:
        m = re.match(r"\s+SQ_INSTS_VALU\s+([0-9.e+]+)", l)
        if m:
            return float(m.group(1))
    raise SystemExit(f"no SQ_INSTS_VALU for {kernel} in {fname}")


def steady(fname):
    kv = {}
    for l in open(P(fname)):
        if "," in l and not l.startswith("#"):
            a, b = l.rstrip("\n").split(",", 1)
            kv[a] = b
    return float(kv["avg_ns"]), int(kv["bytes_per_launch"])


def main():
    perm_rate, other_rate = rates()
    print(f"# VALU model, tools/valu_model.py; rates (wave-instr per CU per ns, 4 waves/SIMD, "
          f"profiles/r03/r03_valu_probe.jsonl): v_perm_b32 {perm_rate:.3f}, others {other_rate:.3f} "
          f"(harmonic mean of v_bitop3/v_and/v_lshrrev/v_xor/v_add)")
    print("shape,valu_per_launch,src_dwords_per_cu,valu_per_src_dword,perm_per_src_dword,"
          "valu_ms,hbm_ms_at_copy_ceiling,measured_ms,valu_busy,frac_of_8TBs,frac_of_copy_ceiling")
    for label, f, hdr, kern, k, p, n, s, xor, st in SHAPES:
        v = valu_count(f, hdr, kern)
        ns, nbytes = steady(st)
        src_dwords = k * n * s / 256.0  # one wave-instruction covers 64 lanes x 4 B of a source
        per = v / src_dwords
        looked = (p - 1) * (k - 1) if xor else p * k
        perm = 3.0 * looked / k
        per_cu = src_dwords / CUS
        valu_ns = per_cu * (perm / perm_rate + max(per - perm, 0.0) / other_rate)
        hbm_ns = nbytes / COPY_CEILING * 1e9
        print(f"{label},{v:.4g},{per_cu:.4g},{per:.2f},{perm:.2f},{valu_ns / 1e6:.3f},{hbm_ns / 1e6:.3f},"
              f"{ns / 1e6:.3f},{valu_ns / ns:.2f},{nbytes / ns / 8000.0:.4f},{hbm_ns / ns:.3f}")


if __name__ == "__main__":
    sys.exit(main())
