"""CPU tier: the drop-in boundary — libisal_hip.so loads and exports exactly the
functions include/*.h declare (no compute calls: no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import ecutil

HEADERS = ["erasure_code.h", "gf_vect_mul.h", "isal_api.h", "isal_hip.h", "raid.h"]

# Reference data-path + support symbols the boundary must provide (SURVEY.md §8b,
# reference isa-l.def:5-57,114-124 restricted to erasure coding).
REFERENCE_EC_ABI = {
    "ec_init_tables", "ec_init_tables_base", "ec_encode_data", "ec_encode_data_base",
    "ec_encode_data_update", "ec_encode_data_update_base", "gf_vect_dot_prod",
    "gf_vect_dot_prod_base", "gf_vect_mad", "gf_vect_mad_base", "gf_vect_mul",
    "gf_vect_mul_base", "gf_vect_mul_init", "gf_vect_mul_init_base", "gf_mul", "gf_inv",
    "gf_gen_rs_matrix", "gf_gen_cauchy1_matrix", "gf_invert_matrix", "isal_get_version",
    "isal_get_version_str",
}


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(os.path.join(ecutil.REPO, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\([^;{]*\)\s*;", text, flags=re.M):
            names.add(m.group(1))
    return names


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", ecutil.ENGINE_LIB], check=True,
                         capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_headers_declare_reference_abi():
    assert REFERENCE_EC_ABI <= declared_functions()


def test_library_exports_every_declared_symbol(engine):
    declared = declared_functions()
    exported = exported_symbols()
    missing = declared - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    extra = {s for s in exported - declared if not s.startswith("_")}
    assert not extra, f"exported but undeclared: {sorted(extra)}"


def test_library_loads_via_dlopen_and_resolves(engine):
    L = ctypes.CDLL(ecutil.ENGINE_LIB)
    for name in sorted(declared_functions()):
        assert getattr(L, name) is not None
    f = L.isal_hip_target
    f.restype = ctypes.c_char_p
    assert f() == b"gfx950"


def test_library_is_gfx950_only():
    """The shared object embeds a gfx950 code object and no other GPU target."""
    data = open(ecutil.ENGINE_LIB, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets


def test_library_has_no_oracle_dependency():
    out = subprocess.run(["nm", "-D", ecutil.ENGINE_LIB], check=True, capture_output=True,
                         text=True).stdout
    assert "oracle_" not in out
    ldd = subprocess.run(["ldd", ecutil.ENGINE_LIB], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "isal_ref" not in ldd
