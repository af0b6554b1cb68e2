"""CPU tier: the drop-in boundary — libisal_hip.so loads and exports exactly the
functions include/*.h declare (no compute calls: no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import ecutil

HEADERS = ["erasure_code.h", "gf_vect_mul.h", "isal_api.h", "isal_hip.h", "raid.h", "crc.h", "crc64.h"]

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


def test_extension_api_rejects_bad_arguments_without_gpu(engine):
    """isal_hip.h calls validate before touching the GPU and return ISAL_HIP_EINVAL (-1)."""
    L = engine.lib()
    h = ctypes.c_void_p()
    u8p = ctypes.POINTER(ctypes.c_ubyte)
    tbl = (ctypes.c_ubyte * 64)()
    ptrs = (u8p * 4)()
    ok_args = dict(len_=64, k=2, rows=2, n=1)
    cases = [(-1, 2, 2, 1), (64, 2, 0, 1), (64, 2, 2, 0), (64, -1, 2, 1)]
    for len_, k, rows, n in cases:
        assert L.isal_hip_batch_create(ctypes.byref(h), len_, k, rows, tbl, n, ptrs, ptrs) == -1
    assert L.isal_hip_batch_create(None, 64, 2, 2, tbl, 1, ptrs, ptrs) == -1
    assert L.isal_hip_batch_create(ctypes.byref(h), 64, 2, 2, None, 1, ptrs, ptrs) == -1
    assert L.isal_hip_batch_encode(None, None) == -1
    assert L.isal_hip_batch_update(None, 0, None) == -1
    assert L.isal_hip_batch_destroy(None) == 0
    for name in ("isal_hip_batch_crc64", "isal_hip_batch_encode_crc64"):
        fn = getattr(L, name)
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_ulonglong, ctypes.c_void_p, ctypes.c_void_p]
        assert fn(None, 0, 0, None, None) == -1  # no batch
    for name in ("isal_hip_batch_encode_crc", "isal_hip_batch_crc"):
        fn = getattr(L, name)
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
        assert fn(None, 0, None, None) == -1
    f = L.isal_hip_pipe_create
    f.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    assert f(ctypes.byref(h), 64, 2, 2, ctypes.cast(tbl, ctypes.c_void_p), 3, 7) == -1  # bad mode
    assert f(ctypes.byref(h), 0, 2, 2, ctypes.cast(tbl, ctypes.c_void_p), 3, 0) == -1
    assert f(ctypes.byref(h), 64, 2, 2, ctypes.cast(tbl, ctypes.c_void_p), 0, 0) == -1
    assert L.isal_hip_pipe_flush(None) == -1
    assert L.isal_hip_pipe_destroy(None) == 0
    del ok_args


def test_raid_argument_contracts_without_gpu(engine):
    """raid.h return codes that need no data pass (reference raid_base.c / pq_gen_avx512.asm)."""
    L = engine.lib()
    arr = (ctypes.c_void_p * 4)()
    for name in ("xor_gen", "xor_gen_base"):
        assert getattr(L, name)(2, 64, arr) == 1  # vects < 3
    for name in ("pq_gen", "pq_gen_base", "pq_check", "pq_check_base"):
        assert getattr(L, name)(3, 64, arr) == 1  # vects < 4
    for name in ("xor_check", "xor_check_base"):
        assert getattr(L, name)(1, 64, arr) == 1  # vects < 2
    assert L.pq_gen(4, 33, arr) == 1  # len % 32 on the dispatched path
    assert L.pq_gen(4, 0, arr) == 0


def test_numa_lookup_against_a_faked_sysfs(engine, tmp_path):
    """isal_hip_multi pins each device's worker to its NUMA node's CPUs; the
    lookup (PCI bus id -> numa_node -> cpulist) checked against a fake tree."""
    root = tmp_path / "sys"
    dev = root / "bus" / "pci" / "devices" / "0000:c5:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    none = root / "bus" / "pci" / "devices" / "0000:05:00.0"
    none.mkdir(parents=True)
    (none / "numa_node").write_text("-1\n")
    for n, lst in ((0, "0-3,8-11\n"), (1, "4-7,12,14-15\n")):
        d = root / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(lst)
    r = str(root)
    # bus ids come from hipDeviceGetPCIBusId in upper case; sysfs is lower case
    assert engine.pci_numa_node("0000:C5:00.0", r) == 1
    assert engine.pci_numa_node("0000:05:00.0", r) == -1  # no NUMA affinity reported
    assert engine.pci_numa_node("0000:99:00.0", r) == -1  # no such device
    assert engine.numa_node_cpus(0, r) == [0, 1, 2, 3, 8, 9, 10, 11]
    assert engine.numa_node_cpus(1, r) == [4, 5, 6, 7, 12, 14, 15]
    assert engine.numa_node_cpus(2, r) is None
    (root / "devices" / "system" / "node" / "node2").mkdir()
    (root / "devices" / "system" / "node" / "node2" / "cpulist").write_text("3-1\n")
    assert engine.numa_node_cpus(2, r) is None  # malformed range
    # hostile ranges end at once (CPU numbers beyond CPU_SETSIZE are malformed)
    for bad in ("0-9223372036854775807\n", "5-100000\n", "0-1023,0-1023,0-1023\n", "99999999999999999999\n"):
        (root / "devices" / "system" / "node" / "node2" / "cpulist").write_text(bad)
        assert engine.numa_node_cpus(2, r) is None, bad
    (root / "devices" / "system" / "node" / "node2" / "cpulist").write_text("0-1023\n")
    assert engine.numa_node_cpus(2, r) == list(range(1024))
    # the real tree of this host parses (node 0 exists on every Linux box with NUMA)
    if os.path.exists("/sys/devices/system/node/node0/cpulist"):
        assert engine.numa_node_cpus(0, None)


def test_route_device_choice_with_fabricated_attributes(engine):
    """The drop-in calls' device choice (isal_hip_route_device, isal_hip.h
    "Several GPUs"): the reference API has no device argument
    (erasure_code.h:108-110), so a call runs on the GPU holding its
    device-resident shards. Driven here with fabricated pointer attributes:
    host-only calls, a foreign device, two devices in one call, managed
    memory, page-locked memory of the run device and of another one."""
    PG, DV, MG, PN = engine.MEM_PAGEABLE, engine.MEM_DEVICE, engine.MEM_MANAGED, engine.MEM_PINNED
    rd = engine.route_device
    # host shards only: the caller's current device, nothing in place
    assert rd([PG] * 6, [-1] * 6, 0) == (0, -1, [0] * 6)
    assert rd([PG] * 3, [-1] * 3, 5) == (5, -1, [0] * 3)
    # device shards on a GPU other than the current one: that GPU
    assert rd([DV] * 4 + [PG], [3] * 4 + [-1], 0) == (3, -1, [1, 1, 1, 1, 0])
    assert rd([PG, DV, PG], [-1, 7, -1], 2) == (7, -1, [0, 1, 0])
    # device shards on two GPUs: refused, naming the first shard on the second
    dev, bad, _ = rd([DV, DV, DV, DV], [2, 2, 5, 2], 2)
    assert (dev, bad) == (-2, 2)
    dev, bad, _ = rd([PG, DV, MG, DV], [-1, 1, -1, 0], 0)
    assert (dev, bad) == (-2, 3)
    # managed memory binds no device and is used in place on any
    assert rd([MG, DV, MG], [-1, 4, -1], 1) == (4, -1, [1, 1, 1])
    assert rd([MG, MG], [-1, -1], 6) == (6, -1, [1, 1])
    # page-locked memory: in place only on the GPU it was registered with
    assert rd([PN, DV, PN], [0, 2, 2], 0) == (2, -1, [0, 1, 1])
    assert rd([PN, PN], [1, 0], 0) == (0, -1, [0, 1])
    # the caller's device unknown and no device shard: no device
    assert rd([PG, PN], [-1, 0], -1) == (-1, -1, [0, 0])
    # no shards; bad arguments
    assert rd([], [], 3)[0] == 3
    L = engine.lib()
    assert L.isal_hip_route_device(-1, None, None, 0, None, None) == -3
    assert L.isal_hip_route_device(2, None, None, 0, None, None) == -3
    # a 64-shard stripe spread over 8 GPUs: the first foreign shard is reported
    kinds, devs = [DV] * 64, [i // 8 for i in range(64)]
    assert rd(kinds, devs, 0)[:2] == (-2, 8)

