"""CPU tier: the built kernel objects, checked without a GPU.

1. Every kernel a host launcher can launch has device code. A HIP object
   holds host-side kernel handles (one per kernel the launchers name) and a
   bundled gfx950 code object; a handle whose kernel is missing from the code
   object is only found when the launch aborts the caller's process
   ("Cannot find Symbol", the r05e abort, DESIGN.md §3 "Kernel registry").
   Here: for every kernel object of the library, the handles' names are a
   subset of the code object's kernel descriptors (*.kd).
2. The LDS-DMA encode (ec_encode_glds) counts its outstanding loads with fixed
   vmcnt waits that assume the ring's global_load_lds DMAs are the only vector
   memory operations in flight (ec_kernels.hip:237-330; the compiler's waitcnt
   pass does not see inline asm). In the disassembly no other vector memory
   instruction may sit between a DMA and the vmcnt(0) that drains them.
"""
import glob
import os
import re
import subprocess

import pytest

import ecutil

LLVM = "/opt/rocm/lib/llvm/bin"
BUILD = os.path.join(ecutil.REPO, "isa-l_amd", "build")
OBJECTS = sorted(glob.glob(os.path.join(BUILD, "*kernels.o")) + glob.glob(os.path.join(BUILD, "crc*_fused_p*.o")))


def _run(*args):
    return subprocess.run(args, check=True, capture_output=True, text=True).stdout


@pytest.fixture(scope="module")
def code_objects(tmp_path_factory):
    if not OBJECTS or not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("kernel objects not built here (make -C isa-l_amd)")
    out = {}
    d = tmp_path_factory.mktemp("co")
    for o in OBJECTS:
        name = os.path.basename(o)[:-2]
        fb, co = d / f"{name}.fatbin", d / f"{name}.co"
        _run(f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", o, str(d / f"{name}.tmp.o"))
        _run(f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
             "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}")
        out[o] = str(co)
    return out


def _host_kernel_handles(obj):
    """Kernel handles of a HIP host object: 8-byte OBJECT symbols in
    .data.rel.ro named like the kernels (their launch stubs are
    __device_stub__<name>)."""
    secs = {}
    for line in _run(f"{LLVM}/llvm-readelf", "-S", "-W", obj).splitlines():
        m = re.match(r"\s*\[\s*(\d+)\]\s+(\S+)", line)
        if m:
            secs[m.group(1)] = m.group(2)
    names = set()
    stubs = 0
    for line in _run(f"{LLVM}/llvm-readelf", "--symbols", "-W", obj).splitlines():
        f = line.split()
        if len(f) < 8:
            continue
        if "__device_stub__" in f[7]:
            stubs += 1
        if f[3] == "OBJECT" and f[2] == "8" and secs.get(f[6]) == ".data.rel.ro" and f[7].startswith("_Z"):
            names.add(f[7])
    return names, stubs


def _device_kernels(co):
    names = set()
    for line in _run(f"{LLVM}/llvm-readelf", "--symbols", "-W", co).splitlines():
        f = line.split()
        if len(f) >= 8 and f[7].endswith(".kd"):
            names.add(f[7][:-3])
    return names


def test_every_launchable_kernel_has_device_code(code_objects):
    total = 0
    for obj, co in code_objects.items():
        host, stubs = _host_kernel_handles(obj)
        dev = _device_kernels(co)
        assert host, f"{obj}: no kernel handles found"
        assert len(host) == stubs, (obj, len(host), stubs)
        missing = sorted(host - dev)
        assert not missing, f"{os.path.basename(obj)}: launchers name kernels with no device code: {missing[:5]}"
        total += len(host)
    assert total > 100, total


VMEM = re.compile(r"\s(global|buffer|flat)_(load|store|atomic)\w*")
INSN = re.compile(r"^\s+(\S+)(.*?)//\s*([0-9A-F]+):")
TARGET = re.compile(r"<[^>+]+\+0x([0-9a-f]+)>")


def _dma_window_violations(asm):
    """Forward may-analysis over the kernel's control-flow graph: a state is
    'a ring DMA may be outstanding'; a global_load_lds sets it, a waitcnt with
    vmcnt(0) clears it. Returns the vector memory instructions reached while it
    is set (the counted waits would then count them too), and the DMA count."""
    ins = []
    for line in asm.splitlines():
        m = INSN.match(line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), line))
    if not ins:
        return [], 0
    base = ins[0][0]
    index = {addr: i for i, (addr, _, _) in enumerate(ins)}
    succ = []
    for i, (addr, op, line) in enumerate(ins):
        nxt = [i + 1] if i + 1 < len(ins) else []
        t = TARGET.search(line)
        tgt = [index[base + int(t.group(1), 16)]] if t and (base + int(t.group(1), 16)) in index else []
        if op == "s_endpgm" or op.startswith("s_setpc"):
            succ.append([])
        elif op == "s_branch":
            succ.append(tgt)
        elif op.startswith("s_cbranch"):
            succ.append(tgt + nxt)
        else:
            succ.append(nxt)
    state = [False] * len(ins)  # DMA may be outstanding on entry
    seen = [False] * len(ins)
    work = [0]
    seen[0] = True
    bad = set()
    while work:
        i = work.pop()
        addr, op, line = ins[i]
        out = state[i]
        if op.startswith("global_load_lds"):
            out = True
        elif op == "s_waitcnt" and re.search(r"vmcnt\(0\)", line):
            out = False
        elif out and VMEM.search(" " + op):
            bad.add(line.strip())
        for j in succ[i]:
            if not seen[j] or (out and not state[j]):
                seen[j] = True
                state[j] = state[j] or out
                work.append(j)
    return sorted(bad), sum(op.startswith("global_load_lds") for _, op, _ in ins)


def test_glds_counted_waits_see_only_the_ring_dmas(code_objects):
    co = next(c for o, c in code_objects.items() if o.endswith("ec_kernels.o"))
    kernels = sorted(k for k in _device_kernels(co) if "ec_encode_glds" in k)
    assert kernels, "no ec_encode_glds kernels in ec_kernels.o"
    for k in kernels:
        asm = _run(f"{LLVM}/llvm-objdump", "-d", f"--disassemble-symbols={k}", co)
        bad, dmas = _dma_window_violations(asm)
        assert dmas >= 4, (k, dmas)
        assert not bad, f"{k}: vector memory ops inside the counted DMA window: {bad[:4]}"


def test_dma_window_analysis_catches_a_stray_load():
    """The analysis itself: a load between a DMA and its vmcnt(0), on one
    branch of two, is reported; the same load after the drain is not."""
    sym = "k"

    def asm(body):
        out, a = [], 0x1000
        for op in body:
            out.append(f"\t{op}  // {a:012X}: 00000000")
            a += 4
        return "\n".join(out)

    ok = asm(["global_load_lds_dwordx4 v1, s[2:3] nt", "s_waitcnt vmcnt(0)",
              "global_load_dwordx4 v[0:3], v1, s[4:5]", "s_endpgm"])
    assert _dma_window_violations(ok)[0] == []
    branchy = asm(["global_load_lds_dwordx4 v1, s[2:3] nt", f"s_cbranch_scc1 1 <{sym}+0x10>",
                   "s_waitcnt vmcnt(0)", "s_branch 0 <k+0x14>", "buffer_load_dword v2, v1, s[4:7], 0 offen",
                   "s_endpgm"])
    bad, dmas = _dma_window_violations(branchy)
    assert dmas == 1 and len(bad) == 1 and "buffer_load_dword" in bad[0], bad


def test_every_kernel_handle_is_in_the_runtime_registry(code_objects, engine):
    """Every launch goes through ISAL_LAUNCH (ec_device.h), so the registry
    isal_hip_selftest_kernels walks on the GPU holds exactly the kernels the
    objects have host handles for (no GPU needed to count them here)."""
    handles = sum(len(_host_kernel_handles(o)[0]) for o in code_objects)
    rc, n = engine.selftest_kernels()
    assert n == handles, (n, handles)
    if rc == -2:  # no GPU in this tier: the runtime was not asked
        return
    assert rc == 0, rc
