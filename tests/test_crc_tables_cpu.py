"""CPU tier: the CRC kernels' chain algebra on the engine's own host tables.

tests/host_tables/*.c include the table builders (isa-l_amd/csrc/crc64_host.c,
crc_host.c) and emulate every lane of one block exactly as the kernels chain
(crc64_kernels.hip: slicing-by-8 pre-shifted chains in the byte-swapped
u-domain and the checksum-only kernel's field tables; crc_kernels.hip:
byte-position P / P' and field F / F' tables), join the lanes and compare with
the bit-serial / bytewise CRC of the block — all eight crc64.h flavours and
crc32_iscsi. The GPU tests check the kernels themselves against the oracle;
this pins the host-side tables without a GPU.
"""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host_tables")
CSRC = os.path.join(os.path.dirname(HERE), os.pardir, "isa-l_amd", "csrc")


@pytest.mark.parametrize("src", ["crc64_chain_check.c", "crc32c_chain_check.c"])
def test_crc_chain_algebra(tmp_path, src):
    exe = tmp_path / src.replace(".c", "")
    r = subprocess.run(["gcc", "-O2", "-Wall", "-I", CSRC, "-o", str(exe), os.path.join(HERE, src),
                        "-lpthread"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
