"""CPU tier: the engine's host code under AddressSanitizer + UBSan (SURVEY.md
§5; the reference runs UBSan over its tests, tools/test_checks.sh:47).

  * tests/sanitize/abi_edges.c — every host path of the C ABI with edge
    arguments, checked against the oracle;
  * the reference's own EC / RAID test programs, compiled with the sanitizers
    and linked against the sanitized engine (isa-l_amd/lib/asan/).
Both run on the CPU route (no GPU in this tier). Leak checking is on for
abi_edges; the reference's test programs do not free their own buffers (e.g.
gf_vect_mul_base_test.c:55-57), so for them it is off.
"""
import os
import subprocess

import pytest

import ecutil
from test_cpu_route import CONFORMANCE, run_programs

SAN_ENV = dict(os.environ, ISAL_HIP_BACKEND="cpu",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
ASAN_BUILD = os.path.join(ecutil.ENGINE_DIR, "build", "asan")


@pytest.fixture(scope="module")
def sanitized_builds():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ecutil.REPO, "tests", "sanitize")],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    if os.path.isdir("/root/reference/erasure_code"):
        r = subprocess.run(["make", "-s", "-C", ecutil.ORACLE_DIR, "conformance_asan", "-j8"],
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-3000:]


def test_abi_edges_under_asan_ubsan(sanitized_builds):
    r = subprocess.run([os.path.join(ASAN_BUILD, "abi_edges")], capture_output=True, text=True,
                       timeout=600, env=SAN_ENV)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "abi_edges: Pass" in r.stdout


def test_reference_test_programs_under_asan_ubsan(sanitized_builds):
    env = dict(SAN_ENV, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    res = run_programs(os.path.join(ecutil.REF_DIR, "conformance_asan"), CONFORMANCE, env)
    if all(v is None for v in res.values()):
        pytest.skip("not built (make -C oracle conformance_asan needs /root/reference)")
    for name, v in res.items():
        assert v is not None, f"{name} not built"
        rc, out = v
        assert rc == 0 and "pass" in out.lower(), (name, out)
