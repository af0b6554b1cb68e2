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


# ---------------------------------------------------------------------------
# libFuzzer (the reference fuzzes init / encode / dot_prod / mad with
# len in [0, 16384], tests/fuzz/ec_fuzz_test.c). Three targets, each bounded:
#   ec_fuzz_test, raid_fuzz_test  the reference's own harnesses, unmodified,
#                                 linked against the engine (crash / ASan /
#                                 UBSan / leak oracle);
#   ec_diff_fuzz                  tests/fuzz/ec_diff_fuzz.c: every input through
#                                 the engine and the oracle, outputs compared.
# ---------------------------------------------------------------------------

FUZZ_DIR = os.path.join(ecutil.ENGINE_DIR, "build", "fuzz")
FUZZ_SECONDS = int(os.environ.get("ISAL_FUZZ_SECONDS", "20"))
# report_globals=0: this toolchain's static link registers some TUs' globals
# twice (a false odr-violation at start-up); heap, stack and UB checks stay on
FUZZ_ENV = dict(os.environ, ISAL_HIP_BACKEND="cpu", ASAN_OPTIONS="report_globals=0:detect_leaks=1",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def fuzz_builds():
    targets = ["all"] + (["ref"] if os.path.isdir("/root/reference/tests/fuzz") else [])
    r = subprocess.run(["make", "-s", "-C", os.path.join(ecutil.REPO, "tests", "fuzz"), "-j8"] + targets,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("target,layout", [("ec_diff_fuzz", "diff"), ("ec_fuzz_test", "ec"),
                                           ("raid_fuzz_test", "raid")])
def test_libfuzzer_targets(fuzz_builds, tmp_path, target, layout):
    import sys

    exe = os.path.join(FUZZ_DIR, target)
    if not os.path.exists(exe):
        pytest.skip(f"{target} not built (the reference's harnesses need /root/reference)")
    corpus = tmp_path / "corpus"
    subprocess.run([sys.executable, os.path.join(ecutil.REPO, "tests", "fuzz", "seeds.py"), layout, str(corpus)],
                   check=True, capture_output=True)
    r = subprocess.run([exe, f"-max_total_time={FUZZ_SECONDS}", "-max_len=300000", "-print_final_stats=1",
                        f"-artifact_prefix={tmp_path}/", str(corpus)],
                       capture_output=True, text=True, timeout=FUZZ_SECONDS + 300, env=FUZZ_ENV, cwd=tmp_path)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    runs = [int(l.split(":")[-1]) for l in out.splitlines() if l.startswith("stat::number_of_executed_units")]
    assert runs and runs[0] >= 200, out[-2000:]  # the seeds alone are ~150-200 inputs
