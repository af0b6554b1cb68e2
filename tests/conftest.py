import os
import sys

import pytest

# Exactly one HIP runtime per process: torch's (see isal_amd._one_hip_runtime).
import torch  # noqa: F401,E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import ecutil  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libisal_hip.so on the GPU)")


@pytest.fixture(scope="session")
def oracle():
    return ecutil.oracle()


@pytest.fixture(scope="session")
def engine():
    """The product library (isa-l_amd/lib/libisal_hip.so) through its Python mirror."""
    ecutil.build_engine()
    import isal_amd

    isal_amd.lib()
    return isal_amd


@pytest.fixture(scope="session")
def gpu():
    """Fails (does not skip) when the GPU is missing: -m gpu runs must not pass vacuously."""
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch.device("cuda:0")


def pytest_runtest_teardown(item):
    """ISAL_TEST_RSS_LOG=<file>: append each test's id, the process's peak RSS
    after it and the current RSS split (anonymous / file-backed / shmem, MiB),
    to find the test that sets the suite's peak and what kind of pages it is."""
    path = os.environ.get("ISAL_TEST_RSS_LOG")
    if path:
        import resource

        cur = {}
        with open("/proc/self/status") as st:
            for line in st:
                if line.startswith(("RssAnon", "RssFile", "RssShmem")):
                    key, val = line.split(":")
                    cur[key] = int(val.split()[0]) // 1024
        with open(path, "a") as f:
            f.write(f"{item.nodeid} {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss // 1024} "
                    + " ".join(f"{k_}={v}" for k_, v in cur.items()) + "\n")


def pytest_terminal_summary(terminalreporter):
    """Peak resident memory of the test process (the GPU tier's full-size
    C2/C3/C4 host arrays are freed after each test; DESIGN §5 records it)."""
    import resource

    kb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    terminalreporter.write_line(f"peak RSS of the test process: {kb / 1024:.0f} MiB")
