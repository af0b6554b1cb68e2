#!/bin/bash
# r06ah: drop-in product tables limited to k <= 12: drop-in / kernel-argument tests (new shapes).
set -o pipefail
O=gpurun_out/r06ah; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dropin or kernel_args or karg or concurrent or selftest" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
