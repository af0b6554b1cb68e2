#!/bin/bash
# r06ad: randomized batch-encode shapes against the oracle (new test).
set -o pipefail
O=gpurun_out/r06ad; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "random_shapes" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -6 $O/pytest.txt
