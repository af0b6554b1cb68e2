#!/bin/bash
# r06n: full GPU suite with the LDS product tables for 7-8 row passes, smoke, default bench line.
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 600 $O/bench.json
