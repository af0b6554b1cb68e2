#!/bin/bash
# r06b: checksum entry points on device buffers, crc64_funcs_test (gpu/auto), mailbox slow branch.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "crc_entry or crc64_device_buffer or slow_stream or crc64_funcs or selftest or one_context or visible_to_other or failure_aborts" \
  > $O/pytest.txt 2>&1 || { tail -80 $O/pytest.txt; exit 1; }
tail -15 $O/pytest.txt
