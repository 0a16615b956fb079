#!/usr/bin/env bash
# GPU box: ring-tag check of the diagnostic build + the host-symbol zero-copy stress test.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -k "ring_tags" tests/test_gpu_decode.py::test_host_symbols_zero_copy_stress -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r4h.log 2>&1 || { tail -40 gpurun_out/pytest_r4h.log; exit 1; }
tail -5 gpurun_out/pytest_r4h.log
