#!/usr/bin/env bash
# GPU box: fused-decode parity tests, then the decode part of the configs bench.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_decode.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { tail -40 gpurun_out/pytest_fused.log; exit 1; }
tail -3 gpurun_out/pytest_fused.log
