#!/usr/bin/env bash
# GPU box: the fused-decode parity tests (both step orderings), then the ordering A/B.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused_decode.py tests/test_gpu_decode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1 || { tail -60 gpurun_out/pytest_r3b.log; exit 1; }
tail -3 gpurun_out/pytest_r3b.log
timeout -k 10 300 python3 tools/ab_decode_select.py > gpurun_out/ab_select_r3b.jsonl 2> gpurun_out/ab_select_r3b.err
cat gpurun_out/ab_select_r3b.jsonl
