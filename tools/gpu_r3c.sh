#!/usr/bin/env bash
# GPU box: fused-decode parity (both orderings) + ordering A/B; then the streaming kernel's
# per-role cycle table under a set of timing experiments (make lib-exp).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused_decode.py tests/test_gpu_decode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3c.log 2>&1 || { tail -60 gpurun_out/pytest_r3c.log; exit 1; }
tail -3 gpurun_out/pytest_r3c.log
timeout -k 10 300 python3 tools/ab_decode_select.py > gpurun_out/ab_select_r3c.jsonl 2> gpurun_out/ab_select_r3c.err
cat gpurun_out/ab_select_r3c.jsonl
bash tools/gpu_exp_diag.sh 0 8 1024 1032 32 1064 2048 2056 3080
