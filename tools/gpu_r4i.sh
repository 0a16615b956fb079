#!/usr/bin/env bash
# GPU box (round 4): fused-decode parity suites at the working tree, then configs[4] v2 / tone
# timings of the working tree against the named var_* builds (tools/gpu_decode_var.sh).
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4i}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_decode.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
timeout -k 10 600 bash tools/gpu_decode_var.sh "$@" > gpurun_out/ab_${TAG}.txt 2>&1 || { tail -5 gpurun_out/ab_${TAG}.txt; exit 1; }
cat gpurun_out/ab_${TAG}.txt
