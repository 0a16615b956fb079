#!/usr/bin/env bash
# GPU box (round 4): F4 parity suite at the working tree, then F4 kernel times of the working
# tree against the named var_* builds (tools/gpu_f4_ab.sh).
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4q}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_v2_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
timeout -k 10 900 bash tools/gpu_f4_ab.sh "$@" > gpurun_out/ab_${TAG}.txt 2>&1 || { tail -5 gpurun_out/ab_${TAG}.txt; exit 1; }
cat gpurun_out/ab_${TAG}.txt
