#!/usr/bin/env bash
# GPU box: the full GPU suite, then configs[4] split A/B (per-utterance descriptors in the segmented kernel).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r3u.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r3u.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r3u.log
timeout -k 10 200 python3 tools/ab_long_split.py > gpurun_out/ab_long_r3u.jsonl 2>&1 || { cat gpurun_out/ab_long_r3u.jsonl; exit 1; }
cat gpurun_out/ab_long_r3u.jsonl
