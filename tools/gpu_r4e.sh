#!/usr/bin/env bash
# GPU box (round 4): fused decodes -- parity suites, per-phase diag cycles, configs timings.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4e}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_decode.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
timeout -k 10 120 python3 tools/diag_decode.py > gpurun_out/diag_decode_${TAG}.txt 2>&1 || { tail -5 gpurun_out/diag_decode_${TAG}.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/diag_decode_${TAG}.txt
timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err || { tail -5 gpurun_out/configs_${TAG}.err; exit 1; }
cat gpurun_out/configs_${TAG}.jsonl
