#!/usr/bin/env bash
# GPU-box round check: parity tests, one bench line, the other configs, rocprof kernel stats +
# PMC traffic. Usage (via gpurun): bash tools/gpu_check.sh <tag>
set -euo pipefail
TAG=${1:-r1}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
tail -3 gpurun_out/pytest_gpu_${TAG}.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err
cat gpurun_out/configs_${TAG}.jsonl
bash tools/profile_gpu.sh "$TAG"
