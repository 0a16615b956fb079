#!/usr/bin/env bash
# GPU box: the parity suite, one bench line, kernel stats + PMC traffic of the bench.
# Usage: bash tools/gpu_check3.sh <tag>
set -euo pipefail
TAG=${1:-r3}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_${TAG}.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
bash tools/profile_gpu.sh "$TAG"
