#!/usr/bin/env bash
# GPU box (round 4 final): the round check (tools/gpu_r4z.sh: GPU suite, smoke, bench, rocprof
# kernel stats + PMC passes), then every BASELINE config's timing (tools/bench_configs.py).
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r4x}
bash tools/gpu_r4z.sh "$TAG" || exit 1
timeout -k 10 400 python3 tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err || { tail -5 gpurun_out/configs_${TAG}.err; exit 1; }
cat gpurun_out/configs_${TAG}.jsonl
