#!/usr/bin/env bash
# GPU box: full parity suite, bench line, N=2 rehearsal (gloo, two ranks on one GPU), the other
# configs, per-step symbol latency, rocprof kernel stats + PMC traffic. Usage: bash tools/gpu_round.sh <tag>
set -euo pipefail
TAG=${1:-r2}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG}.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > gpurun_out/bench2_${TAG}.json 2> gpurun_out/bench2_${TAG}.err
cat gpurun_out/bench2_${TAG}.json
timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err
cat gpurun_out/configs_${TAG}.jsonl
timeout -k 10 200 python3 tools/bench_step_symbols.py > gpurun_out/steps_${TAG}.json 2> gpurun_out/steps_${TAG}.err
cat gpurun_out/steps_${TAG}.json
timeout -k 10 200 python3 tools/bench_cliff.py > gpurun_out/cliff_${TAG}.jsonl 2> gpurun_out/cliff_${TAG}.err
cat gpurun_out/cliff_${TAG}.jsonl
bash tools/profile_gpu.sh "$TAG"
bash tools/profile_long.sh "$TAG"
