#!/usr/bin/env bash
# GPU box: per-step symbols with the step kernel's own completion word (sync mode 3) + their
# timings; segmented kernel with per-utterance descriptors: parity + configs[4] A/B.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fwd_bwd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3s.log 2>&1 || { tail -40 gpurun_out/pytest_r3s.log; exit 1; }
tail -2 gpurun_out/pytest_r3s.log
timeout -k 10 200 python3 tools/ab_long_split.py > gpurun_out/ab_long_r3s.jsonl 2>&1 || { cat gpurun_out/ab_long_r3s.jsonl; exit 1; }
cat gpurun_out/ab_long_r3s.jsonl
timeout -k 10 300 python3 tools/bench_step_symbols.py > gpurun_out/steps_r3s.json 2> gpurun_out/steps_r3s.err
cat gpurun_out/steps_r3s.json
