#!/usr/bin/env bash
# GPU box: decode + reference-symbol parity, decode ordering A/B, decode phase cycles (diag),
# per-step symbol latency with the three completion modes.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused_decode.py tests/test_gpu_decode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1 || { tail -60 gpurun_out/pytest_r3e.log; exit 1; }
tail -3 gpurun_out/pytest_r3e.log
timeout -k 10 300 python3 tools/ab_decode_select.py > gpurun_out/ab_select_r3e.jsonl 2> gpurun_out/ab_select_r3e.err
cat gpurun_out/ab_select_r3e.jsonl
timeout -k 10 300 python3 tools/bench_step_symbols.py > gpurun_out/steps_r3e.json 2> gpurun_out/steps_r3e.err
cat gpurun_out/steps_r3e.json
