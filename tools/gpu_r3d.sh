#!/usr/bin/env bash
# GPU box: fused-decode phase cycles (diag build) and the per-step symbol latency breakdown.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/diag_decode.py > gpurun_out/diag_decode_r3d.jsonl 2> gpurun_out/diag_decode_r3d.err
cat gpurun_out/diag_decode_r3d.jsonl
timeout -k 10 300 python3 tools/bench_step_symbols.py > gpurun_out/steps_r3d.json 2> gpurun_out/steps_r3d.err
cat gpurun_out/steps_r3d.json
