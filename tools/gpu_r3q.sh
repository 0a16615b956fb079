#!/usr/bin/env bash
# GPU box: the round check (tools/gpu_round.sh) plus the chain lane-mask A/B at configs[1].
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_libs.py 256 200 80 20 4 product ssnt-tts-rust_amd/lib/var_mask/libssnt_tts_c.so > gpurun_out/ab_mask_r3q.jsonl 2>&1 || { cat gpurun_out/ab_mask_r3q.jsonl; exit 1; }
cat gpurun_out/ab_mask_r3q.jsonl
bash tools/gpu_round.sh r3m
