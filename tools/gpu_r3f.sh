#!/usr/bin/env bash
# GPU box: per-step symbol latency (completion modes), then the long-form wide-kernel depth A/B.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab_libs.py 64 2000 400 3 4 product ssnt-tts-rust_amd/lib/var_w32_16/libssnt_tts_c.so ssnt-tts-rust_amd/lib/var_w24_24/libssnt_tts_c.so > gpurun_out/ab_wide_r3f.jsonl 2> gpurun_out/ab_wide_r3f.err
cat gpurun_out/ab_wide_r3f.jsonl
