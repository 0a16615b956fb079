#!/usr/bin/env bash
# GPU box: headline A/B of the gradient waves' pre-cut poll interval (s_sleep 1 / 4 / 12).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab_libs.py 256 200 80 20 6 product ssnt-tts-rust_amd/lib/var_nap4/libssnt_tts_c.so ssnt-tts-rust_amd/lib/var_nap12/libssnt_tts_c.so > gpurun_out/ab_nap_r3x.jsonl 2>&1 || { cat gpurun_out/ab_nap_r3x.jsonl; exit 1; }
cat gpurun_out/ab_nap_r3x.jsonl
