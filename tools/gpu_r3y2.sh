#!/usr/bin/env bash
# GPU box: headline A/B of the chains' spin behaviour (priority drop / sleep while waiting).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=ssnt-tts-rust_amd/lib
timeout -k 10 500 python3 tools/ab_libs.py 256 200 80 20 6 product $L/var_y1/libssnt_tts_c.so $L/var_y2/libssnt_tts_c.so $L/var_y3/libssnt_tts_c.so > gpurun_out/ab_yield.jsonl 2>&1 || { cat gpurun_out/ab_yield.jsonl; exit 1; }
cat gpurun_out/ab_yield.jsonl
