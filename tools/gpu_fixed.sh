#!/usr/bin/env bash
# GPU box: graph-timed kernel time of each fixed-mask library (tools/build_fixed.sh).
# Usage: bash tools/gpu_fixed.sh <tag> "B T U" mask1 mask2 ...
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; SHAPE=$2; shift 2
for m in "$@"; do
  SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/fix$m/libssnt_tts_c.so timeout -k 10 60 python3 tools/ab_exp_graph.py $SHAPE $m | tee -a gpurun_out/fixed_$TAG.jsonl
done
