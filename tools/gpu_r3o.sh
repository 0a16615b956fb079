#!/usr/bin/env bash
# GPU box: configs[4] segmented-kernel prefetch-depth A/B (product vs 32-row phase 1 / both phases), split on/off.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=ssnt-tts-rust_amd/lib
for v in product var_wd32a var_wd32; do
  if [ "$v" = product ]; then unset SSNT_TTS_C_LIB; else export SSNT_TTS_C_LIB=$PWD/$L/$v/libssnt_tts_c.so; fi
  echo "== $v"
  timeout -k 10 200 python3 tools/ab_long_split.py 2>&1 | grep -v amdgpu.ids
done
