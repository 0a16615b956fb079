#!/usr/bin/env bash
# GPU box: configs[4] segmented kernel after the vmcnt-pad fix: product vs 32-row phase 1, split on/off.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=ssnt-tts-rust_amd/lib
for v in product var_n32a; do
  if [ "$v" = product ]; then unset SSNT_TTS_C_LIB; else export SSNT_TTS_C_LIB=$PWD/$L/$v/libssnt_tts_c.so; fi
  echo "== $v"
  timeout -k 10 200 python3 tools/ab_long_split.py 2>&1 | grep -v amdgpu.ids
done
unset SSNT_TTS_C_LIB
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 200 --timeout-method thread -k "wide or config5 or beyond_512 or workspace or config4" 2>&1 | tail -3
