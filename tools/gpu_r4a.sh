#!/usr/bin/env bash
# GPU box (round 4, first call): the store-data hazard study -- the product, the
# per-utterance-descriptor streaming kernel as reverted in round 3 (var_desc) and the same kernel
# with the two wait states after each wide store (var_desc_nop), grad pre-filled with NaN and
# compared with the oracle; then the chain-step micro-benchmarks.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/ssnt-tts-rust_amd/lib
for v in product var_desc var_desc_nop; do
  lib=$L/libssnt_tts_c.so; [ $v != product ] && lib=$L/$v/libssnt_tts_c.so
  echo "== $v B=5 T=90 U=80"
  SSNT_TTS_C_LIB=$lib timeout -k 10 120 python3 tools/debug_desc.py 5 90 80 4 2>&1 | grep -v amdgpu.ids | grep "^rep" || exit 1
  echo "== $v B=256 T=200 U=80"
  SSNT_TTS_C_LIB=$lib timeout -k 10 120 python3 tools/debug_desc.py 256 200 80 3 2>&1 | grep -v amdgpu.ids | grep "^rep" || exit 1
done
echo "== micro_step"; timeout -k 10 120 tools/micro/bin/micro_step || exit 1
echo "== micro_batch"; timeout -k 10 120 tools/micro/bin/micro_batch || exit 1
