#!/usr/bin/env bash
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== product"; timeout -k 10 120 python3 tools/debug_desc.py 5 90 80 2 2>&1 | grep -v amdgpu.ids
echo "== var_desc"; SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/var_desc/libssnt_tts_c.so timeout -k 10 120 python3 tools/debug_desc.py 5 90 80 3 2>&1 | grep -v amdgpu.ids
SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/var_desc/libssnt_tts_c.so timeout -k 10 120 python3 tools/debug_desc.py 256 200 80 2 2>&1 | grep -v amdgpu.ids
