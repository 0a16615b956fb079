#!/usr/bin/env bash
# GPU box: headline A/B of the junk-area layout (consecutive 16-byte junk slots) + its parity.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=ssnt-tts-rust_amd/lib
SSNT_TTS_C_LIB=$PWD/$L/var_junk/libssnt_tts_c.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 200 --timeout-method thread -k "full_lengths or config2 or ragged" > gpurun_out/pytest_junk.log 2>&1 || { tail -30 gpurun_out/pytest_junk.log; exit 1; }
tail -1 gpurun_out/pytest_junk.log
timeout -k 10 400 python3 tools/ab_libs.py 256 200 80 20 8 product $L/var_junk/libssnt_tts_c.so > gpurun_out/ab_junk.jsonl 2>&1 || { cat gpurun_out/ab_junk.jsonl; exit 1; }
cat gpurun_out/ab_junk.jsonl
