#!/usr/bin/env bash
# GPU box: streaming kernel with per-utterance descriptors -- fwd-bwd parity, configs[1] A/B vs
# the previous streaming kernel (same other objects), configs[4] after the split default change.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fwd_bwd.py tests/test_gpu_pair.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3t.log 2>&1 || { tail -40 gpurun_out/pytest_r3t.log; exit 1; }
tail -2 gpurun_out/pytest_r3t.log
timeout -k 10 300 python3 tools/ab_libs.py 256 200 80 20 6 product ssnt-tts-rust_amd/lib/var_oldstream/libssnt_tts_c.so > gpurun_out/ab_stream_r3t.jsonl 2>&1 || { cat gpurun_out/ab_stream_r3t.jsonl; exit 1; }
cat gpurun_out/ab_stream_r3t.jsonl
