#!/usr/bin/env bash
# GPU box (round 4): F4 parity suite against each named var_* build, then F4 kernel times of the
# product against them (tools/gpu_f4_ab.sh). Tuning study only.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4s}
for n in "$@"; do
  SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/var_$n/libssnt_tts_c.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_v2_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_$n.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/pytest_${TAG}_$n.log)"
done
timeout -k 10 900 bash tools/gpu_f4_ab.sh "$@" > gpurun_out/ab_${TAG}.txt 2>&1 || { tail -5 gpurun_out/ab_${TAG}.txt; exit 1; }
cat gpurun_out/ab_${TAG}.txt
