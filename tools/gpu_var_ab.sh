#!/usr/bin/env bash
# GPU box: for each named var_* tuning build, the headline bench (kernel time) and the full-size
# parity test; names prefixed "d" are diag builds and print their per-role cycle table instead.
# Tuning study only. Usage: bash tools/gpu_var_ab.sh base r2 dr2
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in "$@"; do
  d=ssnt-tts-rust_amd/lib/var_$n
  if [[ $n == d* ]]; then
    SSNT_DIAG_LIB=var_$n timeout -k 10 120 python3 tools/diag_fwd_bwd.py > gpurun_out/diag_$n.txt 2>&1 || { echo "diag $n failed"; tail -5 gpurun_out/diag_$n.txt; exit 1; }
    echo "== $n"; grep -v amdgpu.ids gpurun_out/diag_$n.txt
    continue
  fi
  export SSNT_TTS_C_LIB=$PWD/$d/libssnt_tts_c.so
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/v_$n.json 2>gpurun_out/v_$n.err || { echo "$n bench failed"; tail -3 gpurun_out/v_$n.err; exit 1; }
  timeout -k 10 200 python3 -m pytest tests/test_gpu_fwd_bwd.py -q -x -k "config2_full and default" --timeout 150 > gpurun_out/vt_$n.log 2>&1; rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/v_$n.json')); print('$n', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), 'parity rc=$rc')"
  [ $rc -eq 0 ] || exit 1
  unset SSNT_TTS_C_LIB
done
