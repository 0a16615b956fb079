#!/usr/bin/env bash
# GPU box: headline bench (kernel time) + the full-size parity test for each built variant
# (tools/build_variants.sh). Tuning study only.
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in ssnt-tts-rust_amd/lib/var_*/; do
  n=$(basename $d)
  export SSNT_TTS_C_LIB=$PWD/$d/libssnt_tts_c.so
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/v_$n.json 2>gpurun_out/v_$n.err || { echo "$n bench failed"; tail -3 gpurun_out/v_$n.err; exit 1; }
  timeout -k 10 200 python3 -m pytest tests/test_gpu_fwd_bwd.py -q -x -k "config2_full and default" --timeout 150 > gpurun_out/vt_$n.log 2>&1; rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/v_$n.json')); print('$n', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), 'parity rc=$rc')"
  [ $rc -eq 0 ] || exit 1
done
