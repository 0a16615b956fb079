#!/usr/bin/env bash
# GPU box: configs[4] v2 / tone and configs[2] v1 fused-decode times of the product library and each named var_*
# build, alternating (the bench_configs timers; CPU baseline skipped). Tuning study only.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in prod "$@" prod "$@"; do
  if [ $n = prod ]; then unset SSNT_TTS_C_LIB; else export SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/var_$n/libssnt_tts_c.so; fi
  timeout -k 10 120 python3 - "$n" <<'PY' 2>&1 | grep -v amdgpu.ids
import json, sys
sys.path.insert(0, "tools")
import bench_configs as bc
bc.cpu_time = lambda fn, min_s=0: 1.0
v2 = bc.v2_decode_config(64, 400, 2000, 16, 4, iters=10)
tone = bc.tone_decode_config(64, 400, 5, 4, iters=10)
v1 = bc.decode_config(256, 200, 80, 4, iters=10)
print(sys.argv[1], "v2", round(v2["gpu_us"], 1), "tone", round(tone["gpu_us"], 1), "v1", round(v1["gpu_us"], 1))
PY
done
