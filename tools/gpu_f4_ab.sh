#!/usr/bin/env bash
# GPU box: configs[4] F4 (v2 duration fwd-bwd) kernel times of the product library and each
# named var_* build, alternating, same box (rocprof kernel stats). Tuning study only.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
cat > gpurun_out/f4_ab.py <<'PY'
import sys, json
sys.path.insert(0, "tools")
import bench_configs as bc
bc.cpu_time = lambda f: 1.0
print(json.dumps(bc.v2_fwd_bwd_config(64, 400, 2000, 16, iters=10)))
PY
for n in prod "$@" prod "$@"; do
  if [ $n = prod ]; then unset SSNT_TTS_C_LIB; else export SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/var_$n/libssnt_tts_c.so; fi
  rm -rf gpurun_out/prof_f4_$n
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f4_$n -o kt -- python3 gpurun_out/f4_ab.py > gpurun_out/f4_ab_$n.log 2>&1 || { tail -20 gpurun_out/f4_ab_$n.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_f4_$n/kt_kernel_stats.csv')):
    if 'f4' in r['Name']:
        print('$n', r['Name'][30:70], r['Calls'], round(float(r['AverageNs'])/1e3, 2))
"
done
