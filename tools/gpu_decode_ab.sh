#!/usr/bin/env bash
# GPU box: fused-decode parity tests, then configs[2] / v2 / tone decode kernel times (rocprof).
# Usage (via gpurun): bash tools/gpu_decode_ab.sh <tag>
set -euo pipefail
TAG=${1:-dec}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dec_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_dec_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_dec_${TAG}.log
cat > gpurun_out/dec_${TAG}.py <<'PY'
import sys, json
sys.path.insert(0, "tools")
import bench_configs as bc
bc.cpu_time = lambda f: 1.0
print(json.dumps(bc.decode_config(256, 200, 80, 4, iters=20)))
print(json.dumps(bc.v2_decode_config(64, 400, 2000, 16, 4, iters=10)))
print(json.dumps(bc.tone_decode_config(64, 400, 5, 4, iters=10)))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec_${TAG} -o kt -- python3 gpurun_out/dec_${TAG}.py > gpurun_out/dec_${TAG}.log 2>&1 || { tail -20 gpurun_out/dec_${TAG}.log; exit 1; }
grep -o '"config": "[^"]*"\|"gpu_us": [0-9.]*' gpurun_out/dec_${TAG}.log | paste - -
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_dec_${TAG}/kt_kernel_stats.csv')):
    if 'fused' in r['Name'] or 'paths' in r['Name']:
        print(r['Name'][:100], r['Calls'], float(r['AverageNs'])/1e3)
"
