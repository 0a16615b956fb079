#!/usr/bin/env bash
# GPU box (round 4): F4 sweep with padded row buffers -- parity suite, then configs[4] F4 kernel
# stats (rocprof) of the product library.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4d}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_v2_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
cat > gpurun_out/f4_once.py <<'PY'
import sys, json
sys.path.insert(0, "tools")
import bench_configs as bc
bc.cpu_time = lambda fn, min_s=0: 1.0
print(json.dumps(bc.v2_fwd_bwd_config(64, 400, 2000, 16, iters=10)))
PY
rm -rf gpurun_out/prof_f4_${TAG}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f4_${TAG} -o kt -- python3 gpurun_out/f4_once.py > gpurun_out/f4_${TAG}.log 2>&1 || { tail -20 gpurun_out/f4_${TAG}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/f4_${TAG}.log | tail -1
python3 - "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_f4_{sys.argv[1]}/**/kt_kernel_stats.csv", recursive=True) + glob.glob(f"gpurun_out/prof_f4_{sys.argv[1]}/kt_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    if "f4" in r["Name"]:
        print(r["Name"][30:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
