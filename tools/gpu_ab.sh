#!/usr/bin/env bash
# GPU-box A/B (via gpurun): kernel variants at config 2, plain and with the fused loss sum.
# Usage: bash tools/gpu_ab.sh "0 7"
set -o pipefail
VARS=${1:-"0 7"}
mkdir -p gpurun_out
timeout -k 10 300 python3 - "$VARS" > gpurun_out/ab.log 2>&1 <<'PY' || exit 1
import sys, json
sys.path.insert(0, "tools")
from ab_fwd_bwd import bench_shape
v = tuple(int(x) for x in sys.argv[1].split())
print("plain", json.dumps(bench_shape(256, 200, 80, variants=v, rounds=5)))
print("sum  ", json.dumps(bench_shape(256, 200, 80, variants=v, rounds=5, use_sum=True)))
PY
cat gpurun_out/ab.log
