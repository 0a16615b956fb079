#!/usr/bin/env bash
# GPU-box tuning sweep (via gpurun): fwd-bwd parity, per-wave diag of each wave mix, in-process A/B.
# Usage: bash tools/gpu_mix_sweep.sh "0 5"   (variants; default all)
set -o pipefail
VARS=${1:-"0 2 3 4 5 6"}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fb.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_fb.log; [ $rc -eq 0 ] || exit $rc
for v in $VARS; do
  SSNT_DIAG_LIB=diag SSNT_VARIANT=$v timeout -k 10 120 python3 tools/diag_fwd_bwd.py > gpurun_out/diag_v$v.log 2>&1 || exit 1
done
timeout -k 10 200 python3 - "$VARS" > gpurun_out/ab.log 2>&1 <<'PY' || exit 1
import sys, json
sys.path.insert(0, "tools")
from ab_fwd_bwd import bench_shape
print(json.dumps(bench_shape(256, 200, 80, variants=tuple(int(v) for v in sys.argv[1].split()), rounds=5)))
PY
cat gpurun_out/ab.log
