#!/usr/bin/env bash
# Round 5: segmented kernel, split vs one workgroup per direction across shapes (64-step
# publications), parity of the wide cases first. Usage: bash tools/gpu_r5i.sh TAG
set -uo pipefail
TAG=${1:-r5i}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
SSNT_AB_TESTS=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -k "wide or long or 512 or config5" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/${TAG}_pytest.log | tail -40; exit $rc; }
for shape in "64 2000 400" "32 2000 400" "64 1100 1024" "64 760 700" "64 520 500" "64 400 300" "128 1100 1024" "64 1200 400" "128 2000 400"; do
  timeout -k 10 200 python3 tools/ab_long_modes.py $shape 0 1 2>&1 | grep '"form"' | tee -a gpurun_out/${TAG}_shapes.jsonl || exit 1
done
