#!/usr/bin/env bash
# GPU box: segmented-kernel parity (split + one-workgroup forms), configs[4] split A/B, long profile.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 200 --timeout-method thread -k "wide or config5 or beyond_512 or workspace or loss_sum or config4" > gpurun_out/pytest_wide_r3n.log 2>&1 || { tail -60 gpurun_out/pytest_wide_r3n.log; exit 1; }
tail -3 gpurun_out/pytest_wide_r3n.log
timeout -k 10 200 python3 tools/ab_long_split.py > gpurun_out/ab_long_split_r3n.jsonl 2>&1 || { cat gpurun_out/ab_long_split_r3n.jsonl; exit 1; }
cat gpurun_out/ab_long_split_r3n.jsonl
bash tools/profile_long.sh r3n
