#!/usr/bin/env bash
# GPU box: segmented kernel, one vs two workgroups per direction across U (feasible lattices).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for shp in "64 1100 1024" "64 760 700" "64 520 500" "64 400 300" "128 1100 1024" "32 2000 400"; do
  timeout -k 10 200 python3 tools/ab_long_split.py $shp 1 2>&1 | grep -v amdgpu.ids | head -2
done
