#!/usr/bin/env bash
# GPU-box experiment sweep (via gpurun): diag of the experiment build (make lib-exp) under
# SSNT_EXP bit masks. Usage: bash tools/gpu_exp_sweep.sh <variant> "<exp masks>"
set -o pipefail
V=${1:-5}
MASKS=${2:-"0 1 2 4"}
mkdir -p gpurun_out
for m in $MASKS; do
  SSNT_DIAG_LIB=exp SSNT_EXP=$m SSNT_VARIANT=$V timeout -k 10 120 python3 tools/diag_fwd_bwd.py > gpurun_out/exp_v${V}_m$m.log 2>&1 || exit 1
done
