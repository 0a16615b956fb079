#!/usr/bin/env bash
# GPU box: the experiment build (make lib-exp) of the streaming kernel under a matrix of SSNT_EXP
# knobs, with per-role cycle totals (tools/diag_fwd_bwd.py). Timing study only.
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for e in "$@"; do
  SSNT_DIAG_LIB=exp SSNT_EXP=$e timeout -k 10 120 python3 tools/diag_fwd_bwd.py > gpurun_out/exp_$e.txt 2>&1 || { cat gpurun_out/exp_$e.txt; exit 1; }
  cat gpurun_out/exp_$e.txt
done
