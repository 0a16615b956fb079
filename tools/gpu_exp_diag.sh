#!/usr/bin/env bash
# GPU box: the experiment build's per-role cycle table (tools/diag_fwd_bwd.py) for each SSNT_EXP
# mask given. Timing experiments only (most masks give wrong results).
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for e in "$@"; do
  SSNT_DIAG_LIB=exp SSNT_EXP=$e timeout -k 10 120 python3 tools/diag_fwd_bwd.py > gpurun_out/exp_$e.txt 2>&1 || { echo "exp $e failed"; tail -5 gpurun_out/exp_$e.txt; exit 1; }
  echo "== exp $e"; grep -E "launch|chain|conv f0|grad f0" gpurun_out/exp_$e.txt
done
