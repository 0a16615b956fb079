#!/usr/bin/env bash
# GPU box: the whole parity suite, the alignment/shape cliff table, per-step symbols.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r3g.log 2>&1 || { tail -60 gpurun_out/pytest_r3g.log; exit 1; }
tail -3 gpurun_out/pytest_r3g.log
timeout -k 10 300 python3 tools/bench_cliff.py > gpurun_out/cliff_r3g.jsonl 2> gpurun_out/cliff_r3g.err
cat gpurun_out/cliff_r3g.jsonl
for sh in "256 200 80" "64 200 80" "16 200 80" "1 200 80" "64 2000 400" "16 2000 400" "1 2000 400"; do
  timeout -k 10 120 python3 tools/time_fwd_bwd.py $sh 5 >> gpurun_out/bscale_r3g.jsonl 2>> gpurun_out/bscale_r3g.err
done
cat gpurun_out/bscale_r3g.jsonl
