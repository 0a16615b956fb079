#!/usr/bin/env bash
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ring_depth or config2 or lds_edge" > gpurun_out/pytest_r3i.log 2>&1 || { tail -40 gpurun_out/pytest_r3i.log; exit 1; }
tail -2 gpurun_out/pytest_r3i.log
timeout -k 10 200 python3 tools/ab_ring3.py 256 200 80 > gpurun_out/ab_ring_r3i.jsonl 2> gpurun_out/ab_ring_r3i.err
timeout -k 10 200 python3 tools/ab_ring3.py 1 200 80 >> gpurun_out/ab_ring_r3i.jsonl 2>> gpurun_out/ab_ring_r3i.err
cat gpurun_out/ab_ring_r3i.jsonl
