#!/usr/bin/env bash
# GPU box: F4 with the transposed class butterfly -- parity, configs[4] timing + kernel stats.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_f4_r3w
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_v2_fwd_bwd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_f4_r3w.log 2>&1 || { tail -40 gpurun_out/pytest_f4_r3w.log; exit 1; }
tail -2 gpurun_out/pytest_f4_r3w.log
timeout -k 10 200 python3 tools/f4_run_once.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f4_r3w -o kt -- python3 tools/f4_run_once.py > gpurun_out/prof_f4_r3w/kt.log 2>&1
cat gpurun_out/prof_f4_r3w/kt_kernel_stats.csv | cut -c1-200
