#!/usr/bin/env bash
# GPU box: long-row kernel parity, configs timing, rocprof stats + PMC traffic of configs[4].
set -euo pipefail
TAG=${1:-r2w}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_${TAG}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wide_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_wide_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_wide_${TAG}.log
timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err
cat gpurun_out/configs_${TAG}.jsonl
O=gpurun_out/prof_${TAG}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/run_long.py 5 > $O/kt.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt2 -o kt -- python3 tools/run_long.py 5 2 > $O/kt2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 tools/run_long.py 2 > $O/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 tools/run_long.py 2 > $O/write.log 2>&1
cut -d, -f1-4 $O/kt/kt_kernel_stats.csv | head -8
