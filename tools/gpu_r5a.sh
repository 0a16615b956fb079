#!/usr/bin/env bash
# Round-5 first GPU check: full GPU suite (debug64 tolerance tests included), bench line,
# rocprof kernel stats of the bench. Usage: bash tools/gpu_r5a.sh
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA -k "debug64" > gpurun_out/r5a_debug64.log 2>&1
rc=$?; tail -15 gpurun_out/r5a_debug64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || exit 1
cat gpurun_out/r5a_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5a_prof -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5a_prof.log 2>&1 || exit 1
head -5 gpurun_out/r5a_prof/kt_kernel_stats.csv
