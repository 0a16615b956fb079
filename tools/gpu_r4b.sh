#!/usr/bin/env bash
# GPU box (round 4): the rows kernel -- fwd-bwd parity suite, then the bench line and a rocprof
# kernel trace of it. Usage: bash tools/gpu_r4b.sh <tag>
set -uo pipefail
TAG=${1:-r4b}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fb_${TAG}.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_fb_${TAG}.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { cat gpurun_out/bench_${TAG}.err | tail -20; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --variant 13 > gpurun_out/bench_stream_${TAG}.json 2>&1 || exit 1
cat gpurun_out/bench_stream_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}/kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || exit 1
find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1 | xargs cat | head -5
