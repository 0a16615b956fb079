#!/usr/bin/env bash
# GPU box (round 4 close): the full GPU suite, smoke, the bench line, then the bench under
# rocprofv3 (kernel stats + FETCH_SIZE / WRITE_SIZE passes) for profiles/.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4z}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -5 gpurun_out/smoke_${TAG}.log; exit 1; }
grep -v amdgpu.ids gpurun_out/smoke_${TAG}.log | tail -2
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -5 gpurun_out/bench_${TAG}.err; exit 1; }
tail -1 gpurun_out/bench_${TAG}.json
bash tools/profile_gpu.sh ${TAG} > gpurun_out/profile_${TAG}.log 2>&1 || { tail -5 gpurun_out/profile_${TAG}.log; exit 1; }
tail -3 gpurun_out/profile_${TAG}.log
