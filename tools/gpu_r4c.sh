#!/usr/bin/env bash
# GPU box: rows kernel vs streaming kernel at configs[1] -- bench lines and per-role diag tables.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4c}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
for v in 0 14 13; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --variant $v > gpurun_out/bench_v${v}_${TAG}.json 2>&1 || exit 1
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(r['roofline']['kernel'], round(r['roofline']['kernel_ms']*1e3,2), 'us/launch', round(r['ms_per_step']*1e3,2), 'us/step')" gpurun_out/bench_v${v}_${TAG}.json
done
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
for v in 0 13; do
  SSNT_VARIANT=$v timeout -k 10 120 python3 tools/diag_fwd_bwd.py > gpurun_out/diag_v${v}_${TAG}.txt 2>&1 || { tail -5 gpurun_out/diag_v${v}_${TAG}.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/diag_v${v}_${TAG}.txt
done
timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err || { tail -5 gpurun_out/configs_${TAG}.err; exit 1; }
cat gpurun_out/configs_${TAG}.jsonl
