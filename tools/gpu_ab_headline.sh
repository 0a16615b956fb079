#!/usr/bin/env bash
# GPU box: fwd-bwd parity (all variants), then the headline bench (default kernel) and its
# kernel stats. Usage (via gpurun): bash tools/gpu_ab_headline.sh <tag>
set -euo pipefail
TAG=${1:-ab}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_ab_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_ab_${TAG}.log
timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2>gpurun_out/bench_${TAG}.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}.json')); print(d['ms_per_step'], d['roofline'], d['value'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o kt -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}.log 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_${TAG}/kt_kernel_stats.csv')):
    print(r['Name'][:90], r['Calls'], float(r['AverageNs'])/1e3)
"
