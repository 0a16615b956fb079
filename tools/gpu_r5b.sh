#!/usr/bin/env bash
# Round 5: full GPU suite including the A/B-only forms, bench line, tone-waves A/B, rocprof
# kernel stats of the decode workloads + F4 and of the bench. Usage: bash tools/gpu_r5b.sh TAG
set -uo pipefail
TAG=${1:-r5b}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
SSNT_AB_TESTS=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/${TAG}_pytest.log | tail -40; exit $rc; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python3 tools/ab_tone_waves.py > gpurun_out/${TAG}_tone_waves.json 2>&1 || exit 1
cat gpurun_out/${TAG}_tone_waves.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_dec -o kt -- python3 tools/prof_decode.py 10 > gpurun_out/${TAG}_dec.log 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/${TAG}_dec/kt_kernel_stats.csv | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_long -o kt -- python3 tools/ab_long_modes.py 0 1 2 > gpurun_out/${TAG}_long.log 2>&1 || exit 1
grep -h split_mode gpurun_out/${TAG}_long.log
cut -d, -f1-4 gpurun_out/${TAG}_long/kt_kernel_stats.csv | grep wide
