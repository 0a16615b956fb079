#!/usr/bin/env bash
# GPU box: configs[4] long-form fwd-bwd under rocprofv3 -- kernel trace + stats, then one
# FETCH_SIZE and one WRITE_SIZE pass; summary into profiles/<tag>_long_*. Usage: bash tools/profile_long.sh <tag>
set -euo pipefail
TAG=${1:-r2}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_long_${TAG}
mkdir -p "$OUT" profiles
RUN=(python3 tools/long_run_once.py 5)
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- "${RUN[@]}" > "$OUT/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- "${RUN[@]}" > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- "${RUN[@]}" > "$OUT/write.log" 2>&1
python3 tools/pmc_long.py "$OUT" "$TAG"
