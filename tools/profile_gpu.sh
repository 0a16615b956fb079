#!/usr/bin/env bash
# Run on the GPU box (via gpurun): kernel trace + stats of the bench, then one rocprofv3 pass
# per PMC counter (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), then summarise into
# profiles/. Usage: bash tools/profile_gpu.sh <tag>   (e.g. r1)
set -euo pipefail
TAG=${1:-r1}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT" profiles
BENCH=(python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline)

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- "${BENCH[@]}" \
  > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- "${BENCH[@]}" \
  > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- "${BENCH[@]}" \
  > "$OUT/write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT" "$TAG"
# profiles/ is written on the box too, but only gpurun_out/ travels back: re-run
# tools/pmc_traffic.py locally on gpurun_out/prof_<tag> to refresh the committed summaries.
