#!/usr/bin/env bash
# PMC sweep of the fwd-bwd kernel (GPU box, via gpurun): one rocprofv3 pass per counter group.
# Usage: bash tools/pmc_sweep.sh <tag> "<group1>" "<group2>" ...   (a group = space-separated
# counters collected in one pass). Output: gpurun_out/pmc_<tag>/<i>/...counter_collection.csv
set -euo pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
ROOT=$PWD
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  OUT=$ROOT/gpurun_out/pmc_$TAG/$i
  mkdir -p "$OUT"
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT" -o p -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/log.txt" 2>&1
  i=$((i+1))
done
python3 "$ROOT/tools/pmc_table.py" "$ROOT/gpurun_out/pmc_$TAG"
