#!/usr/bin/env bash
# PMC passes over an arbitrary command (GPU box). Usage:
#   bash tools/pmc_cmd.sh <tag> "<counters pass1>" ["<counters pass2>" ...] -- <cmd...>
set -euo pipefail
TAG=$1; shift
groups=()
while [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
cd "$(dirname "$0")/.."
ROOT=$PWD
export TMPDIR=/tmp
i=0
for grp in "${groups[@]}"; do
  OUT=$ROOT/gpurun_out/pmc_$TAG/$i
  mkdir -p "$OUT"
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT" -o p -- "$@" > "$OUT/log.txt" 2>&1
  i=$((i+1))
done
python3 "$ROOT/tools/pmc_table.py" "$ROOT/gpurun_out/pmc_$TAG"
