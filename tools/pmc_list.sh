#!/usr/bin/env bash
# GPU box: list the PMC counters rocprofv3 offers here (to pick SQ passes)
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/pmc_list.txt | sort -u > gpurun_out/pmc_sq.txt || true
wc -l gpurun_out/pmc_sq.txt
