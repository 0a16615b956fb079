#!/usr/bin/env bash
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/ab_exp.py 1 200 80 0 8 2048 2056 3080 6152 7176 > gpurun_out/ab_exp_r3j.jsonl 2> gpurun_out/ab_exp_r3j.err
timeout -k 10 200 python3 tools/ab_exp.py 256 200 80 0 8 2056 3080 7176 >> gpurun_out/ab_exp_r3j.jsonl 2>> gpurun_out/ab_exp_r3j.err
cat gpurun_out/ab_exp_r3j.jsonl
