#!/usr/bin/env bash
# GPU box: streaming-kernel timing masks (make lib-expnd), graph-timed (tools/ab_exp_graph.py).
# bits: 3 chains never poll converters, 10 chains read no factors, 11 no release polls,
# 12 chains alone (other roles exit; only with 3 and 11), 5 no chain row stores, 7 converters
# alone, 13 two rows per dependent chain step (three-term recurrence)
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
M="0 8192 2056 10248 6152 7176 6184 14344 4224"
timeout -k 10 120 python3 tools/ab_exp_graph.py 256 200 80 $M | tee gpurun_out/ab_exp_r3k2.jsonl
timeout -k 10 120 python3 tools/ab_exp_graph.py 1 200 80 $M | tee -a gpurun_out/ab_exp_r3k2.jsonl
timeout -k 10 120 python3 tools/ab_exp_graph.py 256 100 80 $M | tee -a gpurun_out/ab_exp_r3k2.jsonl
