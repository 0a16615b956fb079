#!/usr/bin/env bash
# GPU-box A/B (via gpurun): default ring (8 slots) vs the 16-slot variant (8) at lattices whose
# rows still fit LDS beside the bigger ring, plus the default at config 2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_ring.py > gpurun_out/ab_ring.log 2>&1 || exit 1
cat gpurun_out/ab_ring.log
