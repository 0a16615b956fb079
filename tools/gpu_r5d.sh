#!/usr/bin/env bash
# Round 5: segmented kernel parity (all wide cases, A/B forms included) and configs[4] phase times
# under rocprofv3. Usage: bash tools/gpu_r5d.sh TAG
set -uo pipefail
TAG=${1:-r5d}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
SSNT_AB_TESTS=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -k "wide or long or 512 or config5" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/${TAG}_pytest.log | tail -40; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_long -o kt -- python3 tools/ab_long_modes.py 0 1 2 > gpurun_out/${TAG}_long.log 2>&1 || exit 1
grep -h form gpurun_out/${TAG}_long.log
python3 - gpurun_out/${TAG}_long/kt_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "ssnt" in n:
        print(n[n.index("k_"):n.index("(ssnt::")], r["Calls"], round(float(r["AverageNs"]) / 1000, 1))
PY
