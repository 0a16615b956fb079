#!/usr/bin/env bash
# Round 5: segmented kernel A/B at configs[4] and two more long shapes (forms 0 / 1), parity
# first, phase times under rocprofv3. Usage: bash tools/gpu_r5j.sh TAG
set -uo pipefail
TAG=${1:-r5j}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
SSNT_AB_TESTS=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fwd_bwd.py -k "wide or long or 512 or config5" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/${TAG}_pytest.log | tail -40; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_long -o kt -- python3 tools/ab_long_modes.py 0 1 > gpurun_out/${TAG}_long.log 2>&1 || exit 1
grep -h '"form"' gpurun_out/${TAG}_long.log
python3 - gpurun_out/${TAG}_long/kt_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "ssnt" in n:
        print(n[n.index("k_"):n.index("(ssnt::")], r["Calls"], round(float(r["AverageNs"]) / 1000, 1))
PY
for shape in "32 2000 400" "64 760 700"; do
  timeout -k 10 200 python3 tools/ab_long_modes.py $shape 0 1 2>&1 | grep '"form"' || exit 1
done
