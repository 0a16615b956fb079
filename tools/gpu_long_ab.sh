#!/usr/bin/env bash
# GPU box: configs[4] segmented-kernel phase times (rocprof kernel stats) of the product library
# and each named var_* build, alternating. Tuning / traffic study only.
set -uo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in prod "$@" prod "$@"; do
  if [ $n = prod ]; then unset SSNT_TTS_C_LIB; else export SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/var_$n/libssnt_tts_c.so; fi
  rm -rf gpurun_out/prof_long_$n
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_long_$n -o kt -- python3 tools/long_run_once.py 5 > gpurun_out/long_ab_$n.log 2>&1 || { tail -5 gpurun_out/long_ab_$n.log; }
  python3 - "$n" <<'PY'
import csv, glob, sys
n = sys.argv[1]
f = glob.glob(f"gpurun_out/prof_long_{n}/**/kt_kernel_stats.csv", recursive=True) + glob.glob(f"gpurun_out/prof_long_{n}/kt_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    if "wide" in r["Name"]:
        print(n, r["Name"][36:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
