set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5s_prof -o run -- python3 tools/probe_f4_window.py 5 1600 1700 1900 2000 2100 2400 2900 3400 > gpurun_out/r5s.log 2>&1
find gpurun_out/r5s_prof -name "*kernel_trace.csv" | head -3
