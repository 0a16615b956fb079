set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5y_smoke.log 2>&1
tail -1 gpurun_out/r5y_smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r5y_bench.json 2> gpurun_out/r5y_bench.err
cat gpurun_out/r5y_bench.json
