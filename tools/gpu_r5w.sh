set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SSNT_AB_TESTS=1 timeout -k 10 600 python -u -m pytest tests -m "gpu and ab" -x -q --timeout 200 --timeout-method thread > gpurun_out/r5w_ab_tests.log 2>&1
tail -3 gpurun_out/r5w_ab_tests.log
