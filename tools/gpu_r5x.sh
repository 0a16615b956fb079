set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/ssnt-tts-rust_amd/lib
for i in 1 2 3; do
  for v in base f4new; do
    SSNT_TTS_C_LIB=$L/$v/libssnt_tts_c.so timeout -k 10 120 python -u tools/time_f4.py $v >> gpurun_out/r5x_time.jsonl
  done
done
SSNT_TTS_C_LIB=$L/f4new/libssnt_tts_c.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5x_prof -o run -- python3 tools/time_f4.py prof > gpurun_out/r5x_prof.log 2>&1
SSNT_TTS_C_LIB=$L/f4new/libssnt_tts_c.so timeout -k 10 600 python -u -m pytest tests/test_gpu_v2_fwd_bwd.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x_tests.log 2>&1
tail -2 gpurun_out/r5x_tests.log
