set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SH="64 2000 400 32 2000 400 64 1100 1024 64 760 700 64 1200 400"
for i in 1 2; do
  SSNT_TTS_C_LIB=$PWD/ssnt-tts-rust_amd/lib/old/libssnt_tts_c.so timeout -k 10 150 python -u tools/time_long.py old $SH >> gpurun_out/r5p_time.jsonl
  timeout -k 10 150 python -u tools/time_long.py new $SH >> gpurun_out/r5p_time.jsonl
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 300 --timeout-method thread -k "wide or long or split or debug64" > gpurun_out/r5p_tests.log 2>&1
tail -3 gpurun_out/r5p_tests.log
