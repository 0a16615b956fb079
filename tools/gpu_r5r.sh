set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SH="64 2000 400 32 2000 400 64 1200 400 64 520 500"
L=$PWD/ssnt-tts-rust_amd/lib
for i in 1 2; do
  for v in old p2d24; do
    SSNT_TTS_C_LIB=$L/$v/libssnt_tts_c.so timeout -k 10 150 python -u tools/time_long.py $v $SH >> gpurun_out/r5r_time.jsonl
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_fwd_bwd.py -x -q --timeout 300 --timeout-method thread -k "wide or long or split" > gpurun_out/r5r_tests.log 2>&1
tail -2 gpurun_out/r5r_tests.log
