set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/ssnt-tts-rust_amd/lib
for i in 1 2 3; do
  for v in base pair2; do
    SSNT_TTS_C_LIB=$L/$v/libssnt_tts_c.so timeout -k 10 150 python -u tools/time_long.py $v 256 200 80 256 200 128 256 200 65 >> gpurun_out/r5v_time.jsonl
  done
done
