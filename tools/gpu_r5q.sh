set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SH="64 2000 400 32 2000 400 64 1100 1024 64 1200 400"
L=$PWD/ssnt-tts-rust_amd/lib
for i in 1 2; do
  for v in old r256p64 r256p128; do
    SSNT_TTS_C_LIB=$L/$v/libssnt_tts_c.so timeout -k 10 150 python -u tools/time_long.py $v $SH >> gpurun_out/r5q_time.jsonl
  done
done
