set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$PWD/ssnt-tts-rust_amd/lib
for i in 1 2 3; do
  for v in base noconv; do
    SSNT_TTS_C_LIB=$L/$v/libssnt_tts_c.so timeout -k 10 150 python -u tools/time_long.py $v 256 200 80 >> gpurun_out/r5t_time.jsonl
  done
done
