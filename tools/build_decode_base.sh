#!/usr/bin/env bash
# Build the committed fused_decode.hip (HEAD) into ssnt-tts-rust_amd/lib/var_old/ beside the
# working-tree library, for tools/gpu_decode_ab2.sh old. Tuning study only.
set -euo pipefail
cd "$(dirname "$0")/.."
L=ssnt-tts-rust_amd/lib
mkdir -p $L/var_old
git show HEAD:ssnt-tts-rust_amd/csrc/fused_decode.hip > ssnt-tts-rust_amd/csrc/_fused_old.hip
trap 'rm -f ssnt-tts-rust_amd/csrc/_fused_old.hip' EXIT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I include -I ssnt-tts-rust_amd/csrc -c ssnt-tts-rust_amd/csrc/_fused_old.hip -o $L/var_old/fused_decode.o
objs=$(ls $L/obj/*.o | grep -v fused_decode.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/var_old/libssnt_tts_c.so $L/var_old/fused_decode.o $objs -Wl,-soname,libssnt_tts_c.so
