#!/usr/bin/env bash
# Build the committed (HEAD) version of one kernel source into ssnt-tts-rust_amd/lib/var_old/,
# linked with the working tree's other product objects, for same-box A/B timing against the
# working tree (tools/gpu_decode_var.sh old, tools/gpu_f4_ab.sh old). Usage:
#   bash tools/build_head_variant.sh v2_fwd_bwd.hip     (tuning study only)
set -euo pipefail
cd "$(dirname "$0")/.."
SRCF=${1:?source file under csrc/}
L=ssnt-tts-rust_amd/lib
mkdir -p $L/var_old
git show HEAD:ssnt-tts-rust_amd/csrc/$SRCF > ssnt-tts-rust_amd/csrc/_head_variant.hip
trap 'rm -f ssnt-tts-rust_amd/csrc/_head_variant.hip' EXIT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden \
  -I include -I ssnt-tts-rust_amd/csrc -c ssnt-tts-rust_amd/csrc/_head_variant.hip -o $L/var_old/head.o
objs=$(ls $L/obj/*.o | grep -v "/${SRCF%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/var_old/libssnt_tts_c.so $L/var_old/head.o $objs -Wl,-soname,libssnt_tts_c.so
