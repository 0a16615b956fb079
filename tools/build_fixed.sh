#!/usr/bin/env bash
# Build one library per experiment mask with the mask baked in at compile time
# (-DSSNT_EXP_FIXED: no runtime bit tests inside the chain steps, so the timing is the product
# kernel's code minus what the mask removes). Only fwd_bwd_stream.hip is rebuilt; the other
# objects come from `make lib`. Usage: bash tools/build_fixed.sh mask1 mask2 ...
set -euo pipefail
cd "$(dirname "$0")/.."
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I include -I ssnt-tts-rust_amd/csrc"
L=ssnt-tts-rust_amd/lib
OTHERS=$(ls $L/obj/*.o | grep -v 'fwd_bwd_stream\|fwd_bwd_pair\|/fwd_bwd.o')
for m in "$@"; do
  (
    mkdir -p $L/fix$m/obj
    for f in fwd_bwd fwd_bwd_stream fwd_bwd_pair; do
      /opt/rocm/bin/hipcc $HIPFLAGS -DSSNT_EXP -DSSNT_EXP_FIXED=$m -c ssnt-tts-rust_amd/csrc/$f.hip -o $L/fix$m/obj/$f.o &
    done
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/fix$m/libssnt_tts_c.so $L/fix$m/obj/*.o $OTHERS -Wl,-soname,libssnt_tts_c.so
  ) &
done
wait
