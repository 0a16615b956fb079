#!/usr/bin/env bash
# Build tuning variants of the library: fwd_bwd_stream.hip recompiled with -D overrides, linked
# with the product objects into ssnt-tts-rust_amd/lib/var_<name>/. Usage:
#   bash tools/build_variants.sh name1 "-DSSNT_T_CDEPTH=12" name2 "-DSSNT_T_CPRIO=2" ...
# (select one with SSNT_TTS_C_LIB=.../var_<name>/libssnt_tts_c.so). Tuning study only.
# SRC=<file>.hip (default fwd_bwd_stream.hip) picks the source file the -D overrides apply to.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s lib
L=ssnt-tts-rust_amd/lib
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I include -I ssnt-tts-rust_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p $L/var_$name
  /opt/rocm/bin/hipcc $FLAGS $defs -c ssnt-tts-rust_amd/csrc/${SRC:-fwd_bwd_stream.hip} -o $L/var_$name/${SRC:-fwd_bwd_stream.hip}.o &
done
wait
for d in $L/var_*/; do
  vo=$(ls $d/*.hip.o 2>/dev/null) || continue  # (make-built study libraries: var_desc*)
  objs=$(ls $L/obj/*.o | grep -v "/$(basename $vo .hip.o).o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libssnt_tts_c.so $vo $objs -Wl,-soname,libssnt_tts_c.so
done
