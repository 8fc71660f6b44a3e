#!/bin/bash
# Build a variant of libpdvc_hip.so with one source recompiled under extra -D flags (kernel tuning experiments):
#   tools/variant_lib.sh seqattn.hip out.so -DSQ_WPE=4
# Load it with PDVC_HIP_LIB=out.so.  Needs the regular build's objects (build_native.py) first.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/dense-video-captioning_amd
SRC=$1; OUT=$2; shift 2
OBJ=/tmp/variant_$$.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I "$ROOT/include" \
  -I "$PKG/csrc" "$@" -c "$PKG/csrc/$SRC" -o $OBJ
OBJS=$(ls $PKG/build/gfx950/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS $OBJ
rm -f $OBJ
