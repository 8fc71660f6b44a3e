#!/bin/bash
# CPU sanitizer pass: the plain-C oracle (oracle/msda_oracle.c) and the
# library's host-only C++ (csrc/detok.cpp, csrc/pdvc_status.cpp) built with -fsanitize=address,undefined by gcc/g++,
# then
#   (1) a C++ driver of the host entry points' edge cases (tools/sanitize/host_check.cpp), run directly;
#   (2) pytest -m "not gpu" with the ASan runtime preloaded, the oracle loaded from the sanitized build
#       (PDVC_ORACLE_LIB) and the host entry points from the sanitized host library (PDVC_HOST_ASAN_LIB,
#       tests/test_host_native.py).  Any ASan / UBSan report aborts the run (halt_on_error, -fno-sanitize-recover).
# CPU only; outputs under oracle/_asan/ (git-ignored).  Usage: bash tools/sanitize/run.sh [pytest args]
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/oracle/_asan
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1"
gcc $SAN -fPIC -shared -ffp-contract=off -o "$OUT/libmsda_oracle.so" "$ROOT/oracle/msda_oracle.c" -lm
g++ $SAN -fPIC -shared -std=c++17 -I "$ROOT/include" -o "$OUT/libpdvc_host.so" \
    "$ROOT/dense-video-captioning_amd/csrc/detok.cpp" "$ROOT/dense-video-captioning_amd/csrc/pdvc_status.cpp"
g++ $SAN -std=c++17 -I "$ROOT/include" -o "$OUT/host_check" "$ROOT/tools/sanitize/host_check.cpp" \
    -L "$OUT" -lpdvc_host -Wl,-rpath,"$OUT"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:alloc_dealloc_mismatch=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
"$OUT/host_check"
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
cd "$ROOT"
LD_PRELOAD="$PRE" PDVC_ORACLE_LIB="$OUT/libmsda_oracle.so" PDVC_HOST_ASAN_LIB="$OUT/libpdvc_host.so" \
    python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
