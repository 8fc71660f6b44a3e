#!/bin/bash
# Same-box A/B of two builds of libpdvc_hip.so on the MSDA kernels: rocprofv3 kernel stats of tools/kbench.py (the
# fused op at PDVC's encoder / decoder shapes) and tools/dropin_prof.py (the drop-in operator), alternating the builds.
#   LIBS="libpdvc_hip var_old" bash tools/lib_ab.sh TAG
set -o pipefail
TAG=${1:-lib_ab}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for L in ${LIBS:-libpdvc_hip var_old}; do
    for tool in kbench dropin_prof; do
      PDVC_HIP_LIB=dense-video-captioning_amd/lib/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/${tool}_${L}_$rep" -o run -- python -u tools/$tool.py --videos 256 --reps 5 > "$OUT/${tool}_${L}_$rep.log" 2>&1 \
          || { tail -20 "$OUT/${tool}_${L}_$rep.log"; exit 1; }
      ks=$(find "$OUT/${tool}_${L}_$rep" -name "*kernel_stats.csv" | head -1)
      echo "== $tool $L rep $rep"; python tools/profsum.py "$ks" 0 8
    done
  done
done
