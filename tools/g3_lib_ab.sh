#!/bin/bash
# gemm3p / gemm3w timings of the default library against variant builds (LIBS), alternating, two rounds:
#   LIBS="libpdvc_hip var_x" bash tools/g3_lib_ab.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do
  for L in ${LIBS:-libpdvc_hip}; do
    PDVC_HIP_LIB=dense-video-captioning_amd/lib/$L.so PDVC_GEMM3_NO_BLASLT=1 timeout -k 10 200 python -u tools/gemm3_bench.py \
        --only ${OPS:-fwdp,dgradp} --shapes ${SHAPES:-512x512,2048x512} --no-err --iters 10 > $OUT/${L}_$rep.log 2>&1 || exit 1
    grep '"op"' $OUT/${L}_$rep.log | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print('$L', $rep, r['op'], r['M'], r['N'], r['K'], '%.1f TF/s (%.3f ms)' % (r['ours_tfs'], r['ours_ms']))
"
  done
done
