#!/bin/bash
# gemm3p ablations (profiles/r05_gemm3_ablation.txt): the default library against variant builds of gemm3.hip
# (tools/variant_lib.sh gemm3.hip dense-video-captioning_amd/lib/var_g3_16.so -DG3_ABLATE=16, var_g3_al2.so -DG3_AL2=1,
# var_g3_al2e.so -DG3_AL2=1 -DG3_ABLATE=16), 983040 x 512 x {512, 2048}.   tools/g3_ablate.sh OUTTAG
O=gpurun_out/$1; mkdir -p $O
for L in ${LIBS:-libpdvc_hip var_g3_16 var_g3_al2 var_g3_al2e}; do
  for mnk in 983040,512,512 983040,512,2048; do
    PDVC_HIP_LIB=dense-video-captioning_amd/lib/$L.so timeout -k 10 120 python -u tools/gemm3_bench.py --mnk $mnk --no-err --iters 10 ${ACCUM:+--accum} 2>&1 | grep '"op"' | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print('$L', r['op'], r['M'], r['N'], r['K'], 'ours %.1f TF/s (%.3f ms)' % (r['ours_tfs'], r['ours_ms']))
" || exit 1
  done
done
