#!/bin/bash
# gemm3 timings, default against an environment variant (same library, same box), alternating, two rounds:
#   VAR="PDVC_G3_MF16=1" bash tools/g3_env_ab.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do
  for arm in a b; do
    E=""; [ $arm = b ] && E="$VAR"
    env $E PDVC_GEMM3_NO_BLASLT=1 timeout -k 10 200 python -u tools/gemm3_bench.py \
        --only ${OPS:-fwdp,dgradp,wgrad} --shapes ${SHAPES:-512x512,2048x512} --no-err --iters 10 > $OUT/${arm}_$rep.log 2>&1 || exit 1
    grep '"op"' $OUT/${arm}_$rep.log | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print('$arm', $rep, r['op'], r['M'], r['N'], r['K'], '%.1f TF/s (%.3f ms)' % (r['ours_tfs'], r['ours_ms']))
"
  done
done
