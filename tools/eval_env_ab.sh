#!/bin/bash
# The eval line (bench.py --mode eval, its default 1024 videos), defaults against an environment variant, alternating
# on one box, two rounds:   VAR="PDVC_POST_GATE=0" bash tools/eval_env_ab.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
for rep in 1 2; do
  for arm in a b; do
    E=""; [ $arm = b ] && E="$VAR"
    env $E timeout -k 10 300 python -u bench.py --mode eval --no-cpu-baseline > "$OUT/${arm}_$rep.json" \
        2> "$OUT/${arm}_$rep.err" || { tail -20 "$OUT/${arm}_$rep.err"; exit 1; }
    python -c "
import json; d = json.loads(open('$OUT/${arm}_$rep.json').read().strip().splitlines()[-1])
print('$arm', $rep, '${E:-default}', '%.1f videos/s' % d['value'], '%.2f ms/step' % d['ms_per_step'])"
  done
done
