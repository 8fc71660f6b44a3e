#!/bin/bash
# The eval line, defaults against an environment variant, alternating on one box, three rounds, with each run's
# per-step wall times (the outlier steps):   VAR="PDVC_GC_FREEZE=0" bash tools/eval_env_ab3.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
for rep in 1 2 3; do
  for arm in a b; do
    E=""; [ $arm = b ] && E="$VAR"
    env $E timeout -k 10 300 python -u bench.py --mode eval --no-cpu-baseline --steps 12 > "$OUT/${arm}_$rep.json" \
        2> "$OUT/${arm}_$rep.err" || { tail -20 "$OUT/${arm}_$rep.err"; exit 1; }
    python -c "
import json; d = json.loads(open('$OUT/${arm}_$rep.json').read().strip().splitlines()[-1])
print('$arm', $rep, '${E:-default}', '%.1f videos/s' % d['value'], 'median %.1f' % d['per_step']['median_videos_per_s'], 'walls', d['per_step']['wall_ms_all'])"
  done
done
