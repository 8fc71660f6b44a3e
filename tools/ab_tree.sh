#!/bin/bash
# Same-box A/B of two code trees (GPU box, repo root): HEAD against an older tree copied under $OLD (default _r05,
# git-ignored), alternating, two rounds each:  bash tools/ab_tree.sh TAG [bench.py args]
set -o pipefail
TAG=$1; shift
OLD=${OLD:-_r05}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for run in new1 old1 new2 old2; do
  if [[ $run == old* ]]; then dir=$OLD; else dir=.; fi
  (cd "$dir" && timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@") > "$OUT/$run.json" 2> "$OUT/$run.err" \
      || { tail -5 "$OUT/$run.err"; exit 1; }
  echo "$run $(grep -o '"value": [0-9.]*' "$OUT/$run.json")"
done
