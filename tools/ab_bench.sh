#!/bin/bash
# Same-box A/B of bench.py (GPU box, repo root): default, variant, default, variant.
#     [BENCH_ARGS="--stream ragged"] bash tools/ab_bench.sh TAG "ENV=VALUE [ENV2=VALUE2]"
set -o pipefail
TAG=$1
VAR=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for run in a1 b1 a2 b2; do
  if [[ $run == b* ]]; then
    env $VAR timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/$run.json" 2> "$OUT/$run.err" || { tail -5 "$OUT/$run.err"; exit 1; }
  else
    timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/$run.json" 2> "$OUT/$run.err" || { tail -5 "$OUT/$run.err"; exit 1; }
  fi
  echo "$run $(grep -o '"value": [0-9.]*' "$OUT/$run.json")"
done
