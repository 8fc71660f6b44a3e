#!/bin/bash
# Every bench line of HEAD on one box (GPU box, repo root), each under its own time limit; stops at the first failure.
#   bash tools/all_lines.sh TAG   -> gpurun_out/TAG/bench_<line>.json
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
run() {  # name, seconds, bench.py arguments
  local n=$1 s=$2; shift 2
  echo "[$(date +%T)] $n: bench.py $*"
  timeout -k 10 "$s" python -u bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" \
      || { echo "$n failed"; tail -20 "$OUT/bench_$n.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$n.json')); print('  $n', round(d['value'], 1), d['unit'])"
}
run headline 400
run ragged 400 --stream ragged --no-cpu-baseline
run yc2_bf16 400 --workload yc2_tsp_bf16 --no-cpu-baseline
run newmodel 500 --workload yc2_newmodel --no-cpu-baseline
run anet_c3d 500 --workload anet_c3d --no-cpu-baseline
run eval 400 --mode eval --no-cpu-baseline
