#!/bin/bash
# Round-2 bench lines of every BASELINE config (one GPU box pass, each step under its own limit, stop at the first
# failure).  Usage: bash tools/r02_lines.sh TAG
set -o pipefail
TAG=${1:-r02_lines}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, then bench.py arguments
  local n=$1; shift
  echo "[$(date +%T)] $n"
  timeout -k 10 500 python -u bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" \
      || { echo "$n failed"; tail -20 "$OUT/bench_$n.err"; exit 1; }
  cut -c1-200 "$OUT/bench_$n.json"
}
run yc2_bf16 --workload yc2_tsp_bf16 --no-cpu-baseline
run yc2_newmodel --workload yc2_newmodel --no-cpu-baseline
run anet_c3d --workload anet_c3d --no-cpu-baseline
run eval --mode eval --videos-per-gpu 256 --steps 3 --warmup 1 --no-cpu-baseline
echo "[$(date +%T)] done"
