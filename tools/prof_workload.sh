#!/bin/bash
# Kernel trace of one bench workload's replayed step (GPU box): tools/profsteps.py breakdown + rocprof summary.
#   bash tools/prof_workload.sh TAG WORKLOAD
set -o pipefail
OUT=gpurun_out/$1; WL=$2; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python -u bench.py --workload "$WL" --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > "$OUT/prof_bench.json" \
    2> "$OUT/prof.err" || { echo "rocprof bench failed"; tail -30 "$OUT/prof.err"; exit 1; }
kt=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python tools/profsteps.py "$kt" 45 > "$OUT/replay_steps.txt" && head -40 "$OUT/replay_steps.txt"
rm -f $(find "$OUT" -name "*.csv" -size +20M)
