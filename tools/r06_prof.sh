#!/bin/bash
# Kernel traces of HEAD (GPU box): the headline bench's replayed step (tools/profsteps.py, tools/g3launches.py) and
# the eval line's steps (tools/gaps.py).   bash tools/r06_prof.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
    || { echo "rocprof bench failed"; tail -30 "$OUT/prof.err"; exit 1; }
kt=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python tools/profsteps.py "$kt" 45 > "$OUT/replay_steps.txt" && head -50 "$OUT/replay_steps.txt"
python tools/g3launches.py "$kt" > "$OUT/g3launches.txt" && tail -12 "$OUT/g3launches.txt"
ks=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python tools/profsum.py "$ks" 0 45 > "$OUT/prof_summary.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/evalprof" -o run \
    -- python -u bench.py --mode eval --videos-per-gpu 256 --steps 8 --warmup 2 --no-cpu-baseline > "$OUT/eval_prof.json" \
    2> "$OUT/evalprof.err" || { echo "rocprof eval failed"; tail -30 "$OUT/evalprof.err"; exit 1; }
kt=$(find "$OUT/evalprof" -name "*kernel_trace.csv" | head -1)
python tools/gaps.py "$kt" > "$OUT/eval_gaps.txt"; cat "$OUT/eval_gaps.txt"
rm -f $(find "$OUT" -name "*.csv" -size +20M)  # keep the merge under gpurun's cap
