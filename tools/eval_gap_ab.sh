#!/bin/bash
# Eval-line idle gaps under host settings (GPU box), one rocprofv3 --kernel-trace run per arm:
#   bash tools/eval_gap_ab.sh TAG [name:ENV=value ...]      (default arms: the defaults, PostProcess inline,
#                                                             the deferred host half without its gate)
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
ARMS=("$@"); [ ${#ARMS[@]} -eq 0 ] && ARMS=("default:" "nodefer:PDVC_POST_DEFER=0" "nogate:PDVC_POST_GATE=0")
for spec in "${ARMS[@]}"; do
  arm=${spec%%:*}; E=${spec#*:}
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$arm" -o run \
      -- python -u bench.py --mode eval --videos-per-gpu 256 --steps 8 --warmup 2 --no-cpu-baseline > "$OUT/$arm.json" \
      2> "$OUT/$arm.err" || { echo "$arm failed"; tail -20 "$OUT/$arm.err"; exit 1; }
  kt=$(find "$OUT/$arm" -name "*kernel_trace.csv" | head -1)
  echo "== $arm ($E)"; tail -1 "$OUT/$arm.json" | cut -c1-120; python tools/gaps.py "$kt" | tail -7
  python tools/evalbreak.py "$kt" 25 > "$OUT/${arm}_kernels.txt"
  rm -f "$kt"
done
