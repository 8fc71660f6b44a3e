#!/bin/bash
# Eval-line idle gaps under three host settings (GPU box): the defaults, the host half of PostProcess inline
# (PDVC_POST_DEFER=0), and the default 5 ms GIL switch interval (PDVC_EVAL_SWITCH_INTERVAL=0.005).
#   bash tools/eval_gap_ab.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
for arm in default nodefer si5ms; do
  E=""; [ $arm = nodefer ] && E="PDVC_POST_DEFER=0"; [ $arm = si5ms ] && E="PDVC_EVAL_SWITCH_INTERVAL=0.005"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$arm" -o run \
      -- python -u bench.py --mode eval --videos-per-gpu 256 --steps 8 --warmup 2 --no-cpu-baseline > "$OUT/$arm.json" \
      2> "$OUT/$arm.err" || { echo "$arm failed"; tail -20 "$OUT/$arm.err"; exit 1; }
  kt=$(find "$OUT/$arm" -name "*kernel_trace.csv" | head -1)
  echo "== $arm"; python tools/gaps.py "$kt" | tail -7
  rm -f "$kt"
done
