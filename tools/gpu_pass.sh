#!/bin/bash
# One GPU pass: each step writes its own timestamped log under gpurun_out/$PASS (a rerun never overwrites a failing
# log); a step that fails, aborts or times out ends the pass (no GPU work after it).
#   tools/gpu_pass.sh PASS 'label|seconds|command' ...
PASS=$1; shift
OUT=gpurun_out/$PASS
mkdir -p "$OUT"
for spec in "$@"; do
  label=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  log="$OUT/${label}_$(date +%H%M%S).log"
  echo "== $label ($secs s): $cmd" | tee -a "$OUT/pass.txt"
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "   rc=$rc log=$log" | tee -a "$OUT/pass.txt"
  grep -v amdgpu.ids "$log" | tail -n 25
  if [ $rc -ne 0 ]; then echo "pass $PASS stopped at $label (rc=$rc)"; exit $rc; fi
done
