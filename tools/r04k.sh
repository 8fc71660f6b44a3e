#!/bin/bash
# round-4 GPU pass K: value walk depth 16 (4 waves/SIMD) vs 8, and the ops tests at the QU=3 default
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -1 $O/ops.log
for ug in 0 16 0 16; do
  echo "[$(date +%T)] PDVC_VALUE_UG=$ug"
  PDVC_VALUE_UG=$ug timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/u$ug -o kb_$RANDOM -- python -u tools/kbench.py --videos 1024 --reps 4 2>&1 | grep -E "^(encoder)" || exit 1
done
for ug in 0 16; do
  for f in $(find $O/u$ug -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"ug$ug {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}\") for r in csv.DictReader(open(sys.argv[1])) if 'bwd_value' in r['Name'] or 'bwd_query' in r['Name']]" $f
  done
done
