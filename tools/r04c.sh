#!/bin/bash
# round-4 GPU pass C: the wave-uniform value walk -- ops parity, then A/B against the 16-lane-group walk
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] ops tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -2 $O/ops.log
for q in 0 1 0 1; do
  echo "[$(date +%T)] kbench PDVC_VAL_Q4=$q"
  PDVC_VAL_Q4=$q timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kb_q$q -o kb_$RANDOM -- python -u tools/kbench.py --videos 1024 --reps 4 2>&1 | grep -E "^(encoder|decoder)" | tee -a $O/kbench_q$q.log || exit 1
done
for q in 0 1; do
  for f in $(find $O/kb_q$q -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"q$q {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:100]}\") for r in csv.DictReader(open(sys.argv[1])) if 'msda1d_bwd_value' in r['Name']]" $f
  done
done | tee $O/kb_ab.txt
