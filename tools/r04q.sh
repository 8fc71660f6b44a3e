#!/bin/bash
# round-4 GPU pass Q: value-gradient query chunk at T = 1024 (occupancy vs a second accumulating pass)
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
for qc in 0 960 640 0 960; do
  echo "[$(date +%T)] PDVC_VAL_QCHUNK=$qc"
  PDVC_VAL_QCHUNK=$qc timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q$qc -o kb_$RANDOM -- python -u tools/kbench.py --videos 512 --reps 4 --T 1024 2>&1 | grep -E "^encoder" || exit 1
done
for qc in 0 960 640; do
  for f in $(find $O/q$qc -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"qc$qc {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}\") for r in csv.DictReader(open(sys.argv[1])) if 'bwd_value' in r['Name']]" $f
  done
done
for ab in 0 1 0 1; do
  echo "[$(date +%T)] PDVC_WIN_ABLATE=$ab (forward, T=1024)"
  PDVC_WIN_ABLATE=$ab timeout -k 10 120 python -u tools/kbench.py --videos 512 --reps 4 --T 1024 2>&1 | grep -E "^encoder" || exit 1
done
