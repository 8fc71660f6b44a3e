#!/bin/bash
# round-4 GPU pass J: value-gradient workgroups per CU (L2 working set of the dOut gathers) and the QU=3 interleave
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
for kib in 0 64 0 64 40; do
  echo "[$(date +%T)] PDVC_VAL_LDS_KIB=$kib"
  PDVC_VAL_LDS_KIB=$kib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$kib -o kb_$RANDOM -- python -u tools/kbench.py --videos 1024 --reps 4 2>&1 | grep -E "^(encoder|decoder)" || exit 1
done
for kib in 0 64 40; do
  for f in $(find $O/k$kib -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"lds$kib {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}\") for r in csv.DictReader(open(sys.argv[1])) if 'bwd_value' in r['Name']]" $f
  done
done
