#!/bin/bash
# round-4 GPU pass L: the drop-in operator's kernels at the encoder shape (256 videos)
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o dropin -- python -u tools/dropin_prof.py > $O/dropin.log 2>&1 || { tail -20 $O/dropin.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
python -c "import csv,sys; [print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Name'][:100]}\") for r in csv.DictReader(open(sys.argv[1]))]" $f | sort -k5 -n -r | head -20
grep "encoder" $O/dropin.log | head -3
