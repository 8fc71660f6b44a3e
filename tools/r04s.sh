#!/bin/bash
# round-4 GPU pass S: parity of the kept changes (windowed forward skips the level-0 window a wave has no sample in;
# drop-in backward-query prefetch; value walk mask from LDS), then the T = 1024 forward and the drop-in backward
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] parity"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
  tests/test_gpu_bf16.py > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2 3; do
  echo "[$(date +%T)] kbench T=1024"
  timeout -k 10 120 python -u tools/kbench.py --videos 512 --reps 4 --T 1024 2>&1 | grep -E "^encoder" || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/win -o kb -- python -u tools/kbench.py \
  --videos 512 --reps 4 --T 1024 > $O/win.log 2>&1 || { tail -20 $O/win.log; exit 1; }
for f in $(find $O/win -name "*kernel_stats.csv"); do
  python -c "import csv,sys; [print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}\") for r in csv.DictReader(open(sys.argv[1])) if 'msda1d' in r['Name']]" $f
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dropin -o dp -- python -u tools/dropin_prof.py \
  > $O/dropin.log 2>&1 || { tail -20 $O/dropin.log; exit 1; }
tail -3 $O/dropin.log
for f in $(find $O/dropin -name "*kernel_stats.csv"); do
  python -c "import csv,sys; [print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}\") for r in csv.DictReader(open(sys.argv[1])) if 'msda' in r['Name']]" $f
done
