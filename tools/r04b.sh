#!/bin/bash
# round-4 GPU pass B: determinism with every dropout off, value-walk A/B (kbench, csv kernel stats), replay check
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] determinism probe"
timeout -k 10 400 python -u tools/determinism_probe.py --videos 256 > $O/det256.log 2>&1 || { tail -20 $O/det256.log; exit 1; }
grep -v Warning $O/det256.log | tail -16
for pf in 0 4 0 4; do
  echo "[$(date +%T)] kbench PDVC_VAL_PF=$pf"
  PDVC_VAL_PF=$pf timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kb_pf$pf -o kb -- python -u tools/kbench.py --videos 1024 --reps 4 >> $O/kbench_pf$pf.log 2>&1 || exit 1
done
for pf in 0 4; do
  for f in $(find $O/kb_pf$pf -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"pf$pf {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:110]}\") for r in csv.DictReader(open(sys.argv[1])) if 'msda1d' in r['Name']]" $f
  done
done | tee $O/kb_ab.txt
echo "[$(date +%T)] scale test"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_step_graph_scale.py > $O/scale_test.log 2>&1; tail -15 $O/scale_test.log
echo "[$(date +%T)] graph replays vs eager, 256 videos"
timeout -k 10 400 python -u tools/check_graph_replays.py --videos 256 > $O/replays256.log 2>&1 || { tail -20 $O/replays256.log; exit 1; }
grep -v Warning $O/replays256.log | tail -6
