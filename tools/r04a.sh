#!/bin/bash
# round-4 GPU pass A: launcher / DP / memset / ops tests, value-walk A/B (kbench), determinism probe
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_launcher.py \
    tests/test_gpu_dp.py tests/test_gpu_graph_memset.py tests/test_gpu_ops.py tests/test_gpu_batch.py tests/test_gpu_model.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for pf in 0 4 0 4; do
  echo "[$(date +%T)] kbench PDVC_VAL_PF=$pf"
  PDVC_VAL_PF=$pf timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kb_pf$pf -o kb -- python -u tools/kbench.py --videos 1024 --reps 4 >> $O/kbench_pf$pf.log 2>&1 || exit 1
done
for pf in 0 4; do
  for f in $(find $O/kb_pf$pf -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"pf$pf {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:110]}\") for r in csv.DictReader(open(sys.argv[1])) if 'msda1d' in r['Name']]" $f
  done
done | tee $O/kb_ab.txt
echo "[$(date +%T)] determinism probe"
timeout -k 10 400 python -u tools/determinism_probe.py --videos 256 > $O/det256.log 2>&1 || { tail -20 $O/det256.log; exit 1; }
tail -30 $O/det256.log
