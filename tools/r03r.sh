# round-3 GPU pass: wave-uniform value-gradient walk (W1) -- full GPU suite, per-kernel device times with the walk
# on and off (PDVC_VALUE_W1=0), bench lines (headline, cfg-2 bf16)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03r}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log; ok $rc
PDVC_VALUE_W1=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests_w0.log 2>&1; rc=$?
tail -2 $O/tests_w0.log; ok $rc
for w in 1 0; do
  PDVC_VALUE_W1=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kp$w -o run -- python -u tools/kbench.py --videos 1024 --reps 5 > $O/kbp$w.txt 2>&1; rc=$?
  ks=$(find $O/kp$w -name "*kernel_stats.csv" | head -1)
  echo "W1=$w: $(grep -E 'encoder|decoder' $O/kbp$w.txt | tr '\n' ' ')"; python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "msda1d" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:70]}')
PY
  ok $rc
done
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 300 $O/bench.json; tail -2 $O/bench.err; ok $rc
echo "[$(date +%T)] bench yc2_tsp_bf16"
timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16.json 2> $O/bench_bf16.err; rc=$?
tail -c 200 $O/bench_bf16.json; ok $rc
echo "[$(date +%T)] done"
