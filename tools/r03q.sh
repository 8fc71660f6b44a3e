# round-3 GPU pass: packed-FMA pyramid forward (MSDA op tests, kernel timings) and the value-gradient ablations
# (PDVC_VAL_ABLATE=1: sort only, 2: walk without the gathers), per-kernel device times by rocprofv3
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03q}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_modules.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; ok $rc
for T in 512 256; do
  timeout -k 10 120 python -u tools/kbench.py --videos 1024 --reps 10 --T $T > $O/kb_T$T.txt 2>&1; rc=$?
  echo "T=$T: $(grep -E 'encoder|decoder' $O/kb_T$T.txt | tr '\n' ' ')"; ok $rc
done
for ab in 0 1 2; do
  PDVC_VAL_ABLATE=$ab timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kp$ab -o run -- python -u tools/kbench.py --videos 1024 --reps 5 > $O/kbp$ab.txt 2>&1; rc=$?
  ks=$(find $O/kp$ab -name "*kernel_stats.csv" | head -1)
  echo "ablate=$ab"; python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "msda1d" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:70]}')
PY
  ok $rc
done
echo "[$(date +%T)] memset diagnosis"
PDVC_ZERO_MEMSET=1 timeout -k 10 300 python -u tools/diag_memset_graph.py $O/memset > $O/memset.log 2>&1; rc=$?
grep -v "^replay [02]" $O/memset.log | tail -60; ok $rc
echo "[$(date +%T)] done"
