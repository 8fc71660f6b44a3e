# round-3 GPU pass: value-gradient zero-fill moved ahead of the scan -- MSDA op tests, per-kernel times
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c2}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; ok $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kp -o run -- python -u tools/kbench.py --videos 1024 --reps 5 > $O/kbp.txt 2>&1; rc=$?
ks=$(find $O/kp -name "*kernel_stats.csv" | head -1)
python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "msda1d" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:70]}')
PY
ok $rc
