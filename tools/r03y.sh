# round-3 GPU pass: backward-query prefetch (MSDA op tests, kernel timing) and the torch-memory memset capture probe
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03y}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
timeout -k 10 120 python -u tools/memset_torch_probe.py > $O/memset_torch.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/memset_torch.txt; ok $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; ok $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kp -o run -- python -u tools/kbench.py --videos 1024 --reps 5 > $O/kbp.txt 2>&1; rc=$?
grep -E "enc|dec" $O/kbp.txt
ks=$(find $O/kp -name "*kernel_stats.csv" | head -1)
python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "msda1d" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:70]}')
PY
ok $rc
echo "[$(date +%T)] done"
