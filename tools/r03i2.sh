# round-3 GPU pass: backward-query pyramid kernel staged by LDS-DMA -- MSDA op tests, per-kernel times (two
# kbench runs), a short headline bench (graph node counts in the line)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03i2}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; ok $rc
for i in 1 2; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kp$i -o run -- python -u tools/kbench.py --videos 1024 --reps 5 > $O/kbp$i.txt 2>&1; rc=$?
ks=$(find $O/kp$i -name "*kernel_stats.csv" | head -1)
python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "msda1d" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:70]}')
PY
ok $rc
done
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/bench.json 2> $O/bench.err; rc=$?
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config'].get('graph_nodes_per_replay'))"; ok $rc
