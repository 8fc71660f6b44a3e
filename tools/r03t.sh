# round-3 GPU pass: native set criterion -- its parity tests against the torch form, the model/batch fixtures,
# full GPU suite, rocprof kernel stats + launch count of the headline bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03t}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] setcrit tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_setcrit.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests_setcrit.log 2>&1; rc=$?
tail -15 $O/tests_setcrit.log; ok $rc
echo "[$(date +%T)] full suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -6 $O/tests.log; ok $rc
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -12 $O/prof_summary.txt; fi
tail -c 300 $O/prof_bench.json
ok $rc
echo "[$(date +%T)] opparents"
timeout -k 10 300 python -u tools/opparents.py --videos 256 --top 60 > $O/opparents.txt 2>&1; rc=$?
grep -A40 "ops per owner" $O/opparents.txt | head -30; ok $rc
echo "[$(date +%T)] done"
