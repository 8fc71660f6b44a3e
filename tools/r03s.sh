# round-3 GPU pass: streaming MHA backward -- module tests (both backward kernels vs float64 and each other), backward
# timing, MSDA op tests, rocprof kernel stats of the headline bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03s}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_ops.py tests/test_gpu_batch.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; ok $rc
timeout -k 10 200 python -u tools/mha_bwd_bench.py > $O/mha_bwd.txt 2>&1; rc=$?; grep BWD2 $O/mha_bwd.txt; ok $rc
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -30 $O/prof_summary.txt; fi
tail -c 400 $O/prof_bench.json
ok $rc
echo "[$(date +%T)] done"
