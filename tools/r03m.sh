# round-3 GPU pass: full GPU suite, bf16 cast census, bench lines (headline, cfg-2 bf16, ragged stream graphed and
# eager), rocprof kernel stats of the headline bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03m; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -8 $O/tests.log; ok $rc
for qu in 1 3 5; do
  PDVC_BQ_QU=$qu timeout -k 10 120 python -u tools/kbench.py --videos 1024 --reps 10 > $O/kb_qu$qu.txt 2>&1; rc=$?
  echo "QU=$qu: $(grep encoder $O/kb_qu$qu.txt)"; ok $rc
done
PDVC_BQ_QU=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/ops_qu5.log 2>&1; rc=$?
tail -3 $O/ops_qu5.log; ok $rc
echo "[$(date +%T)] bf16 casts"
PDVC_CAST_LOG=1 timeout -k 10 200 python -u tools/diag_bf16_casts.py --videos 128 > $O/casts.txt 2>&1; rc=$?
head -30 $O/casts.txt; ok $rc
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 300 $O/bench.json; tail -2 $O/bench.err; ok $rc
echo "[$(date +%T)] bench yc2_tsp_bf16"
timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16.json 2> $O/bench_bf16.err; rc=$?
tail -c 300 $O/bench_bf16.json; tail -2 $O/bench_bf16.err; ok $rc
echo "[$(date +%T)] bench ragged (graph)"
timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged.json 2> $O/bench_ragged.err; rc=$?
tail -c 200 $O/bench_ragged.json; ok $rc
echo "[$(date +%T)] bench ragged (eager)"
timeout -k 10 500 python -u bench.py --stream ragged --graph none --steps 4 --warmup 1 --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged_eager.json 2> $O/bench_ragged_eager.err; rc=$?
tail -c 200 $O/bench_ragged_eager.json; ok $rc
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -30 $O/prof_summary.txt; fi
ok $rc
echo "[$(date +%T)] done"
