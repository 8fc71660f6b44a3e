# round-3 GPU pass at the restored HEAD: full GPU suite + smoke, MSDA kernel timings, bench lines (headline,
# cfg-2 bf16, ragged stream), rocprof kernel stats of the headline bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03o}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -8 $O/tests.log; ok $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; ok $rc
for T in 512 256; do
  timeout -k 10 120 python -u tools/kbench.py --videos 1024 --reps 10 --T $T > $O/kb_T$T.txt 2>&1; rc=$?
  echo "T=$T: $(grep -E 'encoder|decoder' $O/kb_T$T.txt | tr '\n' ' ')"; ok $rc
done
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 300 $O/bench.json; tail -2 $O/bench.err; ok $rc
echo "[$(date +%T)] bench yc2_tsp_bf16"
timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16.json 2> $O/bench_bf16.err; rc=$?
tail -c 300 $O/bench_bf16.json; tail -2 $O/bench_bf16.err; ok $rc
echo "[$(date +%T)] bench ragged (graph)"
timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged.json 2> $O/bench_ragged.err; rc=$?
tail -c 200 $O/bench_ragged.json; ok $rc
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -30 $O/prof_summary.txt; fi
ok $rc
echo "[$(date +%T)] done"
