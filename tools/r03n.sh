# round-3 GPU pass: the value-gradient kernel without the bf16 store spill -- MSDA/bf16 tests, kernel timing,
# bench lines (headline, cfg-2 bf16), the memset-in-graph diagnosis, rocprof kernel stats of the headline bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03n; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16.py tests/test_gpu_attn_block.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log; ok $rc
for T in 512 256; do
  timeout -k 10 120 python -u tools/kbench.py --videos 1024 --reps 10 --T $T > $O/kb_T$T.txt 2>&1; rc=$?
  echo "T=$T: $(grep -E 'encoder|decoder' $O/kb_T$T.txt | tr '\n' ' ')"; ok $rc
done
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 200 $O/bench.json; tail -2 $O/bench.err; ok $rc
echo "[$(date +%T)] bench yc2_tsp_bf16"
timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16.json 2> $O/bench_bf16.err; rc=$?
tail -c 200 $O/bench_bf16.json; tail -2 $O/bench_bf16.err; ok $rc
echo "[$(date +%T)] memset diagnosis"
PDVC_ZERO_MEMSET=1 timeout -k 10 200 python -u tools/diag_memset_graph.py $O/memset > $O/memset.log 2>&1; rc=$?
grep -v "^    " $O/memset.log | tail -40; ok $rc
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -24 $O/prof_summary.txt; fi
ok $rc
echo "[$(date +%T)] done"
