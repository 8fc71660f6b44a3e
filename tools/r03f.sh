# round-3 GPU pass: tests (every failure listed), pyramid-forward ablations, bench lines (default, ragged stream
# graphed and eager), the memset-in-graph diagnosis, rocprof kernel stats.  A step that crashes, aborts or times
# out (exit > 1) ends the script; a Python failure (exit 1) is recorded and the next step runs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03f; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; ok $rc
for a in 0 1 2 3; do
  PDVC_PYR_ABLATE=$a timeout -k 10 120 python -u tools/kbench.py --videos 256 --reps 20 > $O/kb_$a.txt 2>&1; rc=$?
  grep -E "encoder|decoder" $O/kb_$a.txt; ok $rc
done
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 600 $O/bench.json; ok $rc
echo "[$(date +%T)] bench ragged (graph)"
timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline > $O/bench_ragged.json 2> $O/bench_ragged.err; rc=$?
tail -c 400 $O/bench_ragged.json; tail -3 $O/bench_ragged.err; ok $rc
echo "[$(date +%T)] bench ragged (eager)"
timeout -k 10 500 python -u bench.py --stream ragged --graph none --steps 4 --warmup 1 --no-cpu-baseline --no-gemm-roofline > $O/bench_ragged_eager.json 2> $O/bench_ragged_eager.err; rc=$?
tail -c 400 $O/bench_ragged_eager.json; tail -3 $O/bench_ragged_eager.err; ok $rc
echo "[$(date +%T)] memset diagnosis"
PDVC_ZERO_MEMSET=1 timeout -k 10 200 python -u tools/diag_memset_graph.py $O/memset > $O/memset.log 2>&1; rc=$?
tail -40 $O/memset.log; ok $rc
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -30 $O/prof_summary.txt; fi
ok $rc
echo "[$(date +%T)] done"
