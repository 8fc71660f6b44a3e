# round-3 GPU pass B: the tests that failed in pass A, the bf16 cast census, bench lines (headline, cfg-2 bf16,
# ragged stream graphed and eager), the memset-in-graph diagnosis, rocprof kernel stats; last, the capacity
# capture diagnosis after an eager step (native backtrace on a segfault).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py tests/test_gpu_configs.py tests/test_gpu_bf16.py tests/test_gpu_attn_block.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; ok $rc
echo "[$(date +%T)] bf16 casts"
PDVC_CAST_LOG=1 timeout -k 10 200 python -u tools/diag_bf16_casts.py --videos 128 > $O/casts.txt 2>&1; rc=$?
head -45 $O/casts.txt; ok $rc
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 300 $O/bench.json; tail -2 $O/bench.err; ok $rc
echo "[$(date +%T)] bench yc2_tsp_bf16"
timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16.json 2> $O/bench_bf16.err; rc=$?
tail -c 300 $O/bench_bf16.json; tail -2 $O/bench_bf16.err; ok $rc
echo "[$(date +%T)] bench ragged (graph)"
timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged.json 2> $O/bench_ragged.err; rc=$?
tail -c 300 $O/bench_ragged.json; tail -3 $O/bench_ragged.err; ok $rc
echo "[$(date +%T)] bench ragged (eager)"
timeout -k 10 500 python -u bench.py --stream ragged --graph none --steps 4 --warmup 1 --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged_eager.json 2> $O/bench_ragged_eager.err; rc=$?
tail -c 300 $O/bench_ragged_eager.json; tail -3 $O/bench_ragged_eager.err; ok $rc
echo "[$(date +%T)] memset diagnosis"
PDVC_ZERO_MEMSET=1 timeout -k 10 200 python -u tools/diag_memset_graph.py $O/memset > $O/memset.log 2>&1; rc=$?
tail -30 $O/memset.log; ok $rc
echo "[$(date +%T)] capacity capture after an eager step"
timeout -k 10 200 python -u tools/diag_capacity_capture.py --eager-first --release --no-sync-debug > $O/cap_diag.log 2>&1; rc=$?
grep -v "^    " $O/cap_diag.log | tail -60; ok $rc
echo "[$(date +%T)] done"
