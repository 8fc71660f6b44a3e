# round-3 PMC traffic passes (one rocprofv3 --pmc run per counter; kernel trace only beside it) for the MSDA kernels
# and the library GEMMs of an eager step at the headline workload; the ragged-stream bench with the asynchronous
# StepGraph.load; last, the capacity step-graph test.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for k in msda1d Cijk_; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=fetch; [ $c = WRITE_SIZE ] && d=write
    echo "[$(date +%T)] pmc $k $c"
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$k" --output-format csv -d "$O/$k/$d" \
        -- python -u bench.py --steps 2 --warmup 1 --graph none --no-cpu-baseline --no-dropin --no-gemm-roofline \
        > "$O/${k}_$d.json" 2> "$O/${k}_$d.err"; rc=$?
    if [ $rc -ne 0 ]; then echo "pmc $k $c rc=$rc"; tail -20 "$O/${k}_$d.err"; exit $rc; fi
  done
done
python tools/pmc_traffic.py "$O/msda1d" msda1d_fwd_pyr "$O/msda1d_fwd_pyr_traffic.json" | tail -4
python tools/pmc_traffic.py "$O/msda1d" msda1d_fwd_buf "$O/msda1d_fwd_buf_traffic.json" | tail -4
python tools/pmc_traffic.py "$O/msda1d" msda1d_bwd_query_pyr "$O/msda1d_bwd_query_pyr_traffic.json" | tail -4
python tools/pmc_traffic.py "$O/msda1d" msda1d_bwd_value "$O/msda1d_bwd_value_enc_traffic.json" --largest-grid | tail -6
python tools/pmc_gemm.py "$O/Cijk_" 3 "$O/gemm_traffic.json" | tail -12
echo "[$(date +%T)] bench ragged (graph, async load)"
timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged.json 2> $O/bench_ragged.err; rc=$?
tail -c 300 $O/bench_ragged.json; tail -3 $O/bench_ragged.err; ok $rc
echo "[$(date +%T)] capacity step graph test"
timeout -k 10 200 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_bf16.py -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; ok $rc
echo "[$(date +%T)] done"
