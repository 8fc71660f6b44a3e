# round-3 PMC traffic passes (one rocprofv3 --pmc run per counter, kernel-trace allowed beside it):
# MSDA forward, MSDA backward (query + value kernels) and the library GEMMs of an eager step, headline workload
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O
for k in msda1d_fwd msda1d_bwd Cijk_; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=fetch; [ $c = WRITE_SIZE ] && d=write
    echo "[$(date +%T)] pmc $k $c"
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex "$k" --output-format csv -d "$O/$k/$d" \
        -- python -u bench.py --steps 2 --warmup 1 --graph none --no-cpu-baseline --no-dropin --no-gemm-roofline \
        > "$O/${k}_$d.json" 2> "$O/${k}_$d.err" || { echo "pmc $k $c failed"; tail -20 "$O/${k}_$d.err"; exit 1; }
  done
done
python tools/pmc_traffic.py "$O/msda1d_fwd" msda1d_fwd "$O/msda1d_fwd_traffic.json" | tail -3
python tools/pmc_traffic.py "$O/msda1d_bwd" msda1d_bwd_query "$O/msda1d_bwd_query_traffic.json" | tail -3
python tools/pmc_traffic.py "$O/msda1d_bwd" msda1d_bwd_value "$O/msda1d_bwd_value_traffic.json" | tail -3
python tools/pmc_gemm.py "$O/Cijk_" 3 "$O/gemm_traffic.json"
echo "[$(date +%T)] done"
