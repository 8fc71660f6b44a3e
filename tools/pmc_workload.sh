# PMC traffic passes (one rocprofv3 --pmc run per counter) of the MSDA forward / backward kernels and the library
# GEMMs of one bench workload:  WL=yc2_tsp_bf16 TAG=r03u bash tools/pmc_workload.sh
# -> gpurun_out/$TAG/<kernel>_traffic_$WL.json (copy into profiles/ as r03_<kernel>_traffic_$WL.json)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
WL=${WL:-yc2_tsp_bf16}
O=gpurun_out/${TAG:-pmc_$WL}; mkdir -p $O
for k in msda1d_fwd msda1d_bwd Cijk_ gemm3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=fetch; [ $c = WRITE_SIZE ] && d=write
    echo "[$(date +%T)] pmc $k $c"
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex "$k" --output-format csv -d "$O/$k/$d" \
        -- python -u bench.py --workload $WL --steps 2 --warmup 1 --graph none --no-cpu-baseline --no-dropin \
        --no-gemm-roofline > "$O/${k}_$d.json" 2> "$O/${k}_$d.err" || { echo "pmc $k $c failed"; tail -20 "$O/${k}_$d.err"; exit 1; }
  done
done
python tools/pmc_traffic.py "$O/msda1d_fwd" msda1d_fwd_pyr "$O/msda1d_fwd_pyr_traffic_$WL.json" | tail -2
python tools/pmc_traffic.py "$O/msda1d_fwd" msda1d_fwd_buf "$O/msda1d_fwd_buf_traffic_$WL.json" | tail -2
python tools/pmc_traffic.py "$O/msda1d_fwd" msda1d_fwd_win "$O/msda1d_fwd_win_traffic_$WL.json" | tail -2
python tools/pmc_traffic.py "$O/msda1d_bwd" msda1d_bwd_query_pyr "$O/msda1d_bwd_query_pyr_traffic_$WL.json" | tail -2
python tools/pmc_traffic.py "$O/msda1d_bwd" msda1d_bwd_query_dot "$O/msda1d_bwd_query_dot_traffic_$WL.json" --largest-grid | tail -2
python tools/pmc_traffic.py "$O/msda1d_bwd" msda1d_bwd_value "$O/msda1d_bwd_value_enc_traffic_$WL.json" --large-launches | tail -2
python tools/pmc_gemm.py "$O/Cijk_" 3 "$O/gemm_traffic_$WL.json" | tail -3
python tools/pmc_gemm.py "$O/gemm3" 3 "$O/gemm3_traffic_$WL.json" "gemm3p?_kernel|gemm3w_kernel" | tail -3
echo "[$(date +%T)] done"
