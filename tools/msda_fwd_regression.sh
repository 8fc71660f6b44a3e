#!/bin/bash
# the unchanged encoder MSDA forward ran ~14 % slower inside the round-5 step.  The same
# kernels measured in three settings with one counter set each (effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration,
# MI355X_MICROARCH.md DVFS; duration from the same pass's kernel trace):
#   standalone  tools/kbench.py --videos 1024 (random projections)
#   step        bench.py eager steps (--graph none), its inputs from gemm3p (the default)
#   step_nog3   the same with PDVC_GEMM3=0 (the projections on hipBLASLt, as round 4)
# then tools/msda_fwd_regression.py summarises.   bash tools/msda_fwd_regression.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
KR="msda1d_fwd_pyr2|msda1d_bwd_query_pyr|msda1d_bwd_value|gemm3p_kernel"
STEP="python -u bench.py --steps 2 --warmup 1 --graph none --no-cpu-baseline --no-dropin --no-gemm-roofline"
for arm in standalone step step_nog3; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then CT="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS"
    else CT="FETCH_SIZE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; fi
    echo "[$(date +%T)] $arm pass $pass"
    case $arm in
      standalone) timeout -s KILL 240 rocprofv3 --pmc $CT --kernel-trace --kernel-include-regex "$KR" --output-format csv \
                    -d "$OUT/$arm/p$pass" -- python -u tools/kbench.py --videos 1024 --reps 3 > "$OUT/$arm.p$pass.log" 2>&1 ;;
      step) timeout -s KILL 300 rocprofv3 --pmc $CT --kernel-trace --kernel-include-regex "$KR" --output-format csv \
                    -d "$OUT/$arm/p$pass" -- $STEP > "$OUT/$arm.p$pass.log" 2>&1 ;;
      step_nog3) PDVC_GEMM3=0 timeout -s KILL 300 rocprofv3 --pmc $CT --kernel-trace --kernel-include-regex "$KR" \
                    --output-format csv -d "$OUT/$arm/p$pass" -- $STEP > "$OUT/$arm.p$pass.log" 2>&1 ;;
    esac
    rc=$?; [ $rc -ne 0 ] && { echo "$arm pass $pass failed ($rc)"; tail -20 "$OUT/$arm.p$pass.log"; exit 1; }
  done
done
python tools/msda_fwd_regression.py "$OUT" | tee "$OUT/summary.txt"
