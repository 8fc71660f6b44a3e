#!/bin/bash
# round-4 GPU pass I: backward-query interleave (PDVC_BQ_QU) A/B and PMC counters of the encoder MSDA backward kernels
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
for qu in 1 3 5 1; do
  echo "[$(date +%T)] kbench PDVC_BQ_QU=$qu"
  PDVC_BQ_QU=$qu timeout -k 10 120 python -u tools/kbench.py --videos 1024 --reps 4 2>&1 | grep -E "^encoder" | tee -a $O/kbench_qu$qu.log || exit 1
done
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INST_LEVEL_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i + 1))
  echo "[$(date +%T)] pmc pass $i"
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "msda1d_bwd" --output-format csv \
      -d "$O/p$i" -- python -u tools/kbench.py --videos 1024 --reps 2 > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$O/p$i.log"; exit 1; }
done
python tools/pmc_counters.py "$O" > "$O/counters.txt" && cat "$O/counters.txt"
