#!/bin/bash
# PMC passes over the MSDA kernels at the bench's encoder/decoder shapes (GPU box, repo root):
#     bash tools/msda_pmc.sh TAG [VIDEOS]
# one rocprofv3 run per counter set (hardware limits per pass), then tools/pmc_counters.py.
set -o pipefail
TAG=${1:-pmc}
V=${2:-256}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INST_LEVEL_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  echo "[$(date +%T)] pass $i: $set"
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "msda1d|mha_|relu_dropout|addnorm" --output-format csv \
      -d "$OUT/p$i" -- python -u tools/kbench.py --videos "$V" --reps 2 > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
python tools/pmc_counters.py "$OUT" > "$OUT/counters.txt" && cat "$OUT/counters.txt"
