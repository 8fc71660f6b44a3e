#!/bin/bash
# PMC passes over the gemm3 kernels (GPU box, repo root):  bash tools/gemm3_pmc.sh TAG [OPS]
# one rocprofv3 run per counter set, each under its own KILL timeout, then tools/pmc_counters.py.
set -o pipefail
TAG=${1:-g3pmc}
OPS=${2:-fwdp,wgrad}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export PDVC_GEMM3_NO_BLASLT=1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  echo "[$(date +%T)] pass $i: $set"
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "gemm3" --output-format csv \
      -d "$OUT/p$i" -- python -u tools/gemm3_bench.py --no-err --iters 2 --only "$OPS" --shapes 512x512 > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
python tools/pmc_counters.py "$OUT" > "$OUT/counters.txt" && cat "$OUT/counters.txt"
