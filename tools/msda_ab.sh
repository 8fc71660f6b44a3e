#!/bin/bash
# MSDA backward A/B on the GPU box: parity of the MSDA op tests under both backward-query kernels, then kernel
# timings (tools/kbench.py) and a rocprofv3 kernel split, old (PDVC_MSDA_BWDQ=0) vs new.  Usage: bash tools/msda_ab.sh TAG
set -o pipefail
TAG=${1:-msda_ab}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py tests/test_gpu_model.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -1 "$OUT/pytest_new.log"
for v in ${ABVALS:-0 1}; do
  env ${ABVAR:-PDVC_MSDA_BWDQ}=$v timeout -k 10 200 python -u tools/kbench.py --videos ${VIDEOS:-256} > "$OUT/kbench_$v.txt" 2>&1 \
      || { tail -20 "$OUT/kbench_$v.txt"; exit 1; }
  echo "${ABVAR:-PDVC_MSDA_BWDQ}=$v"; grep -v amdgpu.ids "$OUT/kbench_$v.txt"
done
for v in ${ABVALS:-0 1}; do
  env ${ABVAR:-PDVC_MSDA_BWDQ}=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o run \
      -- python -u tools/kbench.py --videos ${VIDEOS:-256} --reps 5 > "$OUT/prof_$v.log" 2>&1 || { tail -20 "$OUT/prof_$v.log"; exit 1; }
  ks=$(find "$OUT/prof_$v" -name "*kernel_stats.csv" | head -1)
  echo "${ABVAR:-PDVC_MSDA_BWDQ}=$v kernels:"; python tools/profsum.py "$ks" 0 8
done
