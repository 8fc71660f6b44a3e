#!/bin/bash
# Decoder self-attention forward A/B on the GPU box: the module tests (MHA routes vs float64) with the lean forward,
# then rocprofv3 kernel stats of a short bench under PDVC_MHA_FWD2=0 and =1.  Usage: bash tools/mha_ab.sh TAG
set -o pipefail
TAG=${1:-mha_ab}
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_model.py tests/test_gpu_batch.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in 0 1; do
  PDVC_MHA_FWD2=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o run \
      -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gemm-roofline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
      || { tail -20 "$OUT/bench_$v.err"; exit 1; }
  ks=$(find "$OUT/prof_$v" -name "*kernel_stats.csv" | head -1)
  echo "FWD2=$v"; grep -E "mha_" "$ks" | cut -d, -f1-4 | cut -c1-160
done
