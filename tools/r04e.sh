#!/bin/bash
# round-4 GPU pass E: caption recurrence over live row ranges -- model tests, then the ragged bench A/B
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_batch_gt.py \
    tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_bf16.py tests/test_gpu_dp.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sr in 1 0; do
  echo "[$(date +%T)] ragged bench PDVC_STEP_RANGES=$sr"
  PDVC_STEP_RANGES=$sr timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged_sr$sr.json 2> $O/bench_ragged_sr$sr.err || { tail -20 $O/bench_ragged_sr$sr.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_ragged_sr$sr.json')); print(d['value'], d['ms_per_step'])"
done
echo "[$(date +%T)] long-pyramid ops tests"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "long_pyramids" > $O/ops_long.log 2>&1 || { tail -30 $O/ops_long.log; exit 1; }
tail -2 $O/ops_long.log
for w in 0 1; do
  echo "[$(date +%T)] kbench T=1024 PDVC_MSDA_WIN=$w"
  PDVC_MSDA_WIN=$w timeout -k 10 120 python -u tools/kbench.py --videos 512 --reps 4 --T 1024 2>&1 | grep -E "^(encoder|decoder)" | tee -a $O/kbench_T1024_win$w.log || exit 1
done
