#!/bin/bash
# round-4 GPU pass G: word gates over the loss-carrying tokens -- caption/model tests, ragged bench, its replay profile
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_batch_gt.py \
    tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_bf16.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "[$(date +%T)] ragged bench"
timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin > $O/bench_ragged.json 2> $O/bench_ragged.err || { tail -20 $O/bench_ragged.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_ragged.json')); print(d['value'], d['ms_per_step'])"
echo "[$(date +%T)] ragged stream under rocprofv3"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_rag -o rag -- python -u bench.py --stream ragged --steps 6 --warmup 2 --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/prof_rag.json 2> $O/prof_rag.err || { tail -20 $O/prof_rag.err; exit 1; }
kt=$(find $O/prof_rag -name "*kernel_trace.csv" | head -1); python tools/profsteps.py "$kt" 45 > $O/prof_rag_steps.txt; head -24 $O/prof_rag_steps.txt
