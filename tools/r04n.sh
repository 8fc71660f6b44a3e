#!/bin/bash
# round-4 GPU pass N: bf16 mode with the recurrence's per-step GEMMs on bf16 -- tests, then the cfg-2 line A/B
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py > $O/bf16_tests.log 2>&1 || { tail -40 $O/bf16_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/bf16_tests.log | tail -12
for r in 1 0; do
  echo "[$(date +%T)] yc2_tsp_bf16 PDVC_BF16_RECURRENCE=$r"
  PDVC_BF16_RECURRENCE=$r timeout -k 10 500 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16_r$r.json 2> $O/bench_bf16_r$r.err || { tail -20 $O/bench_bf16_r$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_bf16_r$r.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['gemm_device_ms_per_step'])"
done
