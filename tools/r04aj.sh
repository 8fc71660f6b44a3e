#!/bin/bash
# round-4 GPU pass AJ: add-norm kernels with double-buffered row loads (PDVC_AN_PF, default on): parity of both forms,
# the model-level suites, then A/B of the headline and bf16 bench lines
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04aj; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for v in 1 0; do
  echo "[$(date +%T)] add-norm parity PDVC_AN_PF=$v"
  PDVC_AN_PF=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_addnorm.py > $O/an$v.log 2>&1; rc=$?; tail -1 $O/an$v.log; ok $rc
done
echo "[$(date +%T)] model-level suites"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_modules.py \
  tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_bf16.py tests/test_gpu_configs.py > $O/parity.log 2>&1
rc=$?; tail -1 $O/parity.log; ok $rc
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2))" $1; }
for v in 1 0 1 0; do
  echo "[$(date +%T)] anet_tsp PDVC_AN_PF=$v"
  PDVC_AN_PF=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_$v.json 2> $O/anet_$v.err; rc=$?; ok $rc; show $O/anet_$v.json
done
echo "[$(date +%T)] rocprof kernel stats, both forms"
for v in 1 0; do
  PDVC_AN_PF=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- \
    python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/prof$v.json \
    2> $O/prof$v.err; rc=$?; ok $rc
  ks=$(find $O/prof$v -name "*kernel_stats.csv" | head -1)
  grep -h "addnorm" "$ks" | cut -d, -f1-4 | cut -c1-160
done
