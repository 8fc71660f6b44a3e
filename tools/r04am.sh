#!/bin/bash
# round-4 GPU pass AM: the stride-2 conv's W0 tap as in-place strided batched GEMMs (PDVC_CONV_BMM, default on):
# parity (model-level suites), then the headline A/B
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04am; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] parity"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_groupnorm.py \
  tests/test_gpu_modules.py tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_bf16.py \
  tests/test_gpu_configs.py > $O/parity.log 2>&1; rc=$?; tail -1 $O/parity.log; ok $rc
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2))" $1; }
for v in 1 0 1 0; do
  echo "[$(date +%T)] anet_tsp PDVC_CONV_BMM=$v"
  PDVC_CONV_BMM=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_$v.json 2> $O/anet_$v.err; rc=$?; ok $rc; show $O/anet_$v.json
done
for v in 1 0; do
  echo "[$(date +%T)] yc2_bf16 PDVC_CONV_BMM=$v"
  PDVC_CONV_BMM=$v timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin \
    --no-gemm-roofline > $O/bf16_$v.json 2> $O/bf16_$v.err; rc=$?; ok $rc; show $O/bf16_$v.json
done
