#!/bin/bash
# round-4 GPU pass AC: the fused caption step backward (pdvc_cap_softattn_backward_f32)
# (PDVC_CAP_FUSED_BWD, default on; the forward then skips the samples and att): parity (ABI test + the model-level suites), then A/B of the headline and bf16 bench lines
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ac; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] fused-step ABI parity"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
  -k cap_softattn > $O/abi.log 2>&1; rc=$?; tail -2 $O/abi.log; ok $rc
echo "[$(date +%T)] parity"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
  tests/test_gpu_modules.py tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_bf16.py \
  tests/test_gpu_configs.py > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; ok $rc
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2), {k: (v['launches'], round(v['avg_us'],1)) for k, v in d['kernels'].items() if 'cap' in k or 'softattn' in k})" $1; }
for v in 1 0 1 0; do
  echo "[$(date +%T)] anet_tsp PDVC_CAP_FUSED_BWD=$v"
  PDVC_CAP_FUSED_BWD=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_d$v.json 2> $O/anet_d$v.err; rc=$?; ok $rc; show $O/anet_d$v.json
done
for v in 1 0; do
  echo "[$(date +%T)] yc2_bf16 PDVC_CAP_FUSED_BWD=$v"
  PDVC_CAP_FUSED_BWD=$v timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin \
    --no-gemm-roofline > $O/bf16_d$v.json 2> $O/bf16_d$v.err; rc=$?; ok $rc; show $O/bf16_d$v.json
done
