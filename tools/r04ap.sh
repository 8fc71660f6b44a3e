#!/bin/bash
# round-4 GPU pass AP: rank-1 caption sample gradients (PDVC_CAP_RANK1, default on): the fused backward no longer
# writes p_k * dres 16 times per row; the value-gradient pass forms it.  Parity (ABI + model-level), then A/B
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ap; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] ABI parity"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
  -k "cap_value_grad_rank1 or cap_softattn" > $O/abi.log 2>&1; rc=$?; tail -1 $O/abi.log; ok $rc
echo "[$(date +%T)] model-level suites"
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_modules.py \
  tests/test_gpu_model.py tests/test_gpu_batch.py tests/test_gpu_bf16.py tests/test_gpu_configs.py > $O/parity.log 2>&1
rc=$?; tail -1 $O/parity.log; ok $rc
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2), {k: (v['launches'], round(v['avg_us'],1)) for k, v in d['kernels'].items() if 'softattn' in k})" $1; }
for v in 1 0 1 0; do
  echo "[$(date +%T)] anet_tsp PDVC_CAP_RANK1=$v"
  PDVC_CAP_RANK1=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_$v.json 2> $O/anet_$v.err; rc=$?; ok $rc; show $O/anet_$v.json
done
for v in 1 0; do
  echo "[$(date +%T)] yc2_bf16 PDVC_CAP_RANK1=$v"
  PDVC_CAP_RANK1=$v timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin \
    --no-gemm-roofline > $O/bf16_$v.json 2> $O/bf16_$v.err; rc=$?; ok $rc; show $O/bf16_$v.json
done
for v in 1 0; do
  PDVC_CAP_RANK1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- \
    python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/prof$v.json \
    2> $O/prof$v.err; rc=$?; ok $rc
done
echo done
