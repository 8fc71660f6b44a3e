#!/bin/bash
# round-4 GPU pass W: XCD-aware wave order of the caption gather kernels (PDVC_CAP_XCD, default on): parity, then
# A/B of the headline and bf16 bench lines (their per-launch cap_gather times)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] parity"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_modules.py \
  tests/test_gpu_model.py tests/test_gpu_batch.py > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; ok $rc
for v in 1 0 1 0; do
  echo "[$(date +%T)] anet_tsp PDVC_CAP_XCD=$v"
  PDVC_CAP_XCD=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_x$v.json 2> $O/anet_x$v.err; rc=$?; ok $rc
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), {k: round(v['avg_us'],1) for k, v in d['kernels'].items() if 'cap' in k})" $O/anet_x$v.json
done
for v in 1 0; do
  echo "[$(date +%T)] yc2_bf16 PDVC_CAP_XCD=$v"
  PDVC_CAP_XCD=$v timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin \
    --no-gemm-roofline > $O/bf16_x$v.json 2> $O/bf16_x$v.err; rc=$?; ok $rc
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), {k: round(v['avg_us'],1) for k, v in d['kernels'].items() if 'cap' in k})" $O/bf16_x$v.json
done
