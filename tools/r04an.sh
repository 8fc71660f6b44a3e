#!/bin/bash
# round-4 GPU pass AN: the fused caption backward re-forming its tanh rows from the U corners (PDVC_CAP_BWD_KEEP=0,
# 168 registers: three waves per SIMD) against holding them (252: two waves)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04an; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for v in 0 1; do
  echo "[$(date +%T)] ABI parity PDVC_CAP_BWD_KEEP=$v"
  PDVC_CAP_BWD_KEEP=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_ops.py -k cap_softattn > $O/abi$v.log 2>&1; rc=$?; tail -1 $O/abi$v.log; ok $rc
done
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2), {k: (v['launches'], round(v['avg_us'],1)) for k, v in d['kernels'].items() if 'softattn' in k})" $1; }
for v in 0 1 0 1; do
  echo "[$(date +%T)] anet_tsp PDVC_CAP_BWD_KEEP=$v"
  PDVC_CAP_BWD_KEEP=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_$v.json 2> $O/anet_$v.err; rc=$?; ok $rc; show $O/anet_$v.json
done
for v in 0 1; do
  echo "[$(date +%T)] yc2_bf16 PDVC_CAP_BWD_KEEP=$v"
  PDVC_CAP_BWD_KEEP=$v timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin \
    --no-gemm-roofline > $O/bf16_$v.json 2> $O/bf16_$v.err; rc=$?; ok $rc; show $O/bf16_$v.json
done
