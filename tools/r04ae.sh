#!/bin/bash
# round-4 GPU pass AE: the fused caption step kernels with 1-sample chunks (160 / 252 registers) against 4-sample
# chunks (228 / 449): parity of both forms (ABI tests), then A/B of the headline and bf16 bench lines
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ae; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for c in 1 4; do
  echo "[$(date +%T)] ABI parity, chunk $c"
  PDVC_CAP_FWD_CH=$c PDVC_CAP_BWD_CH=$c timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_ops.py -k cap_softattn > $O/abi$c.log 2>&1; rc=$?; tail -1 $O/abi$c.log; ok $rc
done
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2), {k: (v['launches'], round(v['avg_us'],1)) for k, v in d['kernels'].items() if 'softattn' in k})" $1; }
for c in 1 4 1 4; do
  echo "[$(date +%T)] anet_tsp chunk $c"
  PDVC_CAP_FWD_CH=$c PDVC_CAP_BWD_CH=$c timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin \
    --no-gemm-roofline > $O/anet_c$c.json 2> $O/anet_c$c.err; rc=$?; ok $rc; show $O/anet_c$c.json
done
for c in 1 4; do
  echo "[$(date +%T)] yc2_bf16 chunk $c"
  PDVC_CAP_FWD_CH=$c PDVC_CAP_BWD_CH=$c timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 \
    --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/bf16_c$c.json 2> $O/bf16_c$c.err; rc=$?; ok $rc
  show $O/bf16_c$c.json
done
