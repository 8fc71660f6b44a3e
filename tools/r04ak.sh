#!/bin/bash
# round-4 GPU pass AK: relu-dropout kernels with 4 element groups per lane in flight (PDVC_FFN_U, default on):
# parity of both forms, then the headline A/B and per-kernel times
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ak; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for v in 4 1; do
  echo "[$(date +%T)] ffn parity PDVC_FFN_U=$v"
  PDVC_FFN_U=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_ffn.py tests/test_gpu_bf16.py > $O/ffn$v.log 2>&1; rc=$?; tail -1 $O/ffn$v.log; ok $rc
done
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],2))" $1; }
for v in 4 1 4 1; do
  echo "[$(date +%T)] anet_tsp PDVC_FFN_U=$v"
  PDVC_FFN_U=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-dropin --no-gemm-roofline \
    > $O/anet_$v.json 2> $O/anet_$v.err; rc=$?; ok $rc; show $O/anet_$v.json
done
for v in 4 1; do
  PDVC_FFN_U=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- \
    python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/prof$v.json \
    2> $O/prof$v.err; rc=$?; ok $rc
done
echo done
