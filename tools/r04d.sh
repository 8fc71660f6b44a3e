#!/bin/bash
# round-4 GPU pass D: scale test, headline bench line, ragged stream with / without packed caption tokens
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
echo "[$(date +%T)] scale test"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_step_graph_scale.py > $O/scale_test.log 2>&1 || { tail -30 $O/scale_test.log; exit 1; }
tail -2 $O/scale_test.log
echo "[$(date +%T)] headline bench"
timeout -k 10 500 python -u bench.py > $O/bench_anet_tsp.json 2> $O/bench_anet_tsp.err || { tail -20 $O/bench_anet_tsp.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_anet_tsp.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gather']['frac'], d['roofline_gather_bwd']['frac'])"
grep -c "AccumulateGrad node's stream" $O/bench_anet_tsp.err || true
for pk in 1 0; do
  echo "[$(date +%T)] ragged bench PDVC_TOKENS_PACKED=$pk"
  PDVC_TOKENS_PACKED=$pk timeout -k 10 500 python -u bench.py --stream ragged --no-cpu-baseline --no-gemm-roofline > $O/bench_ragged_pk$pk.json 2> $O/bench_ragged_pk$pk.err || { tail -20 $O/bench_ragged_pk$pk.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_ragged_pk$pk.json')); print(d['value'], d['ms_per_step'], d['config']['stream'])"
done
