#!/bin/bash
# round-4 GPU pass AH: the eval line again (the closing pass measured 1 368 videos/s against 1 463-1 537 before; the
# eval path's greedy step does not use the fused caption kernels), three runs, one with PDVC_CAP_FUSED=0
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ah; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for v in 1 0 1; do
  echo "[$(date +%T)] eval PDVC_CAP_FUSED=$v"
  PDVC_CAP_FUSED=$v timeout -k 10 300 python -u bench.py --mode eval --videos-per-gpu 256 --steps 3 --warmup 1 \
    --no-cpu-baseline > $O/eval_$v.json 2> $O/eval_$v.err; rc=$?; ok $rc; tail -1 $O/eval_$v.json | cut -c1-200
done
