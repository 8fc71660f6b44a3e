#!/bin/bash
# round-4 GPU pass X: the bf16 mixed-output GEMM TunableOp probe, then pass W (caption gather XCD order A/B)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out/r04v
echo "[$(date +%T)] bf16 TunableOp probe"
timeout -k 10 400 python -u tools/bf16_tunable_probe.py --out gpurun_out/r04v/bf16_tunable.csv > gpurun_out/r04v/probe.log 2>&1
rc=$?; tail -20 gpurun_out/r04v/probe.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04w.sh
