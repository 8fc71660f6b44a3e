#!/bin/bash
# round-4 GPU pass AD: the model-level suite alone with the fused caption backward (pass AC aborted inside the
# step-graph capture test), HIP errors logged
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ad; mkdir -p $O
AMD_LOG_LEVEL=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_model.py \
  > $O/model.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" $O/model.log | tail -30; exit $rc
