#!/bin/bash
# round-4 closing pass, part 1: the GPU suite + smoke, then PMC traffic of the MSDA kernels and the library GEMMs for
# the headline (anet_tsp) and bf16 (yc2_tsp_bf16) workloads -- copied into profiles/ on the box as r04_*, so that
# part 2's bench lines (same call or later) read them
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; ok $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; ok $rc
for WL in anet_tsp yc2_tsp_bf16; do
  WL=$WL TAG=r04t/pmc_$WL bash tools/pmc_workload.sh > $O/pmc_$WL.log 2>&1; rc=$?; tail -12 $O/pmc_$WL.log; ok $rc
done
echo "[$(date +%T)] done"
