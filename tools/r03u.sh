# round-3 GPU pass: MSDA op tests (value-gradient flush change), graph node census (memcpy nodes vs .grad buffers),
# the memset-in-graph diagnosis with the node walk, PMC traffic passes of the cfg-2 bf16 workload
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03u}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; ok $rc
timeout -k 10 120 python -u tools/kbench.py --videos 1024 --reps 10 > $O/kb.txt 2>&1; rc=$?; grep -E "enc|dec" $O/kb.txt; ok $rc
echo "[$(date +%T)] node census"
timeout -k 10 300 python -u tools/diag_graph_nodes.py --videos 16 > $O/nodes.txt 2>&1; rc=$?
grep -v "^  rc" $O/nodes.txt | tail -8; grep "^  rc" $O/nodes.txt | head -12; ok $rc
echo "[$(date +%T)] memset diagnosis"
PDVC_ZERO_MEMSET=1 timeout -k 10 300 python -u tools/diag_memset_graph.py $O/memset > $O/memset.log 2>&1; rc=$?
grep -v "^replay [02]" $O/memset.log | tail -40; ok $rc
echo "[$(date +%T)] pmc yc2_tsp_bf16"
WL=yc2_tsp_bf16 TAG=${TAG:-r03u}/pmc timeout -k 10 700 bash tools/pmc_workload.sh; rc=$?; ok $rc
echo "[$(date +%T)] done"
