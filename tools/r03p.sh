# round-3 GPU diagnosis pass: op attribution of one eager step (launch counts per autograd node / forward op),
# the memset-in-graph diagnosis (PDVC_ZERO_MEMSET=1: library zero-fills as hipMemsetAsync, graph DOT dump)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03p}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] opparents"
timeout -k 10 300 python -u tools/opparents.py --videos 256 --top 70 > $O/opparents.txt 2>&1; rc=$?
grep -A70 "ops per owner" $O/opparents.txt | head -50; ok $rc
echo "[$(date +%T)] memset diagnosis"
PDVC_ZERO_MEMSET=1 timeout -k 10 300 python -u tools/diag_memset_graph.py $O/memset > $O/memset.log 2>&1; rc=$?
grep -v "^    " $O/memset.log | tail -60; ok $rc
echo "[$(date +%T)] done"
