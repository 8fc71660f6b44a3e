# round-3 GPU pass: adversarial memset ordering probe (slow writer ahead of the memset) and the memset nodes of the
# 1024-video step graph with the kernels on either side
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03w}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
timeout -k 10 120 ./tools/memset_graph_probe2.bin > $O/memset_probe2.txt 2>&1; rc=$?; cat $O/memset_probe2.txt; ok $rc
timeout -k 10 300 python -u tools/diag_graph_nodes.py --videos 1024 > $O/nodes_1024.txt 2>&1; rc=$?; grep -v Warning $O/nodes_1024.txt | tail -60; ok $rc
echo "[$(date +%T)] done"
