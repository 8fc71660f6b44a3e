# round-3 GPU pass: memset capture probe 3 (node types, eager launches between replays)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/${TAG:-r03x}; mkdir -p $O
timeout -k 10 120 ./tools/memset_graph_probe3.bin > $O/memset_probe3.txt 2>&1; rc=$?; cat $O/memset_probe3.txt; exit $rc
