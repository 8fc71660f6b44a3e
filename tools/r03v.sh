# round-3 GPU pass: packed in_proj and box refinement (module tests + model/batch fixtures), the memset ordering
# probe, step-graph node census at 16 and 1024 videos, headline bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03v}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; ok $rc
echo "[$(date +%T)] memset probe 2"
timeout -k 10 60 ./tools/memset_graph_probe2.bin > $O/memset_probe2.txt 2>&1; rc=$?; cat $O/memset_probe2.txt; ok $rc
echo "[$(date +%T)] node census"
for v in 16 1024; do
  timeout -k 10 300 python -u tools/diag_graph_nodes.py --videos $v > $O/nodes_$v.txt 2>&1; rc=$?; grep "^videos" $O/nodes_$v.txt; ok $rc
done
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 300 $O/bench.json; tail -2 $O/bench.err; ok $rc
echo "[$(date +%T)] done"
