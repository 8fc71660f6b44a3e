# round-3 GPU pass: memset-node rewrite -- its tests, the whole GPU suite, replayed step vs eager at 16 and 1024 videos
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03a2}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_graph_memset.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests_memset.log 2>&1; rc=$?
tail -12 $O/tests_memset.log; ok $rc
for v in 16 1024; do
  timeout -k 10 400 python -u tools/check_graph_replays.py --videos $v > $O/replays_$v.txt 2>&1; rc=$?
  grep -E "^videos|^replay|Error|error" $O/replays_$v.txt | head -8; ok $rc
done
PDVC_GRAPH_MEMSETS=keep timeout -k 10 400 python -u tools/check_graph_replays.py --videos 1024 > $O/replays_1024_keep.txt 2>&1; rc=$?
grep -E "^videos|^replay" $O/replays_1024_keep.txt | head -8; ok $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; ok $rc
echo "[$(date +%T)] done"
