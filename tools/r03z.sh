# round-3 GPU pass: replayed step graph vs the eager step at bench scale (dropout off)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03z}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
for v in 16 1024; do
  timeout -k 10 400 python -u tools/check_graph_replays.py --videos $v > $O/replays_$v.txt 2>&1; rc=$?
  grep -E "^videos|^replay|Error|error" $O/replays_$v.txt | head -8; ok $rc
done
echo "[$(date +%T)] done"
