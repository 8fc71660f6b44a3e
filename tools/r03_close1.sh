#!/bin/bash
# Round-3 closing GPU pass, part 1: full GPU suite + smoke, graph replays vs eager, the headline bench line.
#     TAG=r03z bash tools/r03_close1.sh (part 2: tools/r03_close2.sh)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f}; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; ok $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; ok $rc
echo "[$(date +%T)] replays vs eager at 1024 videos"
timeout -k 10 400 python -u tools/check_graph_replays.py --videos 1024 > $O/replays_1024.txt 2>&1; rc=$?
grep -E "^videos|^second|^replay" $O/replays_1024.txt | cut -c1-200; ok $rc
run() {  # name, then bench.py arguments
  local n=$1; shift
  echo "[$(date +%T)] $n"
  timeout -k 10 500 python -u bench.py "$@" > "$O/bench_$n.json" 2> "$O/bench_$n.err"; local rc=$?
  tail -1 "$O/bench_$n.json" | cut -c1-160; ok $rc
}
run anet_tsp
echo "[$(date +%T)] done"
