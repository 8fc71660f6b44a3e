#!/bin/bash
# Round-4 closing GPU pass: full GPU suite + smoke, the bench line of every BASELINE config, the ragged stream, and
# rocprof kernel stats of the headline bench.  Each step under its own limit; stop at the first failure.
#     TAG=r04f bash tools/r04_final.sh
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04f}; mkdir -p $O
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
run yc2_bf16 --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin
run ragged --stream ragged --no-cpu-baseline --no-gemm-roofline --no-dropin
run yc2_newmodel --workload yc2_newmodel --no-cpu-baseline --no-dropin
run anet_c3d --workload anet_c3d --no-cpu-baseline --no-dropin
run eval --mode eval --videos-per-gpu 256 --steps 3 --warmup 1 --no-cpu-baseline
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -8 $O/prof_summary.txt; fi
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
if [ -n "$kt" ]; then python tools/profsteps.py "$kt" 45 > $O/prof_steps.txt; head -4 $O/prof_steps.txt; fi
ok $rc
echo "[$(date +%T)] done"
