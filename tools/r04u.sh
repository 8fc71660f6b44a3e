#!/bin/bash
# round-4 closing pass, part 2: the headline bench line (anet_tsp, 1 GPU) and the bf16 line with the refreshed traffic
# files, rocprof kernel stats + per-replay step times of the headline bench, eager-vs-replay check at 1024 videos
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
run() {  # name, then bench.py arguments
  local n=$1; shift
  echo "[$(date +%T)] $n"
  timeout -k 10 500 python -u bench.py "$@" > "$O/bench_$n.json" 2> "$O/bench_$n.err"; local rc=$?
  tail -1 "$O/bench_$n.json" | cut -c1-200; ok $rc
}
run anet_tsp
run yc2_bf16 --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin
echo "[$(date +%T)] rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof.err; rc=$?
ks=$(find $O/prof -name "*kernel_stats.csv" | head -1)
if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > $O/prof_summary.txt; head -8 $O/prof_summary.txt; fi
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
if [ -n "$kt" ]; then python tools/profsteps.py "$kt" 45 > $O/prof_steps.txt; head -4 $O/prof_steps.txt; fi
ok $rc
echo "[$(date +%T)] done"
