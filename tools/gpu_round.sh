#!/bin/bash
# One GPU-box pass over the steps named on the command line, each under its own time limit; the script
# stops at the first failure.  Usage (repo root, GPU box):
#     bash tools/gpu_round.sh TAG [kbench] [tests] [bench] [gemm] [prof] [pmc]
#   kbench  MSDA kernel timings, per-query kernels (PDVC_MSDA_PYR=0) and default (whole-pyramid)
#   tests   pytest -m gpu + smoke()
#   bench   bench.py (the JSON line)
#   gemm    bench.py --gemm hip + tools/gemmbench.py
#   prof    rocprofv3 --kernel-trace --stats of bench.py, summarised by tools/profsum.py
#   pmc     FETCH_SIZE and WRITE_SIZE passes over the roofline kernel -> tools/pmc_traffic.py
# BENCH_ARGS (environment) is appended to the bench.py command lines of bench / prof (e.g. --workload ...).
set -o pipefail
TAG=${1:-r01}
shift
STEPS=" $* "
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
has() { [[ "$STEPS" == *" $1 "* ]]; }

if has kbench; then
  echo "[$(date +%T)] kbench"
  PDVC_MSDA_PYR=0 timeout -k 10 300 python -u tools/kbench.py > "$OUT/kbench_perquery.txt" 2>&1 \
      || { echo "kbench failed"; tail -30 "$OUT/kbench_perquery.txt"; exit 1; }
  timeout -k 10 300 python -u tools/kbench.py > "$OUT/kbench.txt" 2>&1 \
      || { echo "kbench failed"; tail -30 "$OUT/kbench.txt"; exit 1; }
  echo "per-query kernels:"; grep -v amdgpu.ids "$OUT/kbench_perquery.txt"
  echo "default:"; grep -v amdgpu.ids "$OUT/kbench.txt"
fi
if has tests; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then  # the per-query MSDA kernels (whole-pyramid ones off) against the oracle too
    PDVC_MSDA_PYR=0 PDVC_MSDA_G4=0 PDVC_MSDA_BWDQ=0 PDVC_MSDA_FWDBUF=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 \
        --timeout-method thread -k msda1d > "$OUT/pytest_gpu_perquery.log" 2>&1
    rc=$?
    tail -1 "$OUT/pytest_gpu_perquery.log"
  fi
  if [ $rc -eq 0 ]; then  # the buffer-load forward / dot backward-query kernels at the encoder shapes too
    PDVC_MSDA_PYR=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py -m gpu -x -q \
        --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_nopyr.log" 2>&1
    rc=$?
    tail -1 "$OUT/pytest_gpu_nopyr.log"
  fi
  tail -3 "$OUT/pytest_gpu.log"
  if [ $rc -ne 0 ]; then echo "pytest failed rc=$rc"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -30; exit $rc; fi
  echo "[$(date +%T)] smoke"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
if has bench; then
  echo "[$(date +%T)] bench"
  timeout -k 10 400 python -u bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
if has gemm; then
  echo "[$(date +%T)] bench --gemm hip"
  timeout -k 10 400 python -u bench.py --gemm hip --no-cpu-baseline > "$OUT/bench_gemm_hip.json" \
      2> "$OUT/bench_gemm_hip.err" || { echo "bench --gemm hip failed"; tail -30 "$OUT/bench_gemm_hip.err"; exit 1; }
  cat "$OUT/bench_gemm_hip.json"
  timeout -k 10 300 python -u tools/gemmbench.py > "$OUT/gemmbench.txt" 2>&1 \
      || { echo "gemmbench failed"; tail -20 "$OUT/gemmbench.txt"; exit 1; }
  cat "$OUT/gemmbench.txt"
fi
if has prof; then
  echo "[$(date +%T)] rocprofv3 kernel stats"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
      -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin $BENCH_ARGS > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
      || { echo "rocprof failed"; tail -30 "$OUT/prof.err"; exit 1; }
  ks=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
  if [ -n "$ks" ]; then python tools/profsum.py "$ks" 0 45 > "$OUT/prof_summary.txt"; cat "$OUT/prof_summary.txt"; fi
fi
if has pmc; then
  for c in FETCH_SIZE WRITE_SIZE; do
    d=fetch
    [ $c = WRITE_SIZE ] && d=write
    echo "[$(date +%T)] pmc $c"
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex msda1d_fwd --output-format csv \
        -d "$OUT/pmc/$d" -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        > "$OUT/pmc_$d.json" 2> "$OUT/pmc_$d.err" || { echo "pmc $c failed"; tail -20 "$OUT/pmc_$d.err"; exit 1; }
  done
  python tools/pmc_traffic.py "$OUT/pmc" msda1d_fwd "$OUT/msda1d_fwd_traffic.json"
fi
echo "[$(date +%T)] done"
