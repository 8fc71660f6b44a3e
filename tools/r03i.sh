# round-3 GPU pass A: tests (the capacity StepGraph test last, alone), the bf16 cast census, pyramid-forward
# ablations, bench lines (headline, cfg-2 bf16).  A step that crashes, aborts or times out (exit > 1) ends the
# script; a Python failure (exit 1) is recorded and the next step runs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03i; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
CAP=tests/test_gpu_batch.py::test_capacity_step_graph_follows_a_ragged_stream
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf --deselect $CAP > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; ok $rc
echo "[$(date +%T)] bf16 casts"
PDVC_CAST_LOG=1 timeout -k 10 200 python -u tools/diag_bf16_casts.py --videos 128 > $O/casts.txt 2>&1; rc=$?
head -40 $O/casts.txt; ok $rc
for a in 0 1 2 3; do
  PDVC_PYR_ABLATE=$a timeout -k 10 120 python -u tools/kbench.py --videos 256 --reps 20 > $O/kb_$a.txt 2>&1; rc=$?
  grep -E "encoder|decoder" $O/kb_$a.txt; ok $rc
done
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 600 $O/bench.json; ok $rc
echo "[$(date +%T)] bench yc2_tsp_bf16"
timeout -k 10 400 python -u bench.py --workload yc2_tsp_bf16 --no-cpu-baseline --no-dropin > $O/bench_bf16.json 2> $O/bench_bf16.err; rc=$?
tail -c 600 $O/bench_bf16.json; tail -3 $O/bench_bf16.err; ok $rc
echo "[$(date +%T)] capacity step graph test"
timeout -k 10 200 python -u -m pytest $CAP -q --timeout 120 --timeout-method thread -rf > $O/cap_test.log 2>&1; rc=$?
tail -15 $O/cap_test.log; ok $rc
echo "[$(date +%T)] done"
