# diagnosis of the capacity StepGraph capture segfault, then the rest of the GPU suite without that test
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 180 python -u tools/diag_capacity_capture.py > $O/diag.log 2>&1; rc=$?
grep -v "^  File\|^    " $O/diag.log | tail -30; echo "diag rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf \
    --deselect tests/test_gpu_batch.py::test_capacity_step_graph_follows_a_ragged_stream > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log; exit $rc
