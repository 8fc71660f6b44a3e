cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/ops.log 2>&1; rc=$?
tail -15 $O/ops.log
if [ $rc -gt 1 ]; then echo "ops rc=$rc: stop"; exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf --ignore=tests/test_gpu_ops.py > $O/rest.log 2>&1; rc=$?
tail -40 $O/rest.log
exit $rc
