cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_dp.py tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_ops.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r02b/pytest_new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r02b/pytest_new.log | grep -v PASSED | head -40
tail -3 gpurun_out/r02b/pytest_new.log
exit $rc
