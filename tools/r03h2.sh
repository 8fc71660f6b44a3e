# round-3 GPU pass: the step's GEMM table by shape (tools/gemm_table.py, 256 videos)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03h2}; mkdir -p $O
timeout -k 10 500 python -u tools/gemm_table.py --videos 256 > $O/gemm_table.txt 2>&1; rc=$?
tail -5 $O/gemm_table.txt; exit $rc
