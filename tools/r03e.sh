# round-3 GPU pass: the full GPU suite (no -x: every failure listed), then the pyramid-forward ablations
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log
if [ $rc -gt 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
for a in 0 1 2 3; do
  PDVC_PYR_ABLATE=$a timeout -k 10 120 python -u tools/kbench.py --videos 256 --reps 20 > $O/kb_$a.txt 2>&1 || { cat $O/kb_$a.txt; exit 1; }
  grep -E "encoder|decoder" $O/kb_$a.txt
done
exit $rc
