# pyramid-forward ablations at 256 videos (tools/kbench.py): default, no staging, no gather
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/r03d; mkdir -p $O
for a in 0 1 2 0; do
  PDVC_PYR_ABLATE=$a timeout -k 10 120 python -u tools/kbench.py --videos 256 --reps 20 > $O/kb_$a.txt 2>&1 || { cat $O/kb_$a.txt; exit 1; }
  grep encoder $O/kb_$a.txt
done
