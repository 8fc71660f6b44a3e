# round-3 GPU pass: LDS-DMA pyramid forward (msda1d_fwd_pyr2_kernel) parity and A/B against the register-staged
# kernel, then the PMC traffic passes, the ragged-stream bench and the capacity step-graph test (tools/r03k.sh)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03l; mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
echo "[$(date +%T)] MSDA op tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q --timeout 120 --timeout-method thread -rf > $O/ops.log 2>&1; rc=$?
tail -6 $O/ops.log; ok $rc
for T in 512 256; do for n in 256 1024; do for d in 0 1; do
  PDVC_PYR_DMA=$d timeout -k 10 120 python -u tools/kbench.py --videos $n --reps 20 --T $T > $O/kb_T${T}_n${n}_dma$d.txt 2>&1; rc=$?
  echo "T=$T n=$n dma=$d: $(grep encoder $O/kb_T${T}_n${n}_dma$d.txt)"; ok $rc
done; done; done
bash tools/r03k.sh
