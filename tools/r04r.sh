#!/bin/bash
# round-4 GPU pass R: the value walk with held-row stores (PDVC_VAL_DEFER) x walk depth (PDVC_VALUE_UG): parity of the
# new variants, then the encoder backward at 1024 videos per variant (kbench + rocprofv3 kernel stats); then pass Q's
# T = 1024 query-chunk and windowed-forward staging measurements
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
for v in "2 6 1" "2 4 0" "1 8 1"; do
  set -- $v
  echo "[$(date +%T)] parity PDVC_VAL_DEFER=$1 PDVC_VALUE_UG=$2 PDVC_BQ_PF=$3"
  PDVC_VAL_DEFER=$1 PDVC_VALUE_UG=$2 PDVC_BQ_PF=$3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_bf16.py > $O/parity_d$1u$2p$3.log 2>&1 || { tail -40 $O/parity_d$1u$2p$3.log; exit 1; }
  tail -1 $O/parity_d$1u$2p$3.log
done
for v in "0 0 0" "0 0 1" "0 6 0" "2 6 0" "2 4 0" "1 6 0" "2 6 1" "0 0 0" "2 6 1"; do
  set -- $v
  echo "[$(date +%T)] kbench PDVC_VAL_DEFER=$1 PDVC_VALUE_UG=$2 PDVC_BQ_PF=$3"
  PDVC_VAL_DEFER=$1 PDVC_VALUE_UG=$2 PDVC_BQ_PF=$3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/k_d$1u$2p$3 -o kb_$RANDOM -- python -u tools/kbench.py --videos 1024 --reps 4 2>&1 | grep -E "^(encoder|decoder)" || exit 1
done
for d in $O/k_*; do
  for f in $(find $d -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"$(basename $d) {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:96]}\") for r in csv.DictReader(open(sys.argv[1])) if 'bwd_' in r['Name']]" $f
  done
done
for qc in 0 960 640 0 960; do
  echo "[$(date +%T)] PDVC_VAL_QCHUNK=$qc (T=1024)"
  PDVC_VAL_QCHUNK=$qc timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q$qc -o kb_$RANDOM -- python -u tools/kbench.py --videos 512 --reps 4 --T 1024 2>&1 | grep -E "^encoder" || exit 1
done
for qc in 0 960 640; do
  for f in $(find $O/q$qc -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"qc$qc {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}\") for r in csv.DictReader(open(sys.argv[1])) if 'bwd_value' in r['Name']]" $f
  done
done
for ab in 0 1 0 1; do
  echo "[$(date +%T)] PDVC_WIN_ABLATE=$ab (forward, T=1024)"
  PDVC_WIN_ABLATE=$ab timeout -k 10 120 python -u tools/kbench.py --videos 512 --reps 4 --T 1024 2>&1 | grep -E "^encoder" || exit 1
done
for v in "0 0 0" "2 6 1" "0 0 0" "2 6 1"; do
  set -- $v
  echo "[$(date +%T)] drop-in PDVC_VAL_DEFER=$1 PDVC_VALUE_UG=$2 PDVC_BQ_PF=$3"
  PDVC_VAL_DEFER=$1 PDVC_VALUE_UG=$2 PDVC_BQ_PF=$3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/dropin_d$1u$2p$3 -o dp_$RANDOM -- python -u tools/dropin_prof.py 2>&1 | tail -3 || exit 1
done
for d in $O/dropin_*; do
  for f in $(find $d -name "*kernel_stats.csv"); do
    python -c "import csv,sys; [print(f\"$(basename $d) {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4} {r['Name'][:96]}\") for r in csv.DictReader(open(sys.argv[1])) if 'bwd' in r['Name']]" $f
  done
done
