#!/bin/bash
# round-4 GPU pass AL: a second same-box A/B of the add-norm prefetch (PDVC_AN_PF), per-kernel times from rocprof,
# alternating 1,0,1,0
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04al; mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "step rc=$rc: stop"; exit $rc; fi; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  echo "[$(date +%T)] run $i PDVC_AN_PF=$v"
  PDVC_AN_PF=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$i -o run -- \
    python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/b$i.json \
    2> $O/b$i.err; rc=$?; ok $rc
  ks=$(find $O/prof$i -name "*kernel_stats.csv" | head -1)
  python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'addnorm_fwd' in r['Name'] or 'addnorm_bwd' in r['Name']:
        print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg')
PY
done
