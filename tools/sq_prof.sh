#!/bin/bash
# seqattn kernels at the cfg-4 shape (GPU box, repo root): timing, rocprofv3 kernel stats, one SQ counter pass
#     bash tools/sq_prof.sh TAG [VIDEOS]
set -o pipefail
TAG=${1:-sq}
V=${2:-64}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/seqattn_bench.py --videos "$V" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python -u tools/seqattn_bench.py --videos "$V" > "$OUT/prof.txt" 2>&1 || { tail -20 "$OUT/prof.txt"; exit 1; }
ks=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "seqattn" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:90]}')
PY
if [ -n "$SQ_PMC" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $SQ_PMC --kernel-include-regex seqattn --output-format csv -d "$OUT/pmc" -o pmc \
      -- python -u tools/seqattn_bench.py --videos "$V" --reps 2 > "$OUT/pmc.txt" 2>&1 || { tail -5 "$OUT/pmc.txt"; exit 1; }
  pc=$(find "$OUT/pmc" -name "*counter_collection.csv" | head -1)
  python - "$pc" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
fi
