#!/bin/bash
# Per-kernel device times of the MSDA kernels at the bench shapes (GPU box, repo root):
#     bash tools/kbench_prof.sh TAG [VIDEOS]
set -o pipefail
TAG=${1:-kb}
V=${2:-256}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kprof" -o run \
    -- python -u tools/kbench.py --videos "$V" --reps 5 > "$OUT/kbench.txt" 2>&1 || { tail -20 "$OUT/kbench.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/kbench.txt"
ks=$(find "$OUT/kprof" -name "*kernel_stats.csv" | head -1)
python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "msda1d" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:90]}')
PY
