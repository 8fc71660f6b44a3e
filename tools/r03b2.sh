# round-3 GPU pass: decoder value-gradient ablations (PDVC_VAL_ABLATE=3: sort only, 4: walk without gathers)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03b2}; mkdir -p $O
for ab in 0 3 4; do
  PDVC_VAL_ABLATE=$ab timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kp$ab -o run -- python -u tools/kbench.py --videos 1024 --reps 5 > $O/kbp$ab.txt 2>&1 || exit 1
  ks=$(find $O/kp$ab -name "*kernel_stats.csv" | head -1)
  echo "ablate=$ab"; python - "$ks" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "bwd_value" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):4d} calls  {r["Name"][:70]}')
PY
done
