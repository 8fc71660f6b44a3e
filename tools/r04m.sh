#!/bin/bash
# round-4 GPU pass M: the yc2_newmodel line (configs[3]) -- PMC traffic, the bench line with its CPU baseline, rocprof
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
WL=yc2_newmodel TAG=r04m/pmc bash tools/pmc_workload.sh || exit 1
echo "[$(date +%T)] yc2_newmodel bench"
timeout -k 10 600 python -u bench.py --workload yc2_newmodel > $O/bench_yc2_newmodel.json 2> $O/bench_yc2_newmodel.err || { tail -20 $O/bench_yc2_newmodel.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_yc2_newmodel.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gather']['frac'], d['roofline_gather']['traffic'], d['cpu_baseline']['value'])"
echo "[$(date +%T)] yc2_newmodel bench under rocprofv3"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o nm -- python -u bench.py --workload yc2_newmodel --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python tools/profsum.py $f 0 30 > $O/prof_summary.txt; head -20 $O/prof_summary.txt
