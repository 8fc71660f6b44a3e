#!/bin/bash
# round-4 GPU pass F: the anet_c3d line (configs[4], T = 1024) -- PMC traffic of its MSDA kernels and GEMMs, the bench
# line with its CPU baseline, and a rocprofv3 kernel-trace summary of the same command
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
WL=anet_c3d TAG=r04f/pmc bash tools/pmc_workload.sh || exit 1
echo "[$(date +%T)] anet_c3d bench"
timeout -k 10 600 python -u bench.py --workload anet_c3d > $O/bench_anet_c3d.json 2> $O/bench_anet_c3d.err || { tail -20 $O/bench_anet_c3d.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_anet_c3d.json')); print(d['value'], d['ms_per_step'], d['roofline_gather']['frac'], d['roofline_gather_bwd']['frac'], d['cpu_baseline']['value'])"
echo "[$(date +%T)] anet_c3d bench under rocprofv3"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3d -- python -u bench.py --workload anet_c3d --steps 5 --warmup 2 --no-cpu-baseline --no-dropin > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python tools/profsum.py $f 0 30 > $O/prof_summary.txt; head -40 $O/prof_summary.txt
echo "[$(date +%T)] ragged stream under rocprofv3"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_rag -o rag -- python -u bench.py --stream ragged --steps 6 --warmup 2 --no-cpu-baseline --no-dropin --no-gemm-roofline > $O/prof_rag.json 2> $O/prof_rag.err || { tail -20 $O/prof_rag.err; exit 1; }
kt=$(find $O/prof_rag -name "*kernel_trace.csv" | head -1); python tools/profsteps.py "$kt" 45 > $O/prof_rag_steps.txt; head -30 $O/prof_rag_steps.txt
