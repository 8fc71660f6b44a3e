#!/bin/bash
# round-4 GPU pass H: the 1024-video step graph replays against the eager step, every dropout off
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 900 python -u tools/check_graph_replays.py --videos 1024 > $O/replays1024.log 2>&1 || { tail -20 $O/replays1024.log; exit 1; }
grep -v Warning $O/replays1024.log | tail -6
