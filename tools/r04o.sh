#!/bin/bash
# round-4 GPU pass O: which torch ops own the small kernels of the headline step (1024 videos)
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 600 python -u tools/opparents.py --videos 1024 --top 60 > $O/opparents.txt 2>&1 || { tail -20 $O/opparents.txt; exit 1; }
grep -v Warning $O/opparents.txt | head -70
