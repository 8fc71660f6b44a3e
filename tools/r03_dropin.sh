#!/bin/bash
# Drop-in operator on the whole-pyramid kernels: its GPU tests, then its per-launch timings (pyramid and A/B gather).
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03dp}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x --timeout 120 --timeout-method thread -k dropin -rf > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u -c "import json, bench; print(json.dumps(bench.dropin_msda(512)))" > $O/dropin_pyr.json 2> $O/dropin_pyr.err || { tail -5 $O/dropin_pyr.err; exit 1; }
PDVC_DROPIN_PYR=0 timeout -k 10 200 python -u -c "import json, bench; print(json.dumps(bench.dropin_msda(512)))" > $O/dropin_gather.json 2> $O/dropin_gather.err || { tail -5 $O/dropin_gather.err; exit 1; }
cat $O/dropin_pyr.json $O/dropin_gather.json
