"""GPU: `bench.py --gpus 2` with no launcher starts its two rank processes itself (bench.py launch_ranks) and rank 0
reports the whole job: n_gpus 2, global_batch = 2 x videos per GPU, parallelism dp2.  Both ranks share the box's
one GPU (--same-device) over gloo; the driver's 8-GPU run takes the same path with one GPU per rank over RCCL.
The step is the bench's own: the captured step graph with bucket-resident gradients, then finish()'s all-reduce."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_starts_two_ranks_itself():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device", "--dist-backend", "gloo",
           "--videos-per-gpu", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-dropin",
           "--no-gemm-roofline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 8
    assert line["config"]["videos_per_gpu"] == 4
    assert line["config"]["parallelism"] == "dp2"
    assert line["value"] > 0
    assert "AccumulateGrad node's stream does not match" not in r.stderr
