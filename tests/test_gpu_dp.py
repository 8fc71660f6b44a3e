"""Data-parallel equivalence on the real model: two ranks, each running 2 videos
through the training step and GradAllReducer, end with the gradients one process computes for the 4-video
union batch -- within 1e-4 * max|ref| + 1e-7 per tensor, with the same parameters left at grad None (the
reference's never-used ones).  Ranks are fresh processes (tests/dp_worker.py) on cuda:0 over gloo (a 1-GPU
box; the bench's N-GPU runs use RCCL with the same reducer); both the eager step and the StepGraph replay
(forward + losses + backward as one hipGraph, the path bench.py times) are covered; the graph mode's all-reduces
are queued behind the per-bucket events the capture records (GradAllReducer.finish_replay).  The union gradient is
itself the mean of the reference's batch-1 gradients (tests/test_gpu_batch.py pins that)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
import test_gpu_model as TM  # noqa: E402
from parity import assert_close  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def union_grads():
    import weights as W
    from pdvc.data import collate, to_device
    d = TM.load("pdvc_batch3_anet")
    model, criterion = TM.build_filled(d)
    model.train()
    dt = to_device(collate(W.dp_items()), "cuda")
    _, loss = model(dt, criterion, "queries")
    wd = criterion.weight_dict
    sum(loss[k] * wd[k] for k in loss.keys() if k in wd).backward()
    return {n: (None if p.grad is None else p.grad.detach().double().cpu().numpy())
            for n, p in model.named_parameters()}


@pytest.fixture(scope="module")
def union():
    return union_grads()


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_two_ranks_equal_union_batch(tmp_path, union, mode):
    world, port = 2, _free_port()
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dp_worker.py"), str(r), str(world),
                               str(port), outs[r], mode], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors="replace")[-3000:])
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r]}"
    for r in range(world):
        g = np.load(outs[r], allow_pickle=False)
        assert int(g["n_buckets"]) >= 2
        if mode == "graph":  # the replays' all-reduces ran behind the capture's per-bucket events (overlapped)
            assert int(g["overlap"]) == 1, "the capture's bucket events were not usable: reduction not overlapped"
            assert int(g["event_nodes"]) == int(g["n_buckets"]), \
                "the replayed graph must hold one event-record node per bucket (ADVICE round 5)"
        for n, ref in union.items():
            if ref is None:
                assert "none." + n in g.files, f"rank {r}: {n} must stay None"
                continue
            got = g["grad." + n].astype(np.float64)
            assert_close(got, ref, f"rank {r} {mode}: grad {n}")
