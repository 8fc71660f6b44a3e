"""Diagnostic: which autograd graphs stay alive after a training forward/backward (tensors with grad_fn
reachable after the step), and who holds them."""
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dense-video-captioning_amd"), ROOT, os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import test_gpu_model as TM  # noqa: E402
import weights as W  # noqa: E402
from pdvc.data import collate, to_device  # noqa: E402

d = TM.load("pdvc_batch3_anet")
model, criterion = TM.build_filled(d)
model.train()
wd = criterion.weight_dict
dt = to_device(collate(W.batch_items(vocab=29)[1:2]), "cuda")
for it in range(2):
    model.zero_grad(set_to_none=True)
    _, loss = model(dt, criterion, "queries")
    total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    total.backward()
    del loss, total, _
gc.collect()
n = 0
for o in gc.get_objects():
    try:
        if isinstance(o, torch.Tensor) and o.grad_fn is not None:
            n += 1
            refs = [type(r).__name__ + (":" + ",".join(list(r.keys())[:6]) if isinstance(r, dict) else "")
                    for r in gc.get_referrers(o)][:6]
            print("alive:", tuple(o.shape), type(o.grad_fn).__name__, refs, flush=True)
    except Exception:
        pass
print("alive tensors with grad_fn:", n)
print("dt keys:", [k for k in dt.keys()])
