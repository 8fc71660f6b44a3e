"""Diagnostic: StepGraph replay vs eager gradients on small batches (which parameters differ, by how much).
    python tools/diag_batch_graph.py [variant ...]     variants: pad3 (the batch fixture), nopad3, pad1, nopad2
"""
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
from pdvc.step_graph import StepGraph  # noqa: E402


def items(variant):
    it = W.batch_items(vocab=29)
    if variant == "pad3":
        return it
    if variant == "nopad3":
        return [it[0], it[2], W.batch_items(seed=22, vocab=29)[2]]
    if variant == "pad1":
        return [it[1]]
    if variant == "nopad2":
        return [it[0], it[2]]
    raise ValueError(variant)


def run(variant):
    d = TM.load("pdvc_batch3_anet")
    model, criterion = TM.build_filled(d)
    model.train()
    wd = criterion.weight_dict
    mk = (lambda: TM.fixture_dt(TM.load("pdvc_small_anet"))) if variant == "fixture" else \
        (lambda: to_device(collate(items(variant)), "cuda"))
    dt = mk()
    model.zero_grad(set_to_none=True)
    _, loss = model(dt, criterion, "queries")
    t0 = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
    t0.backward()
    ge = {n: (None if p.grad is None else p.grad.detach().clone()) for n, p in model.named_parameters()}
    t0 = t0.item()
    del loss, _
    model.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    dt2 = mk()
    sg = StepGraph(model, criterion, dt2)
    for r in range(2):
        t1 = sg.replay().item()
        torch.cuda.synchronize()
        bad = []
        for n, p in model.named_parameters():
            if ge[n] is None or p.grad is None:
                if (ge[n] is None) != (p.grad is None):
                    bad.append((n, "None mismatch"))
                continue
            err = (ge[n] - p.grad).abs().max().item()
            if err > 1e-5 * max(1.0, ge[n].abs().max().item()):
                bad.append((n, f"{err:.3e} (|g| {ge[n].abs().max().item():.3e})"))
        print(f"[{variant}] replay {r}: total {t1:.6f} vs eager {t0:.6f}; {len(bad)} bad grads", flush=True)
        for b in bad[:40]:
            print("   ", *b, flush=True)


if __name__ == "__main__":
    for v in sys.argv[1:] or ["pad3", "nopad3", "pad1", "nopad2"]:
        run(v)
