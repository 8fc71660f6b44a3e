"""Diagnosis: capture the StepGraph of a capacity-padded batch (pdvc/batch_layout.py) in isolation, with torch's
sync debug mode on (every synchronising call during warm-up or capture is reported with its stack), then replay.

    python tools/diag_capacity_capture.py [--eager-first [--release]] [--no-sync-debug]

--eager-first runs an eager unpadded step on the default stream before the capture and keeps its loss tensors
(hence its autograd graph, whose AccumulateGrad nodes were created on the default stream) alive; --release drops
them first.
"""
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dense-video-captioning_amd"), ROOT, os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import test_gpu_model as TM  # noqa: E402
import weights as W  # noqa: E402
from pdvc.batch_layout import pad_to_capacity  # noqa: E402
from pdvc.data import collate, to_device  # noqa: E402
from pdvc.step_graph import StepGraph  # noqa: E402


def main():
    import ctypes
    import faulthandler
    faulthandler.enable(all_threads=True)
    lib = os.path.join(ROOT, "tools", "native", "libsegv_trace.so")
    if os.path.exists(lib):  # native backtrace on SIGSEGV, chained to faulthandler's Python stacks
        ctypes.CDLL(lib).segv_trace_install()
    d = TM.load("pdvc_batch3_anet")
    model, criterion = TM.build_filled(d)
    model.train()
    items = W.batch_items(vocab=29)
    caps = dict(events=7, rows=16, words=12)
    dt = to_device(pad_to_capacity(collate(items), **caps), "cuda")
    if "--eager-first" in sys.argv:
        wd = criterion.weight_dict
        out, loss = model(to_device(collate([items[2], items[0], items[1]]), "cuda"), criterion, "queries")
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        total.backward()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        total = total.item()
        torch.cuda.synchronize()
        print("eager total", total, len(grads), "grads", flush=True)
        if "--release" in sys.argv:
            del out, loss
        model.zero_grad(set_to_none=True)
        print("eager unpadded step done", flush=True)
    if "--no-sync-debug" not in sys.argv:
        torch.cuda.set_sync_debug_mode("warn")
    warnings.simplefilter("always")
    orig = warnings.showwarning

    def show(message, category, filename, lineno, file=None, line=None):
        print("SYNC WARNING:", message, flush=True)
        traceback.print_stack(limit=12)
    warnings.showwarning = show
    print("capturing", flush=True)
    sg = StepGraph(model, criterion, dt)
    torch.cuda.set_sync_debug_mode(0)
    warnings.showwarning = orig
    print("captured", flush=True)
    for i in range(2):
        print("replay", i, float(sg.replay()), flush=True)


if __name__ == "__main__":
    main()
