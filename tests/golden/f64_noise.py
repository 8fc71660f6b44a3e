#!/usr/bin/env python
"""How much rounding noise do the float32 model fixtures carry?  (Run in the build container only: it imports the
reference from /root/reference through make_golden.py, and writes nothing into the repository.)

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/f64_noise.py

Runs the fixture generators of make_golden.py (whole_model_batch, whole_model, module_captioner, module_layers)
twice -- as they are (float32, the fixtures the tests load) and with the reference model, its inputs and the
float32 constants it builds internally (position_encoding.py:44,49, deformable_transformer.py:70,81,202 and the
`.float()` casts) promoted to float64 -- and prints, per fixture, the largest per-tensor relative difference
max|f32 - f64| / max|f64|.  Measured here (round 3): 3.5e-6 at worst (encoder attention_weights gradients),
except the caption head's alpha_net bias gradient, which is zero in exact arithmetic (softmax shift invariance)
and ~1e-18 in both runs.  This is what justifies the GPU tests' bound 1e-4 * max|ref| + 1e-7 (tests/parity.py).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def run(mode):
    import make_golden as MG  # installs the stubs, chdir to the reference
    import torch
    saved = {}

    def fake_save(name, **arrays):
        saved[name] = {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
                       for k, v in arrays.items()}
    MG.save = fake_save
    if mode == "f64":
        import pdvc.pdvc as P
        from data import video_dataset as VD
        torch.set_default_dtype(torch.float64)

        def promote(kw):
            if kw.get("dtype") is torch.float32:
                kw["dtype"] = torch.float64
            return kw
        for fn in ("arange", "linspace"):
            orig = getattr(torch, fn)
            setattr(torch, fn, (lambda o: lambda *a, **k: o(*a, **promote(k)))(orig))
        cumsum = torch.Tensor.cumsum
        torch.Tensor.cumsum = lambda self, *a, **k: cumsum(self, *a, **promote(k))
        torch.Tensor.float = lambda self: self.double()
        t0 = MG.t
        MG.t = lambda x, dtype=torch.float64, grad=False: t0(x, torch.float64, grad)
        build0, collate0 = P.build, VD.collate_fn

        def build64(args):
            m, c, p = build0(args)
            return m.double(), c, p

        def collate64(batch):
            dt = collate0(batch)
            for k, v in list(dt.items()):
                if isinstance(v, torch.Tensor) and v.is_floating_point():
                    dt[k] = v.double()
            dt["video_target"] = [{k: (v.double() if isinstance(v, torch.Tensor) and v.is_floating_point() else v)
                                   for k, v in t.items()} for t in dt["video_target"]]
            return dt
        P.build, VD.collate_fn = build64, collate64
    for gen in ("whole_model_batch", "whole_model", "module_captioner", "module_layers"):
        getattr(MG, gen)()
    return saved


def full(d, k):
    if k in d:
        return d[k].astype(np.float64)
    g = d[k + ".A"].astype(np.float64) @ d[k + ".B"].astype(np.float64)
    return g.reshape(tuple(int(x) for x in d[k + ".shape"]))


def main():
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(1) as pool:
        f32 = pool.apply(run, ("f32",))
    with mp.get_context("spawn").Pool(1) as pool:
        f64 = pool.apply(run, ("f64",))
    for name in f32:
        a, b = f32[name], f64[name]
        keys = {k.rsplit(".", 1)[0] if k.endswith((".A", ".B", ".err", ".shape")) else k for k in a}
        rows = []
        for k in keys:
            try:
                x, y = full(a, k), full(b, k)
            except KeyError:
                continue
            if x.dtype.kind != "f" or x.size == 0 or x.shape != y.shape or not np.abs(y).max():
                continue
            rows.append((float(np.abs(x - y).max() / np.abs(y).max()), k, float(np.abs(y).max())))
        rows.sort(reverse=True)
        print(f"{name}: {len(rows)} tensors; largest relative f32-vs-f64 differences:")
        for r in rows[:4]:
            print("   %.2e  %s  (max|f64| %.2e)" % r)


if __name__ == "__main__":
    main()
