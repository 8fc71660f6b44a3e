"""Add-norm kernels at the encoder's shape (1024 videos x 960 positions, d = 512, dropout 0.1): per-launch device time
of pdvc_add_dropout_layernorm_forward/backward_f32 (HIP events, median) and the HBM rate of their streamed tensors
(forward: read x, s, write y = 3 rows*d*4 bytes; backward: read x, s, dy, write dx, ds = 5).  Round 3 measured a
next-row prefetch and larger forward grids with it (profiles/r03_addnorm_prefetch_rejected.jsonl: no gain -- the
kernels already stream at 5.2-5.4 TB/s, 83-86 % of the guide's 6.29 TB/s float4 copy) and removed them.

    python tools/an_bench.py [--rows 983040] [--d 512] [--reps 20]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dense-video-captioning_amd"))
from pdvc.ops.functions.addnorm import BWD_PARTS, an_backward, an_forward  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024 * 960)
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.rows, a.d, device=dev, generator=g)
    s = torch.randn(a.rows, a.d, device=dev, generator=g)
    dy = torch.randn(a.rows, a.d, device=dev, generator=g)
    w = torch.rand(a.d, device=dev, generator=g) + 0.5
    b = torch.randn(a.d, device=dev, generator=g)
    y, dx, ds = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
    mean = torch.empty(a.rows, device=dev)
    rstd = torch.empty_like(mean)
    dw, db, dsum = torch.empty_like(w), torch.empty_like(w), torch.empty_like(w)
    ws = torch.empty(3 * BWD_PARTS * a.d, device=dev)
    fwd = lambda: an_forward(x, s, w, b, 0.1, 1234, None, 1e-5, y, mean, rstd)  # noqa: E731
    bwd = lambda: an_backward(x, s, w, mean, rstd, dy, 0.1, 1234, None, dx, ds, dw, db, dsum, ws)  # noqa: E731
    tf, tb = timed(fwd, a.reps), timed(bwd, a.reps)
    nb = a.rows * a.d * 4
    out = {"rows": a.rows, "d": a.d, "PDVC_AN_PF": os.environ.get("PDVC_AN_PF", "1"),
           "PDVC_AN_FWD_BLOCKS": os.environ.get("PDVC_AN_FWD_BLOCKS", "1024"),
           "fwd_us": 1e3 * tf, "fwd_tbs": 3 * nb / (tf * 1e-3) / 1e12,
           "bwd_us": 1e3 * tb, "bwd_tbs": 5 * nb / (tb * 1e-3) / 1e12,
           "checksum": [float(y.double().sum()), float(dx.double().sum()), float(ds.double().sum()),
                        float(dw.double().sum()), float(dsum.double().sum())]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
