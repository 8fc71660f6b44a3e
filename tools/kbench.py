"""Standalone timing of the MSDA kernels at the PDVC encoder/decoder shapes (HIP events, interleaved reps).

    python tools/kbench.py [--videos 32] [--reps 20]
Prints per-kernel average microseconds and algorithmic GB/s (SURVEY.md section 8(d) byte model)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dense-video-captioning_amd"))
import torch  # noqa: E402

from pdvc.ops.functions import MSDA1dFunction  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--T", type=int, default=512)
    a = ap.parse_args()
    T_l = tuple(a.T // 2 ** i for i in range(4))
    S = sum(T_l)
    M, D, N = 8, 64, a.videos
    torch.manual_seed(0)
    dev = "cuda"
    for name, Lq in (("encoder", S), ("decoder", 100)):
        value = torch.randn(N, S, M, D, device=dev, requires_grad=True)
        proj = torch.cat([torch.randn(N, Lq, M * 16, device=dev) * 2, torch.randn(N, Lq, M * 16, device=dev)], -1)
        proj.requires_grad_()
        if Lq == S:
            ref = torch.cat([(torch.arange(t, device=dev) + 0.5) / t for t in T_l])[None, :, None, None]
            ref = ref.expand(N, S, 4, 1).contiguous()
        else:
            ref = torch.rand(N, Lq, 4, 1, device=dev)
        out = MSDA1dFunction.apply(value, None, proj, ref, T_l, 0, M * 16)
        g = torch.randn_like(out)
        fwd = lambda: MSDA1dFunction.apply(value, None, proj, ref, T_l, 0, M * 16)
        bwd = lambda: torch.autograd.grad(out, (value, proj), g, retain_graph=True)
        tf = timeit(fwd, a.reps)
        tb = timeit(bwd, a.reps)
        e = 4
        fb = N * S * M * D * e + N * Lq * M * 16 * 12 + N * Lq * M * D * e
        bb = 3 * N * S * M * D * e + N * Lq * M * D * e + 2 * N * Lq * M * 16 * 12
        print(f"{name:8s} N={N} Lq={Lq}: fwd {tf:8.1f} us ({fb / tf / 1e3:7.1f} GB/s alg)  "
              f"bwd {tb:8.1f} us ({bb / tb / 1e3:7.1f} GB/s alg)  [ablate={os.environ.get('PDVC_PYR_ABLATE', '0')}]",
              flush=True)


if __name__ == "__main__":
    main()
