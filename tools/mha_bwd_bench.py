"""Decoder self-attention backward timing at the bench shape (HIP events, median of reps), both MFMA backward kernels:
    python tools/mha_bwd_bench.py [--videos 1024] [--reps 10]
PDVC_MHA_BWD2=1: the 51-KiB streaming kernel (mha_bwd_mfma2_kernel), 0: the 133-KiB one (mha_bwd_mfma_kernel)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dense-video-captioning_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--Q", type=int, default=100)
    a = ap.parse_args()
    from pdvc.ops.functions.attention import QuerySelfAttentionFunction
    torch.manual_seed(0)
    N, M, E, Q = a.videos, 8, 512, a.Q
    qk = torch.randn(N, Q, 2 * E, device="cuda", requires_grad=True)
    v = torch.randn(N, Q, E, device="cuda", requires_grad=True)
    g = torch.randn(N, Q, E, device="cuda")
    for mode in ("0", "1", "0", "1"):
        os.environ["PDVC_MHA_BWD2"] = mode
        out = QuerySelfAttentionFunction.apply(qk, v, None, M, 0.1, 5)
        ts = []
        for _ in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.autograd.grad(out, (qk, v), g, retain_graph=True)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts = sorted(ts[2:])
        print(f"PDVC_MHA_BWD2={mode}: backward {ts[len(ts) // 2]:8.1f} us median (N={N}, Q={Q})", flush=True)


if __name__ == "__main__":
    main()
