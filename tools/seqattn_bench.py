"""Device time of the dual-modality front-end's attention core (csrc/seqattn.hip) at the cfg-4 shape
(T = 512 queries and keys, 32 heads of 24, fp32), per launch, forward and backward, with HIP events around
back-to-back launches of the C ABI (no autograd, no allocation inside the timed region):
    python tools/seqattn_bench.py [--videos 64] [--reps 20]
Prints ms per launch and the algorithmic rate: 4*T*T*D flops per (video, head) forward (scores + P.V) and
10*T*T*D backward (scores recomputed once, dP, dQ, dK, dV -- the kernels execute 14*T*T*D: the dk/dv kernel
recomputes the scores and dP of the dq kernel), against the 157.3 TFLOP/s fp32 MFMA peak."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dense-video-captioning_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=64)
    ap.add_argument("--T", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from pdvc import _native as _n
    N, T, H, D = a.videos, a.T, 32, 24
    E = H * D
    qkv = torch.randn(N, T, 3 * E, device="cuda")
    g = torch.randn(N, T, E, device="cuda")
    out = torch.empty(N, T, E, device="cuda")
    lse = torch.empty(N, H, T, device="cuda")
    ws = torch.empty(N * H * T, device="cuda")
    gq, gk, gv = (torch.empty(N, T, E, device="cuda") for _ in range(3))
    q, k, v = (_n.ptr_any(qkv[..., i * E:(i + 1) * E]) for i in range(3))
    st = _n.stream()

    def fwd():
        _n.call("pdvc_seq_attention_forward_f32", q, 3 * E, k, 3 * E, v, 3 * E, N, T, T, H, D,
                _n.ptr(out), _n.ptr(lse), st)

    def bwd():
        _n.call("pdvc_seq_attention_backward_f32", q, 3 * E, k, 3 * E, v, 3 * E, _n.ptr(out), _n.ptr(g),
                _n.ptr(lse), N, T, T, H, D, _n.ptr(ws), _n.ptr(gq), E, _n.ptr(gk), E, _n.ptr(gv), E, st)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    tf, tb = timed(fwd), timed(bwd)
    ff = 4.0 * N * H * T * T * D
    print(f"videos {N} T {T} H {H} D {D}: forward {tf:.3f} ms ({ff / tf / 1e9:.1f} TFLOP/s), backward {tb:.3f} ms "
          f"({2.5 * ff / tb / 1e9:.1f} TFLOP/s); {1e3 * (tf + tb) / N:.1f} us per video per attention block")


if __name__ == "__main__":
    main()
