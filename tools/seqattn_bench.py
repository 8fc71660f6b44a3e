"""Device time of the dual-modality front-end's attention core (csrc/seqattn.hip) at the cfg-4 shape
(T = 512 queries and keys, 32 heads of 24, fp32), per video, forward and backward, with HIP events:
    python tools/seqattn_bench.py [--videos 64]
Prints ms per launch and the scalar-FP32 rate: 4*T*T*D flops per (video, head) forward (scores + P.V) and
8*T*T*D backward (scores recomputed twice, dP and dS products), against the 157.3 TFLOP/s FP32 vector peak."""
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
    a = ap.parse_args()
    from pdvc.ops.functions.seq_attention import SeqAttentionFunction
    N, T, H, D = a.videos, a.T, 32, 24
    E = H * D
    qkv = torch.randn(N, T, 3 * E, device="cuda", requires_grad=True)
    g = torch.randn(N, T, E, device="cuda")

    def run():
        out = SeqAttentionFunction.apply(qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:], H)
        return out

    for _ in range(3):
        run().backward(g)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    reps = 10
    fwd = bwd = 0.0
    for _ in range(reps):
        e[0].record()
        out = run()
        e[1].record()
        out.backward(g)
        e[2].record()
        torch.cuda.synchronize()
        fwd += e[0].elapsed_time(e[1])
        bwd += e[1].elapsed_time(e[2])
    fwd, bwd = fwd / reps, bwd / reps
    ff = 4.0 * N * H * T * T * D
    print(f"videos {N} T {T} H {H} D {D}: forward {fwd:.3f} ms ({ff / fwd / 1e9:.1f} TFLOP/s), backward incl. "
          f"autograd copies {bwd:.3f} ms ({2 * ff / bwd / 1e9:.1f} TFLOP/s); {1e3 * (fwd + bwd) / N:.1f} us per video "
          f"per attention block")


if __name__ == "__main__":
    main()
