"""Does PyTorch TunableOp (exhaustive hipBLASLt / rocBLAS solution search per GEMM shape) beat the default
heuristic on the encoder's GEMMs?  python tools/tunable_probe.py [--rows 245760]
Times the three large-M GEMMs of an encoder linear (forward addmm, dgrad mm, split-K wgrad bmm) with the default
selection, then tunes them and times again."""
import argparse
import os
import sys

import torch


def timeit(f, reps=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=245760)
    ap.add_argument("--out", default="gpurun_out/tunable_probe.csv")
    a = ap.parse_args()
    M = a.rows
    dev = "cuda"
    cases = []
    for K, N in ((512, 512), (512, 256), (512, 2048), (2048, 512)):
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        b = torch.randn(N, device=dev)
        gy = torch.randn(M, N, device=dev)
        fl = 2.0 * M * N * K
        cases += [
            (f"fwd addmm  K={K} N={N}", fl, lambda x=x, W=W, b=b: torch.addmm(b, x, W.t())),
            (f"fwd mm     K={K} N={N}", fl, lambda x=x, W=W: torch.mm(x, W.t())),
            (f"dgrad mm   K={K} N={N}", fl, lambda gy=gy, W=W: torch.mm(gy, W)),
            (f"wgrad bmm64 K={K} N={N}", fl,
             lambda gy=gy, x=x, N=N, K=K: torch.bmm(gy.view(64, -1, N).transpose(1, 2), x.view(64, -1, K))),
        ]
    base = {}
    for name, fl, f in cases:
        s = timeit(f)
        base[name] = s
        print(f"default {name:26s} {s * 1e6:8.1f} us {fl / s / 1e12:6.1f} TF/s", flush=True)
    import torch.cuda.tunable as tun
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(a.out)
    tun.set_max_tuning_duration(30)
    tun.set_max_tuning_iterations(10)
    for name, fl, f in cases:
        f()
        torch.cuda.synchronize()
        print(f"tuned   {name}", flush=True)
    tun.tuning_enable(False)
    for name, fl, f in cases:
        s = timeit(f)
        print(f"tunable {name:26s} {s * 1e6:8.1f} us {fl / s / 1e12:6.1f} TF/s  ({base[name] / s:.3f}x)", flush=True)
    tun.write_file()
    print("results:", tun.get_results()[:20] if hasattr(tun, "get_results") else "", file=sys.stderr)


if __name__ == "__main__":
    main()
