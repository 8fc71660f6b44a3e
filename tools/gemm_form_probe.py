"""Does a batched form beat the plain GEMM on the encoder's dominant projection shape? (diagnostic)
    python tools/gemm_form_probe.py [--M 983040]
Times y = x W^T + b at (M, 512) x (512, 512) as addmm and as baddbmm over B row chunks with a broadcast weight
(stride-0 batch), each with TunableOp searching its solutions first, with HIP events."""
import argparse
import os
import sys

import torch


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=983040)
    a = ap.parse_args()
    import torch.cuda.tunable as tun
    os.makedirs("gpurun_out", exist_ok=True)
    tun.set_filename("gpurun_out/probe_tunable.csv")
    tun.set_max_tuning_iterations(5)
    tun.set_max_tuning_duration(20)
    tun.enable(True)
    tun.tuning_enable(True)
    M, K, N = a.M, 512, 512
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    b = torch.randn(N, device="cuda")
    fl = 2.0 * M * N * K
    ms = timeit(lambda: torch.addmm(b, x, w.t()))
    print(f"addmm            {ms:7.3f} ms  {fl / ms / 1e9:6.1f} TF/s", flush=True)
    ms = timeit(lambda: torch.mm(x, w))
    print(f"mm (dgrad form)  {ms:7.3f} ms  {fl / ms / 1e9:6.1f} TF/s", flush=True)
    for B in (4, 16, 64):
        xb = x.view(B, M // B, K)
        wb = w.t().unsqueeze(0).expand(B, K, N)
        bb = b.view(1, 1, N)
        ms = timeit(lambda: torch.baddbmm(bb, xb, wb))
        print(f"baddbmm B={B:3d}    {ms:7.3f} ms  {fl / ms / 1e9:6.1f} TF/s", flush=True)
        wd = w.unsqueeze(0).expand(B, N, K)
        ms = timeit(lambda: torch.bmm(xb, wd))
        print(f"bmm dgrad B={B:3d}  {ms:7.3f} ms  {fl / ms / 1e9:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
