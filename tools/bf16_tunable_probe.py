"""Does PyTorch TunableOp tune the bf16 mode's GEMMs (bf16 operands, fp32 output: aten.mm.dtype /
aten.addmm.dtype, pdvc/precision.py) and does the tuned solution beat hipBLASLt's default heuristic?
    python tools/bf16_tunable_probe.py [--rows 491520] [--out gpurun_out/bf16_tunable.csv]
Times the yc2_tsp_bf16 encoder's large-M GEMM shapes (forward, dgrad, wgrad) with the default selection, then with
TunableOp tuning on, and reports whether the tuning file received entries for them."""
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
    ap.add_argument("--rows", type=int, default=491520)
    ap.add_argument("--out", default="gpurun_out/bf16_tunable.csv")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    R = a.rows
    shapes = [  # (name, A (m, k), B (k, n), transposes) of y = A @ B with fp32 output
        ("fwd 512->512", (R, 512), (512, 512)),
        ("fwd 512->2048", (R, 512), (512, 2048)),
        ("fwd 2048->512", (R, 2048), (2048, 512)),
        ("wgrad 512x512 (K=rows)", (512, R), (R, 512)),
    ]
    cases = []
    for name, sa, sb in shapes:
        A = torch.randn(*sa, device=dev).to(torch.bfloat16)
        B = torch.randn(*sb, device=dev).to(torch.bfloat16)
        cases.append((name, A, B, 2.0 * sa[0] * sa[1] * sb[1]))
    op = torch.ops.aten.mm.dtype
    res = {}
    # the split-K form the step uses for weight gradients (pdvc/ops/functions/linear.py wgrad_mm), bf16 operands
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dense-video-captioning_amd")]
    from pdvc.ops.functions.linear import wgrad_splits
    s_ = wgrad_splits(R)
    gy = torch.randn(R, 512, device=dev).to(torch.bfloat16)
    x = torch.randn(R, 512, device=dev).to(torch.bfloat16)
    bop = torch.ops.aten.bmm.dtype
    t = timeit(lambda: bop(gy.reshape(s_, R // s_, 512).transpose(1, 2), x.reshape(s_, R // s_, 512), torch.float32).sum(0))
    print(f"split-K wgrad 512x512 over {s_} chunks: {t * 1e3:8.3f} ms  {2.0 * R * 512 * 512 / t / 1e12:7.1f} TF/s", flush=True)
    for name, A, B, fl in cases:
        t = timeit(lambda: op(A, B, torch.float32))
        res[name] = [t]
        print(f"default  {name:26s} {t * 1e3:8.3f} ms  {fl / t / 1e12:7.1f} TF/s", flush=True)
    import torch.cuda.tunable as tun
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(a.out)
    tun.set_max_tuning_iterations(20)
    tun.set_max_tuning_duration(50)
    for name, A, B, fl in cases:
        op(A, B, torch.float32)
        torch.cuda.synchronize()
    tun.tuning_enable(False)
    for name, A, B, fl in cases:
        t = timeit(lambda: op(A, B, torch.float32))
        res[name].append(t)
        print(f"tunable  {name:26s} {t * 1e3:8.3f} ms  {fl / t / 1e12:7.1f} TF/s  ({res[name][0] / t:.3f}x)", flush=True)
    results = tun.get_results()
    print("tuned entries:", len(results))
    for r in list(results)[:12]:
        print("  ", str(r)[:200])


if __name__ == "__main__":
    sys.exit(main())
