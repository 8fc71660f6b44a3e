"""fp32 GEMM rates of the step's dominant shapes under torch's BLAS backends (diagnostic).
    python tools/gemmbench.py"""
import torch


def rate(M, N, K, ta, tb, reps=20):
    a = torch.randn((K, M) if ta else (M, K), device="cuda")
    b = torch.randn((N, K) if tb else (K, N), device="cuda")
    A = a.t() if ta else a
    B = b.t() if tb else b
    for _ in range(3):
        A @ B
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        A @ B
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    return 2 * M * N * K / t / 1e12, t * 1e6


SHAPES = [  # (M, N, K, A transposed, B transposed): forward x W^T, dgrad g W, wgrad g^T x
    (30720, 512, 512, False, True), (30720, 512, 512, False, False), (512, 512, 30720, True, False),
    (30720, 256, 512, False, True), (4096, 512, 512, False, True), (3584, 5748, 512, False, True),
    (3584, 512, 5748, False, False), (5748, 512, 3584, True, False), (256, 2576, 512, False, True),
]

def rate_pdvc(M, N, K, ta, tb, reps=20):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "dense-video-captioning_amd"))
    from pdvc.ops.functions import matmul
    a = torch.randn((K, M) if ta else (M, K), device="cuda")
    b = torch.randn((N, K) if tb else (K, N), device="cuda")
    A = a.t() if ta else a
    B = b.t() if tb else b
    wgrad = ta and not tb and K >= 4096
    C = torch.zeros(M, N, device="cuda")
    f = (lambda: matmul(A, B, out=C, accumulate=True)) if wgrad else (lambda: matmul(A, B))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    return 2 * M * N * K / t / 1e12, t * 1e6


def rate_splitk_bmm(M, N, K, splits, reps=20):
    """wgrad dW (M,N) = dy^T (M,K) x (K,N) as a batched GEMM over `splits` K-chunks + a sum (torch)."""
    dy = torch.randn(K, M, device="cuda")
    x = torch.randn(K, N, device="cuda")
    f = lambda: torch.bmm(dy.view(splits, K // splits, M).transpose(1, 2), x.view(splits, K // splits, N)).sum(0)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    return 2 * M * N * K / t / 1e12, t * 1e6


if __name__ == "__main__":
    for splits in (2, 4, 8, 16):
        for (M, N, K) in ((512, 512, 30720), (256, 512, 30720), (512, 768, 16384)):
            tf, us = rate_splitk_bmm(M, N, K, splits)
            print(f"{'torch bmm split-K x' + str(splits):28s} M={M:6d} N={N:5d} K={K:6d}: {tf:6.1f} TF/s {us:8.1f} us",
                  flush=True)
    for s in SHAPES:
        tf, us = rate_pdvc(*s)
        print(f"{'pdvc_gemm_f32':28s} M={s[0]:6d} N={s[1]:5d} K={s[2]:6d} tA={int(s[3])} tB={int(s[4])}: {tf:6.1f} TF/s {us:8.1f} us",
              flush=True)
    libs = ["default"]
    try:
        cur = torch.backends.cuda.preferred_blas_library()
        libs = [str(cur)]
        for name in ("hipblaslt", "rocblas"):
            if name not in str(cur).lower():
                libs.append(name)
    except Exception as e:  # noqa: BLE001
        print("preferred_blas_library unavailable:", e)
    for lib in libs:
        if lib != libs[0]:
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as e:  # noqa: BLE001
                print(lib, "unavailable:", e)
                continue
        for s in SHAPES:
            tf, us = rate(*s)
            print(f"{lib:28s} M={s[0]:6d} N={s[1]:5d} K={s[2]:6d} tA={int(s[3])} tB={int(s[4])}: {tf:6.1f} TF/s {us:8.1f} us",
                  flush=True)
