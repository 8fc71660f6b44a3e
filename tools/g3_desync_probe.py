"""Does dephasing the K = 512 gemm3p tiles help? (diagnostic; round 6)  The step's 983040 x 512 x 512 products run one
workgroup per CU in lockstep waves of 256 tiles, so every tile's 256 KiB epilogue leaves in one chip-wide burst.  Arms,
each the same total work, timed with events on the launching stream after warm-up:
  one     a single launch (the step's form);
  two     the rows in two halves on two streams, started together (each half ~128 CUs, still in phase);
  twoD    the same with the second half's stream delayed by D microseconds (torch.cuda._sleep) so the two halves'
          epilogues alternate.
    python tools/g3_desync_probe.py [--delays 10,20,40,60]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dense-video-captioning_amd"))
from pdvc import _native as _n  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--delays", default="10,20,40,60")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    M, N, K = 983040, 512, 512
    x = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda")
    planes = torch.empty(3 * N * K, dtype=torch.int16, device="cuda")
    _n.call("pdvc_split3_planes_f32", _n.ptr_any(W), K, 1, N, K, _n.ptr_any(planes), _n.stream())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    # cycles per microsecond for torch.cuda._sleep (the shader clock, ~2 GHz under this load)
    cyc_per_us = 2000

    def gemm(r0, rows, stream):
        with torch.cuda.stream(stream):
            _n.call("pdvc_gemm3p_f32", rows, N, K, _n.ptr_any(x[r0:]), K, _n.ptr(planes), _n.ptr_any(y[r0:]), N,
                    _n.ptr(b), 1, ctypes_stream(stream))

    def ctypes_stream(stream):
        import ctypes
        return ctypes.c_void_p(stream.cuda_stream)

    def run(arm, delay_us=0):
        if arm == "one":
            gemm(0, M, main_s)
            return
        h = M // 2
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        gemm(0, h, s1)
        if delay_us:
            with torch.cuda.stream(s2):
                torch.cuda._sleep(int(delay_us * cyc_per_us))
        gemm(h, M - h, s2)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

    arms = [("one", 0), ("two", 0)] + [("two", int(d)) for d in a.delays.split(",")]
    for rep in range(2):
        for arm, d in arms:
            for _ in range(3):
                run(arm, d)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run(arm, d)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            print(f"rep {rep} {arm}{d if d else '':<4} {ms:.3f} ms  {2 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
