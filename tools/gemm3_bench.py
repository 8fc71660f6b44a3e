"""pdvc_gemm3_f32 (fp32 GEMM by exact three-term bf16 split, csrc/gemm3.hip) against hipBLASLt fp32 (torch) on the
encoder's nn.Linear shapes: forward (x W^T + b), data gradient (dy W) and weight gradient (dy^T x over all rows).
Prints TF/s (algorithmic fp32 flops) and the error of both against float64 (max |c - ref| / sum_k |a||b|, and
relative to max |ref|).

    python tools/gemm3_bench.py [--rows 983040] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dense-video-captioning_amd"))
from pdvc import _native as _n  # noqa: E402


def gemm3(M, N, K, A, lda, akc, B, ldb, bkc, C, ldc, bias=None, epi=0, splits=1, ws=None):
    _n.call("pdvc_gemm3_f32", M, N, K, _n.ptr_any(A), lda, akc, _n.ptr_any(B), ldb, bkc, _n.ptr_any(C), ldc,
            _n.ptr(bias), epi, splits, None if ws is None else _n.ptr_any(ws), _n.stream())


def gemm3p(M, N, K, A, lda, B, ldb, bkc, planes, C, ldc, bias=None, epi=0):
    _n.call("pdvc_split3_planes_f32", _n.ptr_any(B), ldb, bkc, N, K, _n.ptr_any(planes), _n.stream())
    _n.call("pdvc_gemm3p_f32", M, N, K, _n.ptr_any(A), lda, _n.ptr_any(planes), _n.ptr_any(C), ldc, _n.ptr(bias), epi,
            _n.stream())


def gemm1p(M, N, K, A, lda, B, ldb, bkc, plane, C, ldc, bias=None, epi=0):
    _n.call("pdvc_round_plane_f32", _n.ptr_any(B), ldb, bkc, N, K, _n.ptr_any(plane), _n.stream())
    _n.call("pdvc_gemm1p_f32", M, N, K, _n.ptr_any(A), lda, _n.ptr_any(plane), _n.ptr_any(C), ldc, _n.ptr(bias), epi,
            _n.stream())


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def err(c, ref, scale):
    d = (c.double() - ref).abs()
    return {"max_rel_sum": float((d / scale.clamp_min(1e-300)).max()), "max_rel_ref": float(d.max() / ref.abs().max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=983040)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", type=int, default=64)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="", help="comma list of ops (fwd,dgrad,wgrad); empty = all")
    ap.add_argument("--shapes", default="512x512,256x512,512x256", help="OxI list")
    ap.add_argument("--no-err", action="store_true")
    ap.add_argument("--mnk", default="", help="fwdp only at M,N,K (e.g. 245760,512,2048)")
    ap.add_argument("--accum", action="store_true", help="with --mnk: also the accumulate epilogue")
    ap.add_argument("--bf16", action="store_true",
                    help="the bf16 mode's product: gemm1p against cast + hipBLASLt bf16 (fp32 result), M,N,K list")
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = "cuda"
    M = a.rows
    res = []
    only = set(a.only.split(",")) if a.only else {"fwd", "dgrad", "wgrad", "fwdp", "dgradp"}
    ref_lib = os.environ.get("PDVC_GEMM3_NO_BLASLT") is None

    def run(op, Mo, No, Ko, ours, blaslt, check):
        fl = 2.0 * Mo * No * Ko
        r = {"op": op, "M": Mo, "N": No, "K": Ko}
        r["ours_ms"] = timeit(ours, a.iters)
        r["ours_tfs"] = fl / r["ours_ms"] / 1e9
        if ref_lib:
            r["blaslt_ms"] = timeit(blaslt, a.iters)
            r["blaslt_tfs"] = fl / r["blaslt_ms"] / 1e9
        if not a.no_err:
            r["err_ours"], r["err_blaslt"] = check()
        res.append(r)
        print(json.dumps(r), flush=True)

    if a.bf16:
        aten = torch.ops.aten
        for mnk in (a.mnk or "245760,512,512,0;245760,2048,512,0;245760,512,2048,3;245760,256,512,1").split(";"):
            Mx, Nx, Kx, epi = (int(v) for v in mnk.split(","))
            x = torch.randn(Mx, Kx, device=dev)
            W = torch.randn(Nx, Kx, device=dev) / Kx ** 0.5
            b = torch.randn(Nx, device=dev)
            y = torch.randn(Mx, Nx, device=dev)
            y0 = y.clone()
            plane = torch.empty(Nx * Kx, dtype=torch.int16, device=dev)
            bb = b if epi in (1, 2) else None
            ours = lambda: gemm1p(Mx, Nx, Kx, x, Kx, W, Kx, 1, plane, y, Nx, bb, epi)  # noqa: E731
            x16 = x.to(torch.bfloat16)

            def theirs(cast=True):
                xb = x.to(torch.bfloat16) if cast else x16
                wb = W.to(torch.bfloat16)
                if epi == 3:
                    return aten.addmm.dtype_out(y, xb, wb.t(), torch.float32, out=y)
                if epi == 0:
                    return aten.mm.dtype(xb, wb.t(), torch.float32)
                r = aten.addmm.dtype(b, xb, wb.t(), torch.float32)
                return r.relu_() if epi == 2 else r
            fl = 2.0 * Mx * Nx * Kx
            r = {"op": f"bf16 epi{epi}", "M": Mx, "N": Nx, "K": Kx}
            y.copy_(y0)
            ours()
            torch.cuda.synchronize()
            sub = 4096
            ref = x[:sub].to(torch.bfloat16).double() @ W.to(torch.bfloat16).double().t()
            if epi in (1, 2):
                ref = ref + b.double()
            if epi == 2:
                ref = ref.clamp_min(0)
            if epi == 3:
                ref = ref + y0[:sub].double()
            scale = x[:sub].double().abs() @ W.double().abs().t()
            r["err_ours_vs_bf16_operands"] = float(((y[:sub].double() - ref).abs() / scale).max())
            r["ours_ms"] = timeit(ours, a.iters)
            r["ours_tfs"] = fl / r["ours_ms"] / 1e9
            r["blaslt_cast_ms"] = timeit(theirs, a.iters)
            r["blaslt_precast_ms"] = timeit(lambda: theirs(False), a.iters)
            r["blaslt_precast_tfs"] = fl / r["blaslt_precast_ms"] / 1e9
            res.append(r)
            print(json.dumps(r), flush=True)
            del x, W, y, y0, x16
            torch.cuda.empty_cache()
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        return
    if a.mnk:
        Mx, Nx, Kx = (int(v) for v in a.mnk.split(","))
        x = torch.randn(Mx, Kx, device=dev)
        W = torch.randn(Nx, Kx, device=dev)
        b = torch.randn(Nx, device=dev)
        y = torch.empty(Mx, Nx, device=dev)
        planes = torch.empty(3 * Nx * Kx, dtype=torch.int16, device=dev)
        run("fwdp", Mx, Nx, Kx, lambda: gemm3p(Mx, Nx, Kx, x, Kx, W, Kx, 1, planes, y, Nx, b, 1),
            lambda: torch.addmm(b, x, W.t()), lambda: ({}, {}))
        if a.accum:  # the accumulate epilogue (C += A B^T): the FFN's residual + input-gradient GEMM
            run("fwdp_accum", Mx, Nx, Kx, lambda: gemm3p(Mx, Nx, Kx, x, Kx, W, Kx, 1, planes, y, Nx, None, 3),
                lambda: y.addmm_(x, W.t()), lambda: ({}, {}))
        return
    for (O, I) in [tuple(int(v) for v in sh.split("x")) for sh in a.shapes.split(",")]:
        x = torch.randn(M, I, device=dev)
        W = torch.randn(O, I, device=dev) / I ** 0.5
        b = torch.randn(O, device=dev)
        dy = torch.randn(M, O, device=dev)
        y = torch.empty(M, O, device=dev)
        dx = torch.empty(M, I, device=dev)
        dW = torch.empty(O, I, device=dev)
        ws = torch.empty(a.splits * O * I, device=dev)
        planes = torch.empty(3 * O * I, dtype=torch.int16, device=dev)
        sub = 4096
        s = 64

        def chk_fwd():
            ref = torch.addmm(b.double(), x[:sub].double(), W.double().t())
            scale = x[:sub].double().abs() @ W.double().abs().t() + b.double().abs()
            return err(y[:sub], ref, scale), err(torch.addmm(b, x[:sub], W.t()), ref, scale)

        def chk_dgrad():
            ref = dy[:sub].double() @ W.double()
            scale = dy[:sub].double().abs() @ W.double().abs()
            return err(dx[:sub], ref, scale), err(torch.mm(dy[:sub], W), ref, scale)

        def chk_wgrad():
            ref = dy.double().t() @ x.double()
            scale = dy.double().abs().t() @ x.double().abs()
            theirs = torch.bmm(dy.view(s, M // s, O).transpose(1, 2), x.view(s, M // s, I)).sum(0)
            return err(dW, ref, scale), err(theirs, ref, scale)

        if "fwd" in only:  # y = x W^T + b
            run("fwd", M, O, I, lambda: gemm3(M, O, I, x, I, 1, W, I, 1, y, O, b, 1),
                lambda: torch.addmm(b, x, W.t()), chk_fwd)
        if "dgrad" in only:  # dx = dy W
            run("dgrad", M, I, O, lambda: gemm3(M, I, O, dy, O, 1, W, I, 0, dx, I), lambda: torch.mm(dy, W), chk_dgrad)
        if "fwdp" in only:  # the same with W split once into bf16 planes
            run("fwdp", M, O, I, lambda: gemm3p(M, O, I, x, I, W, I, 1, planes, y, O, b, 1),
                lambda: torch.addmm(b, x, W.t()), chk_fwd)
        if "dgradp" in only:
            run("dgradp", M, I, O, lambda: gemm3p(M, I, O, dy, O, W, I, 0, planes, dx, I), lambda: torch.mm(dy, W),
                chk_dgrad)
        if "wgrad" in only:  # dW = dy^T x over all rows, split
            run("wgrad", O, I, M, lambda: gemm3(O, I, M, dy, O, 0, x, I, 0, dW, I, None, 0, a.splits, ws),
                lambda: torch.bmm(dy.view(s, M // s, O).transpose(1, 2), x.view(s, M // s, I)).sum(0), chk_wgrad)
        del x, W, b, dy, y, dx, dW, ws, planes
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
