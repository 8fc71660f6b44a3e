"""fp32 products of PDVC's large nn.Linear layers on the bf16 matrix cores (csrc/gemm3.hip, pdvc_gemm3*_f32).

gfx950 has no xf32, and its f32-input MFMA runs at 1/16 of the bf16 rate.  pdvc_gemm3 splits each fp32 operand
exactly into three bf16 terms and keeps the six products of order >= 2^-16 (the dropped ones are <= 2^-23 |a||b|,
one fp32 product rounding is 2^-24), accumulating in fp32: an fp32 GEMM whose error against float64 is at or below
hipBLASLt's fp32 GEMM on the same operands (tests/test_gpu_gemm3.py measures both), at up to ~1.8x its rate.

These helpers are drop-in for the torch calls of the projections (pdvc/ops/modules/ms_deform_attn.py:55-58,
deformable_transformer.py:162-189 in the reference -- torch.addmm / mm in the forward, and the input- and
weight-gradient products of their backward), with the same argument meaning:

    addmm_nt(bias, x, W, relu=False)  = torch.addmm(bias, x, W.t())  (+ ReLU)
    mm_nt(x, W)                       = x @ W.t()
    mm_dgrad(dy, W, out=None)         = dy @ W; out given: out += dy @ W  (out.addmm_(dy, W))
    mm_wgrad(gy, x, out=None)         = gy.t() @ x, the reduction over all rows split over workgroups

Shapes the kernels do not take (K not a multiple of 32, unaligned or strided operands, few rows) and the bf16 mode
(pdvc/precision.py, which reroutes torch's GEMMs to bf16 operands) go to torch, i.e. hipBLASLt -- a GPU library
path, never a CPU one.  PDVC_GEMM3=0 sends everything to torch (the A/B switch).
"""
import os

import torch

from pdvc import _native as _n

ENABLED = os.environ.get("PDVC_GEMM3", "1") != "0"
MIN_ROWS = int(os.environ.get("PDVC_GEMM3_MIN_ROWS", "8192"))  # below: launch-bound shapes stay on hipBLASLt
CALLS = {"gemm3": 0, "torch": 0}  # how many products took each path (tests check the encoder takes gemm3)
FLOPS = [0]  # algorithmic 2*M*N*K of every product issued on gemm3 (bench.py's roofline counts them)
EXECUTED_PER_ALGORITHMIC = 6  # bf16 MFMA products per fp32 product (the six split terms)


def _bf16_mode():
    from pdvc.precision import bf16_active
    return bf16_active()


def _rows_ok(t):
    """A 2-D fp32 GPU operand with unit column stride, 16-byte aligned rows."""
    return (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 4 == 0
            and t.data_ptr() % 16 == 0 and t.stride(0) >= t.shape[1])


def _use(M, K, *ops, extra=True):
    if (not extra or not ENABLED or M < MIN_ROWS or K % 32 != 0 or not all(_rows_ok(t) for t in ops)
            or _bf16_mode()):
        CALLS["torch"] += 1
        return False
    CALLS["gemm3"] += 1
    return True


def split_planes(B, b_kc, N, K):
    """The three bf16 planes [3][N][K] of opB[n][k] (b_kc 1: B[n][k]; 0: B[k][n], i.e. opB = B^T)."""
    planes = torch.empty((3, N, K), dtype=torch.int16, device=B.device)
    _n.call("pdvc_split3_planes_f32", _n.ptr_any(B), B.stride(0), int(b_kc), N, K, _n.ptr(planes), _n.stream())
    return planes


def _gemm3p(a, planes, N, out, bias, epi):
    M, K = a.shape
    FLOPS[0] += 2 * M * N * K
    _n.call("pdvc_gemm3p_f32", M, N, K, _n.ptr_any(a), a.stride(0), _n.ptr(planes), _n.ptr_any(out), out.stride(0),
            _n.ptr(bias), epi, _n.stream())
    return out


def addmm_nt(bias, x, W, relu=False, out=None):
    """torch.addmm(bias, x, W.t()) (bias may be None), + ReLU when relu=True; out: an (M, N) row-strided
    destination (written)."""
    M, K = x.shape
    N = W.shape[0]
    ok_out = out is None or (_rows_ok(out) and out.shape == (M, N))
    if not _use(M, K, x, W, extra=W.is_contiguous() and (bias is None or bias.is_contiguous()) and ok_out):
        if out is not None:
            if bias is None:
                torch.mm(x, W.t(), out=out)
            else:
                torch.addmm(bias, x, W.t(), out=out)
            return out.relu_() if relu else out
        if bias is None:
            y = torch.mm(x, W.t())
            return y.relu_() if relu else y
        if relu:
            return torch._addmm_activation(bias, x, W.t(), use_gelu=False)
        return torch.addmm(bias, x, W.t())
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    epi = 0 if bias is None else (2 if relu else 1)
    if bias is None and relu:
        _gemm3p(x, split_planes(W, 1, N, K), N, out, None, 0)
        return out.relu_()
    if generic_wins(M, N, K):  # gemm3p's 256 x 256 tiles would leave the last wave mostly empty
        FLOPS[0] += 2 * M * N * K
        _n.call("pdvc_gemm3_f32", M, N, K, _n.ptr_any(x), x.stride(0), 1, _n.ptr_any(W), W.stride(0), 1,
                _n.ptr_any(out), out.stride(0), _n.ptr(bias), epi, 1, None, _n.stream())
        return out
    return _gemm3p(x, split_planes(W, 1, N, K), N, out, bias, epi)


GENERIC_STAGE_COST = 1.14  # gemm3_kernel's 256 x 128 x 32 stage against gemm3p's 256 x 256 x 16 (same flops)
TILE_MODEL = os.environ.get("PDVC_GEMM3_TILE_MODEL", "1") != "0"


def generic_wins(M, N, K):
    """Launch cost model (one workgroup per CU, whole waves): gemm3p takes ceil(tiles / 256) waves of K / 16
    stages, the generic kernel's 256 x 128 tiles ceil(tiles / 256) waves of K / 32 slower stages.  The generic tile
    wins only where gemm3p's last wave is mostly empty (e.g. 352 tiles: 2 waves against 3 waves of half-depth
    stages) -- at whole or nearly whole waves gemm3p's faster stage decides."""
    if not TILE_MODEL:
        return False
    wp = (((M + 255) // 256) * ((N + 255) // 256) + 255) // 256
    wg = (((M + 255) // 256) * ((N + 127) // 128) + 255) // 256
    return wg * (K / 32) * GENERIC_STAGE_COST < 0.9 * wp * (K / 16)


def addmm_relu_dropout_nt(bias, x, W, p, seed_ptr):
    """dropout(relu(torch.addmm(bias, x, W.t())), p) with the keep mask of pdvc_relu_dropout_forward_f32 for the
    device seed at seed_ptr, as one gemm3 launch (the epilogue does the relu and the mask), or None when the shape
    does not take gemm3 (the caller then runs the GEMM and the relu-dropout pass)."""
    M, K = x.shape
    N = W.shape[0]
    if not (0.0 < p < 1.0) or seed_ptr is None or bias is None or M >= 2 ** 32:
        return None
    if not _use(M, K, x, W, extra=W.is_contiguous() and bias.is_contiguous()):
        return None
    out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    FLOPS[0] += 2 * M * N * K
    planes = split_planes(W, 1, N, K)
    _n.call("pdvc_gemm3p_relu_dropout_f32", M, N, K, _n.ptr_any(x), x.stride(0), _n.ptr(planes), _n.ptr(out), N,
            _n.ptr(bias), float(p), seed_ptr, _n.stream())
    return out


RESID_EPILOGUE = os.environ.get("PDVC_RESID_FUSE", "1") != "0"


def addmm_resid_dropout_nt(bias, x, W, resid, p, seed_ptr):
    """resid + dropout(torch.addmm(bias, x, W.t()), p) -- the residual sub-layer's sum before its LayerNorm -- as one
    gemm3p launch whose epilogue applies the add-norm pass's keep mask for the device seed at seed_ptr
    (pdvc_gemm3p_resid_dropout_f32; p = 0: no mask), or None when the product does not take gemm3p (the caller then
    runs the GEMM and the two-input add-norm pass)."""
    M, K = x.shape
    N = W.shape[0]
    if not RESID_EPILOGUE or bias is None or M >= 2 ** 31 or not (0.0 <= p < 1.0) or (p > 0 and seed_ptr is None):
        return None
    if not _use(M, K, x, W, extra=(W.is_contiguous() and bias.is_contiguous() and resid.is_contiguous()
                                   and resid.shape == (M, N))):
        return None
    if generic_wins(M, N, K):
        return None
    out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    FLOPS[0] += 2 * M * N * K
    planes = split_planes(W, 1, N, K)
    _n.call("pdvc_gemm3p_resid_dropout_f32", M, N, K, _n.ptr_any(x), x.stride(0), _n.ptr(planes), _n.ptr(out), N,
            _n.ptr(bias), _n.ptr(resid), float(p), seed_ptr if p > 0 else None, _n.stream())
    return out


def mm_nt(x, W, out=None):
    return addmm_nt(None, x, W, out=out)


def mm_dgrad(dy, W, out=None, accumulate=True):
    """dy @ W for dy (M, O) and W (O, I): the input gradient of y = x W^T.  out given (M, I): out += dy @ W, or
    out = dy @ W with accumulate=False."""
    M, K = dy.shape
    N = W.shape[1]
    ok = _use(M, K, dy, W, extra=W.is_contiguous() and (out is None or (_rows_ok(out) and out.shape == (M, N))))
    if not ok:
        if out is None:
            return torch.mm(dy, W)
        return out.addmm_(dy, W) if accumulate else torch.mm(dy, W, out=out)
    splits = dgrad_splits(M, N, K)
    if splits > 1 and (out is None or out.is_contiguous()):
        # few output tiles over a deep reduction (the caption logit layer's input gradient: ~8 K rows x 512 over
        # K = 5 760): gemm3p would run one workgroup per tile on a quarter of the CUs, so the reduction is split
        # over workgroups on the generic kernel and the slabs summed in a fixed order (deterministic)
        if out is None:
            out = torch.empty((M, N), dtype=torch.float32, device=dy.device)
            epi = 0
        else:
            epi = 3 if accumulate else 0
        FLOPS[0] += 2 * M * N * K
        ws = torch.empty(splits * M * N, dtype=torch.float32, device=dy.device)
        _n.call("pdvc_gemm3_f32", M, N, K, _n.ptr_any(dy), dy.stride(0), 1, _n.ptr_any(W), W.stride(0), 0,
                _n.ptr(out), N, None, epi, splits, _n.ptr(ws), _n.stream())
        return out
    planes = split_planes(W, 0, N, K)
    if out is None:
        return _gemm3p(dy, planes, N, torch.empty((M, N), dtype=torch.float32, device=dy.device), None, 0)
    return _gemm3p(dy, planes, N, out, None, 3 if accumulate else 0)


def mm_dgrad_dmask(dy, W, hd, p):
    """dy @ W masked as the feed-forward block's relu -> dropout backward: hd > 0 ? (dy @ W) / (1 - p) : 0, with hd
    the forward's relu -> dropout output (M, I) -- one gemm3p launch (pdvc_gemm3p_dmask_f32) -- or None when the
    product does not take gemm3p (the caller runs the GEMM and the relu-dropout backward pass)."""
    M, K = dy.shape
    N = W.shape[1]
    if not (0.0 <= p < 1.0) or dgrad_splits(M, N, K) > 1:
        return None
    if not _use(M, K, dy, W, extra=W.is_contiguous() and hd.is_contiguous() and hd.shape == (M, N)):
        return None
    out = torch.empty((M, N), dtype=torch.float32, device=dy.device)
    FLOPS[0] += 2 * M * N * K
    planes = split_planes(W, 0, N, K)
    _n.call("pdvc_gemm3p_dmask_f32", M, N, K, _n.ptr_any(dy), dy.stride(0), _n.ptr(planes), _n.ptr(out), N,
            _n.ptr(hd), float(p), _n.stream())
    return out


def dgrad_splits(M, N, K):
    """Split-K factor of a data-gradient product: 1 when gemm3p's 256 x 256 tiles already give >= 128 workgroups or
    the reduction is short; else enough K chunks of >= 512 for ~512 workgroups of the generic 256 x 128 tile."""
    if ((M + 255) // 256) * ((N + 255) // 256) >= 128 or K < 1024 or N % 4:
        return 1
    tiles = ((M + 255) // 256) * ((N + 127) // 128)
    return max(1, min((512 + tiles - 1) // tiles, K // 512, 64))


def wgrad_splits(rows, tiles, O=256, I=256):
    """Row chunks of a weight gradient's reduction, by a cost model of gemm3w's launch: one workgroup per CU, so a
    grid of tiles x splits workgroups runs in ceil(/256) waves of ceil(rows / splits / 16) stages each (≈1.9 µs a
    stage, measured at the encoder's shapes), plus the slabs' write and fixed-order sum (8 B per output element and
    split at ≈5 TB/s).  Chunks of at least WGRAD_MIN_CHUNK rows.  (A fixed two-workgroups-per-CU rule left the
    decoder's 8 192-row products at 200 workgroups, 0.78 of a wave, and doubling them to 400 only moved the loss
    into a second wave.)"""
    smax = max(1, min(rows // WGRAD_MIN_CHUNK, 1024))
    if not WGRAD_MODEL:  # the A/B baseline: about two workgroups per CU over the output tiles
        return max(1, min((512 + tiles - 1) // tiles, smax))
    best, best_t = 1, None
    for s in range(1, smax + 1):
        waves = (tiles * s + 255) // 256
        stages = (-(-rows // s) + 15) // 16
        t = waves * stages * 1.9 + (s * O * I * 8 / 5e6 if s > 1 else 0.0)
        if best_t is None or t < best_t - 1e-9:
            best, best_t = s, t
    return best


WGRAD_MIN_CHUNK = int(os.environ.get("PDVC_WGRAD_MIN_CHUNK", "1024"))
WGRAD_MODEL = os.environ.get("PDVC_WGRAD_MODEL", "1") != "0"


# the bias gradient (column sums of gy) taken by the weight-gradient GEMM from the rows it loads (A/B switch)
WGRAD_BIAS = os.environ.get("PDVC_WGRAD_BIAS", "1") != "0"


def wgrad_bias_ok(gy, x, db):
    """Whether mm_wgrad can take gy.sum(0) into db in the same pass (pdvc_gemm3_wgrad_bias_f32's layout rules)."""
    return (WGRAD_BIAS and db.is_cuda and db.dtype == torch.float32 and db.is_contiguous()
            and db.shape == (gy.shape[1],) and db.data_ptr() % 16 == 0 and gy.stride(1) == 1 and x.stride(1) == 1
            and gy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0 and gy.stride(0) % 4 == 0
            and x.stride(0) % 4 == 0 and gy.shape[1] >= 4 and x.shape[1] >= 4)


def mm_wgrad(gy, x, out=None, db=None):
    """gy^T x for gy (rows, O) and x (rows, I): the weight gradient of y = x W^T, deterministic (row chunks summed
    in a fixed order).  out: a contiguous (O, I) destination (written, not accumulated).  db: a contiguous (O,)
    destination for gy.sum(0) (the bias gradient, wgrad_bias_ok), computed by the same kernel from the gy rows it
    loads (pdvc_gemm3_wgrad_bias_f32).  None (nothing written) when the shapes leave gemm3w."""
    rows, O = gy.shape
    I = x.shape[1]
    ok = _use(rows, 32, gy, x, extra=(O % 4 == 0 and I % 4 == 0 and rows % 32 == 0
                                      and (out is None or (out.is_contiguous() and out.shape == (O, I)))))
    if not ok:
        return None
    if db is not None and not wgrad_bias_ok(gy, x, db):
        raise ValueError("mm_wgrad: db needs wgrad_bias_ok(gy, x, db)")
    if out is None:
        out = torch.empty((O, I), dtype=torch.float32, device=gy.device)
    tiles = ((O + 255) // 256) * ((I + 255) // 256)  # gemm3w tiles
    splits = wgrad_splits(rows, tiles, O, I)
    FLOPS[0] += 2 * rows * O * I
    ws = torch.empty(splits * O * I if splits > 1 else 0, dtype=torch.float32, device=gy.device)
    if db is None:
        _n.call("pdvc_gemm3_f32", O, I, rows, _n.ptr_any(gy), gy.stride(0), 0, _n.ptr_any(x), x.stride(0), 0,
                _n.ptr_any(out), I, None, 0, splits, _n.ptr(ws) if splits > 1 else None, _n.stream())
        return out
    dws = torch.empty(splits * O if splits > 1 else 0, dtype=torch.float32, device=gy.device)
    _n.call("pdvc_gemm3_wgrad_bias_f32", O, I, rows, _n.ptr_any(gy), gy.stride(0), _n.ptr_any(x), x.stride(0),
            _n.ptr_any(out), I, 0, splits, _n.ptr(ws) if splits > 1 else None, _n.ptr(db),
            _n.ptr(dws) if splits > 1 else None, _n.stream())
    return out
