"""The base encoder's Conv1d + GroupNorm pyramid (reference: pdvc/base_encoder.py:23-86) on channels-last rows
(N, T, C), the layout the deformable transformer consumes -- no transposes on either side.

  * kernel-1 conv = a Linear over rows (ops/functions/linear.py: hipBLASLt, split-K weight gradient);
  * kernel-3 / stride-2 / pad-1 conv: with T = 2L, the rows (x[2t], x[2t+1]) of a video are one contiguous
    2C-wide row of x.view(N*L, 2C), so y[t] = [x[2t] | x[2t+1]] [W1 | W2]^T + b + x[2t-1] W0^T is one GEMM plus
    the W0 tap of the previous odd row, added shifted by one output row (zero at t = 0: the padding);
  * GroupNorm(G, C) on rows: pdvc_groupnorm_rows_* (csrc/groupnorm.hip).
Same parameters (nn.Conv1d / nn.GroupNorm), same math."""
import os

import torch
import torch.nn.functional as F
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n
from .gemm3 import addmm_nt, mm_dgrad, mm_nt
from .linear import colsum, dense, wgrad_mm

GN_ROWS = 64  # rows per stats chunk (csrc/groupnorm.hip kGnRows)
# the stride-2 conv's previous-odd-row tap in an accumulate epilogue (A/B switch: PDVC_CONV_TAP_EPILOGUE=0)
_TAP_EPILOGUE = os.environ.get("PDVC_CONV_TAP_EPILOGUE", "1") != "0"
# its backward on row-shifted views instead of a shifted copy of the gradient (A/B switch: PDVC_CONV_SHIFT_VIEWS=0)
_SHIFT_VIEWS = os.environ.get("PDVC_CONV_SHIFT_VIEWS", "1") != "0"


class ConvS2RowsFunction(Function):
    """Conv1d(C, O, kernel 3, stride 2, padding 1) on x (N, T, C) rows -> (N, ceil(T/2), O)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N, T, C = x.shape
        Tin = T
        if T % 2:
            x = F.pad(x, (0, 0, 0, 1))  # the extra zero row is the right padding of the last odd window
            T += 1
        L = T // 2
        O = weight.shape[0]
        x = x.contiguous()
        X2 = x.view(N * L, 2 * C)
        w12 = torch.cat([weight[:, :, 1], weight[:, :, 2]], 1)  # (O, 2C): taps on x[2t], x[2t+1]
        w0 = weight[:, :, 0].contiguous()                       # (O, C): tap on x[2t-1]
        y = addmm_nt(bias, X2, w12)
        yv = y.view(N, L, O)
        if _TAP_EPILOGUE and N * L > 1:
            # x[2t+1] W0^T added to output row t+1 by the accumulate epilogue of one GEMM over the rows shifted by
            # one (out = y[1:]); the rows it also reaches across a video boundary (each video's row 0, whose tap is
            # the zero padding) are restored from a copy taken before -- the same values as the separate product
            # and add, without the (N, L, O) intermediate and its add pass
            first = yv[1:, 0].clone()
            mm_dgrad(X2[:-1, C:], w0.t().contiguous(), out=y[1:])
            yv[1:, 0] = first
        else:
            z = mm_nt(X2[:, C:], w0)                     # x[2t+1] W0^T feeds output row t+1
            yv[:, 1:] += z.view(N, L, O)[:, :-1]
        ctx.save_for_backward(X2, w12, w0)
        ctx.shape = (N, T, C, L, O, Tin)
        return yv

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        X2, w12, w0 = ctx.saved_tensors
        N, T, C, L, O, Tin = ctx.shape
        dy2 = dy.reshape(N * L, O).contiguous()
        R = N * L
        if _SHIFT_VIEWS and R >= 64 and R % 32 == 0 and O % 32 == 0 and C % 4 == 0:
            return ConvS2RowsFunction._backward_views(ctx, dy2, X2, w12, w0, N, T, C, L, O, Tin)
        dz = torch.empty_like(dy2).view(N, L, O)  # dy shifted up one row per video, zero at the last (one write)
        dz[:, :-1] = dy2.view(N, L, O)[:, 1:]
        dz[:, -1] = 0.0
        dz2 = dz.view(N * L, O)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            dX2 = mm_dgrad(dy2, w12)
            mm_dgrad(dz2, w0, out=dX2[:, C:])
            gx = dX2.view(N, T, C)[:, :Tin]
        if ctx.needs_input_grad[1]:
            gb = dy2.new_empty(dy2.shape[1]) if ctx.needs_input_grad[2] else None
            g12 = wgrad_mm(dy2, X2, db=gb)  # (the bias gradient from the same pass over dy)
            g0 = wgrad_mm(dz2, X2[:, C:])
            gw = torch.stack([g0, g12[:, :C], g12[:, C:]], 2)
        elif ctx.needs_input_grad[2]:
            gb = colsum(dy2)
        return gx, gw, gb

    @staticmethod
    def _backward_views(ctx, dy2, X2, w12, w0, N, T, C, L, O, Tin):
        """The backward without the shifted gradient dz (dz[r] = dy[r + 1] within a video, 0 at its last row): the W0
        tap's products run on views shifted by one row -- dy2[1:] against the rows before -- and the pairs that cross
        a video boundary are taken out again: the data gradient's rows they reach (each video's last odd row) are
        restored from a copy, and the weight gradient subtracts their (N - 1)-row product.  No (N, L, O) copy."""
        R = N * L
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            dX2 = mm_dgrad(dy2, w12)
            d3 = dX2.view(N, L, 2 * C)
            keep = d3[:-1, -1, C:].clone() if N > 1 else None  # each video's last odd row: its tap is the padding
            mm_dgrad(dy2[1:], w0, out=dX2[:-1, C:])
            if keep is not None:
                d3[:-1, -1, C:] = keep
            gx = d3.view(N, T, C)[:, :Tin]
        if ctx.needs_input_grad[1]:
            gb = dy2.new_empty(O) if ctx.needs_input_grad[2] else None
            g12 = wgrad_mm(dy2, X2, db=gb)  # (the bias gradient from the same pass over dy)
            # g0 = sum over rows r < R - 1 of dy2[r + 1]^T x_odd[r], minus the cross-video pairs: the first R - 32 rows
            # as one split-K product (its row count a multiple of 32), the last 31 and the corrections as small ones
            xo = X2[:, C:]
            g0 = wgrad_mm(dy2[1:R - 31], xo[:R - 32])
            g0.addmm_(dy2[R - 31:].t(), xo[R - 32:R - 1])
            if N > 1:
                g0.addmm_(dy2.view(N, L, O)[1:, 0].t(), xo.view(N, L, C)[:-1, -1], alpha=-1.0)
            gw = torch.stack([g0, g12[:, :C], g12[:, C:]], 2)
        elif ctx.needs_input_grad[2]:
            gb = colsum(dy2)
        return gx, gw, gb


def _fused_forward(x, N, T, C, G, eps, weight, bias, y, ys, y2, mean, rstd, y16=None):
    """The single-pass GroupNorm forward (pdvc_groupnorm_rows_forward_fused_f32: x read once, statistics from
    registers) into y (video stride ys) / y2 / mean / rstd, and y's bf16 rounding into y16 (same offsets) when given;
    False (nothing launched) for shapes it does not serve."""
    try:
        _n.call("pdvc_groupnorm_rows_forward_fused_f32", _n.ptr(x), N, T, C, G, float(eps), _n.ptr(weight),
                _n.ptr(bias), _n.ptr_any(y), ys, _n.ptr(y2), _n.ptr(mean), _n.ptr(rstd),
                None if y16 is None else _n.ptr_any(y16), _n.stream())
        return True
    except _n.NativeError:
        return False


def _fused_backward(x, dy, dys, dy_add, mean, rstd, weight, N, T, C, G, dx):
    """The single-pass GroupNorm backward (pdvc_groupnorm_rows_backward_fused_f32: x and dy read once) into dx;
    returns its (N, 2C) [dgamma | dbeta] partials, or None (nothing launched) for shapes it does not serve."""
    cpart = torch.empty(N, 2 * C, dtype=x.dtype, device=x.device)
    try:
        _n.call("pdvc_groupnorm_rows_backward_fused_f32", _n.ptr(x), _n.ptr_any(dy), dys, _n.ptr(dy_add),
                _n.ptr(mean), _n.ptr(rstd), _n.ptr(weight), N, T, C, G, _n.ptr(cpart), _n.ptr(dx), _n.stream())
        return cpart
    except _n.NativeError:
        return None


class GroupNormRowsFunction(Function):
    """nn.GroupNorm(G, C) of x (N, T, C) rows (statistics per video and group over T x C/G values)."""

    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps):
        x = x.contiguous()
        N, T, C = x.shape
        chunks = (T + GN_ROWS - 1) // GN_ROWS
        kw = dict(dtype=x.dtype, device=x.device)
        y = torch.empty_like(x)
        mean = torch.empty(N * groups, **kw)
        rstd = torch.empty(N * groups, **kw)
        if not _fused_forward(x, N, T, C, groups, eps, weight, bias, y, T * C, None, mean, rstd):
            ws = torch.empty(N * chunks * groups * 3, **kw)
            _n.call("pdvc_groupnorm_rows_forward_f32", _n.ptr(x), N, T, C, groups, float(eps), _n.ptr(weight),
                    _n.ptr(bias), _n.ptr(ws), _n.ptr(y), _n.ptr(mean), _n.ptr(rstd), _n.stream())
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.groups = groups
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, weight, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        N, T, C = x.shape
        G = ctx.groups
        chunks = (T + GN_ROWS - 1) // GN_ROWS
        kw = dict(dtype=x.dtype, device=x.device)
        dx = torch.empty_like(x)
        cpart = _fused_backward(x, dy, T * C, None, mean, rstd, weight, N, T, C, G, dx)
        if cpart is None:
            gws = torch.empty(N * chunks * G * 2 + N * G * 2, **kw)
            cpart = torch.empty(N * chunks, 2 * C, **kw)
            _n.call("pdvc_groupnorm_rows_backward_f32", _n.ptr(x), _n.ptr(dy), _n.ptr(mean), _n.ptr(rstd),
                    _n.ptr(weight), N, T, C, G, _n.ptr(gws), _n.ptr(cpart), _n.ptr(dx), _n.stream())
        gsum = colsum(cpart)
        return dx, gsum[:C].contiguous(), gsum[C:].contiguous(), None, None


class GroupNormFlatFunction(Function):
    """GroupNormRowsFunction writing its result straight into rows [start, start + T) of every video of the
    flattened pyramid `flat` (N, S, C) -- in place, so the levels need no torch.cat (reference:
    deformable_transformer.py:84-106 flattens and concatenates the level outputs).  With `want_copy` it also
    returns the contiguous (N, T, C) result, the input of the next level's convolution; its gradient is added to
    the slice's inside the backward kernels instead of by autograd."""

    @staticmethod
    def forward(ctx, flat, x, weight, bias, groups, eps, start, want_copy, flat16=None):
        x = x.contiguous()
        N, T, C = x.shape
        S = flat.shape[1]
        chunks = (T + GN_ROWS - 1) // GN_ROWS
        kw = dict(dtype=x.dtype, device=x.device)
        y2 = torch.empty_like(x) if want_copy else None
        mean = torch.empty(N * groups, **kw)
        rstd = torch.empty(N * groups, **kw)
        s16 = None if flat16 is None else flat16[:, start:start + T]
        if not _fused_forward(x, N, T, C, groups, eps, weight, bias, flat[:, start:start + T], S * C, y2, mean, rstd,
                              s16):
            ws = torch.empty(N * chunks * groups * 3, **kw)
            _n.call("pdvc_groupnorm_rows_forward_out_f32", _n.ptr(x), N, T, C, groups, float(eps), _n.ptr(weight),
                    _n.ptr(bias), _n.ptr(ws), _n.ptr_any(flat[:, start:start + T]), S * C, _n.ptr(y2), _n.ptr(mean),
                    _n.ptr(rstd), _n.stream())
            if s16 is not None:  # the chunked forms write no bf16 copy: the slice is rounded here
                s16.copy_(flat[:, start:start + T])
        ctx.mark_dirty(flat)
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.meta = (groups, start, S, want_copy)
        return (flat, y2) if want_copy else flat

    @staticmethod
    @once_differentiable
    def backward(ctx, d_flat, d_copy=None):
        x, weight, mean, rstd = ctx.saved_tensors
        G, start, S, want_copy = ctx.meta
        N, T, C = x.shape
        d_flat = d_flat.contiguous() if d_flat is not None else x.new_zeros(N, S, C)
        d_copy = d_copy.contiguous() if d_copy is not None else None
        chunks = (T + GN_ROWS - 1) // GN_ROWS
        kw = dict(dtype=x.dtype, device=x.device)
        dx = torch.empty_like(x)
        cpart = _fused_backward(x, d_flat[:, start:start + T], S * C, d_copy, mean, rstd, weight, N, T, C, G, dx)
        if cpart is None:
            gws = torch.empty(N * chunks * G * 2 + N * G * 2, **kw)
            cpart = torch.empty(N * chunks, 2 * C, **kw)
            _n.call("pdvc_groupnorm_rows_backward_strided_f32", _n.ptr(x), _n.ptr_any(d_flat[:, start:start + T]),
                    S * C, _n.ptr(d_copy), _n.ptr(mean), _n.ptr(rstd), _n.ptr(weight), N, T, C, G, _n.ptr(gws),
                    _n.ptr(cpart), _n.ptr(dx), _n.stream())
        gsum = colsum(cpart)
        # the slice [start, start + T) of the incoming flat was overwritten: only the earlier levels' functions
        # (which read their own slices) consume this gradient, so it passes through unmasked
        return d_flat, dx, gsum[:C].contiguous(), gsum[C:].contiguous(), None, None, None, None, None


def group_norm_rows_ok(gn, x):
    C = x.shape[-1]
    cpg = C // gn.num_groups
    return (x.is_cuda and x.dtype == torch.float32 and gn.affine and C % 4 == 0 and 256 % (C // 4) == 0
            and cpg % 4 == 0 and (cpg // 4) & (cpg // 4 - 1) == 0)


def group_norm_rows_into(gn, x, flat, start, want_copy, flat16=None):
    """group_norm_rows(gn, x) written into flat[:, start:start + T] (see GroupNormFlatFunction), and its bf16 rounding
    into the same rows of flat16 when given (the bf16 mode).  Returns the new flat (and the contiguous result when
    want_copy)."""
    return GroupNormFlatFunction.apply(flat, x, gn.weight, gn.bias, gn.num_groups, gn.eps, start, want_copy, flat16)


def conv1d_rows(conv, x):
    """nn.Conv1d (kernel 1, or kernel 3 / stride 2 / padding 1) applied to x (N, T, C) rows."""
    k = conv.weight.shape[2]
    if k == 1:
        return dense(x, conv.weight[:, :, 0], conv.bias)
    if not (k == 3 and conv.stride[0] == 2 and conv.padding[0] == 1 and conv.dilation[0] == 1 and conv.groups == 1):
        raise NotImplementedError("conv1d_rows supports kernel 1, or kernel 3 with stride 2 / padding 1")
    return ConvS2RowsFunction.apply(x, conv.weight, conv.bias)


def group_norm_rows(gn, x):
    """nn.GroupNorm applied to x (N, T, C) rows (falls back to torch off the GPU / for other group shapes)."""
    if not group_norm_rows_ok(gn, x):
        return F.group_norm(x.transpose(1, 2), gn.num_groups, gn.weight, gn.bias, gn.eps).transpose(1, 2)
    return GroupNormRowsFunction.apply(x, gn.weight, gn.bias, gn.num_groups, gn.eps)
