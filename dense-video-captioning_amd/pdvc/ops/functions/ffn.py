"""The transformer feed-forward sub-layer as one autograd node:
    out = norm(x + dropout_out(linear2(dropout_act(relu(linear1(x))))))
(reference: DeformableTransformerEncoderLayer.forward_ffn, deformable_transformer.py:140-145; the decoder's
forward_ffn, :233-237).  Same arithmetic as the module chain; what changes is where the passes over the
(rows x d_ffn) and (rows x d) tensors go:
  * relu + dropout runs in linear1's gemm3 epilogue when linear1 takes gemm3 (pdvc_gemm3p_relu_dropout_f32),
    else as one in-place HIP pass (csrc/ffn.hip) -- the same mask bits either way; its backward runs in linear2's
    data-gradient epilogue (pdvc_gemm3p_dmask_f32) with linear1's bias gradient a column sum, else as one pass
    that also sums that gradient (no byte mask either way: the forward output itself says where relu passed and
    dropout kept);
  * the residual gradient from the layer norm and linear1's input gradient meet in the dgrad GEMM's epilogue
    (dx = dx_residual + dh W1, beta = 1) instead of an autograd add;
  * the residual sum x + dropout(linear2(h)) is formed in linear2's gemm3 epilogue (pdvc_gemm3p_resid_dropout_f32,
    the add-norm pass's mask bits) and the residual epilogue pdvc_add_dropout_layernorm (csrc/addnorm.hip) reads it
    alone each way.
Both dropout masks are counter hashes of seeds drawn on the GPU (graph-safe), regenerated in the backward.
"""
import ctypes
import os

import torch
import torch.nn.functional as F
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n
from pdvc.precision import attach_bf16, bf16_active, shadow_for
from .addnorm import BWD_PARTS, an_backward, an_forward
from . import linear as _lin
from .gemm3 import addmm_nt, addmm_relu_dropout_nt, addmm_resid_dropout_nt, mm_dgrad, mm_dgrad_dmask
from .linear import CU, wgrad_mm


# False (or PDVC_FFN_FUSE=0): linear1, then the relu-dropout pass (the A/B and the bit-identity test)
FUSE_RELU_DROPOUT = os.environ.get("PDVC_FFN_FUSE", "1") != "0"


def _seed_ptrs(seeds):
    """(act, out) device pointers of the two int64 seeds drawn by ffn_block, or (NULL, NULL)."""
    if seeds is None:
        return None, None
    base = _n.ptr(seeds).value
    return ctypes.c_void_p(base), ctypes.c_void_p(base + 8)


def _parts(rows, cols):
    cblocks = (cols // 4 + 15) // 16
    return max(1, min(256, (8 * CU) // cblocks, rows // 64))


class FFNBlockFunction(Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, p_act, p_out, eps, seeds):
        shape = x.shape
        d = shape[-1]
        x2 = x.reshape(-1, d).contiguous()
        rows = x2.shape[0]
        seed_act, seed_out = _seed_ptrs(seeds)
        h = None
        if FUSE_RELU_DROPOUT and p_act > 0:  # relu -> dropout in linear1's gemm3 epilogue (same mask bits)
            h = addmm_relu_dropout_nt(b1, x2, w1, float(p_act), seed_act)
        if h is None:
            h = addmm_nt(b1, x2, w1)
            h16 = shadow_for(h)  # bf16 mode: linear2's operand written by the same pass
            if h16 is None:
                _n.call("pdvc_relu_dropout_forward_f32", _n.ptr(h), rows, h.shape[1], float(p_act), 0, seed_act,
                        _n.stream())
            else:
                _n.call("pdvc_relu_dropout_forward_f32_bf16out", _n.ptr(h), rows, h.shape[1], float(p_act), 0,
                        seed_act, _n.ptr(h16), _n.stream())
                attach_bf16(h, h16)
        out = torch.empty_like(x2)
        mean = torch.empty(rows, dtype=x.dtype, device=x.device)
        rstd = torch.empty_like(mean)
        # the residual sum t = x + dropout(linear2(h)) in linear2's epilogue, then the add-norm pass on t alone (one
        # tensor fewer read each way); y is then t, and the backward's add-norm pass takes it with s = None
        t = addmm_resid_dropout_nt(b2, h, w2, x2, float(p_out), seed_out)
        if t is not None:
            y = t
            an_forward(t, None, gamma, beta, 0.0, 0, None, eps, out, mean, rstd)
        else:
            y = addmm_nt(b2, h, w2)
            an_forward(x2, y, gamma, beta, p_out, 0, seed_out, eps, out, mean, rstd)
        ctx.save_for_backward(x2, h, y, w1, w2, gamma, mean, rstd, seeds)
        ctx.meta = (shape, float(p_act), float(p_out), t is not None)
        return out.view(shape)

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        x2, h, y, w1, w2, gamma, mean, rstd, seeds = ctx.saved_tensors
        shape, p_act, p_out, fused_sum = ctx.meta
        rows, d = x2.shape
        fdim = h.shape[1]
        _, seed_out = _seed_ptrs(seeds)
        dout2 = dout.reshape(-1, d).contiguous()
        dx = torch.empty_like(x2)
        dy = torch.empty_like(y)
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(gamma)
        ws = torch.empty(3 * BWD_PARTS * d, dtype=x2.dtype, device=x2.device)
        db2 = torch.empty_like(gamma)  # linear2's bias gradient = column sums of dy, summed by the same pass
        if fused_sum:  # y holds t = x + dropout(linear2(h)): the pass reads it alone
            an_backward(y, None, gamma, mean, rstd, dout2, p_out, 0, seed_out, dx, dy, dgamma, dbeta, db2, ws)
        else:
            an_backward(x2, y, gamma, mean, rstd, dout2, p_out, 0, seed_out, dx, dy, dgamma, dbeta, db2, ws)
        dw2 = wgrad_mm(dy, h)
        db1 = torch.empty(fdim, dtype=h.dtype, device=h.device)
        dh = None
        if FUSE_RELU_DROPOUT and not bf16_active():  # relu -> dropout backward in the dgrad epilogue
            dh = mm_dgrad_dmask(dy, w2, h, p_act)
        if dh is not None:
            dw1 = wgrad_mm(dh, x2, db=db1)  # with linear1's bias gradient from the same pass over dh
            mm_dgrad(dh, w1, out=dx)
            return dx.view(shape), dw1, db1, dw2, db2, dgamma, dbeta, None, None, None, None
        dh = mm_dgrad(dy, w2)
        parts = _parts(rows, fdim)
        ws1 = torch.empty(parts * fdim, dtype=h.dtype, device=h.device)
        dh16 = shadow_for(dh)  # bf16 mode: the operand of linear1's two gradient GEMMs, written by the same pass
        if dh16 is None:
            _n.call("pdvc_relu_dropout_backward_f32", _n.ptr(h), _n.ptr(dh), rows, fdim, p_act, parts, _n.ptr(ws1),
                    _n.ptr(db1), _n.stream())
        else:
            _n.call("pdvc_relu_dropout_backward_f32_bf16out", _n.ptr(h), _n.ptr(dh), rows, fdim, p_act, parts,
                    _n.ptr(ws1), _n.ptr(db1), _n.ptr(dh16), _n.stream())
            attach_bf16(dh, dh16)
        dw1 = wgrad_mm(dh, x2)
        mm_dgrad(dh, w1, out=dx)  # residual gradient + linear1's input gradient in one GEMM (beta = 1)
        return dx.view(shape), dw1, db1, dw2, db2, dgamma, dbeta, None, None, None, None


def use_ffn_block(x):
    """FFNBlockFunction serves fp32 GPU activations on the torch/hipBLASLt GEMM backend."""
    return x.is_cuda and x.dtype == torch.float32 and _lin.BACKEND != "hip"


def ffn_block(x, linear1, linear2, norm, p_act, p_out, training):
    """norm(x + dropout(linear2(dropout(relu(linear1(x)))))) with nn.Linear-like linear1/linear2 and an
    nn.LayerNorm norm.  GPU fp32: FFNBlockFunction; CPU (tests of host logic only): the module chain."""
    if not x.is_cuda:
        h = F.dropout(F.relu(F.linear(x, linear1.weight, linear1.bias)), p_act, training)
        return norm(x + F.dropout(F.linear(h, linear2.weight, linear2.bias), p_out, training))
    p_act = float(p_act) if training else 0.0
    p_out = float(p_out) if training else 0.0
    seeds = None
    if p_act > 0 or p_out > 0:
        seeds = torch.randint(0, 2 ** 62, (2,), device=x.device, dtype=torch.int64)
    return FFNBlockFunction.apply(x, linear1.weight, linear1.bias, linear2.weight, linear2.bias, norm.weight,
                                  norm.bias, p_act, p_out, norm.eps, seeds)
