"""Autograd functions over the MI355X C ABI (include/pdvc_msda.h).

Mirrors pdvc/ops/functions/ms_deform_attn_func.py of the reference:
  * MSDeformAttnFunction        -- same signature/semantics as the reference (:20-38), general 2-D op;
  * ms_deform_attn_core_pytorch -- same signature as the reference core (:41-68, border padding);
    here it runs on the HIP raw-sample kernel (there is no CPU path);
and adds the fused 1-D functions PDVC's modules use:
  * MSDA1dFunction   -- softmax + sampling locations + zero-padded gather-reduce (ms_deform_attn.py:167-192)
  * CapGatherFunction -- sampling locations + border raw samples (ms_deform_attn_for_caption.py:92-121)
"""
import os

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

import MultiScaleDeformableAttention as MSDA
from pdvc import _native as _n
from pdvc.precision import attach_bf16, shadow_for

NUM_SAMPLES = 16  # levels x points on the fused paths
NUM_SAMPLES_FUSED = NUM_SAMPLES


class MSDeformAttnFunction(Function):
    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                im2col_step):
        ctx.im2col_step = im2col_step
        output = MSDA.ms_deform_attn_forward(value, value_spatial_shapes, value_level_start_index,
                                             sampling_locations, attention_weights, ctx.im2col_step)
        ctx.save_for_backward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                              attention_weights)
        return output

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        value, shapes, lsi, loc, attn = ctx.saved_tensors
        gv, gl, ga = MSDA.ms_deform_attn_backward(value, shapes, lsi, loc, attn, grad_output, ctx.im2col_step)
        return gv, None, None, gl, ga, None


class _SampleFunction(Function):
    """Raw bilinear samples (N*M, D, Lq, L, P) with border (or zeros) padding, general 2-D."""

    @staticmethod
    def forward(ctx, value, shapes, lsi, loc, padding):
        value, loc = value.contiguous(), loc.contiguous()
        N, S, M, D = value.shape
        _, Lq, _, L, P, _ = loc.shape
        out = torch.empty((N * M, D, Lq, L, P), dtype=value.dtype, device=value.device)
        if value.dtype != torch.float32:
            raise RuntimeError("ms_deform_attn_core_pytorch on MI355X supports float32")
        _n.call("pdvc_ms_deform_sample_f32", _n.ptr(value), _n.ptr(shapes), _n.ptr(lsi), _n.ptr(loc), N, S, M, D,
                L, Lq, P, padding, _n.ptr(out), _n.stream())
        ctx.save_for_backward(value, shapes, lsi, loc)
        ctx.padding = padding
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad):
        value, shapes, lsi, loc = ctx.saved_tensors
        grad = grad.contiguous()
        N, S, M, D = value.shape
        _, Lq, _, L, P, _ = loc.shape
        gv = torch.empty_like(value)
        gl = torch.empty_like(loc)
        _n.call("pdvc_ms_deform_sample_backward_f32", _n.ptr(value), _n.ptr(shapes), _n.ptr(lsi), _n.ptr(loc),
                _n.ptr(grad), N, S, M, D, L, Lq, P, ctx.padding, _n.ptr(gv), _n.ptr(gl), _n.stream())
        return gv, None, None, gl, None


def ms_deform_attn_core_pytorch(value, value_spatial_shapes, sampling_locations, attention_weights,
                                return_value=False):
    """The reference core's contract (ms_deform_attn_func.py:41-68: grid_sample bilinear, border,
    align_corners=False) on the HIP raw-sample kernel."""
    shapes = torch.as_tensor(value_spatial_shapes, dtype=torch.long, device=value.device).reshape(-1, 2)
    lsi = torch.cat((shapes.new_zeros((1,)), shapes.prod(1).cumsum(0)[:-1]))
    samples = _SampleFunction.apply(value, shapes.contiguous(), lsi.contiguous(), sampling_locations,
                                    _n_pad("border"))
    if return_value:
        return samples
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = sampling_locations.shape
    w = attention_weights.transpose(1, 2).reshape(N * M, 1, Lq, L * P)
    out = (samples.flatten(-2) * w).sum(-1).view(N, M * D, Lq)
    return out.transpose(1, 2).contiguous()


def _n_pad(name):
    return {"zeros": 0, "border": 1}[name]


def _levels(level_T):
    return _n.int_array(level_T), len(level_T)


def msda1d_forward(value, pad_mask, proj, ref, level_T, off_base, logit_base, save=True):
    """pdvc_msda1d_forward_f32 on contiguous value (N,S,M,D), proj (N,Lq,C), ref (N,Lq,L,1|2): returns
    (out (N,Lq,M*D), save_attn, save_loc) -- the last two None when save is False."""
    N, S, M, D = value.shape
    Lq, C = proj.shape[1], proj.shape[2]
    RD = ref.shape[3]
    lvl, nl = _levels(level_T)
    out = torch.empty((N, Lq, M * D), dtype=value.dtype, device=value.device)
    save_attn = save_loc = None
    if save:
        # level-major (N, M, L, Lq, P): the kernels' layout (include/pdvc_msda.h)
        save_attn = torch.empty((N, M, nl, Lq, NUM_SAMPLES // nl), dtype=value.dtype, device=value.device)
        save_loc = torch.empty_like(save_attn)
    args = (_n.ptr(value), _n.ptr(pad_mask), _n.ptr(proj), C, off_base, logit_base, _n.ptr(ref), RD, lvl, nl, N, Lq,
            M, D, NUM_SAMPLES // nl, _n.ptr(out), _n.ptr(save_attn), _n.ptr(save_loc))
    meta = (N, Lq, S, M, D, NUM_SAMPLES)
    out16 = shadow_for(out) if Lq == S else None  # bf16 mode, encoder: the output projection's operand
    if out16 is not None:
        try:
            _n.call("pdvc_msda1d_forward_f32_bf16out", *args, _n.ptr(out16), _n.stream(), meta=meta)
            attach_bf16(out, out16)
            return out, save_attn, save_loc
        except _n.NativeError:  # not the pyramid path: the GEMM casts the output itself
            pass
    _n.call("pdvc_msda1d_forward_f32", *args, _n.stream(), meta=meta)
    return out, save_attn, save_loc


# The softmax backward's row term sum_j a_j dL/da_j: summed over the sampled values inside the kernel (default),
# or PDVC_MSDA_DELTA_OUT=1: computed as <grad_out, out> from the forward output (one more (N,Lq,M*D) read).
_DELTA_FROM_OUT = os.environ.get("PDVC_MSDA_DELTA_OUT", "0") == "1"


# bf16 mode: the decoder's value gradient written with its bf16 rounding too (PDVC_MSDA_DEC_BF16OUT=0: cast pass, A/B)
_DEC_BF16OUT = os.environ.get("PDVC_MSDA_DEC_BF16OUT", "1") != "0"


def msda1d_backward(value, pad_mask, proj, ref, save_attn, save_loc, out, grad_out, level_T, off_base, logit_base,
                    need_ref=False, level_sums=False):
    """pdvc_msda1d_backward_ex_f32: returns (grad_value, grad_proj, grad_ref or None), plus with `level_sums` the
    (N, L, M*D) per-(video, level) column sums of grad_value (the value projection's bias gradient is their
    sum).  `out` (the forward output) is passed to the kernel only under PDVC_MSDA_DELTA_OUT=1."""
    N, S, M, D = value.shape
    Lq, C = proj.shape[1], proj.shape[2]
    RD = ref.shape[3]
    lvl, nl = _levels(level_T)
    gv = torch.empty_like(value)
    gp = torch.zeros_like(proj) if C != 2 * M * NUM_SAMPLES else torch.empty_like(proj)
    gr = torch.empty_like(ref) if need_ref else None
    ls = torch.empty(N, nl, M * D, dtype=value.dtype, device=value.device) if level_sums else None
    args = (_n.ptr(value), _n.ptr(pad_mask), _n.ptr(ref), RD, _n.ptr(proj), C, off_base, logit_base, lvl, nl, N, Lq, M,
            D, NUM_SAMPLES // nl, _n.ptr(grad_out), _n.ptr(out) if _DELTA_FROM_OUT else None, _n.ptr(save_attn),
            _n.ptr(save_loc), _n.ptr(gv), _n.ptr(gp), _n.ptr(gr), _n.ptr(ls))
    meta = (N, Lq, S, M, D, NUM_SAMPLES)
    done = False
    # bf16 mode: the projections' gradient-GEMM operands written beside the gradients -- grad_value's everywhere (the
    # decoder's cross-attention value gradient feeds the memory projections' GEMMs), grad_proj's on the encoder
    gv16 = shadow_for(gv) if (Lq == S or _DEC_BF16OUT) else None
    if gv16 is not None:
        gp16 = shadow_for(gp) if Lq == S else None
        try:
            _n.call("pdvc_msda1d_backward_ex_f32_bf16out", *args, _n.ptr(gv16), _n.ptr(gp16), _n.stream(), meta=meta)
            attach_bf16(gv, gv16)
            attach_bf16(gp, gp16)
            done = True
        except _n.NativeError:  # not the pyramid path: the GEMMs cast the gradients themselves
            pass
    if not done:
        _n.call("pdvc_msda1d_backward_ex_f32", *args, _n.stream(), meta=meta)
    return (gv, gp, gr, ls) if level_sums else (gv, gp, gr)


class MSDA1dFunction(Function):
    """Fused MSDeformAttn core for a 1-D temporal pyramid (GPU semantics: zero padding).

    value (N,S,M,D), or (N,S,M*D) with `heads` = M; pad_mask (N,S) uint8 or None; proj (N,Lq,C) holding offsets
    at [off_base, +M*16) and attention logits at [logit_base, +M*16); ref (N,Lq,L,1|2).  Returns (N,Lq,M*D).

    With a (N,S,M*D) value (a projection's output, as the decoder passes it) the value gradient comes back in that
    shape carrying `_pdvc_level_sums`, its per-(video, level) column sums from the value-gradient kernel: the
    projection's backward (MultiLinearFunction) takes its bias gradient from them instead of re-reading it."""

    @staticmethod
    def forward(ctx, value, pad_mask, proj, ref, level_T, off_base, logit_base, heads=None):
        value, proj, ref = value.contiguous(), proj.contiguous(), ref.contiguous()
        flat = value.dim() == 3
        v4 = value.view(value.shape[0], value.shape[1], heads, -1) if flat else value
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        out, save_attn, save_loc = msda1d_forward(v4, pad_mask, proj, ref, level_T, off_base, logit_base, need)
        if need:
            ctx.save_for_backward(v4, pad_mask, proj, ref, save_attn, save_loc, out)
        ctx.meta = (tuple(level_T), off_base, logit_base, flat)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        value, pad_mask, proj, ref, save_attn, save_loc, out = ctx.saved_tensors
        level_T, off_base, logit_base, flat = ctx.meta
        N, S, M, D = value.shape
        sums = flat and (M * D) % 4 == 0 and ctx.needs_input_grad[0]
        res = msda1d_backward(value, pad_mask, proj, ref, save_attn, save_loc, out, grad_out.contiguous(), level_T,
                              off_base, logit_base, need_ref=ctx.needs_input_grad[3], level_sums=sums)
        gv, gp, gr = res[:3]
        if flat:
            gv = gv.view(N, S, M * D)
            if sums:
                from .linear import tag_level_sums
                tag_level_sums(gv, res[3])
        return gv, None, gp, gr, None, None, None, None


class CapGatherFunction(Function):
    """Caption-head sampling: raw border samples (R, M, 16, D) of value (N,S,M,D) for query rows whose
    video is row_video (R,) int32; offsets (R, C) with the M*16 offsets at column off_col0; ref (R,L,1|2).
    With a 2-wide ref, the first rd1_rows rows are 1-d references (centre only, ref[..., 1] unused)."""

    @staticmethod
    def forward(ctx, value, pad_mask, row_video, offsets, ref, level_T, off_col0, rd1_rows=0):
        value, offsets, ref = value.contiguous(), offsets.contiguous(), ref.contiguous()
        N, S, M, D = value.shape
        R, C = offsets.shape
        RD = ref.shape[2]
        lvl, nl = _levels(level_T)
        samples = torch.empty((R, M, NUM_SAMPLES, D), dtype=value.dtype, device=value.device)
        save_loc = torch.empty((R, M, NUM_SAMPLES), dtype=value.dtype, device=value.device)
        _n.call("pdvc_cap_gather_forward_f32", _n.ptr(value), _n.ptr(pad_mask), _n.ptr(row_video), _n.ptr(offsets),
                C, off_col0, None, _n.ptr(ref), RD, int(rd1_rows), lvl, nl, N, R, M, D, NUM_SAMPLES // nl,
                _n.ptr(samples), _n.ptr(save_loc), _n.stream())
        ctx.save_for_backward(value, pad_mask, row_video, offsets, ref, save_loc)
        ctx.meta = (tuple(level_T), off_col0, int(rd1_rows))
        return samples

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_samples):
        value, pad_mask, row_video, offsets, ref, save_loc = ctx.saved_tensors
        level_T, off_col0, rd1_rows = ctx.meta
        grad_samples = grad_samples.contiguous()
        N, S, M, D = value.shape
        R, C = offsets.shape
        RD = ref.shape[2]
        lvl, nl = _levels(level_T)
        gv = torch.zeros_like(value)
        go = torch.zeros_like(offsets) if C != M * NUM_SAMPLES else torch.empty_like(offsets)
        gr = torch.zeros_like(ref) if ctx.needs_input_grad[4] else None
        _n.call("pdvc_cap_gather_backward_f32", _n.ptr(value), _n.ptr(pad_mask), _n.ptr(row_video),
                _n.ptr(offsets), C, off_col0, None, _n.ptr(ref), RD, rd1_rows, lvl, nl, N, R, M, D, NUM_SAMPLES // nl,
                _n.ptr(save_loc), _n.ptr(grad_samples), _n.ptr(gv), _n.ptr(go), _n.ptr(gr), _n.stream())
        return gv, None, None, go, gr, None, None, None
