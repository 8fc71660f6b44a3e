"""Drop-in replacement of the reference's compiled extension module `MultiScaleDeformableAttention`
(pdvc/ops/src/vision.cpp:13-16, imported at pdvc/ops/functions/ms_deform_attn_func.py:18).

Same two functions, same argument meaning and error behaviour (RuntimeError on CPU tensors,
non-contiguous tensors, or batch % min(batch, im2col_step) != 0 -- ms_deform_attn_cuda.cu:28-52),
backed by the MI355X C ABI (include/pdvc_msda.h) instead of the CUDA kernels.
"""
import torch

from pdvc import _native as _n

__all__ = ["ms_deform_attn_forward", "ms_deform_attn_backward"]


def _dims(value, spatial_shapes, sampling_loc):
    if value.dim() != 4 or sampling_loc.dim() != 6:
        raise RuntimeError("value must be (N,S,M,D) and sampling_loc (N,Lq,M,L,P,2)")
    N, S, M, D = value.shape
    L = spatial_shapes.shape[0]
    Lq, P = sampling_loc.shape[1], sampling_loc.shape[4]
    return N, S, M, D, L, Lq, P


def _sfx(value):
    if value.dtype == torch.float32:
        return "f32"
    if value.dtype == torch.float64:
        return "f64"
    raise RuntimeError(f"ms_deform_attn supports float32/float64 (AT_DISPATCH_FLOATING_TYPES), got {value.dtype}")


def _check(*tensors):
    for t in tensors:
        if not t.is_cuda:
            raise RuntimeError("Not implemented on the CPU")
        if not t.is_contiguous():
            raise RuntimeError("input tensors have to be contiguous")


def ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step):
    _check(value, spatial_shapes, level_start_index, sampling_loc, attn_weight)
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, sampling_loc)
    out = torch.empty((N, Lq, M * D), dtype=value.dtype, device=value.device)
    _n.call("pdvc_ms_deform_attn_forward_" + _sfx(value), _n.ptr(value), _n.ptr(spatial_shapes),
            _n.ptr(level_start_index), _n.ptr(sampling_loc), _n.ptr(attn_weight), N, S, M, D, L, Lq, P,
            int(im2col_step), _n.ptr(out), _n.stream())
    return out


def ms_deform_attn_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output,
                            im2col_step):
    grad_output = grad_output.contiguous()
    _check(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output)
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, sampling_loc)
    gv = torch.empty_like(value)
    gl = torch.empty_like(sampling_loc)
    ga = torch.empty_like(attn_weight)
    _n.call("pdvc_ms_deform_attn_backward_" + _sfx(value), _n.ptr(value), _n.ptr(spatial_shapes),
            _n.ptr(level_start_index), _n.ptr(sampling_loc), _n.ptr(attn_weight), _n.ptr(grad_output), N, S, M,
            D, L, Lq, P, int(im2col_step), _n.ptr(gv), _n.ptr(gl), _n.ptr(ga), _n.stream())
    return [gv, gl, ga]
