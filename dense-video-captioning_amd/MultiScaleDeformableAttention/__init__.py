"""Drop-in replacement of the reference's compiled extension module `MultiScaleDeformableAttention`
(pdvc/ops/src/vision.cpp:13-16, imported at pdvc/ops/functions/ms_deform_attn_func.py:18).

Same two functions, same argument meaning and error behaviour (RuntimeError on CPU tensors,
non-contiguous tensors, or batch % min(batch, im2col_step) != 0 -- ms_deform_attn_cuda.cu:28-52),
backed by the MI355X C ABI (include/pdvc_msda.h) instead of the CUDA kernels.

The reference's `data<int64_t>()` / `data<scalar_t>()` accessors raise on a dtype mismatch; the C ABI takes
raw pointers, so those checks are made here: spatial_shapes and level_start_index int64, sampling_loc,
attn_weight and grad_output of value's dtype, and every shape consistent with value's (N, S, M, D) --
a wrong dtype or shape raises RuntimeError instead of being reinterpreted by the kernel.
"""
import torch

from pdvc import _native as _n

__all__ = ["ms_deform_attn_forward", "ms_deform_attn_backward"]


def _dims(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output=None):
    if value.dim() != 4 or sampling_loc.dim() != 6:
        raise RuntimeError("value must be (N,S,M,D) and sampling_loc (N,Lq,M,L,P,2)")
    for name, t in (("spatial_shapes", spatial_shapes), ("level_start_index", level_start_index)):
        if t.dtype != torch.int64:
            raise RuntimeError(f"{name} must be int64 (data<int64_t>()), got {t.dtype}")
    for name, t in (("sampling_loc", sampling_loc), ("attn_weight", attn_weight), ("grad_output", grad_output)):
        if t is not None and t.dtype != value.dtype:
            raise RuntimeError(f"{name} must have value's dtype {value.dtype}, got {t.dtype}")
    N, S, M, D = value.shape
    L = spatial_shapes.shape[0]
    Lq, P = sampling_loc.shape[1], sampling_loc.shape[4]
    if tuple(spatial_shapes.shape) != (L, 2) or tuple(level_start_index.shape) != (L,):
        raise RuntimeError(f"spatial_shapes must be (L,2) and level_start_index (L,), got "
                           f"{tuple(spatial_shapes.shape)} and {tuple(level_start_index.shape)}")
    if tuple(sampling_loc.shape) != (N, Lq, M, L, P, 2):
        raise RuntimeError(f"sampling_loc must be {(N, Lq, M, L, P, 2)}, got {tuple(sampling_loc.shape)}")
    if tuple(attn_weight.shape) != (N, Lq, M, L, P):
        raise RuntimeError(f"attn_weight must be {(N, Lq, M, L, P)}, got {tuple(attn_weight.shape)}")
    if grad_output is not None and tuple(grad_output.shape) != (N, Lq, M * D):
        raise RuntimeError(f"grad_output must be {(N, Lq, M * D)}, got {tuple(grad_output.shape)}")
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
        if t.device != tensors[0].device:
            raise RuntimeError("all tensors must be on the same device")


def ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, im2col_step):
    _check(value, spatial_shapes, level_start_index, sampling_loc, attn_weight)
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, level_start_index, sampling_loc, attn_weight)
    out = torch.empty((N, Lq, M * D), dtype=value.dtype, device=value.device)
    _n.call("pdvc_ms_deform_attn_forward_" + _sfx(value), _n.ptr(value), _n.ptr(spatial_shapes),
            _n.ptr(level_start_index), _n.ptr(sampling_loc), _n.ptr(attn_weight), N, S, M, D, L, Lq, P,
            int(im2col_step), _n.ptr(out), _n.stream())
    return out


def ms_deform_attn_backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output,
                            im2col_step):
    grad_output = grad_output.contiguous()
    _check(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output)
    N, S, M, D, L, Lq, P = _dims(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output)
    gv = torch.empty_like(value)
    gl = torch.empty_like(sampling_loc)
    ga = torch.empty_like(attn_weight)
    if value.dtype == torch.float32:
        # workspace of the 1-D fast path (the level-major location / weight slab its value gradient sorts); the
        # library decides on the device whether the table is a lifted 1-D pyramid
        nws = int(_n.lib().pdvc_ms_deform_attn_workspace_floats(N, M, L, Lq, P))
        ws = torch.empty(max(nws, 1), dtype=torch.float32, device=value.device)
        _n.call("pdvc_ms_deform_attn_backward_ws_f32", _n.ptr(value), _n.ptr(spatial_shapes),
                _n.ptr(level_start_index), _n.ptr(sampling_loc), _n.ptr(attn_weight), _n.ptr(grad_output), N, S, M,
                D, L, Lq, P, int(im2col_step), _n.ptr(gv), _n.ptr(gl), _n.ptr(ga), _n.ptr(ws), nws, _n.stream())
        return [gv, gl, ga]
    _n.call("pdvc_ms_deform_attn_backward_" + _sfx(value), _n.ptr(value), _n.ptr(spatial_shapes),
            _n.ptr(level_start_index), _n.ptr(sampling_loc), _n.ptr(attn_weight), _n.ptr(grad_output), N, S, M,
            D, L, Lq, P, int(im2col_step), _n.ptr(gv), _n.ptr(gl), _n.ptr(ga), _n.stream())
    return [gv, gl, ga]
