"""Iterative box refinement, out = sigmoid(tmp + inverse_sigmoid(reference)), as one native pass each way
(csrc/boxref.hip).  Reference: deformable_transformer.py's refinement (new_reference_points =
(tmp + inverse_sigmoid(reference_points)).sigmoid(); a 1-d reference refines only the centre) and PDVC.forward's
per-layer box heads (pdvc/pdvc.py:245-253); inverse_sigmoid is misc/detr_utils/misc.py:540-544.  torch evaluates
each as ~9 elementwise launches forward and as many backward per decoder layer."""
import torch
from torch.autograd import Function

from pdvc import _native as _n
from pdvc.box_ops import inverse_sigmoid


class BoxRefineFunction(Function):
    @staticmethod
    def forward(ctx, tmp, ref, eps):
        t, r = tmp.contiguous(), ref.contiguous()
        rd = r.shape[-1]
        rows = t.numel() // 2
        if t.shape[-1] != 2 or rd not in (1, 2) or r.numel() != rows * rd:
            raise RuntimeError(f"box refine: tmp (..., 2) and reference (..., 1|2) rows, got {tuple(t.shape)}, "
                               f"{tuple(r.shape)}")
        out = torch.empty_like(t)
        _n.call("pdvc_box_refine_forward_f32", _n.ptr(t), _n.ptr(r), rows, rd, float(eps), _n.ptr(out), _n.stream())
        ctx.save_for_backward(out, r)
        ctx.eps = eps
        return out

    @staticmethod
    def backward(ctx, g):
        out, r = ctx.saved_tensors
        rows = out.numel() // 2
        gt = torch.empty_like(out)
        gr = torch.empty_like(r) if ctx.needs_input_grad[1] else None
        _n.call("pdvc_box_refine_backward_f32", _n.ptr(g.contiguous()), _n.ptr(out), _n.ptr(r), rows, r.shape[-1],
                float(ctx.eps), _n.ptr(gt), _n.ptr(gr) if gr is not None else None, _n.stream())
        return gt, gr, None


def box_refine(tmp, ref, eps=1e-5):
    """sigmoid(tmp + inverse_sigmoid(ref)) for ref (..., 2); for ref (..., 1) only the centre channel is refined."""
    if tmp.is_cuda and tmp.dtype == torch.float32 and ref.dtype == torch.float32:
        return BoxRefineFunction.apply(tmp, ref, eps)
    r = inverse_sigmoid(ref, eps)
    if ref.shape[-1] == 2:
        return (tmp + r).sigmoid()
    return torch.cat([tmp[..., :1] + r, tmp[..., 1:]], -1).sigmoid()
