"""Long-sequence multi-head attention core on the HIP kernels pdvc_seq_attention_* (csrc/seqattn.hip):
softmax(q k^T / sqrt(head_dim)) v per (video, head), no mask, no dropout -- the core of the two
nn.MultiheadAttention(768, 32, batch_first=True) blocks of NewModel's dual-modality front-end
(NewModel.py:41-65).  q, k, v may be column slices of packed in-projections (row stride > width)."""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n

HEAD_DIMS = (16, 24, 32, 48, 64)


def _rowview(t, name):
    """(pointer, row stride) of an (N, T, E) view with unit column stride and batch stride T * row stride."""
    if not t.is_cuda or t.dtype != torch.float32:
        raise RuntimeError(f"seq_attention: {name} must be a float32 GPU tensor")
    N, T, E = t.shape
    if t.stride(2) != 1 or (N > 1 and t.stride(0) != T * t.stride(1)):
        t = t.contiguous()
    return t, _n.ptr_any(t), t.stride(1)


class SeqAttentionFunction(Function):
    @staticmethod
    def forward(ctx, q, k, v, num_heads):
        N, Tq, E = q.shape
        Tk = k.shape[1]
        D = E // num_heads
        if D * num_heads != E or D not in HEAD_DIMS:
            raise RuntimeError(f"seq_attention: head_dim {E}/{num_heads} not in {HEAD_DIMS}")
        if k.shape != (N, Tk, E) or v.shape != (N, Tk, E):
            raise RuntimeError("seq_attention: k and v must be (N, Tk, E) with q's N and E")
        q, qp, ldq = _rowview(q, "q")
        k, kp, ldk = _rowview(k, "k")
        v, vp, ldv = _rowview(v, "v")
        out = torch.empty((N, Tq, E), dtype=q.dtype, device=q.device)
        lse = torch.empty((N, num_heads, Tq), dtype=q.dtype, device=q.device)
        _n.call("pdvc_seq_attention_forward_f32", qp, ldq, kp, ldk, vp, ldv, N, Tq, Tk, num_heads, D,
                _n.ptr(out), _n.ptr(lse), _n.stream())
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.num_heads = num_heads
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        q, k, v, out, lse = ctx.saved_tensors
        H = ctx.num_heads
        N, Tq, E = out.shape
        Tk = k.shape[1]
        grad_out = grad_out.contiguous()
        ws = torch.empty(N * H * Tq, dtype=out.dtype, device=out.device)
        gq = torch.empty((N, Tq, E), dtype=out.dtype, device=out.device)
        gk = torch.empty((N, Tk, E), dtype=out.dtype, device=out.device)
        gv = torch.empty((N, Tk, E), dtype=out.dtype, device=out.device)
        _n.call("pdvc_seq_attention_backward_f32", _n.ptr_any(q), q.stride(1), _n.ptr_any(k), k.stride(1),
                _n.ptr_any(v), v.stride(1), _n.ptr(out), _n.ptr(grad_out), _n.ptr(lse), N, Tq, Tk, H, E // H,
                _n.ptr(ws), _n.ptr(gq), E, _n.ptr(gk), E, _n.ptr(gv), E, _n.stream())
        return gq, gk, gv, None


def seq_attention(q, k, v, num_heads):
    """q (N, Tq, E), k / v (N, Tk, E) -> (N, Tq, E)."""
    return SeqAttentionFunction.apply(q, k, v, num_heads)
