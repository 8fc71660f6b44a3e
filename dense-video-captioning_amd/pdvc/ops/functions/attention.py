"""Decoder query self-attention core on the HIP kernel (pdvc_mha_*): softmax(q*sqrt(1/D) k^T + key padding)
with dropout on the probabilities, times v -- nn.MultiheadAttention's math as the reference decoder layer
uses it (pdvc/deformable_transformer.py:256-258; multi_head_attention_forward with need_weights=True)."""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n

MAX_HEAD_DIM = 64
MAX_QUERIES = 300


class QuerySelfAttentionFunction(Function):
    @staticmethod
    def forward(ctx, qk, v, kpm_u8, num_heads, dropout_p, seed):
        """seed: a Python int, or a 1-element int64 device tensor (drawn on the GPU: graph-capture safe)."""
        qk, v = qk.contiguous(), v.contiguous()
        seed_dev = seed if isinstance(seed, torch.Tensor) else None
        seed_int = 0 if seed_dev is not None else int(seed)
        N, Q, E2 = qk.shape
        E = E2 // 2
        out = torch.empty((N, Q, E), dtype=qk.dtype, device=qk.device)
        lse = torch.empty((N, num_heads, Q), dtype=qk.dtype, device=qk.device)
        _n.call("pdvc_mha_forward_f32", _n.ptr(qk), _n.ptr(v), _n.ptr(kpm_u8), N, Q, num_heads, E // num_heads,
                float(dropout_p), seed_int, _n.ptr(seed_dev), _n.ptr(out), _n.ptr(lse), _n.stream(),
                meta=(N, Q, num_heads))
        ctx.save_for_backward(qk, v, kpm_u8, out, lse, seed_dev)
        ctx.meta = (num_heads, float(dropout_p), seed_int)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        qk, v, kpm_u8, out, lse, seed_dev = ctx.saved_tensors
        num_heads, p, seed = ctx.meta
        grad_out = grad_out.contiguous()
        N, Q, E2 = qk.shape
        D = E2 // 2 // num_heads
        ws = torch.empty(_n.lib().pdvc_mha_workspace_floats(N, Q, num_heads, D), dtype=qk.dtype, device=qk.device)
        gqk = torch.empty_like(qk)
        gv = torch.empty_like(v)
        _n.call("pdvc_mha_backward_f32", _n.ptr(qk), _n.ptr(v), _n.ptr(kpm_u8), _n.ptr(out), _n.ptr(grad_out),
                _n.ptr(lse), N, Q, num_heads, D, p, seed, _n.ptr(seed_dev), _n.ptr(ws),
                _n.ptr(gqk), _n.ptr(gv),
                _n.stream(), meta=(N, Q, num_heads))
        return gqk, gv, None, None, None, None


def query_self_attention(qk, v, key_padding_mask, num_heads, dropout_p):
    """qk (N, Q, 2E) = [q | k] in-projections, v (N, Q, E); key_padding_mask (N, Q) True = ignore."""
    N, Q, E2 = qk.shape
    if E2 // 2 // num_heads > MAX_HEAD_DIM or Q > MAX_QUERIES:
        raise NotImplementedError(f"query self-attention kernel supports head_dim <= {MAX_HEAD_DIM} and <= "
                                  f"{MAX_QUERIES} queries (got head_dim {E2 // 2 // num_heads}, Q {Q})")
    kpm = None if key_padding_mask is None else key_padding_mask.contiguous().view(torch.uint8)
    # the seed is drawn on the GPU (no host round trip; a captured graph draws a fresh one per replay)
    seed = torch.randint(0, 2 ** 62, (1,), device=qk.device, dtype=torch.int64) if dropout_p > 0 else 0
    return QuerySelfAttentionFunction.apply(qk, v, kpm, num_heads, dropout_p, seed)
