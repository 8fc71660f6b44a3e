"""Decoder query self-attention core: softmax(Q K^T / sqrt(d) + key_padding) V with dropout on the
probabilities -- nn.MultiheadAttention's math (torch.nn.functional.multi_head_attention_forward with
need_weights=True: q scaled by 1/sqrt(d), baddbmm with the -inf padding mask, softmax, dropout, bmm)."""
import math

import torch
import torch.nn.functional as F


def query_self_attention(qk, v, key_padding_mask, num_heads, dropout_p):
    """qk (N, Q, 2E) = [q | k] in-projections, v (N, Q, E); key_padding_mask (N, Q) True = ignore."""
    N, Q, E2 = qk.shape
    E = E2 // 2
    D = E // num_heads
    q = qk[..., :E].reshape(N, Q, num_heads, D).transpose(1, 2).reshape(N * num_heads, Q, D)
    k = qk[..., E:].reshape(N, Q, num_heads, D).transpose(1, 2).reshape(N * num_heads, Q, D)
    vv = v.reshape(N, Q, num_heads, D).transpose(1, 2).reshape(N * num_heads, Q, D)
    q = q * math.sqrt(1.0 / float(D))
    if key_padding_mask is not None:
        bias = torch.zeros(N, Q, dtype=q.dtype, device=q.device).masked_fill(key_padding_mask, float("-inf"))
        bias = bias.view(N, 1, 1, Q).expand(-1, num_heads, -1, -1).reshape(N * num_heads, 1, Q)
        attn = torch.baddbmm(bias, q, k.transpose(-2, -1))
    else:
        attn = torch.bmm(q, k.transpose(-2, -1))
    attn = F.softmax(attn, dim=-1)
    if dropout_p > 0.0:
        attn = F.dropout(attn, p=dropout_p)
    out = torch.bmm(attn, vv)
    return out.view(N, num_heads, Q, D).transpose(1, 2).reshape(N, Q, E)
