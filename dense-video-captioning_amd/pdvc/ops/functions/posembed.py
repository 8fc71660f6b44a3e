"""The encoder's positional input lvl_pos (N, S, d): every pyramid level's PositionEmbeddingSine rows plus its
level embedding, concatenated over levels (reference: position_encoding.py:20-75 per level,
deformable_transformer.py:100-112), as one HIP pass (csrc/posembed.hip) instead of ~12 torch launches per
level and 2-3 passes over (N, S, d).  The sine features need no gradient; the backward sums dlvl_pos per
(video, level) in one read: the level-embedding gradient is the sum over videos, the duration embedding's the
sum over levels of its channels."""
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n


class LevelPosRowsFunction(Function):
    @staticmethod
    def forward(ctx, xe, dim_t, dur, level_embed, level_T):
        N, S = xe.shape
        F = dim_t.numel()
        Dd = dur.shape[1]
        C = F + Dd
        lvl = _n.int_array(level_T)
        pos = torch.empty(N, S, C, dtype=torch.float32, device=xe.device)
        _n.call("pdvc_level_pos_rows_forward_f32", _n.ptr(xe), _n.ptr(dim_t), _n.ptr(dur), _n.ptr(level_embed), lvl,
                len(level_T), N, S, F, Dd, _n.ptr(pos), _n.stream())
        ctx.meta = (tuple(level_T), N, S, F, C)
        return pos

    @staticmethod
    @once_differentiable
    def backward(ctx, dpos):
        level_T, N, S, F, C = ctx.meta
        dpos = dpos.contiguous()
        part = torch.empty(N, len(level_T), C, dtype=dpos.dtype, device=dpos.device)
        _n.call("pdvc_level_pos_rows_backward_f32", _n.ptr(dpos), _n.int_array(level_T), len(level_T), N, S, C,
                _n.ptr(part), _n.stream())
        d_dur = part[:, :, F:].sum(1) if ctx.needs_input_grad[2] else None
        d_le = part.sum(0) if ctx.needs_input_grad[3] else None
        return None, None, d_dur, d_le, None


def level_pos_rows(pyr, level_embed):
    """lvl_pos (N, S, d) from a PyramidPosEmbed and the transformer's level_embed (L, d) parameter."""
    pe = pyr.pe
    xe = torch.cat([pe.positions(m) for m in pyr.masks], 1).contiguous()
    dim_t = pe.freqs(xe.device)
    dur = pe.duration_embedding(pyr.duration).float().contiguous()
    level_T = tuple(int(m.shape[1]) for m in pyr.masks)
    return LevelPosRowsFunction.apply(xe, dim_t, dur, level_embed.contiguous(), level_T)


class LevelPosGradFunction(Function):
    """A (N, L, d) zero tensor whose gradient stands for the per-(video, level) column sums of dlvl_pos: the
    encoder attention blocks (ops/functions/attn_block.py) return those sums directly -- computed from their
    query-projection gradients -- so dlvl_pos (N, S, d) is never materialised or accumulated across layers.
    Backward: the level-embedding and duration-embedding gradients, as LevelPosRowsFunction's."""

    @staticmethod
    def forward(ctx, dur, level_embed, N, F):
        ctx.F = F
        return torch.zeros(N, level_embed.shape[0], level_embed.shape[1], dtype=level_embed.dtype,
                           device=level_embed.device)

    @staticmethod
    @once_differentiable
    def backward(ctx, part):
        F = ctx.F
        d_dur = part[:, :, F:].sum(1) if ctx.needs_input_grad[0] else None
        d_le = part.sum(0) if ctx.needs_input_grad[1] else None
        return d_dur, d_le, None, None


def level_pos_rows_split(pyr, level_embed):
    """(lvl_pos without autograd history, grad handle): lvl_pos as level_pos_rows computes it, and the (N, L, d)
    handle through which consumers that can sum their own position gradients per (video, level) return them."""
    pe = pyr.pe
    xe = torch.cat([pe.positions(m) for m in pyr.masks], 1).contiguous()
    dim_t = pe.freqs(xe.device)
    dur = pe.duration_embedding(pyr.duration).float().contiguous()
    level_T = tuple(int(m.shape[1]) for m in pyr.masks)
    with torch.no_grad():
        pos = LevelPosRowsFunction.apply(xe, dim_t, dur.detach(), level_embed.detach().contiguous(), level_T)
    handle = LevelPosGradFunction.apply(dur, level_embed, xe.shape[0], dim_t.numel())
    return pos, handle


def level_row_sums(x, level_T):
    """Per-(video, level) column sums (N, L, C) of x (N, S, C) rows (pdvc_level_pos_rows_backward_f32)."""
    x = x.contiguous()
    N, S, C = x.shape
    part = torch.empty(N, len(level_T), C, dtype=x.dtype, device=x.device)
    _n.call("pdvc_level_pos_rows_backward_f32", _n.ptr(x), _n.int_array(level_T), len(level_T), N, S, C,
            _n.ptr(part), _n.stream())
    return part
