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
from pdvc.precision import attach_bf16, shadow_for


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


class LevelPos:
    """lvl_pos (N, S, d) kept as the inputs of its kernel: consumers that only add it to a tensor (the encoder's
    query input src + pos, deformable_transformer.py:146) get the sum from one pass that generates the position
    rows in registers (pdvc_level_pos_rows_add_f32) -- the (N, S, d) rows are never written or read.  Carries
    no autograd history; `_pdvc_level_grad` is the gradient handle (LevelPosGradFunction)."""

    def __init__(self, xe, dim_t, dur, level_embed, level_T, handle):
        self.xe, self.dim_t, self.dur, self.level_embed, self.level_T = xe, dim_t, dur, level_embed, level_T
        self._pdvc_level_grad = handle
        self.shape = (xe.shape[0], xe.shape[1], dim_t.numel() + dur.shape[1])

    def _call(self, add):
        N, S = self.xe.shape
        out = torch.empty(self.shape, dtype=torch.float32, device=self.xe.device)
        args = (_n.ptr(self.xe), _n.ptr(self.dim_t), _n.ptr(self.dur), _n.ptr(self.level_embed),
                _n.int_array(self.level_T), len(self.level_T), N, S, self.dim_t.numel(), self.dur.shape[1],
                _n.ptr(add), _n.ptr(out))
        out16 = shadow_for(out) if add is not None else None  # bf16 mode: the query projection's operand
        if out16 is None:
            _n.call("pdvc_level_pos_rows_add_f32", *args, _n.stream())
        else:
            _n.call("pdvc_level_pos_rows_add_f32_bf16out", *args, _n.ptr(out16), _n.stream())
            attach_bf16(out, out16)
        return out

    def add_to(self, x):
        """x + lvl_pos for x (N*S, d) or (N, S, d) rows, shaped like x."""
        return self._call(x.contiguous()).view(x.shape)

    def materialize(self):
        return self._call(None)


def level_pos_rows_split(pyr, level_embed):
    """(lvl_pos as a LevelPos, grad handle): the position rows as level_pos_rows computes them, generated where
    they are added, and the (N, L, d) handle through which consumers that can sum their own position gradients
    per (video, level) return them."""
    pe = pyr.pe
    xe = torch.cat([pe.positions(m) for m in pyr.masks], 1).contiguous()
    dim_t = pe.freqs(xe.device)
    dur = pe.duration_embedding(pyr.duration).float().contiguous()
    level_T = tuple(int(m.shape[1]) for m in pyr.masks)
    handle = LevelPosGradFunction.apply(dur, level_embed, xe.shape[0], dim_t.numel())
    pos = LevelPos(xe, dim_t, dur.detach(), level_embed.detach().contiguous(), level_T, handle)
    return pos, handle


def level_row_sums(x, level_T):
    """Per-(video, level) column sums (N, L, C) of x (N, S, C) rows (pdvc_level_pos_rows_backward_f32)."""
    x = x.contiguous()
    N, S, C = x.shape
    part = torch.empty(N, len(level_T), C, dtype=x.dtype, device=x.device)
    _n.call("pdvc_level_pos_rows_backward_f32", _n.ptr(x), _n.int_array(level_T), len(level_T), N, S, C,
            _n.ptr(part), _n.stream())
    return part
