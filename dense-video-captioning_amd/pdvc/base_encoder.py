"""Multi-level temporal conv pyramid + position embeddings (reference: pdvc/base_encoder.py:23-86).

Level 0: Conv1d(k=1) + GroupNorm(32); levels 1..L-1: Conv1d(k=3, s=2, p=1) + GroupNorm(32), level 1 on the
raw features, later levels on the previous level.  Masks of coarser levels are the nearest-neighbour
resampling of the frame mask (base_encoder.py:77).  SURVEY.md section 8(f) rank 1: the pyramid runs on
channels-last rows (N, T, C) end to end -- convolutions as GEMMs over row views (ops/functions/conv_rows.py),
GroupNorm on rows (csrc/groupnorm.hip) -- so neither the input features nor the levels are ever transposed.
Same nn.Conv1d / nn.GroupNorm parameters (state_dict unchanged).
"""
import os

import torch
import torch.nn.functional as F
from torch import nn

from .ops.functions.conv_rows import conv1d_rows, group_norm_rows, group_norm_rows_into, group_norm_rows_ok
from .position_encoding import PositionEmbeddingSine, PyramidPosEmbed
from .precision import attach_bf16, shadow_for

# bf16 mode: the GroupNorm levels write the flat buffer's bf16 rounding (PDVC_GN_SHADOW=0: the GEMM casts it, A/B)
_FLAT_SHADOW = os.environ.get("PDVC_GN_SHADOW", "1") != "0"


class BaseEncoder(nn.Module):
    def __init__(self, num_feature_levels, vf_dim, hidden_dim):
        super().__init__()
        self.pos_embed = PositionEmbeddingSine(hidden_dim // 2, normalize=True)
        self.num_feature_levels = num_feature_levels
        self.hidden_dim = hidden_dim
        if num_feature_levels > 1:
            projs = [nn.Sequential(nn.Conv1d(vf_dim, hidden_dim, kernel_size=1), nn.GroupNorm(32, hidden_dim))]
            in_ch = vf_dim
            for _ in range(num_feature_levels - 1):
                projs.append(nn.Sequential(nn.Conv1d(in_ch, hidden_dim, kernel_size=3, stride=2, padding=1),
                                           nn.GroupNorm(32, hidden_dim)))
                in_ch = hidden_dim
            self.input_proj = nn.ModuleList(projs)
        else:
            self.input_proj = nn.ModuleList([nn.Sequential(nn.Conv2d(vf_dim, hidden_dim, kernel_size=1),
                                                           nn.GroupNorm(32, hidden_dim))])
        for proj in self.input_proj:
            nn.init.xavier_uniform_(proj[0].weight, gain=1)
            nn.init.constant_(proj[0].bias, 0)

    def _proj(self, lvl, x):
        """Conv1d + GroupNorm of level `lvl` on channels-last rows x (N, T, C) -> (N, T_l, d)."""
        conv, gn = self.input_proj[lvl][0], self.input_proj[lvl][1]
        if not isinstance(conv, nn.Conv1d):
            y = self.input_proj[lvl](x.transpose(1, 2)[..., None])[..., 0]
            return y.transpose(1, 2)
        return group_norm_rows(gn, conv1d_rows(conv, x))

    def forward(self, vf, mask, duration):
        """vf (N, L, C); mask (N, L) True = padding; duration (N,).  Returns lists of (N, d, L_l), (N, L_l),
        (N, d, L_l) as the reference -- the (N, d, L_l) tensors are transposed VIEWS of channels-last
        (N, L_l, d) storage, so the transformer's flattening (src.transpose(1, 2)) costs no copy; the position
        embeddings come as a PyramidPosEmbed (indexable like the reference's list)."""
        x = vf.contiguous()
        if self._flat_ok(x):
            return self._forward_flat(x, mask, duration)
        rows = [self._proj(0, x)]
        masks = [mask]
        for lvl in range(1, self.num_feature_levels):
            src = self._proj(lvl, x if lvl == 1 else rows[-1])
            m = F.interpolate(mask[None].float(), size=src.shape[1:2]).to(torch.bool)[0]
            rows.append(src)
            masks.append(m)
        return [r.transpose(1, 2) for r in rows], masks, PyramidPosEmbed(self.pos_embed, masks, duration)


    def _flat_ok(self, x):
        return (self.num_feature_levels > 1 and all(isinstance(p[0], nn.Conv1d) for p in self.input_proj)
                and group_norm_rows_ok(self.input_proj[0][1], x.new_empty(0, self.hidden_dim)))

    def _forward_flat(self, x, mask, duration):
        """forward() with every level's GroupNorm writing into its rows of one (N, sum T_l, d) buffer: the
        returned level tensors are views of it, tagged `_pdvc_flat`, so the transformer's flattening
        (deformable_transformer.py:84-106, a torch.cat) takes the buffer as it is."""
        N, T, _ = x.shape
        Ts = [T]
        for _ in range(1, self.num_feature_levels):
            Ts.append((Ts[-1] + 1) // 2)  # Conv1d(k=3, s=2, p=1)
        flat = x.new_empty(N, sum(Ts), self.hidden_dim)
        # bf16 mode: every level also writes its rows' bf16 rounding, attached to the finished buffer -- the operand of
        # the first encoder layer's projections, which would otherwise be a cast pass over (N, sum T_l, d)
        flat16 = shadow_for(flat) if _FLAT_SHADOW else None
        start, prev, masks = 0, None, [mask]
        for lvl in range(self.num_feature_levels):
            conv, gn = self.input_proj[lvl][0], self.input_proj[lvl][1]
            c = conv1d_rows(conv, x if lvl <= 1 else prev)
            assert c.shape[1] == Ts[lvl]
            want = 0 < lvl < self.num_feature_levels - 1  # the next level's conv input
            out = group_norm_rows_into(gn, c, flat, start, want, flat16)
            flat, prev = out if want else (out, None)
            start += Ts[lvl]
            if lvl:
                masks.append(F.interpolate(mask[None].float(), size=Ts[lvl]).to(torch.bool)[0])
        attach_bf16(flat, flat16)
        levels, start = [], 0
        for t in Ts:
            v = flat[:, start:start + t].transpose(1, 2)
            v._pdvc_flat = (flat, start)
            levels.append(v)
            start += t
        return levels, masks, PyramidPosEmbed(self.pos_embed, masks, duration)


def build_base_encoder(args):
    return BaseEncoder(args.num_feature_levels, args.feature_dim, args.hidden_dim)
