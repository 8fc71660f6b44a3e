"""Multi-level temporal conv pyramid + position embeddings (reference: pdvc/base_encoder.py:23-86).

Level 0: Conv1d(k=1) + GroupNorm(32); levels 1..L-1: Conv1d(k=3, s=2, p=1) + GroupNorm(32), level 1 on the
raw features, later levels on the previous level.  Masks of coarser levels are the nearest-neighbour
resampling of the frame mask (base_encoder.py:77).  Outside the replaced hot path (SURVEY.md section 8(f),
rank 1), but the convolutions are evaluated as GEMMs (hipBLASLt) over strided tap views instead of MIOpen
convolutions: the k=1 conv is one GEMM, the k=3/s=2 conv one GEMM over the three stacked taps.  Same
nn.Conv1d parameters (state_dict unchanged); GroupNorm is torch's.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .position_encoding import PositionEmbeddingSine


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

    @staticmethod
    def conv1d_gemm(conv, x):
        """nn.Conv1d (k=1, or k=3/stride 2/pad 1) on x (N, C, T) as a GEMM; returns (N, O, T_out)."""
        w, b = conv.weight, conv.bias
        k = w.shape[2]
        if k == 1:
            return torch.matmul(w[:, :, 0], x) + b[None, :, None]
        assert k == 3 and conv.stride[0] == 2 and conv.padding[0] == 1
        T = x.shape[2]
        L = (T - 1) // 2 + 1
        xp = F.pad(x, (1, 1))
        taps = torch.cat([xp[:, :, j:j + 2 * L - 1:2] for j in range(3)], 1)  # (N, 3C, L)
        wr = w.permute(0, 2, 1).reshape(w.shape[0], 3 * w.shape[1])          # [tap][c] order
        return torch.matmul(wr, taps) + b[None, :, None]

    def _proj(self, lvl, x):
        conv, gn = self.input_proj[lvl][0], self.input_proj[lvl][1]
        if isinstance(conv, nn.Conv1d):
            return gn(self.conv1d_gemm(conv, x))
        return self.input_proj[lvl](x)

    def forward(self, vf, mask, duration):
        """vf (N, L, C); mask (N, L) True = padding; duration (N,).  -> lists of (N,d,L_l), (N,L_l), (N,d,L_l)."""
        x = vf.transpose(1, 2)
        srcs, masks, poses = [self._proj(0, x)], [mask], [self.pos_embed.embed(mask, duration)]
        for lvl in range(1, self.num_feature_levels):
            src = self._proj(lvl, x if lvl == 1 else srcs[-1])
            m = F.interpolate(mask[None].float(), size=src.shape[-1:]).to(torch.bool)[0]
            srcs.append(src)
            masks.append(m)
            poses.append(self.pos_embed.embed(m, duration, dtype=src.dtype))
        return srcs, masks, poses


def build_base_encoder(args):
    return BaseEncoder(args.num_feature_levels, args.feature_dim, args.hidden_dim)
