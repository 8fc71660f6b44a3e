"""Sine position embedding + duration embedding (reference: pdvc/position_encoding.py:20-75).

The per-video Python loop of duration_embedding (:44-50) is vectorised: out[v, :int(duration_v)] = 1 is
`arange(256) < int(duration_v)`.  Same parameters (`duration_embed_layer`) and outputs.
"""
import math

import torch
from torch import nn


class PositionEmbeddingSine(nn.Module):
    def __init__(self, num_pos_feats=64, temperature=10000, normalize=False, scale=None):
        super().__init__()
        self.num_pos_feats = num_pos_feats
        self.temperature = temperature
        self.normalize = normalize
        if scale is not None and normalize is False:
            raise ValueError("normalize should be True if scale is passed")
        self.scale = 2 * math.pi if scale is None else scale
        self.max_duration = 256
        self.duration_embed_layer = nn.Linear(self.max_duration, self.max_duration)

    def duration_embedding(self, durations):
        d = durations.int()
        steps = torch.arange(self.max_duration, device=durations.device)
        out = (steps[None, :] < d[:, None]).to(self.duration_embed_layer.weight.dtype)
        return self.duration_embed_layer(out)

    def embed(self, mask, duration, dtype=torch.float32):
        """mask (N, L) True = padding; duration (N,) seconds -> pos (N, num_pos_feats + 256, L)."""
        return self.embed_rows(mask, duration, dtype).permute(0, 2, 1)

    def positions(self, mask):
        """Normalised cumulative positions of the valid frames (N, L): the sine features' argument before the
        frequency division (position_encoding.py:53-58)."""
        not_mask = ~mask
        x_embed = not_mask.cumsum(1, dtype=torch.float32)
        if self.normalize:
            eps = 1e-6
            x_embed = (x_embed - 0.5) / (x_embed[:, -1:] + eps) * self.scale
        return x_embed

    def freqs(self, device):
        """The frequency table dim_t (num_pos_feats,) of position_encoding.py:60-61."""
        dim_t = torch.arange(self.num_pos_feats, dtype=torch.float32, device=device)
        return self.temperature ** (2 * (dim_t // 2) / self.num_pos_feats)

    def embed_rows(self, mask, duration, dtype=torch.float32):
        """The same embedding, channels-last: (N, L, num_pos_feats + 256)."""
        x_embed = self.positions(mask)
        dim_t = self.freqs(mask.device)
        pos_x = x_embed[:, :, None] / dim_t
        pos_x = torch.stack((pos_x[:, :, 0::2].sin(), pos_x[:, :, 1::2].cos()), dim=3).flatten(2)
        dur = self.duration_embedding(duration).reshape(-1, 1, self.max_duration).expand(
            pos_x.shape[0], pos_x.shape[1], self.max_duration)
        return torch.cat((pos_x, dur), dim=2).to(dtype)

    def forward(self, tensor_list):
        """Reference calling convention: a NestedTensor-like object with .tensors, .mask, .duration."""
        return self.embed(tensor_list.mask, tensor_list.duration)


class PyramidPosEmbed:
    """The pyramid's position embeddings as BaseEncoder hands them to the transformer: indexable like the
    reference's list of (N, d, T_l) tensors (base_encoder.py:80-85; an element is materialised on access), while
    DeformableTransformer.prepare_encoder_inputs builds all levels + level embeddings directly into the
    flattened (N, S, d) rows in one HIP pass from these inputs (ops/functions/posembed.py)."""

    def __init__(self, pe, masks, duration):
        self.pe = pe
        self.masks = list(masks)
        self.duration = duration

    def __len__(self):
        return len(self.masks)

    def __getitem__(self, i):
        dt = self.duration.dtype if self.duration.is_floating_point() else torch.float32
        return self.pe.embed_rows(self.masks[i], self.duration, dtype=dt).transpose(1, 2)

    def __iter__(self):
        return (self[i] for i in range(len(self)))


def build_position_encoding(position_embedding, N_steps):
    if position_embedding in ("v2", "sine"):
        return PositionEmbeddingSine(N_steps, normalize=True)
    raise ValueError(f"not supported {position_embedding}")
