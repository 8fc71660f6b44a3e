"""MSDeformAttnCap for MI355X -- same constructor, parameters and forward contract as the reference
(pdvc/ops/modules/ms_deform_attn_for_caption.py:30-123): returns the raw border-padded samples
(N*M, D, Lq, L, P).  The caption head itself calls `sample_rows`, which takes a precomputed value and
returns the samples already in the (rows, M, L*P, D) layout the soft attention consumes.
As in the reference, attention_weights and output_proj are owned but unused (no gradient).
"""
import torch
from torch import nn
from torch.nn.init import constant_, xavier_uniform_

from ..functions import CapGatherFunction, ms_deform_attn_core_pytorch, NUM_SAMPLES_FUSED
from .linear import Linear
from .ms_deform_attn import _is_power_of_2, level_lengths, sampling_offsets_init

import warnings


class MSDeformAttnCap(nn.Module):
    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError("d_model must be divisible by n_heads, but got {} and {}".format(d_model, n_heads))
        if not _is_power_of_2(d_model // n_heads):
            warnings.warn("head dim is not a power of 2: the fused HIP caption gather will not be used")
        self.im2col_step = 64
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = Linear(2 * d_model, n_heads * n_levels * n_points)
        self.attention_weights = Linear(2 * d_model, n_heads * n_levels * n_points)
        self.value_proj = Linear(d_model, d_model)
        self.output_proj = Linear(d_model, d_model)
        self._reset_parameters()

    def _reset_parameters(self):
        constant_(self.sampling_offsets.weight.data, 0.)
        with torch.no_grad():
            self.sampling_offsets.bias = nn.Parameter(
                sampling_offsets_init(self.n_heads, self.n_levels, self.n_points, centred=True))
        constant_(self.attention_weights.weight.data, 0.)
        constant_(self.attention_weights.bias.data, 0.)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.)

    @property
    def fused(self):
        D = self.d_model // self.n_heads
        return (self.n_levels == 4 and self.n_points == 4 and D >= 32 and D <= 512 and _is_power_of_2(D))

    def sample_rows(self, value, pad_mask_u8, row_video, offsets, reference_points, level_T, off_col0=0,
                    rd1_rows=0):
        """value (N,S,d) = value_proj(memory) [hoisted by the caller]; offsets (R, C) with the
        M*L*P sampling offsets at off_col0; reference_points (R, L, 1|2) (with a 2-wide reference the first
        rd1_rows rows are 1-d references).  -> (R, M, L*P, D)."""
        N, S, _ = value.shape
        M, D = self.n_heads, self.d_model // self.n_heads
        return CapGatherFunction.apply(value.reshape(N, S, M, D), pad_mask_u8, row_video, offsets,
                                       reference_points, tuple(level_T), off_col0, rd1_rows)

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes, input_level_start_index,
                input_padding_mask=None):
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        T = level_lengths(input_spatial_shapes)
        if sum(T) != Len_in:
            raise AssertionError("sum of level lengths must equal the flattened input length")
        value = self.value_proj(input_flatten)
        M, D, L, P = self.n_heads, self.d_model // self.n_heads, self.n_levels, self.n_points
        offsets = self.sampling_offsets(query)  # (N, Lq, M*L*P)
        if self.fused and query.is_cuda:
            mask = None if input_padding_mask is None else input_padding_mask.contiguous().view(torch.uint8)
            row_video = torch.arange(N, device=query.device, dtype=torch.int32).repeat_interleave(Len_q)
            ref = reference_points.reshape(N * Len_q, L, reference_points.shape[-1])
            s = self.sample_rows(value, mask, row_video, offsets.reshape(N * Len_q, M * L * P), ref, T)
            # (N*Lq, M, L*P, D) -> reference layout (N*M, D, Lq, L, P)
            return s.view(N, Len_q, M, L, P, D).permute(0, 2, 5, 1, 3, 4).reshape(N * M, D, Len_q, L, P)
        # general path: the reference's own math on the HIP raw-sample kernel
        if input_padding_mask is not None:
            value = value.masked_fill(input_padding_mask[..., None], float(0))
        value = value.view(N, Len_in, M, D)
        off = offsets.view(N, Len_q, M, L, P)
        shapes1d = torch.as_tensor(T, dtype=torch.long, device=query.device)
        if reference_points.shape[-1] == 1:
            loc = reference_points[:, :, None, :, None, 0] + off / shapes1d.to(off.dtype)[None, None, None, :, None]
        else:
            loc = reference_points[:, :, None, :, None, 0] + off / P * reference_points[:, :, None, :, None, 1] * 0.5
        loc = torch.stack((loc, 0.5 * loc.new_ones(loc.shape)), -1)
        shapes2d = torch.stack([shapes1d.new_ones(shapes1d.shape), shapes1d], -1)
        return ms_deform_attn_core_pytorch(value, shapes2d, loc, None, return_value=True)
