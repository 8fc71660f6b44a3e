"""MSDeformAttn for MI355X -- same constructor, parameters (state_dict names) and forward signature as
the reference module (pdvc/ops/modules/ms_deform_attn.py:30-126); the core runs in the fused 1-D HIP
kernels (MSDA1dFunction) with the reference GPU semantics (zero padding).  Shapes the fused kernels do not
cover (not 4 levels x 4 points, or head dims outside {16,32,64,128}) go through the general 2-D HIP op
after the reference's own 1-D -> 2-D lift (ms_deform_attn.py:182-185).
"""
import math
import warnings

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.init import constant_, xavier_uniform_

from ..functions import MSDeformAttnFunction, MSDA1dFunction, NUM_SAMPLES_FUSED
from ..functions.linear import dense
from .linear import Linear

FUSED_HEAD_DIMS = (16, 32, 64, 128)


def _is_power_of_2(n):
    if (not isinstance(n, int)) or (n < 0):
        raise ValueError("invalid input for _is_power_of_2: {} (type: {})".format(n, type(n)))
    return (n & (n - 1) == 0) and n != 0


def level_lengths(input_spatial_shapes):
    """Temporal length of every level as a tuple of ints.  The model passes tuples (no host sync);
    a tensor (the reference's calling convention) is read back once."""
    if isinstance(input_spatial_shapes, torch.Tensor):
        known = input_spatial_shapes.__dict__.get("_pdvc_level_T")  # the model's level table: its host tuple
        if known is not None and input_spatial_shapes.dim() == 1:
            return tuple(known)
        v = input_spatial_shapes.detach().reshape(-1).tolist()
        return tuple(int(x) for x in v)
    return tuple(int(x) for x in input_spatial_shapes)


def sampling_offsets_init(n_heads, n_levels, n_points, centred=False):
    """Bias init of sampling_offsets: per-head direction cos(2*pi*m/M) (normalised by max(|cos|,|sin|)),
    times (point index + 1); the caption variant subtracts the per-level mean over points
    (ms_deform_attn.py:62-71, ms_deform_attn_for_caption.py:55-68)."""
    thetas = torch.arange(n_heads, dtype=torch.float32) * (2.0 * math.pi / n_heads)
    dirs = torch.stack([thetas.cos(), thetas.sin()], -1)
    x = dirs[:, 0] / dirs.abs().max(-1)[0]
    grid = x.view(n_heads, 1, 1).expand(n_heads, n_levels, n_points).clone()
    grid = grid * torch.arange(1, n_points + 1, dtype=torch.float32).view(1, 1, n_points)
    if centred:
        grid = grid - grid.mean(2, keepdim=True)
    return grid.reshape(-1)


class MSDeformAttn(nn.Module):
    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        if d_model % n_heads != 0:
            raise ValueError("d_model must be divisible by n_heads, but got {} and {}".format(d_model, n_heads))
        if not _is_power_of_2(d_model // n_heads):
            warnings.warn("head dim is not a power of 2: the fused 1-D HIP path will not be used")
        self.im2col_step = 64
        self.d_model = d_model
        self.n_levels = n_levels
        self.n_heads = n_heads
        self.n_points = n_points
        self.sampling_offsets = Linear(d_model, n_heads * n_levels * n_points)
        self.attention_weights = Linear(d_model, n_heads * n_levels * n_points)
        self.value_proj = Linear(d_model, d_model)
        self.output_proj = Linear(d_model, d_model)
        self._reset_parameters()

    def _reset_parameters(self):
        constant_(self.sampling_offsets.weight.data, 0.)
        with torch.no_grad():
            self.sampling_offsets.bias = nn.Parameter(
                sampling_offsets_init(self.n_heads, self.n_levels, self.n_points))
        constant_(self.attention_weights.weight.data, 0.)
        constant_(self.attention_weights.bias.data, 0.)
        xavier_uniform_(self.value_proj.weight.data)
        constant_(self.value_proj.bias.data, 0.)
        xavier_uniform_(self.output_proj.weight.data)
        constant_(self.output_proj.bias.data, 0.)

    @property
    def fused(self):
        return (self.n_levels * self.n_points == NUM_SAMPLES_FUSED and self.n_levels == 4
                and self.d_model // self.n_heads in FUSED_HEAD_DIMS)

    def project_query(self, query):
        """One GEMM for both query projections: [offsets | attention logits] (N, Lq, 2*M*L*P)."""
        w = torch.cat([self.sampling_offsets.weight, self.attention_weights.weight], 0)
        b = torch.cat([self.sampling_offsets.bias, self.attention_weights.bias], 0)
        return dense(query, w, b)

    def forward(self, query, reference_points, input_flatten, input_spatial_shapes, input_level_start_index,
                input_padding_mask=None, value=None):
        """`value` may carry a precomputed value_proj(input_flatten) (it is identical for every decoder
        layer's caller only when weights are shared; kept for API symmetry)."""
        N, Len_q, _ = query.shape
        N, Len_in, _ = input_flatten.shape
        T = level_lengths(input_spatial_shapes)
        if sum(T) != Len_in:
            raise AssertionError("sum of level lengths must equal the flattened input length")
        if value is None:  # a caller may have projected input_flatten for several consumers at once (pdvc.py trunk)
            value = getattr(input_flatten, "_pdvc_values", {}).get(id(self.value_proj))
        if value is None:
            value = self.value_proj(input_flatten)
        M, D = self.n_heads, self.d_model // self.n_heads
        if self.fused and query.is_cuda and value.dtype == torch.float32:
            mask = None
            if input_padding_mask is not None:
                mask = input_padding_mask.contiguous().view(torch.uint8)
            proj = self.project_query(query)
            if value.shape != (N, Len_in, M * D):  # no reshape node otherwise: the value gradient keeps its sums
                value = value.reshape(N, Len_in, M * D)
            out = MSDA1dFunction.apply(value, mask, proj, reference_points, T, 0, M * NUM_SAMPLES_FUSED, M)
            return self.output_proj(out)
        return self.output_proj(self._lifted_general(query, reference_points, value, T, input_padding_mask))

    def _lifted_general(self, query, reference_points, value, T, input_padding_mask):
        """The reference's module math verbatim in torch ops + the general 2-D HIP op."""
        N, Len_q, _ = query.shape
        Len_in = value.shape[1]
        if input_padding_mask is not None:
            value = value.masked_fill(input_padding_mask[..., None], float(0))
        value = value.view(N, Len_in, self.n_heads, self.d_model // self.n_heads)
        off = self.sampling_offsets(query).view(N, Len_q, self.n_heads, self.n_levels, self.n_points)
        aw = self.attention_weights(query).view(N, Len_q, self.n_heads, self.n_levels * self.n_points)
        aw = F.softmax(aw, -1).view(N, Len_q, self.n_heads, self.n_levels, self.n_points)
        shapes1d = torch.as_tensor(T, dtype=torch.long, device=query.device)
        if reference_points.shape[-1] == 1:
            loc = reference_points[:, :, None, :, None, 0] + off / shapes1d.to(off.dtype)[None, None, None, :, None]
        elif reference_points.shape[-1] == 2:
            loc = reference_points[:, :, None, :, None, 0] \
                + off / self.n_points * reference_points[:, :, None, :, None, 1] * 0.5
        else:
            raise ValueError("Last dim of reference_points must be 1 or 2, but get {} instead.".format(
                reference_points.shape[-1]))
        loc = torch.stack((loc, 0.5 * loc.new_ones(loc.shape)), -1)
        shapes2d = torch.stack([shapes1d.new_ones(shapes1d.shape), shapes1d], -1)
        lsi = torch.cat((shapes1d.new_zeros((1,)), shapes1d.cumsum(0)[:-1]))
        return MSDeformAttnFunction.apply(value.contiguous(), shapes2d.contiguous(), lsi.contiguous(),
                                          loc.contiguous(), aw.contiguous(), self.im2col_step)
