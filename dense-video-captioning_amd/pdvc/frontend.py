"""The dual-modality front-end of cfgs/yc2_newModel_sound.yml (reference: NewModel, NewModel.py:21-65): the T clip
features (TSP / MViTv2, 768-d) attend to themselves, then the per-clip sound features (HuBERT, 768-d) attend to
them, each block followed by a Linear + LayerNorm MLP, residuals as written there:

    f = ln1(mha1(clips, clips, clips)) + clips;   f = mlp_seq1(f) + f
    g = ln2(mha2(sound, f, f)) + f;               g = mlp_seq2(g) + g      -> dt['video_tensor'] of PDVC

Parameter names and shapes are NewModel's (ln1, mha1.{in_proj_weight, in_proj_bias, out_proj.*}, mlp_seq1.{0,1},
ln2, mha2, mlp_seq2), so its front-end state_dict entries load unchanged.  The attention core is the HIP kernel
pdvc_seq_attention_* (T = 512 queries and keys, 32 heads of 24); projections are the library GEMMs.  HuBERT
itself (torchaudio.pipelines.HUBERT_BASE, downloaded at construction, NewModel.py:35-36) is not rebuilt: the
front-end takes the sound features as an input, as NewModel does once they are cached (NewModel.py:98-100).
"""
import torch
import torch.nn.functional as F
from torch import nn

from pdvc.ops.functions.addnorm import layernorm_residual
from pdvc.ops.functions.seq_attention import seq_attention


class FrontEndAttention(nn.Module):
    """nn.MultiheadAttention(E, H, batch_first=True) forward with key = value, no mask, no dropout, and its
    parameter layout (packed in_proj_weight (3E, E) / in_proj_bias, out_proj Linear)."""

    def __init__(self, embed_dim, num_heads):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim))
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        nn.init.xavier_uniform_(self.in_proj_weight)  # torch MultiheadAttention._reset_parameters
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, query, key):
        E = self.embed_dim
        W, b = self.in_proj_weight, self.in_proj_bias
        if query is key:
            qkv = F.linear(query, W, b)  # one GEMM, q / k / v read as column slices (row stride 3E)
            q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
        else:
            q = F.linear(query, W[:E], b[:E])
            kv = F.linear(key, W[E:], b[E:])
            k, v = kv[..., :E], kv[..., E:]
        return self.out_proj(seq_attention(q, k, v, self.num_heads))


class DualModalityFrontEnd(nn.Module):
    def __init__(self, dim=768, num_heads=32):
        super().__init__()
        self.ln1 = nn.LayerNorm(dim)
        self.mha1 = FrontEndAttention(dim, num_heads)
        self.mlp_seq1 = nn.Sequential(nn.Linear(dim, dim), nn.LayerNorm(dim))
        self.ln2 = nn.LayerNorm(dim)
        self.mha2 = FrontEndAttention(dim, num_heads)
        self.mlp_seq2 = nn.Sequential(nn.Linear(dim, dim), nn.LayerNorm(dim))

    # every `ln(h) + residual` is one HIP pass each way (pdvc_layernorm_residual_*); mlp_seq = Linear, LayerNorm
    def visual_self_attention(self, clips):  # NewModel.py:41-52
        f = layernorm_residual(self.mha1(clips, clips), clips, self.ln1)
        return layernorm_residual(self.mlp_seq1[0](f), f, self.mlp_seq1[1])

    def visual_sound_attention(self, clips, sound):  # NewModel.py:54-65
        g = layernorm_residual(self.mha2(sound, clips), clips, self.ln2)
        return layernorm_residual(self.mlp_seq2[0](g), g, self.mlp_seq2[1])

    def forward(self, clips, sound):
        """clips, sound (N, T, dim) -> (N, T, dim), the video_tensor PDVC consumes (NewModel.py:82-87)."""
        return self.visual_sound_attention(self.visual_self_attention(clips), sound)
