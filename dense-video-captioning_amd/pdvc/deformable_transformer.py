"""Deformable transformer for PDVC on MI355X (reference: pdvc/deformable_transformer.py:22-355).

Same module tree and state_dict names as the reference.  The hot blocks run on HIP kernels:
  * encoder self-attention and decoder cross-attention: MSDeformAttn (fused 1-D MSDA kernels);
  * decoder query self-attention: QuerySelfAttention -- nn.MultiheadAttention's parameters and math
    (deformable_transformer.py:231,256-258) with the softmax(QK^T/sqrt(d))V core in a HIP kernel.
Level shapes travel as Python tuples next to the reference's tensors so that no kernel launch needs a
host read-back of `temporal_shapes` (the reference's `assert spatial_shapes.sum() == Len_in` is a sync).
"""
import copy
import math
import os

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.init import constant_, normal_, xavier_uniform_

from . import hostio
from .ops.functions import add_dropout_layernorm

from .box_ops import inverse_sigmoid
from .ops.functions import linear as _lin
from .ops.functions.linear import PackedLinearFunction, add_row_bias, dense, expand_rows
from .ops.modules import MSDeformAttn
from .ops.modules.linear import Linear
from .ops.functions.attention import query_self_attention
from .ops.functions.ffn import ffn_block, use_ffn_block
from .ops.functions.attn_block import encoder_attn_block, use_attn_block
from .ops.functions.boxref import box_refine
from .ops.functions.posembed import level_pos_rows, level_pos_rows_split
from .position_encoding import PyramidPosEmbed


class DeformableTransformer(nn.Module):
    def __init__(self, d_model=256, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=1024,
                 dropout=0.1, activation="relu", return_intermediate_dec=False, num_feature_levels=4,
                 dec_n_points=4, enc_n_points=4):
        super().__init__()
        self.d_model = d_model
        self.nhead = nhead
        self.no_encoder = num_encoder_layers == 0
        self.num_feature_levels = num_feature_levels
        enc_layer = DeformableTransformerEncoderLayer(d_model, dim_feedforward, dropout, activation,
                                                      num_feature_levels, nhead, enc_n_points)
        self.encoder = DeformableTransformerEncoder(enc_layer, num_encoder_layers)
        dec_layer = DeformableTransformerDecoderLayer(d_model, dim_feedforward, dropout, activation,
                                                      num_feature_levels, nhead, dec_n_points)
        self.decoder = DeformableTransformerDecoder(dec_layer, num_decoder_layers, return_intermediate_dec)
        self.level_embed = nn.Parameter(torch.Tensor(num_feature_levels, d_model))
        self.pos_trans = nn.Linear(d_model, d_model * 2)
        self.pos_trans_norm = nn.LayerNorm(d_model * 2)
        self.reference_points = nn.Linear(d_model, 1)
        self._reset_parameters()

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m._reset_parameters()
        xavier_uniform_(self.reference_points.weight.data, gain=1.0)
        constant_(self.reference_points.bias.data, 0.)
        normal_(self.level_embed)

    def get_proposal_pos_embed(self, proposals):
        num_pos_feats, temperature, scale = 256, 10000, 2 * math.pi
        dim_t = torch.arange(num_pos_feats, dtype=torch.float32, device=proposals.device)
        dim_t = temperature ** (2 * (dim_t // 2) / num_pos_feats)
        proposals = proposals.sigmoid() * scale
        pos = proposals[:, :, :, None] / dim_t
        return torch.stack((pos[:, :, :, 0::2].sin(), pos[:, :, :, 1::2].cos()), dim=4).flatten(2)

    @staticmethod
    def get_valid_ratio(mask):
        return torch.sum(~mask, 1).float() / mask.shape[1]

    def prepare_encoder_inputs(self, srcs, masks, pos_embeds):
        """Flatten the pyramid (deformable_transformer.py:84-114).  temporal_shapes is returned as the
        reference's (L,) long tensor; the Python tuple is attached as `self.last_level_T`."""
        src_flatten, mask_flatten, lvl_pos = [], [], []
        level_T = []
        fused_pos = (isinstance(pos_embeds, PyramidPosEmbed) and srcs[0].is_cuda and srcs[0].dtype == torch.float32
                     and self.level_embed.shape[0] == len(srcs))
        for lvl, (src, mask) in enumerate(zip(srcs, masks)):
            level_T.append(int(src.shape[2]))
            src_flatten.append(src.transpose(1, 2))
            if not fused_pos:
                lvl_pos.append(add_row_bias(pos_embeds[lvl].transpose(1, 2), self.level_embed[lvl]))
            mask_flatten.append(mask)
        flat = getattr(srcs[0], "_pdvc_flat", (None, 0))[0]
        tags = [getattr(s, "_pdvc_flat", (None, 0)) for s in srcs]
        if flat is not None and flat.shape[1] == sum(level_T) and all(
                t[0] is flat and t[1] == sum(level_T[:i]) for i, t in enumerate(tags)):
            src_flatten = flat  # the base encoder wrote every level into its rows of one buffer (base_encoder.py)
        else:
            src_flatten = torch.cat(src_flatten, 1)
        mask_flatten = torch.cat(mask_flatten, 1)
        # all levels' sine + duration rows + level embeddings in one HIP pass (ops/functions/posembed.py); when every
        # encoder layer runs the fused attention block, their position gradients come back as per-(video, level)
        # sums through a small handle instead of a (N, S, d) gradient
        if fused_pos and not self.no_encoder and all(layer.block_ok(src_flatten) for layer in self.encoder.layers):
            lvl_pos, _ = level_pos_rows_split(pos_embeds, self.level_embed)  # a LevelPos, with the handle
        elif fused_pos:
            lvl_pos = level_pos_rows(pos_embeds, self.level_embed)
        else:
            lvl_pos = torch.cat(lvl_pos, 1)
        temporal_shapes = hostio.const(("level_T", tuple(level_T)), lambda: torch.tensor(level_T, dtype=torch.long),
                                       src_flatten.device)
        temporal_shapes.__dict__["_pdvc_level_T"] = tuple(level_T)  # _level_T reads it: no device read-back
        level_start_index = torch.cat((temporal_shapes.new_zeros((1,)), temporal_shapes.cumsum(0)[:-1]))
        valid_ratios = torch.stack([self.get_valid_ratio(m) for m in masks], 1)
        self.last_level_T = tuple(level_T)
        return src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos, mask_flatten

    def forward_encoder(self, src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten,
                        mask_flatten):
        if self.no_encoder:
            return src_flatten
        return self.encoder(src_flatten, temporal_shapes, level_start_index, valid_ratios, lvl_pos_embed_flatten,
                            mask_flatten)

    def prepare_decoder_input_query(self, memory, query_embed):
        bs = memory.shape[0]
        query_embed, tgt = torch.chunk(query_embed, 2, dim=1)
        # the Q reference points are the same for every video: one (Q, d) x (d, 1) product, then broadcast
        # (the reference applies the Linear to the expanded (bs, Q, d) tensor: the same values, bs times the work)
        reference_points = self.reference_points(query_embed).sigmoid().unsqueeze(0).expand(bs, -1, -1).contiguous()
        pos_rows, tgt_rows = query_embed, tgt
        query_embed = expand_rows(query_embed, bs)
        tgt = expand_rows(tgt, bs)
        # the (Q, d) rows every video repeats, for the first decoder layer's in_proj (see _shared_rows)
        query_embed.__dict__["_pdvc_rows"] = pos_rows
        tgt.__dict__["_pdvc_rows"] = tgt_rows
        return reference_points, tgt, reference_points, query_embed

    def prepare_decoder_input_proposal(self, gt_reference_points):
        topk_coords_unact = inverse_sigmoid(gt_reference_points)
        pos_trans_out = self.pos_trans_norm(self.pos_trans(self.get_proposal_pos_embed(topk_coords_unact)))
        query_embed, tgt = torch.chunk(pos_trans_out, 2, dim=2)
        return gt_reference_points, tgt, gt_reference_points, query_embed

    def forward_decoder(self, *kargs):
        return self.decoder(*kargs)


def _level_T(temporal_shapes):
    if isinstance(temporal_shapes, torch.Tensor):
        known = temporal_shapes.__dict__.get("_pdvc_level_T")  # the host tuple it was built from (no read-back)
        if known is not None:
            return known
        return tuple(int(x) for x in temporal_shapes.tolist())
    return tuple(int(x) for x in temporal_shapes)


class DeformableTransformerEncoderLayer(nn.Module):
    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        self.self_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.linear1 = Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout2 = nn.Dropout(dropout)
        self.linear2 = Linear(d_ffn, d_model)
        self.dropout3 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, src):
        if self.activation is F.relu and use_ffn_block(src):
            return ffn_block(src, self.linear1, self.linear2, self.norm2, self.dropout2.p, self.dropout3.p,
                             self.training)
        if self.activation is F.relu:
            src2 = self.linear2(self.dropout2(self.linear1(src, relu=True)))
        else:
            src2 = self.linear2(self.dropout2(self.activation(self.linear1(src))))
        return add_dropout_layernorm(src, src2, self.norm2, self.dropout3.p, self.training)

    def block_ok(self, src):
        return use_attn_block(src, self)

    def forward(self, src, pos, reference_points, temporal_shapes, level_start_index, padding_mask=None):
        handle = getattr(pos, "_pdvc_level_grad", None)
        if pos is not None and self.block_ok(src):
            # the sub-layer as one autograd node: gradients of src meet in GEMM epilogues (ops/functions/attn_block.py)
            src = encoder_attn_block(self, src, pos, handle, reference_points, _level_T(temporal_shapes),
                                     padding_mask)
            return self.forward_ffn(src)
        if handle is not None:
            raise RuntimeError("a level-position gradient handle needs the fused encoder attention block")
        src2 = self.self_attn(self.with_pos_embed(src, pos), reference_points, src, temporal_shapes,
                              level_start_index, padding_mask)
        src = add_dropout_layernorm(src, src2, self.norm1, self.dropout1.p, self.training)
        return self.forward_ffn(src)


class DeformableTransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers

    @staticmethod
    def get_reference_points(temporal_shapes, valid_ratios, device):
        """deformable_transformer.py:198-208: centre of every cell of every level, in valid units."""
        refs = []
        for lvl, L_ in enumerate(_level_T(temporal_shapes)):
            ref = torch.linspace(0.5, L_ - 0.5, L_, dtype=torch.float32, device=device)
            refs.append(ref.reshape(-1)[None] / (valid_ratios[:, None, lvl] * L_))
        reference_points = torch.cat(refs, 1)
        reference_points = reference_points[:, :, None] * valid_ratios[:, None]
        return reference_points[:, :, :, None]

    def forward(self, src, temporal_shapes, level_start_index, valid_ratios, pos=None, padding_mask=None):
        level_T = _level_T(temporal_shapes)
        reference_points = self.get_reference_points(level_T, valid_ratios, device=src.device)
        output = src
        for layer in self.layers:
            output = layer(output, pos, reference_points, level_T, level_start_index, padding_mask)
        return output


# The first decoder layer's self-attention input is the same Q query rows for every video (tgt and query_pos are
# prepare_decoder_input_query's expands): its in_proj runs on the Q rows once and the products are broadcast, where
# the reference projects the bs x Q expanded rows (the same values, bs times the work, forward and backward).
SHARED_QUERY_ROWS = os.environ.get("PDVC_SHARED_QUERY_ROWS", "1") != "0"


def _shared_rows(t):
    """The (Q, d) rows a decoder input repeats for every video (prepare_decoder_input_query), or None."""
    return None if t is None else t.__dict__.get("_pdvc_rows")


class QuerySelfAttention(nn.Module):
    """nn.MultiheadAttention(d_model, n_heads, dropout) with identical parameters (in_proj_weight,
    in_proj_bias, out_proj) and forward semantics for the decoder's (batch-first) use; the attention core
    softmax(Q K^T / sqrt(d) + key_padding) V (+ dropout on the probabilities) is a HIP kernel."""

    def __init__(self, embed_dim, num_heads, dropout=0.0):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        self.out_proj = Linear(embed_dim, embed_dim)
        xavier_uniform_(self.in_proj_weight)
        constant_(self.in_proj_bias, 0.)
        constant_(self.out_proj.bias, 0.)

    def forward(self, qk_in, v_in, key_padding_mask=None, batch=None):
        """qk_in (N, Q, E) = tgt + query_pos (query and key input); v_in (N, Q, E) = tgt;
        key_padding_mask (N, Q) True = ignore.  Returns (N, Q, E).  batch: qk_in and v_in are (Q, E) rows shared
        by `batch` videos (projected once, the products broadcast to (batch, Q, *))."""
        E = self.embed_dim
        w, b = self.in_proj_weight, self.in_proj_bias
        if qk_in.is_cuda and qk_in.dtype == torch.float32 and _lin.BACKEND != "hip":
            # both row blocks of in_proj with one packed weight gradient (no per-slice zero fill, copy and add)
            qk, v = PackedLinearFunction.apply(w, b, (2 * E, E), qk_in, v_in)
        else:
            qk = dense(qk_in, w[:2 * E], b[:2 * E])
            v = dense(v_in, w[2 * E:], b[2 * E:])
        if batch is not None:
            qk = expand_rows(qk, batch).contiguous()
            v = expand_rows(v, batch).contiguous()
        p = self.dropout if self.training else 0.0
        out = query_self_attention(qk, v, key_padding_mask, self.num_heads, p)
        return self.out_proj(out)


class DeformableTransformerDecoderLayer(nn.Module):
    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4):
        super().__init__()
        self.cross_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points)
        self.dropout1 = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.self_attn = QuerySelfAttention(d_model, n_heads, dropout=dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(d_model)
        self.linear1 = Linear(d_model, d_ffn)
        self.activation = _get_activation_fn(activation)
        self.dropout3 = nn.Dropout(dropout)
        self.linear2 = Linear(d_ffn, d_model)
        self.dropout4 = nn.Dropout(dropout)
        self.norm3 = nn.LayerNorm(d_model)

    @staticmethod
    def with_pos_embed(tensor, pos):
        return tensor if pos is None else tensor + pos

    def forward_ffn(self, tgt):
        if self.activation is F.relu and use_ffn_block(tgt):
            return ffn_block(tgt, self.linear1, self.linear2, self.norm3, self.dropout3.p, self.dropout4.p,
                             self.training)
        if self.activation is F.relu:
            tgt2 = self.linear2(self.dropout3(self.linear1(tgt, relu=True)))
        else:
            tgt2 = self.linear2(self.dropout3(self.activation(self.linear1(tgt))))
        return add_dropout_layernorm(tgt, tgt2, self.norm3, self.dropout4.p, self.training)

    def forward(self, tgt, query_pos, reference_points, src, src_temporal_shapes, level_start_index,
                src_padding_mask=None, query_mask=None):
        kpm = None if query_mask is None else ~query_mask
        t_rows, p_rows = _shared_rows(tgt), _shared_rows(query_pos)
        if SHARED_QUERY_ROWS and t_rows is not None and p_rows is not None:
            tgt2 = self.self_attn(t_rows + p_rows, t_rows, key_padding_mask=kpm, batch=tgt.shape[0])
        else:
            tgt2 = self.self_attn(self.with_pos_embed(tgt, query_pos), tgt, key_padding_mask=kpm)
        tgt = add_dropout_layernorm(tgt, tgt2, self.norm2, self.dropout2.p, self.training)
        tgt2 = self.cross_attn(self.with_pos_embed(tgt, query_pos), reference_points, src, src_temporal_shapes,
                               level_start_index, src_padding_mask)
        tgt = add_dropout_layernorm(tgt, tgt2, self.norm1, self.dropout1.p, self.training)
        return self.forward_ffn(tgt)


class DeformableTransformerDecoder(nn.Module):
    def __init__(self, decoder_layer, num_layers, return_intermediate=False):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.return_intermediate = return_intermediate
        self.bbox_head = None  # set by PDVC for iterative refinement (deformable_transformer.py:281)

    def forward(self, tgt, reference_points, src, src_temporal_shapes, src_level_start_index, src_valid_ratios,
                query_pos=None, src_padding_mask=None, query_padding_mask=None, disable_iterative_refine=False):
        level_T = _level_T(src_temporal_shapes)
        output = tgt
        intermediate, intermediate_refs, box_out = [], [], []
        for lid, layer in enumerate(self.layers):
            if reference_points.shape[-1] == 2:
                ref_in = reference_points[:, :, None] * torch.stack([src_valid_ratios, src_valid_ratios], -1)[:, None]
            else:
                ref_in = reference_points[:, :, None] * src_valid_ratios[:, None, :, None]
            output = layer(output, query_pos, ref_in, src, level_T, src_level_start_index, src_padding_mask,
                           query_padding_mask)
            if not disable_iterative_refine and self.bbox_head is not None:
                tmp = self.bbox_head[lid](output)
                box_out.append(tmp)
                # (tmp + inverse_sigmoid(ref)).sigmoid(); a 1-d reference refines only the centre
                # (deformable_transformer.py:311-313); detached, so computed outside autograd in one launch
                with torch.no_grad():
                    reference_points = box_refine(tmp.detach(), reference_points.detach())
            if self.return_intermediate:
                intermediate.append(output)
                intermediate_refs.append(reference_points)
        if self.return_intermediate:
            # side results for PDVC's per-layer heads (pdvc.py _layer_heads): every layer's output as its own
            # tensor (the heads read them directly, so no select of the stacked hs reaches the backward) and the
            # refinement's bbox_head outputs -- the heads' bbox_head call on the same rows and weights (the
            # reference evaluates it twice, deformable_transformer.py:305 and pdvc.py:192 / 253), reused instead
            self.__dict__["_side"] = (intermediate, box_out if len(box_out) == len(self.layers) else None)
            return torch.stack(intermediate), torch.stack(intermediate_refs)
        return output, reference_points


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def _get_activation_fn(activation):
    if activation == "relu":
        return F.relu
    if activation == "gelu":
        return F.gelu
    if activation == "glu":
        return F.glu
    raise RuntimeError(f"activation should be relu/gelu, not {activation}.")


def build_deforamble_transformer(args):
    return DeformableTransformer(d_model=args.hidden_dim, nhead=args.nheads, num_encoder_layers=args.enc_layers,
                                 num_decoder_layers=args.dec_layers, dim_feedforward=args.transformer_ff_dim,
                                 dropout=args.transformer_dropout_prob, activation="relu",
                                 return_intermediate_dec=True, num_feature_levels=args.num_feature_levels,
                                 dec_n_points=args.dec_n_points, enc_n_points=args.enc_n_points)


build_deformable_transformer = build_deforamble_transformer
