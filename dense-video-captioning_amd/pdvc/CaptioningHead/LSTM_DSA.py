"""LSTM captioner with deformable soft attention (reference: pdvc/CaptioningHead/LSTM_DSA.py:17-270).

Same parameters/state_dict names (embed, logit, core.rnn.weight_{ih,hh}_l0, core.deformable_att.*,
core.ctx2att, core.h2att, core.alpha_net) and the same per-step math, restructured for MI355X:

  * every matched (decoder layer, video, event) row of a batch is decoded in ONE recurrence (the reference
    runs one Python loop per decoder layer per video and asserts batch size 1, LSTM_DSA.py:59);
  * loop invariants are hoisted out of the recurrence -- value_proj(memory) (the reference recomputes an
    S x d x d GEMM every step, ms_deform_attn_for_caption.py:94), the embedding lookups and their LSTM
    input projection (teacher forcing makes every input token known up front), the event-feature part of
    the sampling-offset and LSTM projections -- and the three h_{t-1} projections (sampling offsets,
    h2att, W_hh) are one GEMM;
  * the caption logits (logit + log_softmax) are one GEMM over all steps after the recurrence;
  * the border-padded deformable sampling is the HIP caption-gather kernel; rows of decoder layer 0 (1-d
    reference) and later layers ((c, len) references) share one launch;
  * training runs the whole recurrence as one autograd function (ops/functions/caption_decode.py): 6 launches
    per step forward and backward (GEMMs + the gather, soft-attention and LSTM-cell kernels), weight gradients
    as single GEMMs over all steps.
The teacher-forced loop length is computed on the host from the caption lengths (the reference stops at the
first all-zero token column, LSTM_DSA.py:103-104): the same steps are computed, without a per-step sync.
"""
import math
import os

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from pdvc import _native as _n
from pdvc.ops.functions import CaptionDecodeFunction
from pdvc.caption_tokens import DeferredLogprobs, pack_rows
from pdvc.ops.functions.gemm3 import addmm_nt, mm_dgrad, mm_nt, mm_wgrad
from pdvc.ops.functions.linear import dense
from pdvc.ops.functions.logprob import logit_pick
from pdvc.ops.modules import MSDeformAttnCap
from pdvc.ops.modules.linear import Linear


# greedy decoding: ctx2att of the samples as a gather of the once-projected memory rows (LSTMDSACaptioner.
# _ctx2att_rows) instead of a GEMM per step; False keeps the GEMM (tests compare the two)
GREEDY_CTX2ATT_GATHER = True
# the greedy step's word / h / attention-gate products on gemm3 (A/B switch: PDVC_GREEDY_GEMM3=0 keeps torch's)
GREEDY_GEMM3 = os.environ.get("PDVC_GREEDY_GEMM3", "1") != "0"
# the greedy step's gathers and soft attention in one launch, samples and att not written (A/B: PDVC_GREEDY_FUSED_ATT=0)
GREEDY_FUSED_ATT = os.environ.get("PDVC_GREEDY_FUSED_ATT", "1") != "0"
# the greedy step's word gates as rows of a per-decode (vocabulary x 4H) table (A/B: PDVC_GREEDY_WORD_TABLE=0)
GREEDY_WORD_TABLE = os.environ.get("PDVC_GREEDY_WORD_TABLE", "1") != "0"
# ... read by the LSTM cell kernel through the word ids, its activations not written (A/B: PDVC_GREEDY_LSTM_GATHER=0)
GREEDY_LSTM_GATHER = os.environ.get("PDVC_GREEDY_LSTM_GATHER", "1") != "0"
# the teacher-forced word gates the same way, with a sorted (atomic-free) backward (A/B: PDVC_WORD_TABLE=0)
WORD_TABLE = os.environ.get("PDVC_WORD_TABLE", "1") != "0"


class _EmbeddingRows(torch.autograd.Function):
    """nn.Embedding's lookup with an atomic scatter-add backward (index_add_).  torch's embedding backward
    sorts the indices and runs rocprim unique-by-key/partition passes; replayed inside a captured hipGraph
    those faulted on MI355X (illegal address in rocprim's partition kernel), and they are ~6 extra launches."""

    @staticmethod
    def forward(ctx, weight, idx):
        ctx.save_for_backward(idx)
        ctx.rows = weight.shape[0]
        return weight.index_select(0, idx.reshape(-1)).view(*idx.shape, weight.shape[1])

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        D = g.shape[-1]
        gw = g.new_zeros((ctx.rows, D)).index_add_(0, idx.reshape(-1), g.reshape(-1, D))
        return gw, None


def _row_sums_ws(n, cols, device):
    """The workspace of pdvc_sorted_row_sums_f32: two rows of `cols` floats per 64 sorted positions."""
    return torch.empty(2 * ((n + 63) // 64) * cols, dtype=torch.float32, device=device)


class _WordGates(torch.autograd.Function):
    """xe = W_x embed(idx) for the teacher-forced recurrence (idx (n, R) step-major) with a backward over the
    positions that carry a gradient only: `act` (K,) lists them as flat step-major positions (entries >= n * R are
    padding).  A position past its caption's last loss-carrying word feeds no loss (LanguageModelCriterion masks it,
    LSTM_DSA.py:48-52, and every later step of its row is masked too), so its gate gradient is exactly zero: the
    weight gradient GEMM, the input gradient GEMM and the embedding scatter-add run over the K listed positions instead
    of all n * R.  (The scatter-add over all positions also piled every padding position's zero onto embedding row 0
    with atomics: 3.4 ms per step on a ragged stream, profiles/r04_*.)"""

    @staticmethod
    def forward(ctx, weight, W_x, idx, act):
        ctx.save_for_backward(weight, W_x, idx, act)
        ctx.table = WORD_TABLE and idx.is_cuda and W_x.shape[0] % 4 == 0
        if ctx.table:  # rows of the batch's (V + 1) x 4H word-gate table (_WordTable)
            return mm_nt(weight, W_x).index_select(0, idx.reshape(-1)).view(*idx.shape, W_x.shape[0])
        xt = weight.index_select(0, idx.reshape(-1))
        return mm_nt(xt, W_x).view(*idx.shape, W_x.shape[0])

    @staticmethod
    def backward(ctx, g):
        weight, W_x, idx, act = ctx.saved_tensors
        N = idx.numel()
        a = act.clamp(max=N - 1)
        gs = g.reshape(N, -1).index_select(0, a)
        ids = idx.reshape(-1).index_select(0, a)
        if ctx.table:  # the listed positions' gradients summed per word (padding entries keyed past the table)
            V = weight.shape[0]
            keys, order = torch.sort(torch.where(act >= N, torch.full_like(ids, V), ids), stable=True)
            dT = torch.empty((V, gs.shape[1]), dtype=gs.dtype, device=gs.device)
            _n.call("pdvc_sorted_row_sums_f32", _n.ptr(gs), gs.stride(0), gs.shape[1], _n.ptr(keys), _n.ptr(order),
                    ids.numel(), V, _n.ptr(dT), dT.stride(0), _n.ptr(_row_sums_ws(ids.numel(), gs.shape[1], gs.device)),
                    _n.stream())
            dW_x = mm_wgrad(dT, weight)
            if dW_x is None:
                dW_x = torch.mm(dT.t(), weight)
            return mm_dgrad(dT, W_x), dW_x, None, None
        gs.masked_fill_((act >= N)[:, None], 0.0)  # padding entries: no contribution
        xs = weight.index_select(0, ids)  # the embedding rows again (not saved: (n R, E) floats)
        dW_x = mm_wgrad(gs, xs)
        if dW_x is None:
            dW_x = torch.mm(gs.t(), xs)
        dw = weight.new_zeros(weight.shape).index_add_(0, ids, mm_dgrad(gs, W_x))
        return dw, dW_x, None, None


class _WordTable(torch.autograd.Function):
    """xe = W_x embed(idx) (idx (n, R) step-major) as rows of the batch's word-gate table T = embed.weight W_x^T
    ((V + 1) x 4H): one (V + 1)-row GEMM and a row gather instead of an (n R)-row GEMM.  Backward: the gathered rows'
    gradients summed per word in a fixed order (a stable sort of idx, pdvc_sorted_row_sums_f32: no atomics), then
    d embed.weight = dT W_x and dW_x = dT^T embed.weight -- two (V + 1)-row GEMMs where the per-position form ran two
    (n R)-row GEMMs and an atomic scatter-add into the embedding.  The same sums as LSTM_DSA.py:229-231 (embed, then
    W_ih over [xt, ...]) in another order."""

    @staticmethod
    def forward(ctx, weight, W_x, idx):
        ctx.save_for_backward(weight, W_x, idx)
        table = mm_nt(weight, W_x)
        return table.index_select(0, idx.reshape(-1)).view(*idx.shape, W_x.shape[0])

    @staticmethod
    def backward(ctx, g):
        weight, W_x, idx = ctx.saved_tensors
        flat = idx.reshape(-1)
        keys, order = torch.sort(flat, stable=True)
        G = g.reshape(flat.numel(), -1)
        if G.stride(1) != 1 or G.stride(0) % 4 or G.data_ptr() % 16:
            G = G.contiguous()
        V, C4 = weight.shape[0], G.shape[1]
        dT = torch.empty((V, C4), dtype=G.dtype, device=G.device)
        _n.call("pdvc_sorted_row_sums_f32", _n.ptr_any(G), G.stride(0), C4, _n.ptr(keys), _n.ptr(order), flat.numel(),
                V, _n.ptr(dT), C4, _n.ptr(_row_sums_ws(flat.numel(), C4, G.device)), _n.stream())
        dw = mm_dgrad(dT, W_x) if ctx.needs_input_grad[0] else None
        dW_x = None
        if ctx.needs_input_grad[1]:
            dW_x = mm_wgrad(dT, weight)
            if dW_x is None:
                dW_x = torch.mm(dT.t(), weight)
        return dw, dW_x, None


def embed_rows(embedding, idx):
    """embedding(idx) for an nn.Embedding without padding_idx/max_norm (the caption head's)."""
    if embedding.padding_idx is not None or embedding.max_norm is not None or not idx.is_cuda:
        return embedding(idx)
    return _EmbeddingRows.apply(embedding.weight, idx)


class LSTMWeights(nn.Module):
    """The parameters of nn.LSTM(input_size, hidden_size, num_layers=1, bias=False) under nn.LSTM's names
    and init (uniform +-1/sqrt(hidden)).  Only the weights are used: the cell runs in the decoder loop."""

    def __init__(self, input_size, hidden_size, num_layers=1):
        super().__init__()
        if num_layers != 1:
            raise NotImplementedError("the caption LSTM supports num_layers=1 (every PDVC config)")
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.weight_ih_l0 = nn.Parameter(torch.empty(4 * hidden_size, input_size))
        self.weight_hh_l0 = nn.Parameter(torch.empty(4 * hidden_size, hidden_size))
        stdv = 1.0 / math.sqrt(hidden_size)
        for w in (self.weight_ih_l0, self.weight_hh_l0):
            nn.init.uniform_(w, -stdv, stdv)


def lstm_cell(gates, c):
    """PyTorch gate order (i, f, g, o); c' = f*c + i*g; h' = o*tanh(c')."""
    i, f, g, o = gates.chunk(4, 1)
    c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    h = torch.sigmoid(o) * torch.tanh(c)
    return h, c


class Captioner(nn.Module):
    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.vocab_size = opt.vocab_size
        self.input_encoding_size = opt.input_encoding_size
        self.rnn_size = opt.rnn_size
        self.num_layers = opt.num_layers
        self.drop_prob_lm = opt.drop_prob
        self.max_caption_len = opt.max_caption_len
        self.ss_prob = 0.0
        self.embed = nn.Embedding(self.vocab_size + 1, self.input_encoding_size)
        self.logit = Linear(self.rnn_size, self.vocab_size + 1)
        self.dropout = nn.Dropout(self.drop_prob_lm)
        self.init_weights()

    def init_weights(self):
        r = 0.1
        self.embed.weight.data.uniform_(-r, r)
        self.logit.bias.data.fill_(0)
        self.logit.weight.data.uniform_(-r, r)

    def init_hidden(self, batch_size):
        w = next(self.parameters())
        return (w.new_zeros(self.num_layers, batch_size, self.rnn_size),
                w.new_zeros(self.num_layers, batch_size, self.rnn_size))

    def build_loss(self, input, target, mask):
        """-(sum_t logp[t, target_t] * mask_t) / (sum mask + 1e-6) (LSTM_DSA.py:48-52), as a gather
        instead of a (rows, steps, vocab) one-hot product."""
        max_len = input.shape[1]
        picked = input.gather(2, target[:, :max_len, None]).squeeze(2)
        return -(picked * mask[:, :max_len]).sum(1) / (mask.sum(1) + 1e-6)

    @staticmethod
    def build_loss_picked(picked, mask):
        """build_loss from the target log-probabilities already gathered (decode_teacher_forced(pick_target=...)):
        -(sum_t picked_t * mask_t) / (sum mask + 1e-6), the same per-row values (LSTM_DSA.py:48-52)."""
        max_len = picked.shape[1]
        return -(picked * mask[:, :max_len]).sum(1) / (mask.sum(1) + 1e-6)


def caption_steps(cap_tensor_cpu):
    """Number of decoder steps of the reference's teacher-forced loop for one video's captions:
    i runs over range(K-1) and stops at the first i >= 1 whose token column is all zero."""
    x = cap_tensor_cpu.numpy() if isinstance(cap_tensor_cpu, torch.Tensor) else np.asarray(cap_tensor_cpu)
    K = x.shape[1]
    if K < 3:
        return max(K - 1, 0)
    zero = np.flatnonzero(np.abs(x[:, 1:K - 1]).sum(0) == 0)
    return int(zero[0]) + 1 if zero.size else K - 1


class ShowAttendTellCore(nn.Module):
    def __init__(self, opt):
        super().__init__()
        self.input_encoding_size = opt.input_encoding_size
        self.rnn_size = opt.rnn_size
        self.num_layers = opt.num_layers
        self.drop_prob_lm = opt.drop_prob
        self.att_feat_size = int(opt.clip_context_dim / opt.cap_nheads)
        self.att_hid_size = opt.att_hid_size
        self.opt = opt
        self.wordRNN_input_feats_type = opt.wordRNN_input_feats_type
        self.input_dim = opt.hidden_dim * 2
        self.rnn = LSTMWeights(self.input_encoding_size + self.input_dim, self.rnn_size, self.num_layers)
        self.att_drop = nn.Dropout(0.5)  # owned by the reference, never applied
        d_model = opt.hidden_dim
        self.n_levels = opt.cap_num_feature_levels
        self.n_heads = opt.cap_nheads
        self.n_points = opt.cap_dec_n_points
        self.deformable_att = MSDeformAttnCap(d_model, self.n_levels, self.n_heads, self.n_points)
        if self.att_hid_size > 0:
            self.ctx2att = nn.Linear(self.att_feat_size, self.att_hid_size)
            self.h2att = nn.Linear(self.rnn_size, self.att_hid_size)
            self.alpha_net = nn.Linear(self.att_hid_size, 1)


# the greedy loop's exit test on the device (decode_greedy): a count read every CHECK_EVERY steps, CHECK_LAG steps late
CHECK_EVERY = 2
CHECK_LAG = 4
_PINNED = {}


def _pinned_counts(n):
    """A pinned host buffer of n int64 (per size, reused; each decode's copies are ordered by its own events)."""
    b = _PINNED.get(n)
    if b is None:
        b = _PINNED[n] = torch.empty(n, dtype=torch.long, pin_memory=torch.cuda.is_available())
    return b


class LSTMDSACaptioner(Captioner):
    def __init__(self, opt):
        super().__init__(opt)
        self.core = ShowAttendTellCore(opt)

    # ------------------------------------------------------------------------------------------------
    # the batched decode engine
    # ------------------------------------------------------------------------------------------------
    def _prepare(self, memory, mask_flatten):
        core = self.core
        # hoisted: identical for every step; the trunk may have projected memory for all its consumers at once
        value = getattr(memory, "_pdvc_values", {}).get(id(core.deformable_att.value_proj))
        if value is None:
            value = core.deformable_att.value_proj(memory)
        mask_u8 = None if mask_flatten is None else mask_flatten.contiguous().view(torch.uint8)
        return value, mask_u8

    def _step_weights(self):
        core = self.core
        H = self.rnn_size
        E = self.input_encoding_size
        Dm = core.input_dim // 2
        W_off, b_off = core.deformable_att.sampling_offsets.weight, core.deformable_att.sampling_offsets.bias
        W_ih, W_hh = core.rnn.weight_ih_l0, core.rnn.weight_hh_l0
        n_off = W_off.shape[0]
        A = core.att_hid_size
        # one GEMM for every h_{t-1} projection: [sampling offsets (h part) ; h2att ; W_hh]
        W_h = torch.cat([W_off[:, :H], core.h2att.weight, W_hh], 0)
        b_h = torch.cat([b_off.new_zeros(n_off), core.h2att.bias, W_hh.new_zeros(W_hh.shape[0])], 0)
        return dict(H=H, E=E, Dm=Dm, n_off=n_off, A=A, W_off_hs=W_off[:, H:], b_off=b_off,
                    W_x=W_ih[:, :E], W_att=W_ih[:, E:E + Dm], W_hs=W_ih[:, E + Dm:], W_h=W_h, b_h=b_h)

    def _step(self, w, h, c, x_gates, hs_part, off_hs, value, mask_u8, row_video, ref_rows, rd1_rows, level_T):
        """One decoder step for all rows (LSTM_DSA.py:231-263)."""
        core = self.core
        n_off, A = w["n_off"], w["A"]
        hp = F.linear(h, w["W_h"], w["b_h"])
        off = hp[:, :n_off] + off_hs
        att_h = hp[:, n_off:n_off + A]
        g_hh = hp[:, n_off + A:]
        clip = core.deformable_att.sample_rows(value, mask_u8, row_video, off.contiguous(), ref_rows, level_T, 0,
                                               rd1_rows)  # (R, M, L*P, D)
        R, M, NS, D = clip.shape
        att = core.ctx2att(clip)  # (R, M, NS, A)
        dot = torch.tanh(att + att_h[:, None, None, :])
        dot = core.alpha_net(dot).squeeze(-1)  # (R, M, NS)
        weight = F.softmax(dot, dim=-1)
        att_res = torch.bmm(weight.reshape(R * M, 1, NS), clip.reshape(R * M, NS, D)).reshape(R, M * D)
        gates = x_gates + hs_part + F.linear(att_res, w["W_att"]) + g_hh
        return lstm_cell(gates, c)

    def _fused_step_ok(self, hs_rows, value, w):
        """The greedy step can run on the teacher-forced recurrence's kernels (the same six launches per step as
        CaptionDecodeFunction.forward): fp32 GPU rows, float4-aligned widths, a soft-attention hidden layer."""
        core = self.core
        M = core.deformable_att.n_heads
        D = value.shape[-1] // M
        return (hs_rows.is_cuda and hs_rows.dtype == torch.float32 and value.dtype == torch.float32
                and w["A"] > 0 and w["A"] % 4 == 0 and D % 4 == 0 and w["H"] % 4 == 0
                and core.deformable_att.fused)

    def _greedy_buffers(self, R, value, w):
        core = self.core
        M = core.deformable_att.n_heads
        D = value.shape[-1] // M
        Ph = w["W_h"].shape[0]
        kw = dict(dtype=value.dtype, device=value.device)
        # (CLIP and ATT, the samples and att rows, only for the three-launch step: allocated there on first use)
        return dict(HP=torch.empty((R, Ph), **kw), CLIP=None, LOC=torch.empty((R, M, 16), **kw), ATT=None,
                    PROBS=torch.empty((R, M, 16), **kw), RES=torch.empty((R, M * D), **kw),
                    GATT=torch.empty((R, 4 * w["H"]), **kw), ACTS=torch.empty((R, 4 * w["H"]), **kw),
                    H=[torch.empty((R, w["H"]), **kw) for _ in range(2)],
                    C=[torch.empty((R, w["H"]), **kw) for _ in range(2)])

    def _ctx2att_rows(self, value, mask_u8):
        """ctx2att of every memory position, once per decode: U = ctx2att(value masked to 0 at padding), (Nv, S, M, A).
        A sample is a border-clamped bilinear blend of value rows whose weights sum to 1, so ctx2att(sample) =
        W (sum_k w_k v_k) + b = sum_k w_k (W v_k + b): the same blend of U rows -- one gather per step instead of
        a (rows x 16) x D x A GEMM per step (LSTM_DSA.py:245: att = self.ctx2att(clip)).  Padded rows are zeroed
        before the projection (their U row is the bias), which reproduces the kernel's zero contribution of a
        padded corner to the sample while the blend weights keep summing to 1."""
        core = self.core
        Nv, S, E = value.shape
        M = core.deformable_att.n_heads
        D = E // M
        v = value.view(Nv, S, M, D)
        if mask_u8 is not None:
            v = v.masked_fill(mask_u8.view(Nv, S, 1, 1).bool(), 0.0)
        U = addmm_nt(core.ctx2att.bias, v.reshape(-1, D), core.ctx2att.weight)
        return U.view(Nv, S, M, -1)

    def _step_fused(self, w, b, t, h, c, x_gates, hs_part, off_hs, value, mask_u8, row_video, ref_rows, rd1_rows,
                    level_T):
        """One decoder step for all rows on the fused kernels of the teacher-forced recurrence
        (ops/functions/caption_decode.py): h-projection GEMM, border sampling at ref (+) (hp offsets + off_hs),
        ctx2att as a second gather of the pre-projected rows U, soft attention (tanh, alpha_net, softmax over the
        16 samples, weighted sum), the attention gate GEMM and the LSTM cell with the four gate addends --
        LSTM_DSA.py:231-263, as _step."""
        from pdvc import _native as _n
        from pdvc.ops.functions.ms_deform_attn_func import NUM_SAMPLES, _levels
        core = self.core
        Nv, S, E = value.shape
        M = core.deformable_att.n_heads
        D = E // M
        R, H = h.shape
        G = 4 * H
        n_off, A = w["n_off"], w["A"]
        Ph = w["W_h"].shape[0]
        lvl, nl = _levels(level_T)
        st = _n.stream()
        HP = b["HP"]
        if GREEDY_GEMM3:
            addmm_nt(w["b_h"], h, w["W_h"], out=HP)
        else:
            torch.addmm(w["b_h"], h, w["W_h"].t(), out=HP)
        ref = ref_rows.contiguous()
        alpha_w = core.alpha_net.weight.view(-1)
        if (GREEDY_FUSED_ATT and b["U"] is not None and A == D == 512 and Ph % 4 == 0 and n_off % 4 == 0
                and all(q.data_ptr() % 16 == 0 for q in (value, b["U"], HP, alpha_w))):
            # the two gathers and the soft attention in one launch (the teacher-forced recurrence's kernel), the
            # samples and att never written: nothing reads them back in a greedy decode
            ah, ldh = _n.rows(HP[:, n_off:n_off + A])
            _n.call("pdvc_cap_softattn_forward_f32", _n.ptr(value), _n.ptr(mask_u8), _n.ptr(b["U"]),
                    _n.ptr(row_video), _n.ptr(HP), Ph, 0, _n.ptr(off_hs.contiguous()), _n.ptr(ref), ref.shape[2],
                    int(rd1_rows), lvl, nl, Nv, R, M, D, NUM_SAMPLES // nl, ah, ldh, _n.ptr(alpha_w),
                    _n.ptr(core.alpha_net.bias), None, _n.ptr(b["LOC"]), None, _n.ptr(b["PROBS"]), _n.ptr(b["RES"]),
                    st)
        else:
            self._gather_softattn(b, value, mask_u8, row_video, HP, Ph, off_hs, ref, rd1_rows, lvl, nl, Nv, R, M, D,
                                  A, n_off, st)
        if GREEDY_GEMM3:
            mm_nt(b["RES"], w["W_att"], out=b["GATT"])
        else:
            torch.mm(b["RES"], w["W_att"].t(), out=b["GATT"])
        gh, ldg = _n.rows(HP[:, n_off + A:])
        h_out, c_out = b["H"][t % 2], b["C"][t % 2]
        if isinstance(x_gates, tuple):  # (word-gate table, word ids): rows read by id, no activations kept
            xtab, ids = x_gates
            _n.call("pdvc_lstm_cell_forward_gather_f32", _n.ptr(xtab), xtab.stride(0), _n.ptr(ids.contiguous()),
                    _n.ptr(b["GATT"]), G, gh, ldg, _n.ptr(hs_part.contiguous()), G, _n.ptr(c.contiguous()), R, H,
                    _n.ptr(h_out), H, _n.ptr(c_out), None, st)
        else:
            xg = x_gates.contiguous()
            _n.call("pdvc_lstm_cell_forward_f32", _n.ptr(xg), G, _n.ptr(b["GATT"]), G, gh, ldg,
                    _n.ptr(hs_part.contiguous()), G, _n.ptr(c.contiguous()), R, H, _n.ptr(h_out), H, _n.ptr(c_out),
                    _n.ptr(b["ACTS"]), st)
        return h_out, c_out

    def _gather_softattn(self, b, value, mask_u8, row_video, HP, Ph, off_hs, ref, rd1_rows, lvl, nl, Nv, R, M, D, A,
                         n_off, st):
        """The greedy step's samples, att and soft attention as three launches (gather, gather or ctx2att GEMM, soft
        attention): the heads the fused kernel does not take."""
        from pdvc.ops.functions.ms_deform_attn_func import NUM_SAMPLES
        core = self.core
        if b["CLIP"] is None:
            b["CLIP"] = torch.empty((R, M, NUM_SAMPLES, D), dtype=value.dtype, device=value.device)
            b["ATT"] = torch.empty((R * M * NUM_SAMPLES, A), dtype=value.dtype, device=value.device)
        _n.call("pdvc_cap_gather_forward_f32", _n.ptr(value), _n.ptr(mask_u8), _n.ptr(row_video), _n.ptr(HP), Ph, 0,
                _n.ptr(off_hs.contiguous()), _n.ptr(ref), ref.shape[2], int(rd1_rows), lvl, nl, Nv, R, M, D,
                NUM_SAMPLES // nl, _n.ptr(b["CLIP"]), _n.ptr(b["LOC"]), st)
        if b["U"] is not None:  # att = ctx2att(clip) as the same sample blend of the projected rows U, no mask
            _n.call("pdvc_cap_gather_forward_f32", _n.ptr(b["U"]), None, _n.ptr(row_video), _n.ptr(HP), Ph, 0,
                    _n.ptr(off_hs.contiguous()), _n.ptr(ref), ref.shape[2], int(rd1_rows), lvl, nl, Nv, R, M, A,
                    NUM_SAMPLES // nl, _n.ptr(b["ATT"]), None, st)
        else:
            torch.addmm(core.ctx2att.bias, b["CLIP"].view(-1, D), core.ctx2att.weight.t(), out=b["ATT"])
        ah, ldh = _n.rows(HP[:, n_off:n_off + A])
        _n.call("pdvc_softattn_forward_f32", _n.ptr(b["ATT"]), ah, ldh, _n.ptr(core.alpha_net.weight.view(-1)),
                _n.ptr(core.alpha_net.bias), _n.ptr(b["CLIP"]), R, M, A, D, _n.ptr(b["RES"]), _n.ptr(b["PROBS"]), st)

    def decode_teacher_forced(self, hs_rows, ref_rows, rd1_rows, row_video, memory, mask_flatten, level_T, seq,
                              n_steps, video_csr=None, pick_target=None, tokens=None, step_ranges=None):
        """hs_rows (R, d) event features; ref_rows (R, L, 2) references (rows < rd1_rows are 1-d: centre in
        [..., 0]); row_video (R,) int32; memory (N, S, d); seq (R, K) long; returns logprobs (R, n_steps, V).
        video_csr (start, rows, max rows per video) of row_video lets the backward sum the value gradient of all
        steps in one destination-sorted pass (no float atomics).  With pick_target (R, >= n_steps) long, returns
        (logprobs, picked) where picked (R, n_steps) = logprobs at the target words (csrc/logprob.hip: log_softmax
        and the loss's gather in one pass, the backward in one pass -- the input of build_loss_picked).  With tokens
        (index, scatter) of pdvc/caption_tokens.py pack_tokens as well, the logit GEMM and that pass run over the packed
        valid tokens only, picked is zero at the other positions, and the logprobs come back as a DeferredLogprobs.
        step_ranges: (host per-step (start, count), device copy) -- the rows of each step when the rows are ordered by
        their video's step count (pdvc.py `_caption_rows`); the other (row, step) hidden states are zeros."""
        core = self.core
        if self.training and self.ss_prob > 0:
            out = self.decode_scheduled_sampling(hs_rows, ref_rows, rd1_rows, row_video, memory, mask_flatten,
                                                 level_T, seq, n_steps)
            if pick_target is None:
                return out
            return out, out.gather(2, pick_target[:, :n_steps, None]).squeeze(2)
        w = self._step_weights()
        value, mask_u8 = self._prepare(memory, mask_flatten)
        if n_steps == 0:
            empty = hs_rows.new_zeros(hs_rows.shape[0], 0, self.vocab_size + 1)
            return empty if pick_target is None else (empty, hs_rows.new_zeros(hs_rows.shape[0], 0))
        if tokens is not None and pick_target is not None and self.embed.padding_idx is None \
                and self.embed.max_norm is None:
            # the word gates' backward over the loss-carrying tokens only (_WordGates): their step-major positions
            R_, n_ = seq.shape[0], n_steps
            sc = tokens[1]
            live = sc < R_ * n_
            act = torch.where(live, (sc % n_) * R_ + torch.div(sc, n_, rounding_mode="floor"),
                              torch.full_like(sc, R_ * n_))
            xe = _WordGates.apply(self.embed.weight, w["W_x"], seq[:, :n_steps].t().contiguous(), act)
        elif (WORD_TABLE and seq.is_cuda and hs_rows.dtype == torch.float32 and self.embed.padding_idx is None
              and self.embed.max_norm is None and w["W_x"].shape[0] % 4 == 0):
            # the word part of the gates as rows of the batch's (V + 1) x 4H table (_WordTable)
            xe = _WordTable.apply(self.embed.weight, w["W_x"], seq[:, :n_steps].t().contiguous())
        else:
            xt = embed_rows(self.embed, seq[:, :n_steps].t())  # (n, R, E): step-major, the recurrence's layout
            xe = dense(xt, w["W_x"])  # loop-invariant gate parts: word part per step, event part per row
        hs_g = dense(hs_rows, w["W_hs"])
        off_hs = F.linear(hs_rows, w["W_off_hs"], w["b_off"])
        Nv, S, _ = value.shape
        M = core.deformable_att.n_heads
        # the projection output itself (no view node): its gradient comes back with the bias gradient's row sums
        Hs = CaptionDecodeFunction.apply(
            value, xe, hs_g, off_hs, ref_rows, w["W_h"], w["b_h"], core.ctx2att.weight,
            core.ctx2att.bias, core.alpha_net.weight.view(-1), core.alpha_net.bias, w["W_att"], mask_u8, row_video,
            tuple(level_T), rd1_rows, video_csr, M, step_ranges)
        Hd = self.dropout(Hs)
        if pick_target is not None and tokens is not None:
            index, scatter = tokens
            R, n, H = Hd.shape
            Hp = pack_rows(Hd.reshape(R * n, H), tokens)
            tgt = pick_target[:, :n_steps].reshape(-1).index_select(0, index)
            _, picked_p = logit_pick(Hp, self.logit, tgt)
            picked = Hp.new_zeros(R * n + 1).index_copy(0, scatter, picked_p)[:R * n].view(R, n)
            return DeferredLogprobs(Hd.detach(), self.logit.weight.detach().clone(),
                                    self.logit.bias.detach().clone()), picked
        if pick_target is not None:
            return logit_pick(Hd, self.logit, pick_target[:, :n_steps])
        return F.log_softmax(self.logit(Hd), dim=-1)

    def decode_scheduled_sampling(self, hs_rows, ref_rows, rd1_rows, row_video, memory, mask_flatten, level_T, seq,
                                  n_steps, generator=None, record=None):
        """The teacher-forced loop with scheduled sampling (LSTM_DSA.py:88-107, training with ss_prob > 0): from
        step 1 on, each row's input word is, with probability ss_prob, drawn from the previous step's distribution
        exp(logprobs) (torch.multinomial over every row, the drawn words substituted where a uniform draw falls
        below ss_prob) instead of the ground-truth word; the drawn words carry no gradient.  Every step's input
        then depends on the previous step's output, so the word gates are formed per step and the steps run
        through autograd (the same per-step math as _step) instead of the whole-sequence CaptionDecodeFunction.
        Rows whose video's loop has already stopped (the reference breaks at the video's first all-zero token
        column) keep stepping with their masked targets, which the loss ignores.  record: a list that receives
        each step's input words (R,) -- tests replay them through the teacher-forced path.  Returns logprobs
        (R, n_steps, V).  (train.py:152-156 assigns the schedule to the caption_head ModuleList, which no
        captioner reads: set Captioner.ss_prob itself to enable it.)"""
        R = hs_rows.shape[0]
        w = self._step_weights()
        value, mask_u8 = self._prepare(memory, mask_flatten)
        hs_part = F.linear(hs_rows, w["W_hs"])
        off_hs = F.linear(hs_rows, w["W_off_hs"], w["b_off"])
        h = hs_rows.new_zeros(R, w["H"])
        c = hs_rows.new_zeros(R, w["H"])
        outs = []
        for i in range(n_steps):
            it = seq[:, i].clone()
            if i >= 1:
                u = torch.rand(R, device=hs_rows.device, generator=generator)
                drawn = torch.multinomial(torch.exp(outs[-1].detach()), 1, generator=generator).view(-1)
                it = torch.where(u < self.ss_prob, drawn, it)
            if record is not None:
                record.append(it)
            x_gates = F.linear(embed_rows(self.embed, it), w["W_x"])
            h, c = self._step(w, h, c, x_gates, hs_part, off_hs, value, mask_u8, row_video, ref_rows, rd1_rows,
                              level_T)
            outs.append(F.log_softmax(self.logit(self.dropout(h)), dim=-1))
        if not outs:
            return hs_rows.new_zeros(R, 0, self.vocab_size + 1)
        return torch.stack(outs, 1)

    @torch.no_grad()
    def decode_greedy(self, hs_rows, ref_rows, rd1_rows, row_video, memory, mask_flatten, level_T, max_len=None,
                      sample_max=1, temperature=1.0, generator=None):
        """Caption decoding for all rows at once (LSTM_DSA.py:118-186); returns seq (R, T) and seqLogprobs
        (R, T) with the reference's unfinished-mask semantics, T <= max_len + 1 steps.  sample_max=1: greedy
        (argmax word and its log-probability).  sample_max=0: the next word is drawn from
        exp(logprobs / temperature) (torch.multinomial, normalised; `generator` seeds it) and its log-probability
        is the untempered logprobs at the drawn word, as LSTM_DSA.py:160-168."""
        R = hs_rows.shape[0]
        max_len = self.max_caption_len if max_len is None else max_len
        w = self._step_weights()
        value, mask_u8 = self._prepare(memory, mask_flatten)
        hs_part = F.linear(hs_rows, w["W_hs"])
        off_hs = F.linear(hs_rows, w["W_off_hs"], w["b_off"])
        h = hs_rows.new_zeros(R, w["H"])
        c = hs_rows.new_zeros(R, w["H"])
        fused = self._fused_step_ok(hs_rows, value, w)
        if fused:
            # the per-step products on the in-tree fp32 GEMM (gemm3, row-major weights: the word and attention
            # parts of W_ih as contiguous copies, once per decode) where the row count takes it, else torch's
            w = dict(w, W_x=w["W_x"].contiguous(), W_att=w["W_att"].contiguous())
            value = value.contiguous()
            step_bufs = self._greedy_buffers(R, value, w)
            A = w["A"]  # the gather kernel's widths: powers of two in [32, 512] (else ctx2att stays a GEMM)
            gather = GREEDY_CTX2ATT_GATHER and 32 <= A <= 512 and A & (A - 1) == 0
            step_bufs["U"] = self._ctx2att_rows(value, mask_u8) if gather else None
        # the word part of the gates for every vocabulary entry, once per decode ((V + 1) x 4H, the embedding table
        # through W_x): each step then gathers its rows instead of embedding and projecting R rows
        xtab = None
        if fused and GREEDY_WORD_TABLE and self.embed.padding_idx is None and self.embed.max_norm is None:
            xtab = mm_nt(self.embed.weight, w["W_x"])
        it = torch.zeros(R, dtype=torch.long, device=hs_rows.device)
        seq, seqlp = [], []
        unfinished = None
        # the reference leaves the loop at the first step whose rows have all finished (LSTM_DSA.py:178-179).  Its
        # test stays on the device: each step's count of unfinished rows goes into alive[t], and the host reads one
        # count per CHECK_EVERY steps, CHECK_LAG steps late (an async copy into pinned memory), so the launches run
        # ahead of the decode instead of waiting for every step's read-back; the steps decoded past the reference's
        # exit are cut off after the loop from the counts (one read): seq and seqlp are exactly the reference's
        dev = hs_rows.device
        alive = torch.ones(max_len + 2, dtype=torch.long, device=dev)
        host = _pinned_counts(max_len + 2)
        pending = []  # (step, event) of the counts copied to the host, oldest first
        for t in range(max_len + 1):
            if t > 0:
                if sample_max and logprobs is None:  # fused: argmax and its log-probability from the logits
                    sample_lp = torch.empty(R, dtype=logits.dtype, device=logits.device)
                    it = torch.empty(R, dtype=torch.long, device=logits.device)
                    _n.call("pdvc_logprob_argmax_f32", _n.ptr(logits), R, logits.shape[1], _n.ptr(it),
                            _n.ptr(sample_lp), _n.stream())
                elif sample_max:
                    sample_lp, it = torch.max(logprobs, 1)
                else:
                    prob = torch.exp(logprobs if temperature == 1.0 else torch.div(logprobs, temperature))
                    it = torch.multinomial(prob, 1, generator=generator)
                    sample_lp = logprobs.gather(1, it)
                    it = it.view(-1)
            if xtab is not None:  # read through the word ids by the LSTM cell kernel: no gathered copy
                x_gates = (xtab, it) if GREEDY_LSTM_GATHER else xtab.index_select(0, it)
            elif fused and GREEDY_GEMM3:
                x_gates = mm_nt(self.embed(it), w["W_x"])
            else:
                x_gates = F.linear(self.embed(it), w["W_x"])
            if fused:
                h, c = self._step_fused(w, step_bufs, t, h, c, x_gates, hs_part, off_hs, value, mask_u8, row_video,
                                        ref_rows, rd1_rows, level_T)
            else:
                h, c = self._step(w, h, c, x_gates, hs_part, off_hs, value, mask_u8, row_video, ref_rows, rd1_rows,
                                  level_T)
            logits = self.logit(self.dropout(h))
            # greedy on the fused path needs only each row's argmax and its log-probability (pdvc_logprob_argmax_f32)
            logprobs = None if (fused and sample_max) else F.log_softmax(logits, dim=1)
            if t >= 1:
                unfinished = (it > 0) if t == 1 else (unfinished & (it > 0))
                torch.sum(unfinished, 0, out=alive[t])
                seq.append(it * unfinished.type_as(it))
                seqlp.append(sample_lp.view(-1))
                if not alive.is_cuda:  # (CPU: the reference's immediate test)
                    if int(alive[t]) == 0:
                        break
                elif t % CHECK_EVERY == 0:
                    host[t].copy_(alive[t], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                    pending.append((t, ev))
                if pending and pending[0][0] <= t - CHECK_LAG:
                    tc, ev = pending.pop(0)
                    ev.synchronize()
                    if int(host[tc]) == 0:
                        break
        if seq:  # the reference's exit: the first step with no unfinished row (its tokens are not appended)
            counts = alive[1:len(seq) + 1].cpu()
            zero = (counts == 0).nonzero()
            if len(zero):
                keep = int(zero[0, 0])
                seq, seqlp = seq[:keep], seqlp[:keep]
        if not seq:
            return None, None
        return torch.stack(seq, 1), torch.stack(seqlp, 1)

    # ------------------------------------------------------------------------------------------------
    # reference-compatible entry points (one video: hs (1, E, d))
    # ------------------------------------------------------------------------------------------------
    def _rows_from_reference(self, hs, reference, others):
        vid_num, query_num, _ = hs.shape
        L = self.core.n_levels
        vr = others["valid_ratios"]
        if reference.shape[-1] == 2:
            ref = reference[:, :, None] * torch.stack([vr] * 2, -1)[:, None]
            rd1 = 0
        else:
            ref = reference[:, :, None] * vr[:, None, :, None]
            ref = torch.cat([ref, torch.zeros_like(ref)], -1)
            rd1 = vid_num * query_num
        ref = ref[:, :, :L].reshape(vid_num * query_num, L, 2)
        row_video = torch.arange(vid_num, device=hs.device, dtype=torch.int32).repeat_interleave(query_num)
        lt = others.get("level_T")  # (a .get default would read the device tensor back even when level_T is given)
        T = tuple(int(x) for x in (lt if lt is not None else others["spatial_shapes"].tolist()))[:L]
        return hs.reshape(vid_num * query_num, -1), ref, rd1, row_video, T

    def forward(self, hs, reference, others, cap_tensor):
        hs_rows, ref, rd1, rv, T = self._rows_from_reference(hs, reference, others)
        seq = cap_tensor.long()
        n_steps = caption_steps(seq.detach().cpu())
        return self.decode_teacher_forced(hs_rows, ref, rd1, rv, others["memory"], others["mask_flatten"], T, seq,
                                          n_steps)

    def sample(self, hs, reference, others, opt={}):
        """opt: sample_max (1 greedy, 0 multinomial), temperature, generator (torch.Generator for the draws);
        beam_size is ignored, as in the reference (read at LSTM_DSA.py:124, never used)."""
        hs_rows, ref, rd1, rv, T = self._rows_from_reference(hs, reference, others)
        seq, lp = self.decode_greedy(hs_rows, ref, rd1, rv, others["memory"], others["mask_flatten"], T,
                                     sample_max=opt.get("sample_max", 1), temperature=opt.get("temperature", 1.0),
                                     generator=opt.get("generator"))
        if seq is None:
            return [], []
        return seq, lp
