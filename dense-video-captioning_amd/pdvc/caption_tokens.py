"""Caption tokens packed by validity: the vocabulary projection and log-softmax over the words the loss reads.

The reference's caption loss (LanguageModelCriterion, pdvc/CaptioningHead/LSTM_DSA.py:48-52) is
    -(sum_t logp[r, t, target_t] * mask[r, t]) / (sum_t mask[r, t] + 1e-6)
with mask = cap_mask[:, 1:]: positions past a caption's end token carry weight 0.  A batch of ragged captions decoded
to one width (the longest caption of the batch, or a capacity-padded stream's 30 tokens, pdvc/batch_layout.py)
spends most of its (rows x steps x vocab) logits on such positions.  Here the logit GEMM and the fused log-softmax +
target pick (csrc/logprob.hip) run over a buffer of `capacity` token rows holding the valid (row, step) positions in
row-major order; the picked log-probabilities are scattered back to (rows, steps), zeros elsewhere -- the loss
multiplies those by mask 0, so every loss and gradient is the unpacked one's (the masked positions' logits get no
gradient in either form).  Every step is a fixed-size device op (a prefix sum, an index copy, gathers), so the
packing is captured in the step graph and a new batch of the stream re-packs on replay; only the capacity is a host
fact (the batch's token count: the sum over its captions, known from the host copy of cap_mask).

`cap_prob_train` (the last decoder layer's full (rows, steps, vocab) log-probabilities, an output of PDVC.forward
that no loss reads, pdvc.py:388-410 in the reference) is not formed in the step: DeferredLogprobs keeps the dropped
hidden states and a copy of the logit layer's weights of this forward and materialises it on first access.
"""
import torch
import torch.nn.functional as F


def token_count(cap_mask_cpu, n_steps):
    """Loss-carrying tokens per decoder layer of a batch: sum over its captions of cap_mask[c, 1 : n_steps + 1]."""
    if n_steps <= 0:
        return 0
    return int(cap_mask_cpu[:, 1:n_steps + 1].sum())


def pack_tokens(valid, capacity):
    """valid (R, n) bool on the device -> (index, scatter): index (capacity,) int64, the flat (r * n + t) position of
    the k-th valid token (row-major), 0 past the last one; scatter (capacity,) int64, the same positions with R * n
    (a dump slot) past the last one.  Fixed shapes, no host read (graph-capturable); the caller guarantees
    valid.sum() <= capacity."""
    R, n = valid.shape
    flat = valid.reshape(-1)
    pos = torch.cumsum(flat.to(torch.int64), 0) - 1
    # (a token past the capacity would be dropped, never written out of bounds; callers size the capacity from the
    # host count, so none is)
    dest = torch.where(flat & (pos < capacity), pos, torch.full_like(pos, capacity))
    src = torch.arange(R * n, device=valid.device, dtype=torch.int64)
    index = torch.zeros(capacity + 1, dtype=torch.int64, device=valid.device).index_copy_(0, dest, src)[:capacity]
    count = flat.sum()
    live = torch.arange(capacity, device=valid.device) < count
    scatter = torch.where(live, index, torch.full_like(index, R * n))
    return index, scatter


class _PackRows(torch.autograd.Function):
    """x (N, H) -> x[index] (capacity, H); backward: the rows written back with index_copy through `scatter` (every
    live position once, the padding into a dump row) -- no float atomics (index_select's backward is an atomic
    index_add_)."""

    @staticmethod
    def forward(ctx, x, index, scatter):
        ctx.save_for_backward(scatter)
        ctx.n = x.shape[0]
        return x.index_select(0, index)

    @staticmethod
    def backward(ctx, g):
        (scatter,) = ctx.saved_tensors
        gx = g.new_zeros((ctx.n + 1, g.shape[1])).index_copy_(0, scatter, g)[:ctx.n]
        return gx, None, None


def pack_rows(x, tokens):
    """The packed token rows of x (N, H), N = rows * steps flattened row-major (pack_tokens' positions)."""
    return _PackRows.apply(x, tokens[0], tokens[1])


class DeferredLogprobs:
    """log_softmax(logit(Hd)) of a (rows, steps) selection, formed when first read.  Hd (R, n, H) are the hidden
    states after the caption dropout of the forward that made them; weight / bias a copy of the logit layer's
    parameters of that forward (so an optimizer step in between does not change the values)."""

    def __init__(self, Hd, weight, bias, rows=None, steps=None):
        self.Hd, self.weight, self.bias = Hd, weight, bias
        self.rows, self.steps = rows, steps
        self._value = None

    def select(self, rows=None, steps=None):
        """rows: (start, length) or an index tensor; steps: how many leading steps."""
        return DeferredLogprobs(self.Hd, self.weight, self.bias, rows, steps)

    def materialize(self):
        if self._value is None:
            h = self.Hd
            if isinstance(self.rows, tuple):
                h = h.narrow(0, self.rows[0], self.rows[1])
            elif self.rows is not None:
                h = h.index_select(0, self.rows)
            if self.steps is not None:
                h = h[:, :self.steps]
            with torch.no_grad():
                self._value = F.log_softmax(F.linear(h, self.weight, self.bias), dim=-1)
        return self._value


class RowSelect:
    """x.index_select(0, rows)[:, :steps], formed when first read (the last layer's rows of the caption log-probabilities:
    an output of the training forward that no loss reads -- a 1.3 GB copy per headline step when formed eagerly)."""

    def __init__(self, x, rows, steps):
        self.x, self.rows, self.steps = x, rows, steps
        self._value = None

    def materialize(self):
        if self._value is None:
            self._value = self.x.index_select(0, self.rows)[:, :self.steps]
        return self._value


class LazyProbs(dict):
    """The caption_probs dict of a step: a DeferredLogprobs / RowSelect value is materialised on access."""

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        return v.materialize() if isinstance(v, (DeferredLogprobs, RowSelect)) else v

    def get(self, k, default=None):
        return self[k] if k in self else default

    def values(self):
        return [self[k] for k in self.keys()]

    def items(self):
        return [(k, self[k]) for k in self.keys()]
