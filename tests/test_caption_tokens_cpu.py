"""CPU: the caption-token packing of the logit projection (pdvc/caption_tokens.py).  pack_tokens lists the valid
(row, step) positions row-major and routes everything past the last one to a dump slot; the packed loss path --
gather the valid rows, log-softmax, pick the target, scatter back to (rows, steps) -- gives the unpacked loss and
gradients exactly (the loss multiplies the other positions by 0); LazyProbs materialises a deferred value on read."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dense-video-captioning_amd"))
from pdvc.caption_tokens import DeferredLogprobs, LazyProbs, pack_rows, pack_tokens, token_count  # noqa: E402


def _mask(R, n, g):
    lens = torch.randint(0, n + 1, (R,), generator=g)
    return torch.arange(n)[None, :] < lens[:, None]


def test_pack_tokens_lists_valid_positions():
    g = torch.Generator().manual_seed(0)
    R, n = 37, 9
    valid = _mask(R, n, g)
    valid[5, 3] = False  # a hole: the packing does not assume prefixes
    cap = int(valid.sum()) + 11
    index, scatter = pack_tokens(valid, cap)
    want = torch.nonzero(valid.reshape(-1)).view(-1)
    k = want.numel()
    assert torch.equal(index[:k], want)
    assert torch.equal(scatter[:k], want)
    assert torch.all(index[k:] == 0) and torch.all(scatter[k:] == R * n)


def test_pack_tokens_drops_overflow_instead_of_writing_out_of_bounds():
    valid = torch.ones(4, 5, dtype=torch.bool)
    index, scatter = pack_tokens(valid, 7)
    assert torch.equal(index, torch.arange(7))
    assert index.shape == (7,)


def _loss(picked, mask):
    return (-(picked * mask).sum(1) / (mask.sum(1) + 1e-6)).sum()


def test_packed_loss_equals_unpacked():
    g = torch.Generator().manual_seed(1)
    R, n, H, V = 23, 7, 16, 31
    valid = _mask(R, n, g)
    Hd = torch.randn(R, n, H, generator=g, dtype=torch.float64, requires_grad=True)
    W = torch.randn(V, H, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(V, generator=g, dtype=torch.float64, requires_grad=True)
    tgt = torch.randint(0, V, (R, n), generator=g)
    m = valid.double()
    lp = F.log_softmax(F.linear(Hd, W, b), -1)
    ref = _loss(lp.gather(2, tgt[..., None]).squeeze(2), m)
    gref = torch.autograd.grad(ref, (Hd, W, b))
    index, scatter = pack_tokens(valid, int(valid.sum()) + 5)
    Hp = pack_rows(Hd.reshape(R * n, H), (index, scatter))
    lpp = F.log_softmax(F.linear(Hp, W, b), -1)
    pk = lpp.gather(1, tgt.reshape(-1).index_select(0, index)[:, None]).squeeze(1)
    picked = Hp.new_zeros(R * n + 1).index_copy(0, scatter, pk)[:R * n].view(R, n)
    got = _loss(picked, m)
    ggot = torch.autograd.grad(got, (Hd, W, b))
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)
    for a, e in zip(ggot, gref):
        torch.testing.assert_close(a, e, rtol=1e-12, atol=1e-12)


def test_token_count_and_lazy_probs():
    mask = torch.tensor([[1, 1, 1, 0], [1, 1, 0, 0], [0, 0, 0, 0]], dtype=torch.bool)
    assert token_count(mask, 3) == 3 and token_count(mask, 1) == 2 and token_count(mask, 0) == 0
    g = torch.Generator().manual_seed(2)
    Hd = torch.randn(6, 4, 8, generator=g)
    W, b = torch.randn(5, 8, generator=g), torch.randn(5, generator=g)
    d = DeferredLogprobs(Hd, W, b)
    full = F.log_softmax(F.linear(Hd, W, b), -1)
    probs = LazyProbs(cap_prob_train=d.select((2, 3), 2), other=1)
    torch.testing.assert_close(probs["cap_prob_train"], full[2:5, :2])
    torch.testing.assert_close(dict(probs.items())["cap_prob_train"], full[2:5, :2])
    assert probs.get("other") == 1
    sel = torch.tensor([5, 0])
    torch.testing.assert_close(LazyProbs(x=d.select(sel, 3))["x"], full[sel][:, :3])


def test_word_gates_backward_over_listed_positions():
    """_WordGates: W_x embed(idx) with its backward restricted to the listed positions equals the full autograd
    backward when the gate gradient is zero everywhere else (padding entries of the list contribute nothing)."""
    from pdvc.CaptioningHead.LSTM_DSA import _WordGates
    g = torch.Generator().manual_seed(5)
    n, R, V, E, G = 6, 9, 13, 8, 12
    idx = torch.randint(0, V, (n, R), generator=g)
    idx[0] = 0  # every row starts at token 0, as the captions do
    weight = torch.randn(V, E, generator=g, dtype=torch.float64, requires_grad=True)
    W = torch.randn(G, E, generator=g, dtype=torch.float64, requires_grad=True)
    keep = torch.rand(n, R, generator=g) < 0.5
    up = torch.randn(n, R, G, generator=g, dtype=torch.float64) * keep[..., None]
    ref = torch.autograd.grad((F.linear(weight[idx], W) * up).sum(), (weight, W))
    act = torch.nonzero(keep.reshape(-1)).view(-1)
    act = torch.cat([act, torch.full((5,), n * R)])  # capacity padding
    out = _WordGates.apply(weight, W, idx, act)
    torch.testing.assert_close(out, F.linear(weight[idx], W))
    got = torch.autograd.grad((out * up).sum(), (weight, W))
    for a, e in zip(got, ref):
        torch.testing.assert_close(a, e, rtol=1e-12, atol=1e-12)
