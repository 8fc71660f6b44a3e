"""GPU: the fused caption-step kernels against the float64 caption-step oracle at full size.

oracle/cap_step.py restates ShowAttendTellCore's soft attention over MSDeformAttnCap's border samples
(pdvc/CaptioningHead/LSTM_DSA.py:231-263, pdvc/ops/modules/ms_deform_attn_for_caption.py:78-123) in float64 on the
CPU, autograd supplying the backward, and is pinned to the reference captioner's fixtures (tests/test_oracle.py).
Here the product kernels run at the headline pyramid T_l = [512, 256, 128, 64] with 64 caption rows over 4 videos and
the 512-wide head every cfg uses:

  pdvc_cap_softattn_forward_f32   -> sampling locations, probabilities p, attended rows res
  pdvc_cap_softattn_backward_f32  -> the gradients of att (= dL/dU per sample), att_h, alpha_net, the sampling
                                     offsets and the reference points
  pdvc_cap_value_grad_rank1_f32   -> the value gradient of the p * dres samples;  pdvc_cap_value_grad_ranged_f32 on
                                     grad_att -> the gradient of the projected rows U = ctx2att(value)

and the value gradient of the reference's form (att = ctx2att(samples), samples of the masked value) must equal
rank1 + ranged(U) @ W_ctx.  Bound (tests/parity.py): every tensor within 1e-4 of its own max |ref|.
"""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from parity import assert_close  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


def cu(a, dtype=None):
    t = torch.as_tensor(np.asarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV).contiguous()


@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("masked", [False, True])
def test_cap_step_kernels_match_float64_oracle(ref_dim, masked):
    from oracle import cap_step as C
    from pdvc import _native as _n
    rng = np.random.RandomState(100 + 10 * ref_dim + masked)
    T_l = [512, 256, 128, 64]
    S, Nv, R, D, M = sum(T_l), 4, 64, 512, 1
    row_video = np.repeat(np.arange(Nv), R // Nv).astype(np.int32)
    value = rng.randn(Nv, S, M, D)
    mask = np.zeros((Nv, S), bool)
    if masked:  # padded tails of two videos' levels (the collate's padding, data/video_dataset.py:15-149)
        mask[1, 400:512] = True
        mask[1, 700:768] = True
        mask[3, 900:960] = True
    W_c = rng.uniform(-1, 1, size=(D, D)) / np.sqrt(D)
    b_c = rng.uniform(-0.1, 0.1, size=D)
    alpha_w = rng.randn(D) * 0.1
    alpha_b = rng.randn(1) * 0.1
    att_h = rng.randn(R, D) * 0.5
    off_h = rng.randn(R, 16) * 3.0
    off_e = rng.randn(R, 16) * 3.0
    if ref_dim == 1:
        ref = rng.uniform(-0.1, 1.1, size=(R, 4, 1))
        rd1 = 0
    else:
        ref = np.concatenate([rng.uniform(0, 1, size=(R, 4, 1)), rng.uniform(0.05, 0.9, size=(R, 4, 1))], -1)
        rd1 = 16  # the first video's rows: decoder layer 0's 1-d reference formula
    dres = rng.randn(R, D)

    # ---- the oracle (float64, CPU), the reference's form
    vt = C.to_f64(value, True)
    mt = torch.as_tensor(mask)
    offt = C.to_f64(off_h + off_e, True)
    reft = C.to_f64(ref, True)
    aht = C.to_f64(att_h, True)
    Wct, bct = C.to_f64(W_c, True), C.to_f64(b_c, True)
    awt, abt = C.to_f64(alpha_w, True), C.to_f64(alpha_b, True)
    loc = C.sampling_locations(offt, reft, T_l, M, 4, rd1_rows=rd1)
    smp = C.step_samples(vt, mt, torch.as_tensor(row_video), loc, T_l)
    att, p, res = C.soft_attention_step(smp, aht, Wct, bct, awt, abt)
    (res * C.to_f64(dres)).sum().backward()

    # ---- the product kernels (fp32, GPU)
    value_masked = np.where(mask[..., None, None], 0.0, value)
    U = value_masked @ W_c.T + b_c  # ctx2att of the masked value rows (what the decoder gathers)
    off_stride = 16 + 4 + D
    hp = np.zeros((R, off_stride))
    hp[:, :16] = off_h
    hp[:, 20:] = att_h
    vg, ug, hpg = cu(value, torch.float32), cu(U, torch.float32), cu(hp, torch.float32)
    maskg = cu(mask.astype(np.uint8)) if masked else None
    rvg, offe = cu(row_video), cu(off_e, torch.float32)
    refg = cu(ref, torch.float32)
    awg, abg = cu(alpha_w, torch.float32), cu(alpha_b, torch.float32)
    ah, ldh = _n.rows(hpg[:, 20:])
    lvl = _n.int_array(T_l)
    geo = (_n.ptr(rvg), _n.ptr(hpg), off_stride, 0, _n.ptr(offe), _n.ptr(refg), ref_dim, rd1, lvl, 4, Nv, R, M, D, 4)
    sloc, probs, resg = (torch.empty(R, M, 16, device=DEV), torch.empty(R, M, 16, device=DEV),
                         torch.empty(R, M * D, device=DEV))
    _n.call("pdvc_cap_softattn_forward_f32", _n.ptr(vg), _n.ptr(maskg), _n.ptr(ug), *geo, ah, ldh, _n.ptr(awg),
            _n.ptr(abg), None, _n.ptr(sloc), None, _n.ptr(probs), _n.ptr(resg), _n.stream())
    assert_close(sloc, loc.detach().reshape(R, M, 16).numpy(), "sampling locations", TOL)
    assert_close(probs, p.detach().numpy(), "probabilities", TOL)
    assert_close(resg, res.detach().numpy(), "attended rows", TOL)
    assert float(p.detach().max()) < 0.9, "the soft attention must not be degenerate"

    dresg = cu(dres, torch.float32)
    datt = torch.empty(R * M * 16, D, device=DEV)
    gaw, gab = torch.empty(R * M, D, device=DEV), torch.empty(R * M, device=DEV)
    dhp = torch.zeros(R, off_stride, device=DEV)
    gr = torch.zeros_like(refg)
    gah, ldgah = _n.rows(dhp[:, 20:])
    _n.call("pdvc_cap_softattn_backward_f32", _n.ptr(vg), _n.ptr(maskg), _n.ptr(ug), *geo, _n.ptr(sloc),
            _n.ptr(probs), _n.ptr(dresg), ah, ldh, _n.ptr(awg), _n.ptr(datt), gah, ldgah, None, _n.ptr(gaw),
            _n.ptr(gab), _n.ptr(dhp), _n.ptr(gr), _n.stream())
    # dL/datt in the oracle: the step again with att = ctx2att(samples) as the leaf
    dU_ref = _datt_reference(smp.detach(), aht.detach(), Wct.detach(), bct.detach(), awt.detach(), abt.detach(),
                             C.to_f64(dres))
    assert_close(datt.view(R, M, 16, D), dU_ref.numpy(), "grad att (dL/dU per sample)", TOL)
    assert_close(dhp[:, 20:], aht.grad.numpy(), "grad att_h", TOL)
    assert_close(gaw.sum(0), awt.grad.numpy(), "grad alpha_net.weight", TOL)
    # the alpha_net bias gradient is zero in exact arithmetic (a softmax is shift-invariant: sum_k dL/de_k = 0 per
    # row); bounded against the scale of its sibling, the alpha_net weight gradient
    assert_close(gab.sum(0, keepdim=True), abt.grad.numpy(), "grad alpha_net.bias", TOL,
                 scale=float(awt.grad.abs().max()))
    assert_close(dhp[:, :16], offt.grad.numpy(), "grad sampling offsets", TOL)
    assert_close(gr, reft.grad.numpy(), "grad reference points", TOL)

    # value gradient: rank-1 samples (p * dres) + the U rows' gradient through ctx2att
    order = np.argsort(row_video, kind="stable").astype(np.int32)
    starts = np.concatenate([[0], np.cumsum(np.bincount(row_video, minlength=Nv))]).astype(np.int32)
    vs, vr = cu(starts), cu(order)
    max_rows = int(np.bincount(row_video, minlength=Nv).max())
    gv = torch.empty(Nv, S, M, D, device=DEV)
    ls = torch.empty(Nv, 4, M * D, device=DEV)
    _n.call("pdvc_cap_value_grad_rank1_f32", _n.ptr(maskg), lvl, 4, Nv, M, D, 4, R, 1, max_rows, _n.ptr(vs),
            _n.ptr(vr), None, _n.ptr(sloc), _n.ptr(dresg), _n.ptr(probs), _n.ptr(gv), _n.ptr(ls), _n.stream())
    gU = torch.empty(Nv, S, M, D, device=DEV)
    lsU = torch.empty(Nv, 4, M * D, device=DEV)
    _n.call("pdvc_cap_value_grad_ranged_f32", None, lvl, 4, Nv, M, D, 4, R, 1, max_rows, _n.ptr(vs), _n.ptr(vr),
            None, _n.ptr(sloc), _n.ptr(datt), _n.ptr(gU), _n.ptr(lsU), _n.stream())
    gv_total = gv.double().cpu() + (gU.double().cpu() @ torch.as_tensor(W_c))
    if masked:  # U = ctx2att(masked value): its gradient reaches only the unmasked rows of the value
        gv_total[torch.as_tensor(mask)] = 0.0
    assert_close(gv_total, vt.grad.numpy(), "grad value (rank-1 samples + U rows through ctx2att)", TOL)
    gUc = gU.double().cpu().reshape(-1, D)
    assert_close(gUc.sum(0), bct.grad.numpy(), "grad ctx2att.bias (the U rows' gradient summed)", TOL)
    assert_close(gUc.t() @ torch.as_tensor(value_masked.reshape(-1, D)), Wct.grad.numpy(),
                 "grad ctx2att.weight (U rows' gradient against the masked value rows)", TOL)


def _datt_reference(smp, att_h, W_c, b_c, alpha_w, alpha_b, dres):
    """dL/d att for L = <dres, res>, att = ctx2att(samples): the oracle's step with att as the leaf."""
    R, M, K, D = smp.shape
    att = (smp @ W_c.t() + b_c).detach().requires_grad_(True)
    dot = torch.tanh(att + att_h.view(R, 1, 1, -1))
    e = dot @ alpha_w.view(-1) + alpha_b.view(())
    p = torch.softmax(e, dim=-1)
    res = (p[..., None] * smp).sum(2).reshape(R, M * D)
    (res * dres).sum().backward()
    return att.grad
