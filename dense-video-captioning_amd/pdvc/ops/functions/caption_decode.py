"""The teacher-forced LSTM-DSA caption recurrence as ONE autograd function (forward and backward).

Reference: ShowAttendTellCore.forward (pdvc/CaptioningHead/LSTM_DSA.py:231-263) called once per token by
Captioner.forward (LSTM_DSA.py:55-109).  Per step and row (h, c start at zero):
    hp      = [W_off_h ; W_h2att ; W_hh] h_{t-1} + [0 ; b_h2att ; 0]            (one GEMM)
    clip    = border samples of value at  ref (+) (hp[:, :16] + off_hs)          (cap-gather kernel)
    att     = ctx2att(clip)                                                      (one GEMM, R*16 rows)
    res     = sum_j softmax_j(alpha_net(tanh(att_j + hp[:, h2att]))) clip_j      (soft-attention kernel)
    gates   = xe_t + W_att res + hp[:, W_hh] + W_hs hs                           (one GEMM + LSTM kernel)
    h, c    = LSTM cell(gates, c)
xe_t = W_x embed(token_t) (step-major, (n, R, 4H)), hs_g = W_hs hs and off_hs = W_off_hs hs + b_off are loop
invariants computed by the caller (with autograd); hs_g is the LSTM kernel's fourth addend, so the (R, n, 4H)
sum xe + hs_g is never formed, and xe's gradient is returned as a view of the step-major
gate gradients (no transposing copy).  Autograd of the stock modules issues ~25 kernels per step forward and ~50
backward; here it is 6 launches per step each way, and every weight gradient is ONE GEMM over all steps
after the backward loop (the per-step activations are kept: ~0.5 MB per row per step at PDVC's shape).
"""
import os

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from pdvc import _native as _n
from pdvc.precision import attach_bf16, bf16_active, fp32_gemms, shadow_for
from .gemm3 import addmm_nt, mm_dgrad
from .linear import colsum, tag_level_sums, wgrad_mm
from .ms_deform_attn_func import NUM_SAMPLES, _levels


# ctx2att of the samples as a gather of the once-projected value rows (see forward); False keeps the per-step GEMM
CTX2ATT_GATHER = True
U_GRAD = True  # the backward in the same form (see forward); False: dW_ctx and dclip from CLIP and dATT per sample
U_MAX_BYTES = 16 << 30  # largest projected-rows buffer of the gather form (bound its memory)
# In the bf16 mode (pdvc/precision.py) the recurrence's per-step GEMMs also run on bf16 operands with fp32 accumulation
# and fp32 results (round 4; PDVC_BF16_RECURRENCE=0 keeps them fp32, the earlier policy).  The step's inputs are
# rounded freshly each step (they are written by the HIP kernels, which the mode's per-tensor rounding cache cannot
# see) and the weights once per pass.
BF16_RECURRENCE = os.environ.get("PDVC_BF16_RECURRENCE", "1") != "0"
# a step's value and projected-row samples and its soft attention in one launch (pdvc_cap_softattn_forward_f32, the
# 512-wide head of every cfg); PDVC_CAP_FUSED=0: the three launches (gather, gather, soft attention)
CAP_FUSED = os.environ.get("PDVC_CAP_FUSED", "1") != "0"
# ... and its backward in one launch (pdvc_cap_softattn_backward_f32, U-gradient form), re-forming the samples and att
# from their corner rows: the forward then writes neither.  PDVC_CAP_FUSED_BWD=0: the two backward launches
CAP_FUSED_BWD = os.environ.get("PDVC_CAP_FUSED_BWD", "1") != "0"
# ... and the sample gradients it would write (p_k * dres, rank 1 per row) formed by the value-gradient pass from the
# per-step dres rows and the probabilities (pdvc_cap_value_grad_rank1_f32); PDVC_CAP_RANK1=0: written and read back
CAP_RANK1 = os.environ.get("PDVC_CAP_RANK1", "1") != "0"
_BF16 = torch.bfloat16


def _aligned16(*ptrs):
    """every pointer 16-B aligned (the fused step reads and writes its rows as float4s)"""
    return all((p.value or 0) % 16 == 0 for p in ptrs)


def _gemm(inp, a, b, out, b16):
    """out = inp + a @ b (inp None: a @ b), fp32 out; b16: a rounded to bf16 here, b already bf16.  inp is a bias
    vector or `out` itself (accumulate).  fp32: b = W^T (a weight's transposed view) or W -- the forward product and
    the input gradient of a projection -- on the split-bf16 GEMM (ops/functions/gemm3.py) where it takes the shape."""
    if b16 is None:
        if b.dim() == 2 and b.stride(0) == 1 and b.t().is_contiguous() and (inp is None or inp.dim() == 1):
            addmm_nt(inp, a, b.t(), out=out)
        elif b.is_contiguous() and (inp is None or inp is out):
            mm_dgrad(a, b, out=out, accumulate=inp is not None)
        elif inp is None:
            torch.mm(a, b, out=out)
        else:
            torch.addmm(inp, a, b, out=out)
    elif inp is None:
        torch.ops.aten.mm.dtype_out(a.to(_BF16), b16, torch.float32, out=out)
    else:
        torch.ops.aten.addmm.dtype_out(inp, a.to(_BF16), b16, torch.float32, out=out)


# the per-step gradients' sums over the steps as one contiguous reduction (PDVC_STEP_SUM_WHOLE=0: two strided ones, A/B)
_STEP_SUM_WHOLE = os.environ.get("PDVC_STEP_SUM_WHOLE", "1") != "0"
# bf16 mode: the caption dU written with its bf16 rounding by its value-gradient pass (PDVC_CAP_DU_SHADOW=0: cast, A/B)
_DU_SHADOW = os.environ.get("PDVC_CAP_DU_SHADOW", "1") != "0"

class CaptionDecodeFunction(Function):
    """value (Nv,S,M,D) = value_proj(memory); xe (n,R,4H); hs_g (R,4H); off_hs (R, M*16); ref (R,L,1|2) (first rd1_rows rows
    1-d when 2-wide); W_h (M*16 + A + 4H, H), b_h; W_ctx (A, D), b_ctx (A); alpha_w (A,), alpha_b (1,);
    W_att (4H, M*D); step_ranges (host per-step (start, count), device (n, 2) int32) or None.  Returns the hidden
    states (R, n, H) (zeros at the (row, step) pairs a range leaves out)."""

    @staticmethod
    def forward(ctx, value, xe, hs_g, off_hs, ref, W_h, b_h, W_ctx, b_ctx, alpha_w, alpha_b, W_att, pad_mask,
                row_video, level_T, rd1_rows, video_csr=None, heads=None, step_ranges=None):
        # value (Nv, S, M, D), or the projection's (Nv, S, M*D) output with `heads` = M: then the value gradient
        # goes back in that shape carrying its per-(video, level) row sums (`_pdvc_level_sums`, as MSDA1dFunction)
        # step_ranges: per step (start, count) -- the rows that step computes (rows ordered by their video's step
        # count, batch_layout.caption_layout(steps=...)); a row stops with its video's loop (LSTM_DSA.py:103-104).
        # The other (step, row) entries of HS, RES, dHP, GAW are zeros, so the all-step weight-gradient GEMMs and
        # sums below are exact; the other per-step buffers are never read there.
        ctx.flat_value = value.dim() == 3
        if ctx.flat_value:
            value = value.view(value.shape[0], value.shape[1], heads, -1)
        value, xe, off_hs, ref = value.contiguous(), xe.contiguous(), off_hs.contiguous(), ref.contiguous()
        hs_g = hs_g.contiguous()
        W_h, W_ctx, W_att = W_h.contiguous(), W_ctx.contiguous(), W_att.contiguous()
        alpha_w, alpha_b = alpha_w.contiguous(), alpha_b.contiguous()
        Nv, S, M, D = value.shape
        n, R, G = xe.shape
        H = G // 4
        ranged = step_ranges is not None
        # step_ranges = (host tuple of (start, count) per step, the same as a (n, 2) int32 device tensor): the device
        # copy is made once per batch by the caller, outside any captured graph
        ranges = tuple(tuple(r) for r in step_ranges[0]) if ranged else ((0, R),) * n
        if len(ranges) != n or any(s0 < 0 or c < 0 or s0 + c > R for s0, c in ranges):
            raise ValueError("caption decode: step_ranges must give one in-bounds (start, count) per step")
        # step t reads step t - 1's state (CS, HS) of each of its rows: every range must lie inside the previous one,
        # else a row entering late reads entries no step wrote
        if any(s1 < s0 or s1 + c1 > s0 + c0 for (s0, c0), (s1, c1) in zip(ranges, ranges[1:])):
            raise ValueError("caption decode: step_ranges must be nested (each step's rows inside the previous step's)")
        A = W_ctx.shape[0]
        NS = NUM_SAMPLES
        n_off = M * NS
        Ph = W_h.shape[0]
        if (Ph != n_off + A + G or W_att.shape != (G, M * D) or off_hs.shape != (R, n_off)
                or hs_g.shape != (R, G)):
            raise ValueError("caption decode: inconsistent weight shapes")
        RD = ref.shape[2]
        lvl, nl = _levels(level_T)
        kw = dict(dtype=value.dtype, device=value.device)
        HP = torch.empty((n, R, Ph), **kw)
        LOC = torch.empty((n, R, M, NS), **kw)
        PROBS = torch.empty((n, R, M, NS), **kw)
        RES = (torch.zeros if ranged else torch.empty)((n, R, M * D), **kw)
        ACTS = torch.empty((n, R, G), **kw)
        CS = torch.empty((n, R, H), **kw)
        HS = (torch.zeros if ranged else torch.empty)((R, n, H), **kw)
        GATT = torch.empty((R, G), **kw)
        zero = torch.zeros((R, H), **kw)
        st = _n.stream()
        # att = ctx2att(clip) is linear in the sample, and a sample is a blend of value rows with weights summing to
        # 1: project the value rows once (padded rows zeroed: their projection is the bias) and blend the projections
        # with the same gather -- U rows N*S instead of a (R*16) x D x A GEMM for each of n steps.  A loop invariant,
        # not part of the recurrence: in the bf16 mode it is a bf16 GEMM like the other projections.
        U = vm = None
        # the projected rows take Nv*S*M*A floats, A/D times the value's (8x at cap_nheads 8): the gather form only
        # while that stays within U_MAX_BYTES (the per-step GEMM needs no such buffer)
        u_bytes = 4 * Nv * S * M * A
        if (CTX2ATT_GATHER and 32 <= A <= 512 and A & (A - 1) == 0 and n * R * M * NS > Nv * S * M
                and u_bytes <= U_MAX_BYTES):
            vm = value if pad_mask is None else value.masked_fill(pad_mask.view(Nv, S, 1, 1).bool(), 0.0)
            U = addmm_nt(b_ctx, vm.view(-1, D), W_ctx).view(Nv, S, M, A)
        # the backward in the same form (U_GRAD): dATT is scattered onto the value rows once (dU), so dW_ctx = dU^T vm
        # and the value gradient's ctx2att part dU W_ctx are GEMMs over N*S rows instead of n*R*16, and the
        # location gradient of att is read off U at the sample corners (pdvc_cap_gather_backward2_f32)
        ctx.u_grad = U is not None and U_GRAD and A == D and video_csr is not None
        # one launch per step for the value and projected-row samples and the soft attention (512-wide heads)
        fused = (CAP_FUSED and U is not None and A == D == 512 and Ph % 4 == 0 and n_off % 4 == 0
                 and _aligned16(_n.ptr(value), _n.ptr(U), _n.ptr(HP), _n.ptr(alpha_w)))
        # ... and its backward: the samples and att are re-formed there, so they are neither written nor kept
        ctx.fused_bwd = fused and ctx.u_grad and CAP_FUSED_BWD
        keep = 0 if ctx.fused_bwd else n
        CLIP = torch.empty((keep, R, M, NS, D), **kw)
        ATT = torch.empty((keep, R * M * NS, A), **kw)
        if ranged and not ctx.u_grad:  # dW_ctx reads CLIP and dATT over every (step, row): no stale entries
            CLIP.zero_()
        ns_ = M * NS
        b16 = BF16_RECURRENCE and bf16_active()
        ctx.b16 = b16
        Wh16 = W_h.t().to(_BF16) if b16 else None
        Wctx16 = W_ctx.t().to(_BF16) if b16 else None
        Watt16 = W_att.t().to(_BF16) if b16 else None
        with fp32_gemms():  # the per-step GEMMs are routed here (_gemm), not by the mode
            for i in range(n):
                s0, c = ranges[i]
                if c == 0:
                    continue
                rs = slice(s0, s0 + c)
                rd1 = min(max(int(rd1_rows) - s0, 0), c)  # the range's rows with a 1-d reference
                hp = HP[i][rs]
                if i == 0:
                    hp.copy_(b_h.expand(c, Ph))  # h_{-1} = 0
                else:
                    _gemm(b_h, HS[rs, i - 1], W_h.t(), hp, Wh16)
                att = None if ctx.fused_bwd else ATT[i][s0 * ns_:(s0 + c) * ns_]
                ah, ldh = _n.rows(hp[:, n_off:n_off + A])
                if fused:  # the two gathers and the soft attention in one launch
                    _n.call("pdvc_cap_softattn_forward_f32", _n.ptr(value), _n.ptr(pad_mask), _n.ptr(U),
                            _n.ptr(row_video[rs]), _n.ptr(hp), Ph, 0, _n.ptr(off_hs[rs]), _n.ptr(ref[rs]), RD, rd1,
                            lvl, nl, Nv, c, M, D, NS // nl, ah, ldh, _n.ptr(alpha_w), _n.ptr(alpha_b),
                            None if ctx.fused_bwd else _n.ptr(CLIP[i][rs]), _n.ptr(LOC[i][rs]), _n.ptr(att),
                            _n.ptr(PROBS[i][rs]), _n.ptr(RES[i][rs]), st)
                else:
                    _n.call("pdvc_cap_gather_forward_f32", _n.ptr(value), _n.ptr(pad_mask), _n.ptr(row_video[rs]),
                            _n.ptr(hp), Ph, 0, _n.ptr(off_hs[rs]), _n.ptr(ref[rs]), RD, rd1, lvl, nl, Nv, c, M, D,
                            NS // nl, _n.ptr(CLIP[i][rs]), _n.ptr(LOC[i][rs]), st)
                    if U is not None:
                        _n.call("pdvc_cap_gather_forward_f32", _n.ptr(U), None, _n.ptr(row_video[rs]), _n.ptr(hp), Ph,
                                0, _n.ptr(off_hs[rs]), _n.ptr(ref[rs]), RD, rd1, lvl, nl, Nv, c, M, A, NS // nl,
                                _n.ptr(att), None, st)
                    else:
                        _gemm(b_ctx, CLIP[i][rs].reshape(-1, D), W_ctx.t(), att, Wctx16)
                    _n.call("pdvc_softattn_forward_f32", _n.ptr(att), ah, ldh, _n.ptr(alpha_w), _n.ptr(alpha_b),
                            _n.ptr(CLIP[i][rs]), c, M, A, D, _n.ptr(RES[i][rs]), _n.ptr(PROBS[i][rs]), st)
                _gemm(None, RES[i][rs], W_att.t(), GATT[:c], Watt16)
                xa, ldx = _n.rows(xe[i][rs])
                gh, ldg = _n.rows(hp[:, n_off + A:])
                ho, ldo = _n.rows(HS[rs, i])
                _n.call("pdvc_lstm_cell_forward_f32", xa, ldx, _n.ptr(GATT), G, gh, ldg, _n.ptr(hs_g[rs]), G,
                        _n.ptr(CS[i - 1][rs] if i > 0 else zero), c, H, ho, ldo, _n.ptr(CS[i][rs]),
                        _n.ptr(ACTS[i][rs]), st)
        ctx.save_for_backward(value, off_hs, ref, W_h, W_ctx, alpha_w, W_att, pad_mask, row_video, HP, CLIP, LOC,
                              ATT, PROBS, RES, ACTS, CS, HS, U if ctx.u_grad else None, vm if ctx.u_grad else None)
        ctx.meta = (tuple(level_T), int(rd1_rows), video_csr, ranges if ranged else None,
                    step_ranges[1] if ranged else None)
        return HS

    @staticmethod
    @once_differentiable
    def backward(ctx, dHS):
        (value, off_hs, ref, W_h, W_ctx, alpha_w, W_att, pad_mask, row_video, HP, CLIP, LOC, ATT, PROBS, RES, ACTS,
         CS, HS, U, vm) = ctx.saved_tensors
        u_grad = ctx.u_grad
        level_T, rd1_rows, video_csr, ranged, sr_dev = ctx.meta
        ranges = ranged if ranged is not None else ((0, HP.shape[1]),) * HP.shape[0]
        dHS = dHS.contiguous()
        Nv, S, M, D = value.shape
        n, R, Ph = HP.shape
        H = HS.shape[2]
        G = 4 * H
        A = W_ctx.shape[0]
        NS = NUM_SAMPLES
        n_off = M * NS
        RD = ref.shape[2]
        lvl, nl = _levels(level_T)
        kw = dict(dtype=value.dtype, device=value.device)
        alloc = torch.zeros if ranged is not None else torch.empty  # ranged: the skipped entries stay zero
        dHP = alloc((n, R, Ph), **kw)
        dATT = (alloc if not u_grad else torch.empty)((n, R * M * NS, A), **kw)
        GAW = alloc((n, R * M, A), **kw)
        GAB = alloc((n, R * M), **kw)
        # with the rows' per-video CSR, every step's sample gradient is kept and the value gradient is one
        # destination-sorted pass after the loop (pdvc_cap_value_grad_f32) instead of per-step atomics
        deferred = video_csr is not None
        # rank-1 sample gradients (fused backward, U-gradient form): the per-step dres rows are kept instead
        rank1 = ctx.fused_bwd and deferred and CAP_RANK1
        dCLIP_all = torch.empty((0 if rank1 else (n if deferred else 1), R, M, NS, D), **kw)
        dRES = torch.empty((R, M * D), **kw)
        dRES_all = torch.empty((n, R, M * D), **kw) if rank1 else None
        dh = torch.empty((R, H), **kw)
        dc = [alloc((R, H), **kw), alloc((R, H), **kw)]
        zero = torch.zeros((R, H), **kw)
        gv = torch.empty_like(value) if deferred else torch.zeros_like(value)
        gr = torch.zeros_like(ref) if ctx.needs_input_grad[3] else None
        st = _n.stream()
        ns_ = M * NS
        b16 = getattr(ctx, "b16", False)
        Watt16 = W_att.to(_BF16) if b16 else None
        Wh16 = W_h.to(_BF16) if b16 else None
        Wctx16 = W_ctx.to(_BF16) if b16 else None
        with fp32_gemms():  # the per-step GEMMs are routed here (_gemm), not by the mode
            for i in reversed(range(n)):
                s0, c = ranges[i]
                rs = slice(s0, s0 + c)
                rd1 = min(max(int(rd1_rows) - s0, 0), c)
                dCLIP = None if rank1 else dCLIP_all[i if deferred else 0][rs]
                if c > 0:
                    last = i == n - 1
                    dhp = dHP[i][rs]
                    gh_, ldgh = _n.rows(dHS[rs, i])
                    dg, lddg = _n.rows(dhp[:, n_off + A:])
                    _n.call("pdvc_lstm_cell_backward_f32", gh_, ldgh, None if last else _n.ptr(dh[rs]), H,
                            None if last else _n.ptr(dc[(i + 1) % 2][rs]), _n.ptr(ACTS[i][rs]),
                            _n.ptr(CS[i - 1][rs] if i > 0 else zero), _n.ptr(CS[i][rs]), c, H, dg, lddg,
                            _n.ptr(dc[i % 2][rs]), st)
                    dres = dRES_all[i][rs] if rank1 else dRES[:c]
                    _gemm(None, dhp[:, n_off + A:], W_att, dres, Watt16)
                    ah, ldh = _n.rows(HP[i][rs][:, n_off:n_off + A])
                    gah, ldgah = _n.rows(dhp[:, n_off:n_off + A])
                    datt = dATT[i][s0 * ns_:(s0 + c) * ns_]
                    gr_ = gr[rs] if gr is not None else None
                    if ctx.fused_bwd:  # the soft attention's and the sampling's backward in one launch
                        _n.call("pdvc_cap_softattn_backward_f32", _n.ptr(value), _n.ptr(pad_mask), _n.ptr(U),
                                _n.ptr(row_video[rs]), _n.ptr(HP[i][rs]), Ph, 0, _n.ptr(off_hs[rs]), _n.ptr(ref[rs]),
                                RD, rd1, lvl, nl, Nv, c, M, D, NS // nl, _n.ptr(LOC[i][rs]), _n.ptr(PROBS[i][rs]),
                                _n.ptr(dres), ah, ldh, _n.ptr(alpha_w), _n.ptr(datt), gah, ldgah, _n.ptr(dCLIP),
                                _n.ptr(GAW[i][s0 * M:(s0 + c) * M]), _n.ptr(GAB[i][s0 * M:(s0 + c) * M]), _n.ptr(dhp),
                                _n.ptr(gr_), st)
                    else:
                        att = ATT[i][s0 * ns_:(s0 + c) * ns_]
                        _n.call("pdvc_softattn_backward_f32", _n.ptr(att), ah, ldh, _n.ptr(alpha_w),
                                _n.ptr(CLIP[i][rs]), _n.ptr(PROBS[i][rs]), _n.ptr(dRES), c, M, A, D, _n.ptr(datt),
                                gah, ldgah, _n.ptr(dCLIP), _n.ptr(GAW[i][s0 * M:(s0 + c) * M]),
                                _n.ptr(GAB[i][s0 * M:(s0 + c) * M]), st)
                        if u_grad:  # dCLIP keeps the soft-attention part only; att's location gradient read off U
                            _n.call("pdvc_cap_gather_backward2_f32", _n.ptr(value), _n.ptr(pad_mask),
                                    _n.ptr(row_video[rs]), _n.ptr(HP[i][rs]), Ph, 0, _n.ptr(off_hs[rs]),
                                    _n.ptr(ref[rs]), RD, rd1, lvl, nl, Nv, c, M, D, NS // nl, _n.ptr(LOC[i][rs]),
                                    _n.ptr(dCLIP), None, _n.ptr(dhp), _n.ptr(gr_), _n.ptr(U), _n.ptr(datt), st)
                        else:
                            if b16:
                                dc_ = dCLIP.reshape(-1, D)
                                _gemm(dc_, datt, W_ctx, dc_, Wctx16)
                            else:
                                dCLIP.reshape(-1, D).addmm_(datt, W_ctx)
                            _n.call("pdvc_cap_gather_backward_f32", _n.ptr(value), _n.ptr(pad_mask),
                                    _n.ptr(row_video[rs]), _n.ptr(HP[i][rs]), Ph, 0, _n.ptr(off_hs[rs]),
                                    _n.ptr(ref[rs]), RD, rd1, lvl, nl, Nv, c, M, D, NS // nl, _n.ptr(LOC[i][rs]),
                                    _n.ptr(dCLIP), None if deferred else _n.ptr(gv), _n.ptr(dhp), _n.ptr(gr_),
                                    st)
                if i > 0:  # dh of step i - 1's rows (rows that stopped at step i have dHP[i] = 0 there)
                    p0, pc = ranges[i - 1]
                    if pc > 0:
                        _gemm(None, dHP[i][p0:p0 + pc], W_h, dh[p0:p0 + pc], Wh16)
        lsums = None
        if deferred:
            vr_start, vr_rows, max_rows = video_csr
            lsums = torch.empty(Nv, nl, M * D, dtype=gv.dtype, device=gv.device) if ctx.flat_value else None
            if rank1:
                _n.call("pdvc_cap_value_grad_rank1_f32", _n.ptr(pad_mask), lvl, nl, Nv, M, D, NS // nl, R, n,
                        int(max_rows), _n.ptr(vr_start), _n.ptr(vr_rows), _n.ptr(sr_dev), _n.ptr(LOC),
                        _n.ptr(dRES_all), _n.ptr(PROBS), _n.ptr(gv), _n.ptr(lsums), st)
            else:
                _n.call("pdvc_cap_value_grad_ranged_f32", _n.ptr(pad_mask), lvl, nl, Nv, M, D, NS // nl, R, n,
                        int(max_rows), _n.ptr(vr_start), _n.ptr(vr_rows), _n.ptr(sr_dev), _n.ptr(LOC),
                        _n.ptr(dCLIP_all), _n.ptr(gv), _n.ptr(lsums), st)
        # weight gradients: one GEMM each over every (step, row)
        d_gates = dHP[..., n_off + A:]                       # (n, R, 4H), row stride Ph: xe's gradient as is
        if _STEP_SUM_WHOLE:  # one reduction over the steps of the contiguous (n, R * Ph) buffer, both slices of it
            d_all = dHP.sum(0)
            d_hs_g, d_off_hs = d_all[:, n_off + A:], d_all[:, :n_off]
        else:  # two reductions over strided column slices (A/B)
            d_hs_g = d_gates.sum(0)
            d_off_hs = dHP[..., :n_off].sum(0)
        if n > 1:
            dW_h = wgrad_mm(dHP[1:].reshape(-1, Ph), HS[:, :-1].transpose(0, 1).reshape(-1, H))
        else:
            dW_h = torch.zeros_like(W_h)
        db_h = colsum(dHP.view(-1, Ph))
        if u_grad:
            # dU = dATT scattered onto the value rows with the sampling weights (no padding mask: U's padded rows are
            # the bias), with its per-(video, level) row sums
            dU = torch.empty((Nv, S, M, A), **kw)
            lsU = torch.empty((Nv, nl, M * A), **kw)
            dU16 = shadow_for(dU) if _DU_SHADOW else None  # bf16 mode: dU's two GEMMs' operand, from the same pass
            args = (None, lvl, nl, Nv, M, A, NS // nl, R, n, int(max_rows), _n.ptr(vr_start), _n.ptr(vr_rows),
                    _n.ptr(sr_dev), _n.ptr(LOC), _n.ptr(dATT), _n.ptr(dU), _n.ptr(lsU))
            if dU16 is None:
                _n.call("pdvc_cap_value_grad_ranged_f32", *args, st)
            else:
                _n.call("pdvc_cap_value_grad_ranged_f32_bf16out", *args, _n.ptr(dU16), st)
                attach_bf16(dU, dU16)
            dU2 = dU.view(-1, A)
            dW_ctx = wgrad_mm(dU2, vm.reshape(-1, D))
            db_ctx = lsU.view(-1, A).sum(0)  # the weights of a sample sum to 1: sum dU = sum dATT
            if pad_mask is None:
                mm_dgrad(dU2, W_ctx, out=gv.view(-1, D))
                if lsums is not None:  # the level sums of gv gain those of dU W_ctx
                    lsums.view(-1, D).addmm_(lsU.view(-1, A), W_ctx)
            else:  # vm = value with its padded rows zeroed: no gradient reaches them
                t = mm_dgrad(dU2, W_ctx).view(Nv, S, M, D)
                gv.add_(t.masked_fill_(pad_mask.view(Nv, S, 1, 1).bool(), 0.0))
                lsums = None  # (the consumer falls back to a column sum)
        else:
            dA2 = dATT.view(-1, A)
            db_ctx = dA2.new_empty(A)
            dW_ctx = wgrad_mm(dA2, CLIP.view(-1, D), db=db_ctx)
        dalpha_w = colsum(GAW.view(-1, A))
        dalpha_b = GAB.sum().reshape(1)
        dW_att = wgrad_mm(d_gates.reshape(-1, G), RES.view(-1, M * D))
        if ctx.flat_value:
            gv = gv.view(Nv, -1, M * D)
            if deferred and lsums is not None:
                tag_level_sums(gv, lsums)
        return (gv, d_gates, d_hs_g, d_off_hs, gr, dW_h, db_h, dW_ctx, db_ctx, dalpha_w, dalpha_b, dW_att, None, None,
                None, None, None, None, None)
