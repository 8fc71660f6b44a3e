"""fp32 matrix products on the gfx950 matrix cores (csrc/gemm.hip, pdvc_gemm_f32) and nn.Linear on them.

`matmul(a, b)` takes op(A) (M,K) and op(B) (K,N) as logical 2-D views and passes their storage order to the
kernel (a row-major or a transposed view of row-major memory both go without a copy).  LinearFunction is
nn.Linear's forward/backward (y = x W^T + b; dx = dy W; dW = dy^T x split over the rows with atomics;
db = sum dy) -- the projections of MSDeformAttn and the FFNs."""
import os

import torch
import torch.nn.functional as F
from torch.autograd import Function

from pdvc import _native as _n
from .gemm3 import addmm_nt, mm_dgrad

CU = 256  # MI355X compute units
# "hip": the projections run on pdvc_gemm_f32; "torch": F.linear (hipBLASLt) -- an A/B switch for bench.py
BACKEND = os.environ.get("PDVC_GEMM", "torch")


def _operand(t):
    """(tensor, transposed flag, leading dimension) for a logical 2-D operand."""
    if t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t, 0, max(t.stride(0), 1)
    if t.stride(0) == 1 and t.stride(1) >= t.shape[0]:
        return t, 1, max(t.stride(1), 1)
    t = t.contiguous()
    return t, 0, max(t.stride(0), 1)


def _split_k(M, N, K):
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    if tiles >= CU or K < 1024:
        return 1
    return max(1, min(2 * CU // tiles, K // 512))


def matmul(a, b, bias=None, relu=False, out=None, accumulate=False):
    """op(a) (M,K) @ op(b) (K,N) (+ bias) (ReLU) -> (M,N) fp32.  accumulate=True adds into `out` (split-K)."""
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("pdvc matmul is fp32")
    M, K = a.shape
    K2, N = b.shape
    if K != K2:
        raise ValueError(f"inner dimensions differ: {tuple(a.shape)} @ {tuple(b.shape)}")
    a, ta, lda = _operand(a)
    b, tb, ldb = _operand(b)
    if accumulate:
        if out is None or bias is not None or relu:
            raise ValueError("accumulate needs `out` and no epilogue")
        epi, split = 3, _split_k(M, N, K)
    else:
        epi = 0 if bias is None else (2 if relu else 1)
        split = 1
        if out is None:
            out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    if bias is not None:
        bias = bias.contiguous()
    if out.stride(1) != 1:
        raise ValueError("out must have unit column stride")
    _n.call("pdvc_gemm_f32", M, N, K, _n.ptr_any(a), lda, ta, _n.ptr_any(b), ldb, tb, _n.ptr_any(out), out.stride(0),
            _n.ptr(bias), epi, split, _n.stream())
    return out


class LinearFunction(Function):
    """y = x W^T + b (ReLU fused when relu=True: the backward masks dy with y > 0)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu=False):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        y = matmul(x2, weight.t(), bias=bias, relu=relu)
        ctx.save_for_backward(x2, weight, y if relu else None)
        ctx.has_bias = bias is not None
        return y.view(*shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, weight, y = ctx.saved_tensors
        gy2 = gy.reshape(-1, weight.shape[0])
        if y is not None:
            gy2 = gy2 * (y > 0)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = matmul(gy2, weight).view(*gy.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            gw = torch.zeros_like(weight)
            matmul(gy2.t(), x2, out=gw, accumulate=True)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy2.sum(0)
        return gx, gw, gb, None


def linear(x, weight, bias=None, relu=False):
    return LinearFunction.apply(x, weight, bias, relu)


# dense(..., relu=True) asks hipBLASLt for the ReLU epilogue instead of a separate pass (same-box A/B 3277 -> 3292
# videos/s); PDVC_RELU_EPILOGUE=0 keeps addmm + relu_
_RELU_EPILOGUE = os.environ.get("PDVC_RELU_EPILOGUE", "1") != "0"


def wgrad_splits(rows):
    """K-chunks for a weight gradient over `rows` rows: hipBLASLt runs dW = dy^T x (512 x 512 outputs, K = N*S
    = 30720) on 128 workgroups at ~70 TF/s; as a batched GEMM over 16 row chunks plus a sum it fills the
    chip at ~135 TF/s (tools/gemmbench.py on MI355X).  1 = a plain GEMM."""
    for s in (64, 32, 16, 8, 4, 2):  # 245760 rows (256 videos): 64 chunks, 146 TF/s (tools/gemm_large.py)
        if rows % s == 0 and rows // s >= 1536:
            return s
    return 1


def colsum(x, out=None):
    """x.sum(0) for a 2-D fp32 GPU tensor: pdvc_colsum_f32 (csrc/colsum.hip) when the rows are long and
    16-byte aligned, else torch.  The bias gradient of every projection.  out: a contiguous (cols,) destination."""
    rows, cols = x.shape
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and cols % 4 == 0 and rows >= 512
            and x.data_ptr() % 16 == 0):
        return x.sum(0) if out is None else torch.sum(x, 0, out=out)
    cblocks = (cols // 4 + 15) // 16
    parts = max(1, min(256, (8 * CU) // cblocks, rows // 64))  # >= 8 workgroups per CU on wide gradients
    ws = torch.empty(parts * cols, dtype=x.dtype, device=x.device)
    if out is None:
        out = torch.empty(cols, dtype=x.dtype, device=x.device)
    _n.call("pdvc_colsum_f32", _n.ptr(x), rows, cols, parts, _n.ptr(ws), _n.ptr(out), _n.stream())
    return out


class AddRowBias(Function):
    """x + bias broadcast over the rows of x (..., C); the bias gradient is a column sum (colsum) instead of
    torch's generic reduction over the broadcast dims (e.g. the transformer's level embedding added to each
    level's positional rows, deformable_transformer.py:110 in the reference)."""

    @staticmethod
    def forward(ctx, x, bias):
        ctx.C = bias.numel()
        return x + bias.view(*([1] * (x.dim() - 1)), -1)

    @staticmethod
    def backward(ctx, dy):
        gb = colsum(dy.reshape(-1, ctx.C).contiguous()) if ctx.needs_input_grad[1] else None
        return dy, gb


def add_row_bias(x, bias):
    return AddRowBias.apply(x, bias)


class ExpandRowsFunction(Function):
    """t (Q, C) broadcast to (bs, Q, C) -- the decoder's query embedding and target rows, the same for every video
    (deformable_transformer.py:186-188 in the reference: query_embed.unsqueeze(0).expand(bs, -1, -1)).  Forward is
    torch's expand (a view); the backward sums the bs gradient slices as one column sum over the (bs, Q*C) view
    (colsum) instead of torch's reduction over the batch dimension."""

    @staticmethod
    def forward(ctx, t, bs):
        ctx.shape = t.shape
        return t.unsqueeze(0).expand(bs, *t.shape)

    @staticmethod
    def backward(ctx, g):
        return colsum(g.reshape(g.shape[0], -1).contiguous()).view(ctx.shape), None


def expand_rows(t, bs):
    """t.unsqueeze(0).expand(bs, ...) with a column-sum backward (ExpandRowsFunction) for fp32 GPU rows."""
    if not (t.is_cuda and t.dtype == torch.float32 and t.requires_grad and _EXPAND_COLSUM):
        return t.unsqueeze(0).expand(bs, *t.shape)
    return ExpandRowsFunction.apply(t, bs)


_EXPAND_COLSUM = os.environ.get("PDVC_EXPAND_COLSUM", "1") != "0"  # A/B switch


def wgrad_mm(gy, x, out=None, db=None):
    """gy^T x for row-major gy (rows, O) and x (rows, I): the weight-gradient product, split over K.  out: a
    contiguous (O, I) destination (a row block of a packed weight's gradient).  db: an (O,) destination for the
    bias gradient gy.sum(0) -- taken by gemm3w from the gy rows it loads when the layout allows (wgrad_bias_ok),
    else a colsum pass."""
    rows = gy.shape[0]
    if gy.shape[1] == 1:  # a 1-wide layer: a weighted column sum, not an (M = 1) GEMM (~1 TB/s on hipBLASLt)
        r = colsum((x * gy).contiguous()).view(1, -1)
        if db is not None:
            colsum(gy, out=db)
        return r if out is None else out.copy_(r)
    from .gemm3 import mm_wgrad, wgrad_bias_ok
    fuse = db is not None and wgrad_bias_ok(gy, x, db)
    r = mm_wgrad(gy, x, out, db if fuse else None)  # fp32 on the bf16 matrix cores when the shape allows it
    if r is not None:
        if db is not None and not fuse:
            colsum(gy, out=db)
        return r
    if db is not None:
        colsum(gy, out=db)
    s = wgrad_splits(rows)
    if s == 1:
        return torch.mm(gy.t(), x) if out is None else torch.mm(gy.t(), x, out=out)
    p = torch.bmm(gy.reshape(s, rows // s, gy.shape[1]).transpose(1, 2), x.reshape(s, rows // s, x.shape[1]))
    return p.sum(0) if out is None else torch.sum(p, 0, out=out)


class PackedLinearFunction(Function):
    """Row blocks of ONE packed nn.Linear weight applied to different inputs, y_i = x_i W[r_i:r_i+1]^T + b[...]:
    nn.MultiheadAttention's in_proj over the (query | key) input and the value input (torch's MHA slices
    in_proj_weight the same way).  The blocks' weight and bias gradients are written into one packed gradient
    (GEMM / column-sum out= views), where per-slice autograd built a zero-filled full-size gradient, copied the
    block in and added the others (SliceBackward: a fill, a copy and an add per slice and step)."""

    @staticmethod
    def forward(ctx, weight, bias, rows, *xs):
        outs = []
        r0 = 0
        for x, r in zip(xs, rows):
            x2 = x.reshape(-1, x.shape[-1])
            y = addmm_nt(bias[r0:r0 + r], x2, weight[r0:r0 + r])
            outs.append(y.view(*x.shape[:-1], r))
            r0 += r
        ctx.rows = rows
        ctx.shapes = [x.shape for x in xs]
        ctx.save_for_backward(weight, *[x.reshape(-1, x.shape[-1]) for x in xs])
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gys):
        weight, *x2s = ctx.saved_tensors
        gw = torch.zeros_like(weight) if any(g is None for g in gys) else torch.empty_like(weight)
        gb = weight.new_zeros(weight.shape[0]) if any(g is None for g in gys) else weight.new_empty(weight.shape[0])
        gxs = []
        r0 = 0
        for g, x2, r, shp in zip(gys, x2s, ctx.rows, ctx.shapes):
            if g is None:
                gxs.append(None)
                r0 += r
                continue
            g2 = g.reshape(-1, r).contiguous()
            w = weight[r0:r0 + r]
            gxs.append(mm_dgrad(g2, w).view(shp) if ctx.needs_input_grad[3 + len(gxs)] else None)
            wgrad_mm(g2, x2, out=gw[r0:r0 + r], db=gb[r0:r0 + r])
            r0 += r
        return (gw, gb, None) + tuple(gxs)


def tag_relu_masked(g, y):
    """Mark g (a gradient w.r.t. the ReLU output y) as already masked by y > 0 -- the data-gradient GEMM that made it
    applied the mask in its epilogue -- so y's producer skips its threshold_backward pass.  Tagged with g's version
    counter like tag_level_sums: a gradient autograd later accumulates into in place loses the tag."""
    g._pdvc_relu_masked = (y, g._version)
    return g


def relu_masked(g, y):
    """Whether g carries tag_relu_masked for exactly this ReLU output y and is unchanged since."""
    ent = getattr(g, "_pdvc_relu_masked", None)
    return (ent is not None and ent[1] == g._version and ent[0].data_ptr() == y.data_ptr()
            and ent[0].shape == y.shape and g.shape[-1] == y.shape[-1])


# the box MLP's ReLU backward in the next layer's data-gradient epilogue (pdvc_gemm3p_dmask_f32 with p = 0: hd > 0 ?
# g : 0, bit for bit threshold_backward) instead of a pass over (rows, O); PDVC_RELU_DMASK=0 is the A/B switch
_RELU_DMASK = os.environ.get("PDVC_RELU_DMASK", "1") != "0"


class TorchLinearFunction(Function):
    """nn.Linear (+ fused ReLU) on hipBLASLt with a split-K weight gradient (see wgrad_splits)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu=False):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        # a strided weight view (the caption LSTM's word part W_ih[:, :E]) as a contiguous copy: the in-tree GEMMs
        # take row-major operands (a 2048 x 512 copy against a 114688-row product)
        weight = weight if weight.is_contiguous() else weight.contiguous()
        if relu and bias is not None and _RELU_EPILOGUE:
            y = addmm_nt(bias, x2, weight, relu=True)  # ReLU in the GEMM epilogue
        else:
            y = addmm_nt(bias, x2, weight)
            if relu:
                y.relu_()
        # x is the output of another ReLU layer of this kind: the input gradient can be masked in its GEMM epilogue
        relu_in = x.__dict__.get("_pdvc_relu_out")
        ctx.save_for_backward(x2, weight, y if relu else None, relu_in)
        ctx.has_bias = bias is not None
        out = y.view(*shape[:-1], weight.shape[0])
        if relu:
            out.__dict__["_pdvc_relu_out"] = y  # (the saved y: its backward checks the tag against it)
        return out

    @staticmethod
    def backward(ctx, gy):
        x2, weight, y, relu_in = ctx.saved_tensors
        O = weight.shape[0]
        gy2 = gy.reshape(-1, O)
        if y is not None and not relu_masked(gy, y):
            gy2 = torch.ops.aten.threshold_backward(gy2, y, 0.0)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = None
            if _RELU_DMASK and relu_in is not None and relu_in.shape == (gy2.shape[0], weight.shape[1]):
                from .gemm3 import mm_dgrad_dmask
                gx = mm_dgrad_dmask(gy2.contiguous(), weight, relu_in, 0.0)
                if gx is not None:
                    gx = tag_relu_masked(gx.view(*gy.shape[:-1], weight.shape[1]), relu_in)
            if gx is None:
                gx = mm_dgrad(gy2, weight).view(*gy.shape[:-1], weight.shape[1])
        want_gb = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            gb = gy2.new_empty(O) if want_gb else None
            gw = wgrad_mm(gy2, x2, db=gb)  # (the bias gradient from the same pass over gy)
        elif want_gb:
            gb = colsum(gy2.contiguous())
        return gx, gw, gb, None


def dense(x, weight, bias=None, relu=False):
    """nn.Linear (+ ReLU) on the backend selected by BACKEND (fp32 CUDA tensors only go to the HIP GEMM)."""
    if x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32:
        if BACKEND == "hip":
            return LinearFunction.apply(x, weight, bias, relu)
        return TorchLinearFunction.apply(x, weight, bias, relu)
    y = F.linear(x, weight, bias)
    return F.relu(y) if relu else y


LEVEL_SUM_USES = [0]  # bias gradients taken from a consumer's row sums (tests check the hand-over happens)


class MultiLinearFunction(Function):
    """Several nn.Linear layers applied to the same input x: (x W_0^T + b_0, x W_1^T + b_1, ...).  Forward is
    one GEMM per layer; the backward accumulates the input gradient of all of them in the epilogues of their
    data-gradient GEMMs (beta = 1) instead of autograd adds over x's shape -- PDVC's encoder memory feeds the
    value projections of every decoder layer and of the caption head (deformable_transformer.py:260-262,
    ms_deform_attn_for_caption.py:70)."""

    @staticmethod
    def forward(ctx, x, *wb):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        ws, bs = wb[0::2], wb[1::2]
        outs = tuple(addmm_nt(b, x2, w).view(*shape[:-1], w.shape[0]) for w, b in zip(ws, bs))
        ctx.save_for_backward(x2, *ws)
        ctx.shape = shape
        return outs

    @staticmethod
    def backward(ctx, *grads):
        x2, *ws = ctx.saved_tensors
        gx = None
        gwb = []
        for g, w in zip(grads, ws):
            if g is None:
                gwb += [None, None]
                continue
            g2 = g.reshape(-1, w.shape[0]).contiguous()
            if gx is None:
                gx = mm_dgrad(g2, w)
            else:
                mm_dgrad(g2, w, out=gx)
            # a fused deformable-attention consumer hands its value gradient over with per-(video, level) row sums
            # (MSDA1dFunction): the bias gradient from those instead of another pass over g
            ls = level_sums_of(g)
            LEVEL_SUM_USES[0] += ls is not None
            if ls is not None and ls.shape[-1] == w.shape[0]:
                gwb += [wgrad_mm(g2, x2), ls.view(-1, ls.shape[-1]).sum(0)]
            else:
                gb = g2.new_empty(w.shape[0])
                gwb += [wgrad_mm(g2, x2, db=gb), gb]
        if gx is None:
            gx = torch.zeros_like(x2)
        return (gx.view(ctx.shape), *gwb)


def tag_level_sums(g, sums):
    """Hand a value gradient over to its projection's backward with its per-(video, level) row sums, tagged with
    the gradient's version counter: if autograd later accumulates a second consumer's gradient into g in place,
    the version moves and the sums are ignored."""
    g._pdvc_level_sums = (sums, g._version)
    return g


def level_sums_of(g):
    """The row sums tag_level_sums attached to g, or None when absent or stale (g modified since tagging)."""
    ent = getattr(g, "_pdvc_level_sums", None)
    if ent is None or ent[1] != g._version:
        return None
    return ent[0]


def multi_dense(x, layers):
    """[layer(x) for layer in layers] for nn.Linear-like layers (with biases) sharing the input x."""
    wb = []
    for layer in layers:
        wb += [layer.weight, layer.bias]
    return MultiLinearFunction.apply(x, *wb)
