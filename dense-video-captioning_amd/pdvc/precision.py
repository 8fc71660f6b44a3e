"""The bf16 mode of the training step (BASELINE.json configs[1]: yc2_tsp_pdvc, "1 x MI355X bf16").

The reference computes in fp32 only (pdvc/ops/src/cuda/ms_deform_attn_cuda.cu:64,134 dispatch floating types;
every nn.Linear is fp32); the fp32 path stays the default and the parity-pinned one.  In the bf16 mode every
fp32 GEMM of the step -- forward projections, FFNs, LSTM gates, logits, and every input- and weight-gradient
GEMM autograd issues for them -- runs on the bf16 matrix cores: both operands are rounded to bf16 (one cast
pass each, ~0.13 ms per 126 M elements) and multiplied by hipBLASLt with fp32 accumulation and an fp32 RESULT
(aten mm/addmm/bmm/baddbmm .dtype overloads).  Everything else keeps fp32 storage: activations, the HIP kernels
(MSDA, caption gather, layer norms, attention), parameters, gradients and the optimizer state.

Measured on MI355X (tools/bf16_torch_probe.py), 245760 x 512 x 512: fp32 1.10 ms; bf16 0.25-0.31 ms + the
0.13 ms cast; logit / LSTM-gate shapes 591 / 1041 TFLOP/s against 132 / 147 in fp32.  (hipBLASLt's
HIPBLAS_COMPUTE_32F_FAST_16BF -- fp32 operands rounded inside the kernel -- ran 510-785 TFLOP/s with
/opt/rocm's library, tools/blaslt_probe.cpp, but the hipBLASLt that torch loads ships no such kernels for
gfx950, so the rounding is an explicit cast here.)

Mechanism: a TorchDispatchMode that reroutes aten mm / addmm / addmm_ / bmm / baddbmm / _addmm_activation
(and their out= forms) on fp32 GPU tensors; each operand's base tensor is rounded once and the rounding reused
by every GEMM that reads it (_bf).  The mode is thread-local state that autograd carries into its
backward threads, so the gradient GEMMs are rerouted too; inside a captured step graph the rerouting happens
once, at capture.  GEMMs below MIN_FLOPS (tiny heads, 1-wide projections) stay fp32: no time to win there.

    with bf16_matmul():
        out, loss = model(dt, criterion, "queries"); total.backward()

Tolerances against the fp32 path: tests/test_gpu_bf16.py and DESIGN.md.
"""
import contextlib
import os
import sys
import threading

import torch
from torch.utils._python_dispatch import TorchDispatchMode

aten = torch.ops.aten
MIN_FLOPS = 1 << 22
# GEMMs the mode saw: (op, M, N, K) -> [calls on the bf16 path, calls kept in fp32 (below MIN_FLOPS)]
STATS = {}
STATS_CAST = [0, 0, 0]  # [bf16 roundings made, reused from the cache, written by the producing kernel]
# PDVC_CAST_LOG=1 (diagnosis, tools/diag_bf16_casts.py): every rounding pass made, as (shape, where it was asked for)
CAST_LOG = [] if os.environ.get("PDVC_CAST_LOG") else None
_F32 = torch.float32
_BF = torch.bfloat16


_CAPTURE = [0]  # capture epoch: bumped by begin_capture() before every graph capture of the step


def begin_capture():
    """Start a new capture epoch: no rounding made before this point is reused inside the capture that follows.

    A rounding cached eagerly (StepGraph's warm-up steps run on the very `dt` tensors the capture then reads)
    would otherwise be a cache hit at capture time, so no cast kernel would be recorded, and every replay after
    `StepGraph.load(next batch)` would multiply the warm-up batch's bf16 features."""
    _CAPTURE[0] += 1


def _epoch():
    return _CAPTURE[0] if torch.cuda.is_current_stream_capturing() else 0


def _bf(t):
    """t rounded to bf16, the rounding cached on t's base tensor: a GEMM operand is usually a view (reshape,
    transpose, split-K chunks) of a tensor that several GEMMs read -- x in the forward product and again in the
    weight gradient, dy in the input- and weight-gradient products, a weight forward and backward -- so each
    base is rounded once.  The cache lives as long as the base (an attribute of it) and is dropped when the
    base's version counter moves (in-place updates, e.g. the optimizer's).  An entry is reused only in the
    epoch that made it: never across the boundary of a graph capture (eager entries inside a capture, or one
    capture's entries in another), so every captured GEMM operand's cast is itself a node of the graph."""
    base = t._base if t._base is not None else t
    if not base.is_contiguous() or base.is_leaf and base.requires_grad:  # parameters: small, updated in place
        return t.to(_BF)
    ent = base.__dict__.get("_pdvc_bf16")
    epoch = _epoch()
    if ent is None or ent[0] != base._version or ent[2] != epoch:
        ent = (base._version, base.to(_BF), epoch)
        base.__dict__["_pdvc_bf16"] = ent
        STATS_CAST[0] += 1
        if CAST_LOG is not None:
            CAST_LOG.append((tuple(base.shape), _origin()))
    else:
        STATS_CAST[1] += 1
    return ent[1].as_strided(t.shape, t.stride(), t.storage_offset() - base.storage_offset())


def _origin():
    """The innermost caller outside this module and torch (file:line function), or "autograd" for a GEMM issued by
    a built-in backward formula (no Python frame of ours on the stack)."""
    f = sys._getframe(2)
    while f is not None:
        fn = f.f_code.co_filename
        if fn != __file__ and "/torch/" not in fn:
            return f"{os.path.basename(fn)}:{f.f_lineno} {f.f_code.co_name}"
        f = f.f_back
    return "autograd"


def _f32_cuda(*ts):
    return all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == _F32 for t in ts)


def _mnk(a, b):
    return a.shape[-2], b.shape[-1], a.shape[-1]


def _big(a, b):
    M, N, K = _mnk(a, b)
    batch = a.shape[0] if a.dim() == 3 else 1
    return 2 * M * N * K * batch >= MIN_FLOPS


class BF16Matmul(TorchDispatchMode):
    """fp32 GPU GEMMs -> bf16 operands, fp32 accumulation and result (see the module docstring)."""

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        r = NotImplemented if getattr(_FP32, "depth", 0) else self._route(func, args, kwargs)
        return func(*args, **kwargs) if r is NotImplemented else r

    @staticmethod
    def _count(key, routed):
        s = STATS.setdefault(key, [0, 0])
        s[0 if routed else 1] += 1
        return routed

    def _route(self, func, args, kw):
        if func in (aten.mm.default, aten.mm.out):
            a, b = args[:2]
            if not (_f32_cuda(a, b) and self._count(("mm",) + _mnk(a, b), _big(a, b))):
                return NotImplemented
            if func is aten.mm.out:
                return aten.mm.dtype_out(_bf(a), _bf(b), _F32, out=kw["out"])
            return aten.mm.dtype(_bf(a), _bf(b), _F32)
        if func in (aten.addmm.default, aten.addmm.out, aten.addmm_.default, aten._addmm_activation.default):
            inp, a, b = args[:3]
            if not (_f32_cuda(inp, a, b) and self._count(("addmm",) + _mnk(a, b), _big(a, b))):
                return NotImplemented
            if func is aten._addmm_activation.default and kw.get("use_gelu", False):
                return NotImplemented
            beta, alpha = kw.get("beta", 1), kw.get("alpha", 1)
            if func is aten.addmm_.default:
                return aten.addmm.dtype_out(inp, _bf(a), _bf(b), _F32, beta=beta, alpha=alpha, out=inp)
            if func is aten.addmm.out:
                return aten.addmm.dtype_out(inp, _bf(a), _bf(b), _F32, beta=beta, alpha=alpha, out=kw["out"])
            y = aten.addmm.dtype(inp, _bf(a), _bf(b), _F32, beta=beta, alpha=alpha)
            return y.relu_() if func is aten._addmm_activation.default else y
        if func in (aten.bmm.default, aten.baddbmm.default):
            if func is aten.bmm.default:
                a, b = args[:2]
                ok = _f32_cuda(a, b)
            else:
                inp, a, b = args[:3]
                ok = _f32_cuda(inp, a, b)
            if not (ok and self._count(("bmm",) + _mnk(a, b) + (a.shape[0],), _big(a, b))):
                return NotImplemented
            if func is aten.bmm.default:
                return aten.bmm.dtype(_bf(a), _bf(b), _F32)
            return aten.baddbmm.dtype(inp, _bf(a), _bf(b), _F32, beta=kw.get("beta", 1), alpha=kw.get("alpha", 1))
        return NotImplemented


@contextlib.contextmanager
def bf16_matmul(enabled=True):
    """Route the fp32 GEMMs issued inside the block (and by the backward passes it starts) to bf16 MFMA."""
    if not enabled:
        yield
        return
    with BF16Matmul():
        yield


_FP32 = threading.local()  # depth > 0 inside fp32_gemms() on this thread: BF16Matmul passes every op through


@contextlib.contextmanager
def fp32_gemms():
    """GEMMs issued inside stay fp32 even under bf16_matmul: for the caption recurrence, whose per-step GEMMs
    feed the next step (bf16 rounding there compounds over the steps) and are small, latency-bound launches
    with little to win.  Only this module's routing is switched off: other dispatch modes (bench.py's GEMM flop
    count) keep seeing the ops (disabling every mode hid the recurrence's GEMMs from the count)."""
    _FP32.depth = getattr(_FP32, "depth", 0) + 1
    try:
        yield
    finally:
        _FP32.depth -= 1


def routed_summary():
    """(GEMM calls on the bf16 path, calls kept fp32) over everything the mode saw."""
    return sum(v[0] for v in STATS.values()), sum(v[1] for v in STATS.values())


def bf16_active():
    """True inside bf16_matmul (on this thread or an autograd thread it carried the mode into): producing kernels
    then also write the bf16 rounding of their output (attach_bf16), so the GEMM that reads it needs no cast."""
    if getattr(_FP32, "depth", 0):
        return False
    from torch.utils._python_dispatch import _get_current_dispatch_mode_stack
    return any(isinstance(m, BF16Matmul) for m in _get_current_dispatch_mode_stack())


SHADOWS = [True]  # the producing kernels write the bf16 operands (False: every operand is a cast pass; tests)


def shadow_for(t):
    """A bf16 buffer of t's shape for the kernel producing t to write t's rounding into (then attach_bf16(t, it)),
    or None outside the bf16 mode."""
    if not (SHADOWS[0] and t.is_cuda and bf16_active()):
        return None
    return torch.empty(t.shape, dtype=_BF, device=t.device)


def attach_bf16(t, t16):
    """Register t16 (t rounded to bf16, written by the kernel that produced t) as t's cached rounding: _bf finds it
    exactly as if it had cast t itself (same version, same capture epoch), so no cast kernel runs."""
    if t16 is None:
        return t
    base = t._base if t._base is not None else t
    if base is t and t.is_contiguous() and t16.shape == t.shape:
        t.__dict__["_pdvc_bf16"] = (t._version, t16, _epoch())
        STATS_CAST[2] += 1
    return t


def drop_cast_cache(tensors):
    """Forget the cached bf16 roundings of these tensors (their bases)."""
    for t in tensors:
        base = t._base if t._base is not None else t
        base.__dict__.pop("_pdvc_bf16", None)
