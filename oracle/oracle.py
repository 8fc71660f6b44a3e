"""ctypes/numpy front-end of the CPU MSDA oracle (oracle/msda_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the *checker*.  The product package never imports this module.

Functions mirror the reference operator signatures:
  msda_forward(value, shapes, lsi, loc, attn, pad)           ~ MSDA.ms_deform_attn_forward
        (pdvc/ops/src/vision.cpp:14, ms_deform_attn_cuda.cu:20-80) for pad='zeros';
        ~ ms_deform_attn_core_pytorch (ms_deform_attn_func.py:41-68) for pad='border'
  msda_backward(value, shapes, lsi, loc, attn, grad_out, pad) ~ MSDA.ms_deform_attn_backward
        (vision.cpp:15, ms_deform_attn_cuda.cu:83-153)
  msda_sample(value, shapes, lsi, loc, pad)                   ~ core(..., return_value=True)
  msda_sample_backward(value, shapes, lsi, loc, grad, pad)
All arrays are numpy; the dtype (float32 / float64) selects the C instantiation.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libmsda_oracle.so")
_lib = None

PAD = {"zeros": 0, "border": 1}


def build(force=False):
    """Compile the oracle with gcc (no GPU needed)."""
    os.makedirs(os.path.dirname(_LIB_PATH), exist_ok=True)
    src = os.path.join(_HERE, "msda_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-o", _LIB_PATH, src, "-lm"])
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        if os.environ.get("PDVC_ORACLE_LIB"):  # the sanitizer pass's build (tools/sanitize/run.sh)
            _lib = ctypes.CDLL(os.environ["PDVC_ORACLE_LIB"])
            return _lib
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _sfx(a):
    if a.dtype == np.float64:
        return "f64"
    if a.dtype == np.float32:
        return "f32"
    raise TypeError(f"oracle supports float32/float64, got {a.dtype}")


def _prep(value, shapes, lsi, loc, *rest):
    dt = value.dtype
    value = np.ascontiguousarray(value)
    shapes = np.ascontiguousarray(np.asarray(shapes, dtype=np.int64).reshape(-1, 2))
    lsi = np.ascontiguousarray(np.asarray(lsi, dtype=np.int64).reshape(-1))
    loc = np.ascontiguousarray(loc, dtype=dt)
    rest = [np.ascontiguousarray(r, dtype=dt) for r in rest]
    N, S, M, D = value.shape
    _, Lq, _, L, P, two = loc.shape
    assert two == 2 and shapes.shape[0] == L
    return value, shapes, lsi, loc, rest, (N, S, M, D, L, Lq, P)


def msda_forward(value, shapes, lsi, loc, attn, pad="zeros"):
    value, shapes, lsi, loc, (attn,), (N, S, M, D, L, Lq, P) = _prep(value, shapes, lsi, loc, attn)
    out = np.zeros((N, Lq, M, D), dtype=value.dtype)
    f = getattr(_load(), "oracle_msda_forward_" + _sfx(value))
    f(_p(value), _p(shapes), _p(lsi), _p(loc), _p(attn), N, S, M, D, L, Lq, P, PAD[pad], _p(out))
    return out.reshape(N, Lq, M * D)


def msda_backward(value, shapes, lsi, loc, attn, grad_out, pad="zeros"):
    value, shapes, lsi, loc, (attn, grad_out), (N, S, M, D, L, Lq, P) = _prep(value, shapes, lsi, loc, attn, grad_out)
    gv = np.zeros_like(value)
    gl = np.zeros_like(loc)
    ga = np.zeros_like(attn)
    f = getattr(_load(), "oracle_msda_backward_" + _sfx(value))
    f(_p(value), _p(shapes), _p(lsi), _p(loc), _p(attn), _p(grad_out), N, S, M, D, L, Lq, P, PAD[pad],
      _p(gv), _p(gl), _p(ga))
    return gv, gl, ga


def msda_sample(value, shapes, lsi, loc, pad="border"):
    value, shapes, lsi, loc, _, (N, S, M, D, L, Lq, P) = _prep(value, shapes, lsi, loc)
    out = np.zeros((N * M, D, Lq, L, P), dtype=value.dtype)
    f = getattr(_load(), "oracle_msda_sample_" + _sfx(value))
    f(_p(value), _p(shapes), _p(lsi), _p(loc), N, S, M, D, L, Lq, P, PAD[pad], _p(out))
    return out


def msda_sample_backward(value, shapes, lsi, loc, grad_samples, pad="border"):
    value, shapes, lsi, loc, (gs,), (N, S, M, D, L, Lq, P) = _prep(value, shapes, lsi, loc, grad_samples)
    gv = np.zeros_like(value)
    gl = np.zeros_like(loc)
    f = getattr(_load(), "oracle_msda_sample_backward_" + _sfx(value))
    f(_p(value), _p(shapes), _p(lsi), _p(loc), _p(gs), N, S, M, D, L, Lq, P, PAD[pad], _p(gv), _p(gl))
    return gv, gl


# ---------------------------------------------------------------------------------------------
# 1-D PDVC helpers: the module-level math around the op (ms_deform_attn.py:163-192), restated in
# numpy so GPU tests of the fused 1-D kernels can be checked against op-level oracle calls.
# ---------------------------------------------------------------------------------------------
def lift_1d(loc1d, T_levels):
    """(N,Lq,M,L,P) x-locations -> (N,Lq,M,L,P,2) with y=0.5 and shapes [[1,T_l]] (ms_deform_attn.py:182-185)."""
    loc = np.stack([loc1d, np.full_like(loc1d, 0.5)], -1)
    shapes = np.stack([np.ones(len(T_levels), np.int64), np.asarray(T_levels, np.int64)], -1)
    lsi = np.concatenate([[0], np.cumsum(T_levels)[:-1]]).astype(np.int64)
    return loc, shapes, lsi
