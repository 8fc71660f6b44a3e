"""ctypes binding of libpdvc_hip.so -- the C ABI declared in include/pdvc_msda.h.

This is the only door from Python into the HIP kernels.  There is deliberately no fallback: if the
library is missing, or a tensor is not on a GPU, calls raise (the reference likewise raises
"Not implemented on the CPU", pdvc/ops/src/ms_deform_attn.h:38,60).
"""
import ctypes
import os

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("PDVC_HIP_LIB", os.path.join(_PKG, "lib", "libpdvc_hip.so"))

_vp, _i, _u8p = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p
_f, _u64 = ctypes.c_float, ctypes.c_uint64

# name -> argtypes (all return int status)
SIGNATURES = {
    "pdvc_ms_deform_attn_forward_f32": [_vp] * 5 + [_i] * 8 + [_vp, _vp],
    "pdvc_ms_deform_attn_forward_f64": [_vp] * 5 + [_i] * 8 + [_vp, _vp],
    "pdvc_ms_deform_attn_backward_f32": [_vp] * 6 + [_i] * 8 + [_vp] * 4,
    "pdvc_ms_deform_attn_backward_f64": [_vp] * 6 + [_i] * 8 + [_vp] * 4,
    "pdvc_ms_deform_attn_backward_ws_f32": [_vp] * 6 + [_i] * 8 + [_vp] * 4 + [ctypes.c_size_t, _vp],
    "pdvc_ms_deform_sample_f32": [_vp] * 4 + [_i] * 8 + [_vp, _vp],
    "pdvc_ms_deform_sample_backward_f32": [_vp] * 5 + [_i] * 8 + [_vp] * 3,
    "pdvc_msda1d_forward_f32": [_vp, _u8p, _vp, _i, _i, _i, _vp, _i, _vp] + [_i] * 6 + [_vp] * 4,
    "pdvc_msda1d_backward_f32": [_vp, _u8p, _vp, _i, _vp, _i, _i, _i, _vp] + [_i] * 6 + [_vp] * 8,
    "pdvc_msda1d_backward_ex_f32": [_vp, _u8p, _vp, _i, _vp, _i, _i, _i, _vp] + [_i] * 6 + [_vp] * 9,
    "pdvc_msda1d_forward_f32_bf16out": [_vp, _u8p, _vp, _i, _i, _i, _vp, _i, _vp] + [_i] * 6 + [_vp] * 5,
    "pdvc_msda1d_backward_ex_f32_bf16out": [_vp, _u8p, _vp, _i, _vp, _i, _i, _i, _vp] + [_i] * 6 + [_vp] * 11,
    "pdvc_cap_gather_forward_f32": [_vp, _u8p, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _vp] + [_i] * 6 + [_vp] * 3,
    "pdvc_cap_gather_backward_f32": [_vp, _u8p, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _vp] + [_i] * 6 + [_vp] * 6,
    "pdvc_cap_gather_backward2_f32": [_vp, _u8p, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _vp] + [_i] * 6 + [_vp] * 8,
    "pdvc_cap_softattn_forward_f32": [_vp, _u8p, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _vp] + [_i] * 6
    + [_vp, _i] + [_vp] * 8,
    "pdvc_cap_softattn_backward_f32": [_vp, _u8p, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _vp] + [_i] * 6
    + [_vp] * 4 + [_i] + [_vp] * 3 + [_i] + [_vp] * 6,
    "pdvc_cap_value_grad_f32": [_u8p, _vp] + [_i] * 8 + [_vp] * 6,
    "pdvc_cap_value_grad_ex_f32": [_u8p, _vp] + [_i] * 8 + [_vp] * 7,
    "pdvc_cap_value_grad_ranged_f32": [_u8p, _vp] + [_i] * 8 + [_vp] * 8,
    "pdvc_cap_value_grad_ranged_f32_bf16out": [_u8p, _vp] + [_i] * 8 + [_vp] * 9,
    "pdvc_cap_value_grad_rank1_f32": [_u8p, _vp] + [_i] * 8 + [_vp] * 9,
    "pdvc_softattn_forward_f32": [_vp, _vp, _i, _vp, _vp, _vp] + [_i] * 4 + [_vp] * 3,
    "pdvc_softattn_backward_f32": [_vp, _vp, _i, _vp, _vp, _vp, _vp] + [_i] * 4 + [_vp, _vp, _i, _vp, _vp, _vp, _vp],
    "pdvc_lstm_cell_forward_f32": [_vp, _i, _vp, _i, _vp, _i, _vp, _i, _vp, _i, _i, _vp, _i, _vp, _vp, _vp],
    "pdvc_lstm_cell_forward_gather_f32": [_vp, _i, _vp, _vp, _i, _vp, _i, _vp, _i, _vp, _i, _i, _vp, _i, _vp, _vp,
                                          _vp],
    "pdvc_lstm_cell_backward_f32": [_vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _i, _i, _vp, _i, _vp, _vp],
    "pdvc_add_dropout_layernorm_forward_f32": [_vp] * 4 + [_i, _i, _f, _u64, _vp, _f] + [_vp] * 4,
    "pdvc_add_dropout_layernorm_backward_f32": [_vp] * 6 + [_i, _i, _f, _u64] + [_vp] * 8,
    "pdvc_layernorm_residual_forward_f32": [_vp] * 4 + [_i, _i, _f] + [_vp] * 4,
    "pdvc_layernorm_backward_f32": [_vp] * 5 + [_i, _i] + [_vp] * 5,
    "pdvc_lsap_f32": [_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp],
    "pdvc_colsum_f32": [_vp, _i, _i, _i, _vp, _vp, _vp],
    "pdvc_relu_dropout_forward_f32": [_vp, ctypes.c_long, _i, _f, _u64, _vp, _vp],
    "pdvc_relu_dropout_backward_f32": [_vp, _vp, _i, _i, _f, _i, _vp, _vp, _vp],
    "pdvc_add_dropout_layernorm_forward_f32_bf16out": [_vp] * 4 + [_i, _i, _f, _u64, _vp, _f] + [_vp] * 5,
    "pdvc_add_dropout_layernorm_backward_f32_bf16out": [_vp] * 6 + [_i, _i, _f, _u64] + [_vp] * 9,
    "pdvc_relu_dropout_forward_f32_bf16out": [_vp, ctypes.c_long, _i, _f, _u64, _vp, _vp, _vp],
    "pdvc_relu_dropout_backward_f32_bf16out": [_vp, _vp, _i, _i, _f, _i, _vp, _vp, _vp, _vp],
    "pdvc_logprob_pick_backward_f32_bf16out": [_vp, _vp, _vp, _i, _i, _vp, _vp, _vp],
    "pdvc_level_pos_rows_add_f32_bf16out": [_vp] * 5 + [_i] * 5 + [_vp] * 4,
    "pdvc_logprob_pick_forward_f32": [_vp, _vp, _i, _i, _vp, _vp, _vp],
    "pdvc_logprob_pick_backward_f32": [_vp, _vp, _vp, _i, _i, _vp, _vp],
    "pdvc_logprob_pick_backward_ld_f32": [_vp, _vp, _vp, _i, _i, _i, _vp, _vp],
    "pdvc_logprob_argmax_f32": [_vp, _i, _i, _vp, _vp, _vp],
    "pdvc_seq_attention_forward_f32": [_vp, ctypes.c_long, _vp, ctypes.c_long, _vp, ctypes.c_long] + [_i] * 5
    + [_vp, _vp, _vp],
    "pdvc_seq_attention_backward_f32": [_vp, ctypes.c_long, _vp, ctypes.c_long, _vp, ctypes.c_long, _vp, _vp, _vp]
    + [_i] * 5 + [_vp, _vp, ctypes.c_long, _vp, ctypes.c_long, _vp, ctypes.c_long, _vp],
    "pdvc_level_pos_rows_forward_f32": [_vp] * 5 + [_i] * 5 + [_vp, _vp],
    "pdvc_level_pos_rows_backward_f32": [_vp, _vp] + [_i] * 4 + [_vp, _vp],
    "pdvc_level_pos_rows_add_f32": [_vp] * 5 + [_i] * 5 + [_vp, _vp, _vp],
    "pdvc_graph_replace_memsets": [_vp, _vp],
    "pdvc_event_create": [_vp],
    "pdvc_event_destroy": [_vp],
    "pdvc_event_record_external": [_vp, _vp],
    "pdvc_stream_wait_event": [_vp, _vp],
    "pdvc_box_refine_forward_f32": [_vp, _vp, ctypes.c_long, _i, _f, _vp, _vp],
    "pdvc_box_refine_backward_f32": [_vp, _vp, _vp, ctypes.c_long, _i, _f, _vp, _vp, _vp],
    "pdvc_match_cost_f32": [_vp] * 4 + [_i] * 4 + [_f] * 6 + [_vp, _vp],
    "pdvc_set_losses_f32": [_vp] * 11 + [_i] * 5 + [_f, _f, _i, _f] + [_vp] * 5,
    "pdvc_set_losses_backward_f32": [_vp] * 4 + [_i] * 4 + [_vp] * 4,
    "pdvc_groupnorm_rows_forward_f32": [_vp, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "pdvc_groupnorm_rows_backward_f32": [_vp] * 5 + [_i] * 4 + [_vp] * 4,
    "pdvc_groupnorm_rows_forward_out_f32": [_vp, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp, ctypes.c_long, _vp, _vp,
                                            _vp, _vp],
    "pdvc_groupnorm_rows_backward_strided_f32": [_vp, _vp, ctypes.c_long] + [_vp] * 4 + [_i] * 4 + [_vp] * 4,
    "pdvc_groupnorm_rows_forward_fused_f32": [_vp, _i, _i, _i, _i, _f, _vp, _vp, _vp, ctypes.c_long, _vp, _vp, _vp,
                                              _vp, _vp],
    "pdvc_groupnorm_rows_backward_fused_f32": [_vp, _vp, ctypes.c_long] + [_vp] * 4 + [_i] * 4 + [_vp] * 3,
    "pdvc_gemm_f32": [_i, _i, _i, _vp, _i, _i, _vp, _i, _i, _vp, _i, _vp, _i, _i, _vp],
    "pdvc_split3_planes_f32": [_vp, ctypes.c_long, _i, _i, _i, _vp, _vp],
    "pdvc_gemm3p_f32": [_i, _i, _i, _vp, ctypes.c_long, _vp, _vp, ctypes.c_long, _vp, _i, _vp],
    "pdvc_gemm3p_relu_dropout_f32": [_i, _i, _i, _vp, ctypes.c_long, _vp, _vp, ctypes.c_long, _vp, _f, _vp, _vp],
    "pdvc_gemm3p_dmask_f32": [_i, _i, _i, _vp, ctypes.c_long, _vp, _vp, ctypes.c_long, _vp, _f, _vp],
    "pdvc_gemm3p_resid_dropout_f32": [_i, _i, _i, _vp, ctypes.c_long, _vp, _vp, ctypes.c_long, _vp, _vp, _f, _vp, _vp],
    "pdvc_round_plane_f32": [_vp, ctypes.c_long, _i, _i, _i, _vp, _vp],
    "pdvc_gemm1p_f32": [_i, _i, _i, _vp, ctypes.c_long, _vp, _vp, ctypes.c_long, _vp, _i, _vp],
    "pdvc_gemm3_f32": [_i, _i, _i, _vp, ctypes.c_long, _i, _vp, ctypes.c_long, _i, _vp, ctypes.c_long, _vp, _i, _i,
                       _vp, _vp],
    "pdvc_sorted_row_sums_f32": [_vp, ctypes.c_long, _i, _vp, _vp, ctypes.c_long, _i, _vp, ctypes.c_long, _vp,
                                 _vp],
    "pdvc_gemm3_wgrad_bias_f32": [_i, _i, _i, _vp, ctypes.c_long, _vp, ctypes.c_long, _vp, ctypes.c_long, _i, _i,
                                  _vp, _vp, _vp, _vp],
    "pdvc_mha_forward_f32": [_vp, _vp, _u8p] + [_i] * 4 + [_f, _u64] + [_vp] * 4,
    "pdvc_mha_backward_f32": [_vp, _vp, _u8p, _vp, _vp, _vp] + [_i] * 4 + [_f, _u64] + [_vp] * 5,
}

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libpdvc_hip.so once; raise loudly if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"libpdvc_hip.so not found at {LIB_PATH}: build it with "
                              f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        L.pdvc_detokenize.argtypes = [_vp, _i, _i, _vp, _vp, _i, _vp, ctypes.c_int64, _vp]
        L.pdvc_detokenize.restype = ctypes.c_int
        L.pdvc_mha_workspace_floats.argtypes = [ctypes.c_int] * 4
        L.pdvc_mha_workspace_floats.restype = ctypes.c_long
        L.pdvc_ms_deform_attn_workspace_floats.argtypes = [ctypes.c_int] * 5
        L.pdvc_ms_deform_attn_workspace_floats.restype = ctypes.c_size_t
        L.pdvc_sorted_row_sums_workspace.argtypes = [ctypes.c_long, ctypes.c_int]
        L.pdvc_sorted_row_sums_workspace.restype = ctypes.c_long
        L.pdvc_last_error.restype = ctypes.c_char_p
        L.pdvc_abi_version.restype = ctypes.c_int
        _lib = L
    return _lib


class KernelTimer:
    """Records HIP events around selected C-ABI launches on the launching (current) stream, so a bench can
    report a kernel's average device duration over its timed region (bench.py's roofline leg)."""

    def __init__(self, names):
        self.names = set(names)
        self.records = []

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, meta in self.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "metas": [], "launch_ms": []})
            ms = e0.elapsed_time(e1)
            d["launches"] += 1
            d["ms"] += ms
            d["metas"].append(meta)
            d["launch_ms"].append(ms)
        return out


TIMER = None


def call(name, *args, meta=None):
    t = TIMER
    if t is not None and name in t.names:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib(), name)(*args)
        e1.record()
        t.records.append((name, e0, e1, meta))
    else:
        rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().pdvc_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed ({rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Tensors must be contiguous and on a GPU."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeError("PDVC HIP ops need GPU tensors (there is no CPU implementation)")
    if not t.is_contiguous():
        raise NativeError("PDVC HIP ops need contiguous tensors")
    return ctypes.c_void_p(t.data_ptr())


def ptr_any(t):
    """Device pointer of a (possibly strided) GPU tensor; the caller passes its strides to the kernel."""
    if not t.is_cuda:
        raise NativeError("PDVC HIP ops need GPU tensors (there is no CPU implementation)")
    return ctypes.c_void_p(t.data_ptr())


def rows(t):
    """(pointer, row stride) of a 2-D row-strided view (unit column stride), e.g. a column block of a wider
    matrix; the kernels take the row stride as an argument."""
    if not t.is_cuda:
        raise NativeError("PDVC HIP ops need GPU tensors (there is no CPU implementation)")
    if t.dim() != 2 or (t.stride(1) != 1 and t.shape[1] > 1):
        raise NativeError(f"expected a 2-D row-strided view, got shape {tuple(t.shape)} strides {t.stride()}")
    return ctypes.c_void_p(t.data_ptr()), t.stride(0)


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_INT_ARRAYS = {}


def int_array(values):
    """Host int32 array (kept alive in a cache: these are per-model constants such as level lengths)."""
    key = tuple(int(v) for v in values)
    hit = _INT_ARRAYS.get(key)
    if hit is None:
        arr = (ctypes.c_int32 * len(key))(*key)
        hit = (arr, ctypes.cast(arr, ctypes.c_void_p))
        _INT_ARRAYS[key] = hit
    return hit[1]


def detokenize(seqs, words, word_off, yield_every=0):
    """pdvc_detokenize over an int64 host array (rows, len): the captions as Python strings.  words: the
    vocabulary bytes concatenated (numpy uint8), word_off: (num_words + 1,) int64 offsets (word 0 unused)."""
    import numpy as np
    seqs = np.ascontiguousarray(seqs, dtype=np.int64)
    rows, length = seqs.shape
    if rows == 0:
        return []
    longest = int(np.diff(word_off).max(initial=0))
    cap = rows * (length * (longest + 1) + 2) + 1
    out = np.empty(cap, dtype=np.uint8)
    ends = np.empty(rows, dtype=np.int64)
    rc = lib().pdvc_detokenize(seqs.ctypes.data, rows, length, words.ctypes.data, word_off.ctypes.data,
                               len(word_off) - 1, out.ctypes.data, cap, ends.ctypes.data)
    if rc != 0:
        raise NativeError(f"pdvc_detokenize failed ({rc}): {lib().pdvc_last_error().decode(errors='replace')}")
    total = int(ends[-1])
    buf = out[:total].tobytes()
    starts = np.concatenate([[0], ends[:-1]]).tolist()
    stops = ends.tolist()
    if buf.isascii():  # one decode, str slices (byte offsets are character offsets)
        text = buf.decode("ascii")
        cut = lambda a, b: text[a:b]  # noqa: E731
    else:
        cut = lambda a, b: buf[a:b].decode("utf-8")  # noqa: E731
    if not yield_every:
        return [cut(a, b) for a, b in zip(starts, stops)]
    # on a worker thread (PostProcess's deferred host half): the GIL handed back every yield_every rows, so the
    # thread that queues GPU work waits for it ~0.1 ms at a time instead of a whole switch interval (5 ms)
    import time
    res = []
    for i in range(0, rows, yield_every):
        res.extend(cut(a, b) for a, b in zip(starts[i:i + yield_every], stops[i:i + yield_every]))
        time.sleep(0)
    return res
