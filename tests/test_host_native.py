"""CPU: the library's host-only entry points (csrc/detok.cpp, csrc/pdvc_status.cpp) on random and edge inputs.

Loads libpdvc_hip.so, or -- in the sanitizer pass (tools/sanitize/run.sh) -- the same sources built alone with
-fsanitize=address,undefined (PDVC_HOST_ASAN_LIB), so that every call below runs under ASan/UBSan there.  The
expected captions follow the reference's Translator.rtranslate (data/video_dataset.py:172-180): the ids up to the
first 0, words joined by single spaces, then a full stop; an id-less row is the empty caption."""
import ctypes
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "dense-video-captioning_amd"))


def _lib():
    path = os.environ.get("PDVC_HOST_ASAN_LIB")
    if not path:
        from pdvc import _native
        path = _native.LIB_PATH
        if not os.path.exists(path):
            pytest.skip("libpdvc_hip.so not built")
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.pdvc_detokenize.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, vp, ctypes.c_int64, vp]
    L.pdvc_detokenize.restype = ctypes.c_int
    L.pdvc_last_error.restype = ctypes.c_char_p
    return L


def _vocab(words):
    enc = [w.encode() for w in words]
    off = np.zeros(len(enc) + 2, np.int64)  # id 0: the end token (no word)
    off[2:] = np.cumsum([len(e) for e in enc])
    return np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy(), off


def _detok(L, seqs, words, off, cap):
    seqs = np.ascontiguousarray(seqs, np.int64)
    rows, length = seqs.shape
    out = np.zeros(max(cap, 1), np.uint8)
    ends = np.zeros(max(rows, 1), np.int64)
    rc = L.pdvc_detokenize(seqs.ctypes.data, rows, length, words.ctypes.data, off.ctypes.data, len(off) - 1,
                           out.ctypes.data, cap, ends.ctypes.data)
    if rc != 0:
        return rc, None
    caps, prev = [], 0
    for r in range(rows):
        caps.append(bytes(out[prev:ends[r]]).decode())
        prev = ends[r]
    return rc, caps


def _expected(seqs, words):
    res = []
    for row in seqs:
        ids = []
        for w in row:
            if w == 0:
                break
            ids.append(int(w))
        res.append(" ".join(words[i - 1] for i in ids) + "." if ids else "")
    return res


def test_detokenize_random_rows_match_rtranslate():
    L = _lib()
    rng = np.random.RandomState(0)
    words = ["w%d" % i + "é" * (i % 3) for i in range(1, 60)]
    wb, off = _vocab(words)
    for rows, length in [(0, 4), (3, 0), (1, 1), (257, 31)]:
        seqs = rng.randint(0, len(words) + 1, size=(rows, length))
        if rows and length:
            seqs[::3, 0] = 0
        rc, caps = _detok(L, seqs, wb, off, 64 * rows * max(length, 1) + 1)
        assert rc == 0 and caps == _expected(seqs, words)


def test_detokenize_errors_do_not_write_past_the_buffer():
    L = _lib()
    words = ["alpha", "beta"]
    wb, off = _vocab(words)
    seqs = np.array([[1, 2, 1]])
    need = len("alpha beta alpha.")
    assert _detok(L, seqs, wb, off, need + 1)[1] == ["alpha beta alpha."]
    for cap in (0, 1, need - 1):
        rc, _ = _detok(L, seqs, wb, off, cap)
        assert rc == -1 and b"output full" in L.pdvc_last_error()
    assert _detok(L, np.array([[3]]), wb, off, 64)[0] == -1
    assert b"outside" in L.pdvc_last_error()
    bad = off.copy()
    bad[2] = bad[3] + 1  # offsets that run backwards: an error, never a negative-length copy
    assert _detok(L, np.array([[2]]), wb, bad, 64)[0] == -1
    assert b"decreases" in L.pdvc_last_error()
