"""CPU: the C-ABI library builds/loads and exports every symbol include/*.h declares (no GPU calls)."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names.update(re.findall(r"\b(pdvc_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    import build_native
    path = build_native.build(verbose=False)
    return ctypes.CDLL(path)


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "pdvc_ms_deform_attn_forward_f32" in syms and "pdvc_ms_deform_attn_backward_f64" in syms
    assert len(syms) >= 12


def test_every_declared_symbol_is_exported(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"symbols declared in include/*.h but not exported: {missing}"


def test_version_and_errors(lib):
    lib.pdvc_abi_version.restype = ctypes.c_int
    lib.pdvc_last_error.restype = ctypes.c_char_p
    assert lib.pdvc_abi_version() == 1
    # argument validation runs on the host: a bad level count is rejected without touching a GPU
    f = lib.pdvc_ms_deform_attn_forward_f32
    f.restype = ctypes.c_int
    rc = f(None, None, None, None, None, 1, 4, 1, 4, 0, 1, 1, 64, None, None)
    assert rc == -1 and b"num_levels" in lib.pdvc_last_error()
    rc = f(None, None, None, None, None, 3, 4, 1, 4, 1, 1, 1, 2, None, None)
    assert rc == -1 and b"im2col_step" in lib.pdvc_last_error()


def test_native_binding_table_matches_header():
    from pdvc import _native
    assert set(_native.SIGNATURES) <= set(declared_symbols())


def declared_prototypes():
    """name -> list of parameter kinds ('p' pointer, 'i' integer/enum, 'f' floating) from include/*.h."""
    protos = {}
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for name, params in re.findall(r"\b(pdvc_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
            kinds = []
            for prm in params.split(","):
                prm = prm.strip()
                if not prm or prm == "void":
                    continue
                kinds.append("p" if "*" in prm else "f" if re.search(r"\b(float|double)\b", prm) else "i")
            protos[name] = kinds
    return protos


def test_native_binding_argument_kinds_match_header():
    """Each ctypes argtypes list in pdvc/_native.py has the header's parameter count, with pointers where the
    prototype has pointers and scalars where it has scalars."""
    from pdvc import _native
    protos = declared_prototypes()
    bad = []
    for name, argtypes in _native.SIGNATURES.items():
        want = protos.get(name)
        assert want is not None, f"{name}: no prototype parsed"
        got = []
        for t in argtypes:
            if t in (ctypes.c_float, ctypes.c_double):
                got.append("f")
            elif t in (ctypes.c_int, ctypes.c_long, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32,
                       ctypes.c_size_t, ctypes.c_longlong, ctypes.c_ulonglong):
                got.append("i")
            else:
                got.append("p")
        if got != want:
            bad.append(f"{name}: binding {''.join(got)} vs header {''.join(want)}")
    assert not bad, "\n".join(bad)
