"""Diagnosis of the round-1/2 memset-in-graph failure: run with PDVC_ZERO_MEMSET=1 so every
library zero-fill is a hipMemsetAsync again, capture the step graph with debug mode on, dump it with
hipGraphDebugDotPrint (torch CUDAGraph.debug_dump), replay it three times against the eager step (the reference-point
gradient taps of tools/diag_refgrad.py) and list every memset node of the instantiated graph with its parameters
and its neighbours.

    PDVC_ZERO_MEMSET=1 python tools/diag_memset_graph.py OUTDIR
"""
import ctypes
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import diag_refgrad as D  # noqa: E402  (installs the gradient taps)
import torch  # noqa: E402


def parse_dot(path):
    text = open(path, errors="replace").read()
    labels, edges = {}, []
    for m in re.finditer(r'"?(\w+)"?\s*\[((?:[^\]"]|"(?:[^"\\]|\\.)*")*)\]', text):
        lab = re.search(r'label\s*=\s*"((?:[^"\\]|\\.)*)"', m.group(2), re.S)
        if lab:
            labels[m.group(1)] = lab.group(1)
    for m in re.finditer(r'"?(\w+)"?\s*->\s*"?(\w+)"?', text):
        edges.append((m.group(1), m.group(2)))
    return labels, edges


def short(label):
    s = re.sub(r"[{}|\\]", " ", label)
    s = re.sub(r"\s+", " ", s).strip()
    return s[:160]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/memset"
    os.makedirs(out, exist_ok=True)
    dot = os.path.join(out, "step_graph.dot")
    d = D.TM.load("pdvc_batch3_anet")
    model, criterion = D.TM.build_filled(d)
    for i, layer in enumerate(model.transformer.decoder.layers):
        layer._lid = i
    model.train()
    wd = criterion.weight_dict
    mk = lambda: D.to_device(D.collate(D.W.batch_items(vocab=29)[1:2]), "cuda")
    out, loss = model(mk(), criterion, "queries")
    sum(loss[k] * wd[k] for k in loss.keys() if k in wd).backward()
    torch.cuda.synchronize()
    del out, loss  # a live eager graph keeps default-stream AccumulateGrad nodes: capture then crashes (step_graph.py)
    eager = {k: v.clone() for k, v in D.BUFS.items()}
    model.zero_grad(set_to_none=True)
    D.BUFS.clear()
    print("PDVC_ZERO_MEMSET =", os.environ.get("PDVC_ZERO_MEMSET"), flush=True)
    sg = D.StepGraph(model, criterion, mk(), debug_dot=dot)
    for r in range(3):
        sg.replay()
        torch.cuda.synchronize()
        for k, v in eager.items():
            err = (D.BUFS[k] - v).abs().max().item() if k in D.BUFS else float("nan")
            print(f"replay {r}: {k:14s} max|diff| {err:.3e}  (|g| {v.abs().max().item():.3e})", flush=True)
    walk_graph(sg.graph.raw_cuda_graph(), dot)


class MemsetParams(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


class Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class KernelParams(ctypes.Structure):
    _fields_ = [("blockDim", Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p), ("gridDim", Dim3),
                ("kernelParams", ctypes.POINTER(ctypes.c_void_p)), ("sharedMemBytes", ctypes.c_uint)]


def walk_graph(raw, dot):
    """Every memset node of the captured step graph (hip graph API through ctypes): its parameters, whether a
    dependency path leads from it to each kernel node that takes a pointer into the zeroed range (the first 24
    argument slots read as 8-byte words), and which other nodes write or read that range -- a missing edge, or an
    edge HIP does not honour on replay."""
    hip = ctypes.CDLL("libamdhip64.so")
    g = ctypes.c_void_p(raw)
    rc = hip.hipGraphDebugDotPrint(g, dot.encode(), ctypes.c_uint(1 << 0))
    print("hipGraphDebugDotPrint rc", rc, "->", dot, os.path.getsize(dot) if os.path.exists(dot) else "no file")
    n = ctypes.c_size_t(0)
    hip.hipGraphGetNodes(g, None, ctypes.byref(n))
    nodes = (ctypes.c_void_p * n.value)()
    hip.hipGraphGetNodes(g, nodes, ctypes.byref(n))
    kinds = defaultdict(int)
    types = {}
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        types[nd] = t.value
        kinds[t.value] += 1
    print("nodes", n.value, "by type (0 kernel, 1 memcpy, 2 memset, 5 empty, 6 wait, 7 record):", dict(kinds))

    def deps(nd, fn):
        k = ctypes.c_size_t(0)
        fn(ctypes.c_void_p(nd), None, ctypes.byref(k))
        arr = (ctypes.c_void_p * max(k.value, 1))()
        fn(ctypes.c_void_p(nd), arr, ctypes.byref(k))
        return [arr[i] for i in range(k.value)]

    succ = {nd: deps(nd, hip.hipGraphNodeGetDependentNodes) for nd in nodes}
    pred_count = defaultdict(int)
    for a, bs in succ.items():
        for b in bs:
            pred_count[b] += 1
    roots = sum(1 for nd in nodes if pred_count[nd] == 0)
    print("edges", sum(len(v) for v in succ.values()), "roots", roots)
    order = {nd: i for i, nd in enumerate(nodes)}
    maps = []  # readable host mappings: an argument slot past a kernel's last argument may hold any value
    for line in open("/proc/self/maps"):
        a, perm = line.split()[:2]
        if perm[0] == "r":
            lo_, hi_ = (int(x, 16) for x in a.split("-"))
            maps.append((lo_, hi_))

    def readable(p):
        return any(lo_ <= p and p + 8 <= hi_ for lo_, hi_ in maps)

    kargs = {}
    for nd in nodes:
        if types[nd] != 0:
            continue
        kp = KernelParams()
        if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(kp)) != 0 or not kp.kernelParams:
            continue
        words = []
        for i in range(24):
            ptr = kp.kernelParams[i]
            if not ptr or not readable(ptr):
                break
            words.append(ctypes.c_uint64.from_address(ptr).value)
        kargs[nd] = (kp.func, words, kp.gridDim.x)

    def reach(a, b):
        seen, stack = {a}, [a]
        while stack:
            x = stack.pop()
            if x == b:
                return True
            for y in succ[x]:
                if y not in seen:
                    seen.add(y)
                    stack.append(y)
        return False

    for nd in nodes:
        if types[nd] != 2:
            continue
        mp = MemsetParams()
        hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(mp))
        lo, hi = mp.dst, mp.dst + mp.elementSize * mp.width * max(mp.height, 1)
        print(f"memset node #{order[nd]}: dst {mp.dst:#x} elementSize {mp.elementSize} width {mp.width} "
              f"height {mp.height} pitch {mp.pitch} value {mp.value}  preds {pred_count[nd]} succs {len(succ[nd])}")
        users = [(o, k) for k, (f, w, gx) in kargs.items() for o in [order[k]] if any(lo <= x < hi for x in w)]
        for o, k in sorted(users)[:12]:
            f, w, gx = kargs[k]
            print(f"    kernel node #{o} func {f:#x} grid {gx}: reachable from the memset: {reach(nd, k)}, "
                  f"memset reachable from it: {reach(k, nd)}")
        others = [order[m] for m in nodes if types[m] == 2 and m != nd]
        if others:
            mset = []
            for m in nodes:
                if types[m] == 2 and m != nd:
                    q = MemsetParams()
                    hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(m), ctypes.byref(q))
                    if q.dst < hi and lo < q.dst + q.elementSize * q.width * max(q.height, 1):
                        mset.append(order[m])
            if mset:
                print("    other memset nodes overlapping this range:", mset)

if __name__ == "__main__":
    main()
