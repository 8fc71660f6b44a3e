"""Node census of the captured training-step graph (bench workload): nodes by type -- the launches of one replay
(rocprof's per-step launch counts of a bench run also hold the eager steps' host copies and bookkeeping).

    python tools/diag_graph_nodes.py [--videos 16]
"""
import argparse
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402


class DlInfo(ctypes.Structure):
    _fields_ = [("dli_fname", ctypes.c_char_p), ("dli_fbase", ctypes.c_void_p), ("dli_sname", ctypes.c_char_p),
                ("dli_saddr", ctypes.c_void_p)]


class MemsetParams(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


class Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class KernelParams(ctypes.Structure):
    _fields_ = [("blockDim", Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p), ("gridDim", Dim3),
                ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


def kernel_name(hip, libc, nd):
    kp = KernelParams()
    if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(kp)) != 0 or not kp.func:
        return "?"
    info = DlInfo()
    if libc.dladdr(ctypes.c_void_p(kp.func), ctypes.byref(info)) and info.dli_sname:
        name = info.dli_sname.decode(errors="replace")
        try:
            import subprocess
            name = subprocess.run(["c++filt", name], capture_output=True, text=True, timeout=5).stdout.strip() or name
        except Exception:
            pass
        return name[:110]
    return f"func {kp.func:#x}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=16)
    a = ap.parse_args()
    import opts
    from pdvc import gemm_tuning
    from pdvc.data import collate, synthetic_videos, to_device
    from pdvc.pdvc import build
    from pdvc.step_graph import StepGraph
    gemm_tuning.enable()
    torch.manual_seed(0)
    args = opts.parse_opts(["--cfg_path", "cfgs/anet_tsp_pdvc.yml", "--device", "cuda"], cfg_root=PKG,
                           feature_dim=768, num_queries=100, frame_embedding_num=512)
    model, criterion, _ = build(args)
    model = model.cuda().train()
    dt = to_device(collate(synthetic_videos(a.videos, 512, 768, 4, 13, args.vocab_size + 1, seed=1000)), "cuda")
    sg = StepGraph(model, criterion, dt, debug_dot="/tmp/step_graph.dot")
    sg.replay()
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    g = ctypes.c_void_p(sg.graph.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    hip.hipGraphGetNodes(g, None, ctypes.byref(n))
    nodes = (ctypes.c_void_p * n.value)()
    hip.hipGraphGetNodes(g, nodes, ctypes.byref(n))
    kinds = collections.Counter()
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        kinds[t.value] += 1
    print(f"videos {a.videos}: nodes {n.value} by type (0 kernel, 1 memcpy, 2 memset, 5 empty, 6 wait, 7 record): "
          f"{dict(kinds)}", flush=True)
    # every memset node: its parameters and the kernels on either side (host stub symbols through dladdr)
    libc = ctypes.CDLL(None)

    def nbrs(nd, fn):
        k = ctypes.c_size_t(0)
        fn(ctypes.c_void_p(nd), None, ctypes.byref(k))
        arr = (ctypes.c_void_p * max(k.value, 1))()
        fn(ctypes.c_void_p(nd), arr, ctypes.byref(k))
        return [arr[i] for i in range(k.value)]

    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        if t.value != 2:
            continue
        mp = MemsetParams()
        hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(mp))
        print(f"memset: {mp.elementSize * mp.width * max(mp.height, 1)} B (elementSize {mp.elementSize}, width "
              f"{mp.width}, height {mp.height})")
        for p_ in nbrs(nd, hip.hipGraphNodeGetDependencies):
            print("    after :", kernel_name(hip, libc, p_))
        for s_ in nbrs(nd, hip.hipGraphNodeGetDependentNodes):
            print("    before:", kernel_name(hip, libc, s_))

if __name__ == "__main__":
    main()
