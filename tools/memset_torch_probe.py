"""Probe 4 (round 3): hipMemsetAsync on torch-allocated memory inside torch.cuda.graph capture.

The failing step graph (tools/diag_memset_graph.py, PDVC_ZERO_MEMSET=1) held 28 memcpy nodes and 1 memset node where
the default build's graph holds 9 and 0: the library's captured hipMemsetAsync calls did not become memset nodes.
Plain-HIP probes (memset_graph_probe2/3.hip, hipMalloc'd buffers) capture memset nodes that re-apply on every replay.
Here: torch tensors of several sizes, hipMemsetAsync through ctypes on the capturing stream between a torch fill and a
torch add, the captured node types, and the buffer after replays with eager torch work between them (1 if the
zero-fill holds, 6 if not).

    python tools/memset_torch_probe.py
"""
import ctypes

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    torch.zeros(1, device="cuda")
    print("allocator settings:", torch.cuda.memory._get_current_allocator() if hasattr(torch.cuda.memory,
          "_get_current_allocator") else "?", flush=True)
    for n in (40, 400, 1200, 4096, 262144):
        buf = torch.empty(n, device="cuda")
        side = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=side):
            buf.fill_(5.0)
            s = torch.cuda.current_stream().cuda_stream
            rc = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, ctypes.c_size_t(n * 4), ctypes.c_void_p(s))
            buf.add_(1.0)
        raw = ctypes.c_void_p(g.raw_cuda_graph())
        k = ctypes.c_size_t(0)
        hip.hipGraphGetNodes(raw, None, ctypes.byref(k))
        nodes = (ctypes.c_void_p * k.value)()
        hip.hipGraphGetNodes(raw, nodes, ctypes.byref(k))
        types = []
        for nd in nodes:
            t = ctypes.c_int(-1)
            hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
            types.append(t.value)
        g.instantiate()
        vals = []
        for r in range(3):
            g.replay()
            torch.cuda.synchronize()
            vals.append((buf[0].item(), buf[-1].item()))
            junk = [torch.full((n + 13 * i,), 7.0, device="cuda") * 2 for i in range(32)]  # eager work, reuse
            del junk
        print(f"n {n:7d}: memset rc {rc}, node types {types}, after replays {vals}", flush=True)


if __name__ == "__main__":
    main()
