"""Diagnosis of the round-1/2 memset-in-graph failure: run with PDVC_ZERO_MEMSET=1 so every
library zero-fill is a hipMemsetAsync again, capture the step graph with debug mode on, dump it with
hipGraphDebugDotPrint (torch CUDAGraph.debug_dump), replay it three times against the eager step (the reference-point
gradient taps of tools/diag_refgrad.py) and list every memset node of the instantiated graph with its parameters
and its neighbours.

    PDVC_ZERO_MEMSET=1 python tools/diag_memset_graph.py OUTDIR
"""
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
    import shutil
    labels, edges = parse_dot(dot)
    print("dot file:", dot, os.path.getsize(dot), "bytes;", len(labels), "labelled nodes", flush=True)
    if not labels:
        print(open(dot, errors="replace").read()[:3000])
    kinds = defaultdict(int)
    for lab in labels.values():
        u = lab.upper()
        k = ("MEMSET" if "MEMSET" in u else "MEMCPY" if "MEMCPY" in u else "EVENT" if "EVENT" in u
             else "EMPTY" if "EMPTY" in u else "KERNEL")
        kinds[k] += 1
    print("graph nodes by kind:", dict(kinds), " edges:", len(edges), flush=True)
    pred, succ = defaultdict(list), defaultdict(list)
    for a, b in edges:
        succ[a].append(b)
        pred[b].append(a)
    for n, lab in labels.items():
        if "MEMSET" in lab.upper():
            print("memset node", n, ":", short(lab))
            for p in pred[n][:4]:
                print("    after :", short(labels.get(p, p)))
            for s_ in succ[n][:4]:
                print("    before:", short(labels.get(s_, s_)))


if __name__ == "__main__":
    main()
