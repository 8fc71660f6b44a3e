"""What a garbage collection INSIDE a hipGraph stream capture can destroy, case by case.

Round 4's GPU pass AC aborted inside the step-graph capture test; StepGraph has since disabled the collector for the
capture (pdvc/step_graph.py).  This probe runs one child process per case: it builds cyclic garbage holding one kind
of object, starts a capture on a side stream (torch.cuda.graph, the same global capture mode StepGraph uses), runs
gc.collect() inside it, finishes the capture and replays once.  The child's exit status and last output lines are
printed per case, so the cases that break a capture are named by evidence, not inferred:

  tensors     cyclic garbage holding CUDA tensors (caching-allocator blocks freed inside the capture)
  autograd    cyclic garbage holding an eager autograd graph (a loss whose backward never ran: saved tensors,
              AccumulateGrad nodes of parameters, made on the default stream)
  graph       cyclic garbage holding an instantiated torch.cuda.CUDAGraph with its private pool's outputs
              (hipGraphExecDestroy / hipGraphDestroy and the pool's release inside the capture)
  event       cyclic garbage holding timing torch.cuda.Events (hipEventDestroy inside the capture)

    python tools/gc_capture_probe.py            # all cases, one child each
    python tools/gc_capture_probe.py --case X   # one case in this process (what the children run)
"""
import argparse
import gc
import os
import subprocess
import sys

CASES = ("none", "tensors", "autograd", "graph", "event")


class Cyc:
    def __init__(self, payload):
        self.payload = payload
        self.me = self  # a reference cycle: only the collector frees it


def make_garbage(case):
    import torch
    dev = "cuda"
    if case == "tensors":
        Cyc([torch.randn(1 << 20, device=dev) for _ in range(8)])
    elif case == "autograd":
        lin = torch.nn.Linear(256, 256).to(dev)
        x = torch.randn(512, 256, device=dev)
        loss = torch.tanh(lin(x)).pow(2).sum()  # backward never runs: the graph keeps its saved tensors
        Cyc((lin, loss))
    elif case == "graph":
        a = torch.randn(1 << 16, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            b = a * 2  # warm-up
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            b = a * 2 + 1
        g.replay()
        torch.cuda.synchronize()
        Cyc((g, b))
    elif case == "event":
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for e in evs:
            e.record()
        torch.cuda.synchronize()
        Cyc(evs)


def run_case(case):
    import torch
    torch.cuda.init()
    x = torch.randn(1 << 16, device="cuda")
    y = x * 3  # warm-up of the captured ops
    y = y + 1
    torch.cuda.synchronize()
    gc.collect()
    gc.disable()  # the garbage below stays pending until the explicit collection inside the capture
    make_garbage(case)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # capture_begin / capture_end directly: torch.cuda.graph would collect on entry
        g.capture_begin()
        y = x * 3
        freed = gc.collect()
        y = y + 1
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ok = torch.allclose(y, x * 3 + 1)
    print(f"case {case}: collected {freed} objects inside the capture, replay {'correct' if ok else 'WRONG'}",
          flush=True)
    return 0 if ok else 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", choices=CASES)
    ap.add_argument("--timeout", type=int, default=120)
    a = ap.parse_args()
    if a.case:
        sys.exit(run_case(a.case))
    for case in CASES:
        p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--case", case], capture_output=True,
                           text=True, timeout=a.timeout)
        lines = [l for l in (p.stdout + p.stderr).splitlines() if l.strip() and "amdgpu.ids" not in l]
        # the message of an abort, not its stack frames
        keep = [l for l in lines if not l.lstrip().startswith("frame #")][:8]
        print(f"== {case}: exit {p.returncode}")
        for l in keep:
            print("   " + l[:400])
        sys.stdout.flush()


if __name__ == "__main__":
    main()
