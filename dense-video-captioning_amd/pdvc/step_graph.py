"""The whole PDVC training forward + losses + backward as ONE captured hipGraph.

The reference's training iteration (train.py:181-187: `model(dt, criterion, ...)`, weighted loss sum,
`backward()`) launches ~1700 kernels per step from Python at PDVC's shapes; the host, not the GPU, then
sets the pace.  Every host decision of the step depends only on the batch's shapes and event/caption counts
(level lengths, matched rows, caption steps), the set matching runs on the GPU (pdvc_lsap_f32), and no
kernel needs a host read-back, so the step is captured once per batch shape and replayed:

    sg = StepGraph(model, criterion, dt)   # warm-up + capture (dt tensors become the graph's inputs)
    sg.load(dt_next)                       # copy a same-shape batch into the captured inputs (optional)

A batch padded to fixed capacities (pdvc/batch_layout.py pad_to_capacity: events per video, caption rows,
caption width) makes every later batch of the stream a same-shape batch, whatever its event counts and caption
lengths: load() then also recomputes the caption rows' bookkeeping on the host and copies it in.
    total = sg.replay()                    # forward + losses + backward; param.grad hold the new gradients

Dropout stays random per replay (torch's graph-safe Philox offsets; the HIP kernels draw their seeds on the
device).  Gradients live in the graph's memory pool: do not set them to None between replays (the optimizer
step and grad clipping run eagerly on them).  A GradAllReducer (data parallel) records an event at each bucket's
last gradient inside the capture, and replay() queues each bucket's all-reduce behind its event on a side stream
(finish_replay: the reduction overlaps the rest of the replay).  With a reducer the gradients are views into its
flat buckets (bucket-resident, pdvc/distributed.py): the captured step begins with the buckets' zero fill and the
backward accumulates into them, so finish() is one all-reduce and one scale per bucket.

Release the autograd graphs of earlier eager steps (their loss tensors) before constructing a StepGraph: they keep
the parameters' AccumulateGrad nodes alive, created on the stream of that eager step, and a capture whose
gradient accumulation then joins the default stream ended in a crash at capture end on ROCm 7
(tests/test_gpu_batch.py test_capacity_step_graph_follows_a_ragged_stream, tools/diag_capacity_capture.py).
"""
import ctypes
import gc
import os
import threading

import torch


def replace_memsets(graph):
    """Rewrite the memset nodes of a captured, not yet instantiated torch.cuda.CUDAGraph(keep_graph=True) as kernel
    nodes (pdvc_graph_replace_memsets, csrc/graphfix.hip): torch's multi-block reductions zero their semaphores with
    4-32 B memsets, and small captured memset nodes did not re-apply on replays after the first (DESIGN.md section 1;
    tools/memset_torch_probe.py, tools/check_graph_replays.py).  PDVC_GRAPH_MEMSETS=keep skips it (diagnosis).
    Returns the number of nodes rewritten."""
    if os.environ.get("PDVC_GRAPH_MEMSETS") == "keep":
        return 0
    from . import _native as _n
    count = ctypes.c_int(0)
    _n.call("pdvc_graph_replace_memsets", ctypes.c_void_p(graph.raw_cuda_graph()), ctypes.byref(count))
    left = graph_node_counts(graph).get("memset", 0)
    if left:  # never instantiate a graph whose memsets may not re-apply
        raise RuntimeError(f"replace_memsets: {left} memset node(s) left in the captured graph")
    return count.value


def graph_node_counts(graph):
    """Nodes of a kept captured graph by type ({"kernel": k, "memcpy": c, ...}): the launches of one replay."""
    hip = ctypes.CDLL("libamdhip64.so")
    raw = ctypes.c_void_p(graph.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    if hip.hipGraphGetNodes(raw, None, ctypes.byref(n)) != 0:
        return {}
    nodes = (ctypes.c_void_p * n.value)()
    hip.hipGraphGetNodes(raw, nodes, ctypes.byref(n))
    names = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
             7: "event_record"}
    out = {}
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        k = names.get(t.value, str(t.value))
        out[k] = out.get(k, 0) + 1
    out["total"] = int(n.value)
    return out


class _RewritingGraph(torch.cuda.CUDAGraph):
    """A CUDAGraph that keeps its hipGraph_t, rewrites its memset nodes and instantiates at capture end (unless the
    caller asked for keep_graph itself, in which case it instantiates when it chooses, as torch's class does)."""

    def __new__(cls, keep_graph=False):
        return super().__new__(cls, True)

    def __init__(self, keep_graph=False):  # the native object is built by __init__: keep the hipGraph_t
        super().__init__(True)
        self._caller_keeps = bool(keep_graph)

    def capture_end(self):
        super().capture_end()
        replace_memsets(self)
        if not self._caller_keeps:
            self.instantiate()


_REWRITE_LOCK = threading.RLock()
_REWRITE_DEPTH = [0]
_REWRITE_SAVED = [None]


class rewriting_graphs:
    """Within this context, graphs torch creates itself (torch.cuda.make_graphed_callables: the trunk graph,
    PDVC.enable_graph) rewrite their memset nodes as StepGraph does.  The patch is process-wide (make_graphed_callables
    looks up torch.cuda.CUDAGraph), so the context holds a lock: another thread that enters it waits, and a thread that
    builds a CUDAGraph outside it while it is active would also get the rewriting class -- do not capture graphs from
    other threads meanwhile.  Re-entrant: a nested use keeps the patch and the outermost exit restores torch's class."""

    def __enter__(self):
        import torch.cuda.graphs as tg
        _REWRITE_LOCK.acquire()
        if _REWRITE_DEPTH[0] == 0:
            _REWRITE_SAVED[0] = (torch.cuda.CUDAGraph, tg.CUDAGraph, gc.isenabled())
            torch.cuda.CUDAGraph = tg.CUDAGraph = _RewritingGraph
            gc.collect()
            gc.disable()  # no collection inside the captures made here (no_gc_capture: a graph destroyed mid-capture)
        _REWRITE_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        import torch.cuda.graphs as tg
        try:
            _REWRITE_DEPTH[0] -= 1
            if _REWRITE_DEPTH[0] == 0:
                torch.cuda.CUDAGraph, tg.CUDAGraph, enabled = _REWRITE_SAVED[0]
                _REWRITE_SAVED[0] = None
                if enabled:
                    gc.enable()
        finally:
            _REWRITE_LOCK.release()
        return False


_DP_OVERLAP = []
_DP_TRIALS = []


def dp_overlap_supported():
    """Whether an event recorded inside a stream capture (GraphEvent, hipEventRecordExternal) gates a stream outside
    the graph on this stack -- probed once, deterministically.  The probe graph first runs a kernel that holds its
    stream until the host sets a flag (pdvc_spin_until_flag: fine-grained pinned memory, bounded at 5 s), then writes
    7 into a marker, records the event and writes 3.  After each replay is queued, a side stream copies the marker
    (the control, no wait), then waits on the event and copies it again.  While the flag is held the control copy
    must finish and read 0 (the side stream does run beside a held replay) and the waited copy must not have
    finished; released, it must read 7 or 3.  A record that does not gate fails the second test every time, not by
    timing (the earlier probe's ungated control could read 3 when the replay happened to finish
    first).  PDVC_DP_OVERLAP=0 turns the overlap off."""
    if os.environ.get("PDVC_DP_OVERLAP", "1") == "0":
        return False
    if not _DP_OVERLAP:
        ok = False
        host = ctypes.c_void_p()
        dev = ctypes.c_void_p()
        from . import _native as _n
        try:
            import time
            from .distributed import GraphEvent
            _n.call("pdvc_host_flag_alloc", ctypes.byref(host), ctypes.byref(dev))
            flag = ctypes.c_int.from_address(host.value)
            mark = torch.zeros(1, device="cuda")
            ev = GraphEvent()
            g = torch.cuda.CUDAGraph()
            recorded = True
            with torch.cuda.graph(g):
                _n.call("pdvc_spin_until_flag", dev, 1, 5000, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                mark.fill_(7.0)
                try:  # a refused record must not raise out of the capture (a torch graph whose capture raised
                    ev.record(captured=True)  # aborts the process when it is destroyed)
                except Exception:  # noqa: BLE001
                    recorded = False
                mark.fill_(3.0)
            if not recorded:
                raise RuntimeError("the event record was refused inside the capture")
            side = torch.cuda.Stream()
            trials = []
            for _ in range(2):
                flag.value = 0
                mark.zero_()
                torch.cuda.synchronize()
                g.replay()
                # on ONE side stream: the control copy, then the wait, then the waited copy -- the control proves this
                # stream runs beside the held replay (a stream that shares the replay's hardware queue would not, and
                # would then hold the waited copy whether or not the event gates it)
                with torch.cuda.stream(side):
                    seen_ctrl = mark.clone()
                    ctrl_done = torch.cuda.Event()
                    ctrl_done.record()
                ev.wait(side)
                with torch.cuda.stream(side):
                    seen = mark.clone()
                    done = torch.cuda.Event()
                    done.record()
                t0 = time.time()
                while not ctrl_done.query() and time.time() - t0 < 2.0:
                    time.sleep(0.001)
                ctrl_ran = ctrl_done.query()
                # a waited copy that the event does not hold runs right behind the control: give it 50 ms to show
                t0 = time.time()
                while not done.query() and time.time() - t0 < 0.05:
                    time.sleep(0.001)
                held = not done.query()
                flag.value = 1
                t0 = time.time()
                while not done.query():
                    if time.time() - t0 > 20.0:
                        raise RuntimeError("the captured event never fired")
                    time.sleep(0.001)
                torch.cuda.synchronize()
                trials.append((ctrl_ran, held, float(seen_ctrl), float(seen)))
            ok = all(c and h and vc == 0.0 and v in (7.0, 3.0) for c, h, vc, v in trials)
            _DP_TRIALS[:] = trials  # (tests/test_gpu_dp_probe.py reads what the probe saw)
            if os.environ.get("PDVC_DP_OVERLAP_DEBUG"):
                print("dp_overlap_supported: (control ran, waiting copy held, control read, waiting read)", trials)
            del g
        except Exception:  # noqa: BLE001 -- any failure: keep the serial reduction
            if os.environ.get("PDVC_DP_OVERLAP_DEBUG"):
                import traceback
                traceback.print_exc()
            ok = False
        finally:
            if host.value:
                torch.cuda.synchronize()
                _n.call("pdvc_host_flag_free", host)
        _DP_OVERLAP.append(ok)
    return _DP_OVERLAP[0]


class StepGraph:
    def __init__(self, model, criterion, dt, transformer_input_type="queries", warmup=2, reducer=None, debug_dot=None):
        self.model, self.criterion, self.dt, self.tit = model, criterion, dt, transformer_input_type
        self.wd = criterion.weight_dict
        self.reducer = reducer
        # host-side facts of the batch, made once here (they would be host round trips inside the capture)
        if "video_target_padded" not in dt:
            from .matcher import padded_targets
            dt["video_target_padded"] = padded_targets(dt["video_target"], dt["video_tensor"].device)
        if "cap_tensor_cpu" not in dt:
            dt["cap_tensor_cpu"] = dt["cap_tensor"].detach().cpu()
        self.signature = self._signature(dt)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: lazy init, allocator pools, cached host->device bookkeeping
            for _ in range(warmup):
                self._zero_grad()
                self._forward_backward()
                if reducer is not None:
                    reducer.finish()
        torch.cuda.current_stream().wait_stream(side)
        self._zero_grad()
        # the captured hipGraph_t is kept (keep_graph) so that its memset nodes are rewritten as kernel nodes before
        # instantiation (replace_memsets: small captured memsets did not re-apply on replays);
        # debug_dot: also dumped by hipGraphDebugDotPrint for tools/diag_memset_graph.py
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        if debug_dot:
            self.graph.enable_debug_mode()
        from .precision import begin_capture
        begin_capture()  # bf16 mode: every operand rounding of the step becomes a node of the graph
        # data parallel: the capture records an event at each bucket's last gradient and every replay's all-reduces
        # wait on those on a side stream (overlapped with the rest of the replay), when this build can record
        # external events inside a capture; otherwise the reducer is suspended and finish() reduces after the replay
        self.overlap = reducer is not None and reducer.flats is not None and dp_overlap_supported()
        if self.overlap:
            reducer.begin_capture()
        elif reducer is not None:
            reducer.suspended = True
        # no garbage collection inside the capture.  Round 5 pinned the mechanism (tools/gc_capture_probe.py,
        # profiles/r05_gc_capture_probe.txt): a collection inside a capture that frees cyclic garbage holding
        # CUDA tensors, an eager autograd graph or events is harmless, but one that frees an unreachable
        # torch.cuda.CUDAGraph (an earlier test's StepGraph or trunk graph) runs ~CUDAGraph, whose hipGraph
        # destruction is refused while a stream captures (hipErrorStreamCaptureUnsupported, HIPGraph.cpp:324) and
        # throws from a destructor: std::terminate, SIGABRT -- round 4's pass-AC abort inside the step-graph capture
        # test, which ran after the model suites that leave such graphs behind.  torch.cuda.graph collects once on
        # entry; tests/test_gpu_capture_gc.py checks no collection starts inside the capture
        gc_enabled = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(self.graph):
                if reducer is not None and reducer.flats is not None:
                    reducer.zero_grad()  # every replay starts from zeroed buckets (a fill node per bucket)
                self.total, self.losses = self._forward_backward()
                if self.overlap:
                    reducer.end_capture()
                    # this graph's event-record nodes refer to these events: kept as long as the graph (a later
                    # capture with the same reducer makes its own, and destroying these would leave dangling nodes)
                    self.events = list(reducer.events)
        finally:
            if gc_enabled:
                gc.enable()
            if reducer is not None:
                reducer.suspended = False
                reducer.capturing = False
        if debug_dot:
            self.graph.debug_dump(debug_dot)
        # the captured outputs, detached: the storage is the graph's, but the autograd graph of the capture (and
        # through it the parameters' AccumulateGrad nodes, made on the capture stream) is released, so eager steps
        # after the capture build their own nodes on their own stream
        self.total = self.total.detach()
        self.losses = {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in self.losses.items()}
        self.memsets_replaced = replace_memsets(self.graph)
        self.node_counts = graph_node_counts(self.graph)  # the launches of one replay, by node type
        self.graph.instantiate()

    def _zero_grad(self):
        if self.reducer is not None:
            self.reducer.zero_grad()  # bucket views once the reducer knows its active set, else set to None
        else:
            self.model.zero_grad(set_to_none=True)

    def _forward_backward(self):
        out, loss = self.model(self.dt, self.criterion, self.tit)
        total = sum(loss[k] * self.wd[k] for k in loss.keys() if k in self.wd)
        total.backward()
        return total, loss

    @staticmethod
    def _signature(dt):
        """The host facts the captured step depends on: events per video and each video's caption step count
        (the reference's loop stops at the video's first all-zero token column, LSTM_DSA.py:88-104) -- or, for a
        capacity-padded batch (pdvc/batch_layout.py), only the capacities and the batch size."""
        from .CaptioningHead.LSTM_DSA import caption_steps
        from .caption_tokens import token_count
        if dt.get("capacity") is not None:
            c = dt["capacity"]
            return ("capacity", len(dt["video_target"]), c["events"], c["rows"], c["words"], c.get("tokens"),
                    tuple(c["alive"]) if c.get("alive") is not None else None)
        counts = [len(t["labels"]) for t in dt["video_target"]]
        cap = dt.get("cap_tensor_cpu")
        cap = dt["cap_tensor"].detach().cpu() if cap is None else cap
        off = [0]
        for c in counts:
            off.append(off[-1] + c)
        steps = [caption_steps(cap[off[v]:off[v + 1]]) for v in range(len(counts))]
        # the caption token count sizes the packed logit projection (pdvc/caption_tokens.py)
        mask = dt.get("cap_mask_cpu")
        mask = dt["cap_mask"].detach().cpu() if mask is None else mask
        return tuple(counts), tuple(steps), token_count(mask, max(steps, default=0))

    def load(self, dt):
        """Copy a batch of the captured shapes (same event and caption counts) into the graph's inputs: the
        features, masks, token rows and the padded targets the device matching reads.  Every copy is queued on
        the current stream behind the previous replay (device-to-device, or from pinned host memory), and the
        host facts come from the batch's host copies (data.to_device keeps them), so load() never waits for the
        GPU: the host prepares batch k + 1 while replay k runs."""
        if bool(dt.get("video_mask_all_valid", False)) != bool(self.dt.get("video_mask_all_valid", False)):
            raise ValueError("StepGraph.load: the batch's padding (video_mask_all_valid) differs from the captured "
                             "batch's; capture a graph for it")
        if "video_target" in dt:
            sig = self._signature(dt)
            if sig != self.signature:
                raise ValueError("StepGraph.load: the batch's event / caption-step counts differ from the captured "
                                 "batch's; capture a graph for it")
            from .matcher import padded_targets
            cap_events = (dt.get("capacity") or {}).get("events")
            new = dt.get("video_target_padded")  # made by data.to_device from the host copies of the targets
            if new is None or new.get("capacity") != cap_events:  # (from device targets: one sync per video)
                new = padded_targets(dt["video_target"], self.dt["video_tensor"].device, cap_events)
            old = self.dt["video_target_padded"]
            for k, v in new.items():
                if isinstance(v, torch.Tensor):
                    old[k].copy_(v, non_blocking=True)
            for k, rep in old.items():  # the per-layer repeats the criterion cached on the dict (repeat_targets)
                if isinstance(k, tuple) and k[0] == "repeat":
                    for kk, v in rep.items():
                        if isinstance(v, torch.Tensor):
                            v.copy_(new[kk].repeat(k[1], *([1] * (v.dim() - 1))), non_blocking=True)
            cpu = dt.get("cap_tensor_cpu")
            self.dt["cap_tensor_cpu"] = dt["cap_tensor"].detach().cpu() if cpu is None else cpu
            mcpu = dt.get("cap_mask_cpu")
            self.dt["cap_mask_cpu"] = dt["cap_mask"].detach().cpu() if mcpu is None else mcpu
            cap_tok = (dt.get("capacity") or {}).get("tokens")
            if cap_tok is not None:
                have = int(self.dt["cap_mask_cpu"][:, 1:dt["capacity"]["words"]].sum())
                if have > cap_tok:
                    raise ValueError(f"StepGraph.load: {have} caption tokens, capacity {cap_tok}")
            if dt.get("capacity") is not None:  # the caption rows' bookkeeping of the new counts
                from .batch_layout import caption_layout, live_rows, refresh_caption_layout
                from .pdvc import video_steps
                counts = [len(t["labels"]) for t in dt["video_target"]]
                cap = dt["capacity"]
                for k, cached in self.dt.items():
                    if isinstance(k, tuple) and k and k[0] == "_caption_rows":
                        _, Ld, N, Q, blocks = k
                        vsteps = None
                        if cached.get("ordered"):  # rows ordered by step count, within the captured live ranges
                            vsteps = video_steps(self.dt["cap_tensor_cpu"], counts)
                            live = live_rows(counts, vsteps, cap["words"] - 1)
                            if any(a > b for a, b in zip(live, cap["alive"])):
                                raise ValueError("StepGraph.load: the batch's live caption rows exceed the capacity")
                        refresh_caption_layout(cached, caption_layout(counts, Ld, N, Q, blocks, cap["rows"],
                                                                      cap["events"], steps=vsteps))
        for k, v in dt.items():
            dst = self.dt.get(k)
            if isinstance(v, torch.Tensor) and isinstance(dst, torch.Tensor) and dst.device.type == "cuda":
                if dst.shape != v.shape:
                    raise ValueError(f"StepGraph.load: {k} has shape {tuple(v.shape)}, captured {tuple(dst.shape)}")
                dst.copy_(v, non_blocking=True)

    def replay(self):
        self.graph.replay()
        if self.reducer is not None:
            if self.overlap:
                self.reducer.finish_replay(self.events)
            else:
                self.reducer.finish()
        return self.total
