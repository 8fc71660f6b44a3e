"""Data-parallel training over RCCL (torch.distributed backend 'nccl' on ROCm) -- new functionality: the
reference trains PDVC on one device only (train.py never wraps the model).

Videos shard naturally: every rank runs its own videos through the whole step and the only exchange is the
gradient average.  GradAllReducer packs gradients into ~bucket_mb flat buckets in reverse registration order
(roughly the order backward produces them) and launches each bucket's all-reduce as soon as its last
gradient is accumulated, so communication overlaps the rest of the backward pass; buckets are launched
strictly in index order so every rank issues the same collective sequence.  Parameters that never receive a
gradient (8 in PDVC: transformer.pos_trans*, and the caption head's unused attention_weights/output_proj,
SURVEY.md section 8(e)) are detected on the first step and excluded, keeping `grad is None` as in the
reference.  A parameter found active on the first step whose gradient is None on a later step (a branch
not taken on this rank) contributes zeros, so every rank still issues the same collectives, and receives the
rank mean like every other.  Semantics: after finish(), every active gradient is the mean over ranks.

Bucket-resident gradients (torch DDP's gradient_as_bucket_view): after the first finish() every active
parameter's `.grad` IS a view into its bucket's flat buffer.  A step that zeroes through `zero_grad()` (one fill
per bucket, no set-to-None) keeps the views: backward's AccumulateGrad adds into them in place, and finish() is one
all-reduce and one scale per bucket -- no concatenation, no copy back.  A caller that sets the gradients to None
instead still gets the right result: a gradient that is not the bucket's view is copied into its slot at launch
and the view is re-bound after the reduce (`copies` counts those copies; 0 on the resident path).

Under a captured step (pdvc/step_graph.py) no host code runs during the backward, so the hooks cannot launch the
collectives.  Instead the capture records an external event at each bucket's last gradient (begin_capture /
end_capture: an event-record node of the graph), and after every replay finish_replay() queues bucket b's
all-reduce on a side stream behind event b: the reduction of the buckets the backward finishes first runs while
the replay is still computing the rest (the overlap torch DDP gets from its hooks in an eager step).
"""
import ctypes
import os

import torch
import torch.distributed as dist


class GraphEvent:
    """A HIP event that a captured graph records for streams outside it (csrc/graphfix.hip: hipEventRecordExternal
    -- torch's ROCm build refuses torch.cuda.Event(external=True)).  record() on a capturing stream adds an
    event-record node that every replay executes; wait(stream) queues a wait for the latest record."""

    def __init__(self):
        from pdvc import _native as _n
        self._n = _n
        h = ctypes.c_void_p()
        _n.call("pdvc_event_create", ctypes.addressof(h))
        self.handle = h

    def record(self, stream=None, captured=False):
        """captured=True: an error unless the stream is capturing (pdvc_event_record_captured) -- the reducer's
        bucket records, which would otherwise be plain records that every replay's all-reduce races past."""
        s = stream if stream is not None else torch.cuda.current_stream()
        fn = "pdvc_event_record_captured" if captured else "pdvc_event_record_external"
        self._n.call(fn, self.handle, ctypes.c_void_p(s.cuda_stream))

    def wait(self, stream):
        self._n.call("pdvc_stream_wait_event", ctypes.c_void_p(stream.cuda_stream), self.handle)

    def __del__(self):
        try:
            self._n.call("pdvc_event_destroy", self.handle)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


def _graph_event():
    return GraphEvent()


def init_distributed(backend=None):
    """Initialise from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).  Returns
    (rank, world_size, local_rank); world_size 1 without initialisation when not launched distributed."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, init_method="env://")
    return rank, world, local


def broadcast_parameters(module, src=0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        with torch.no_grad():
            for t in list(module.parameters()) + list(module.buffers()):
                dist.broadcast(t.data, src)


class GradAllReducer:
    def __init__(self, params, bucket_mb=25.0, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        seen, uniq = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        self.bucket_bytes = int(bucket_mb * 1024 * 1024)
        self.active = None  # params known to receive gradients (set after the first step)
        self.suspended = False  # True while a step graph is captured: finish() then reduces every bucket
        self.flats = None  # one flat buffer per bucket once the active set is known
        self.copies = 0  # gradients copied into a bucket (not resident); stays 0 when zero_grad() is used
        self.capturing = False  # inside begin_capture() .. end_capture(): bucket completions record events
        self.events = None  # one external event per bucket, recorded by the captured step (finish_replay)
        self._side = None
        self._hooks = []
        self._build(self.params)

    # ------------------------------------------------------------------------------------------------
    def _build(self, params):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        # buckets by (dtype, device) -- a bucket's flat buffer has one dtype -- each filled in reverse registration
        # order up to bucket_bytes; the kinds in order of first appearance, so every rank builds the same sequence
        self.buckets = []
        open_ = {}  # (dtype, device) -> [params, bytes]
        for p in reversed(params):
            key = (p.dtype, p.device)
            nbytes = p.numel() * p.element_size()
            cur = open_.get(key)
            if cur is not None and cur[0] and cur[1] + nbytes > self.bucket_bytes:
                self.buckets.append(cur[0])
                cur = None
            if cur is None:
                cur = open_[key] = [[], 0]
            cur[0].append(p)
            cur[1] += nbytes
        for cur in open_.values():
            if cur[0]:
                self.buckets.append(cur[0])
        self.bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.bucket_of[id(p)] = bi
        for p in params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset()

    def _make_flats(self):
        """One flat buffer per bucket (dtype and device of its parameters) and each parameter's view into it."""
        self.flats, self.views = [], {}
        for b in self.buckets:
            flat = torch.zeros(sum(p.numel() for p in b), dtype=b[0].dtype, device=b[0].device)
            off = 0
            for p in b:
                n = p.numel()
                self.views[id(p)] = flat[off:off + n].view_as(p)
                off += n
            self.flats.append(flat)

    def _resident(self, p):
        v = self.views[id(p)]
        return p.grad is not None and p.grad.data_ptr() == v.data_ptr() and p.grad.shape == v.shape

    def _reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.next_launch = 0
        self.works = []  # (bucket index, flat, work)

    def zero_grad(self):
        """Zero every bucket (one fill each) and bind the active parameters' gradients to their views; the next
        backward accumulates into the buckets in place.  Before the first finish() this is zero_grad(set_to_none)."""
        if self.flats is None:
            for p in self.params:
                p.grad = None
            return
        for f in self.flats:
            f.zero_()
        for p in self.active:
            if not self._resident(p):
                p.grad = self.views[id(p)]
        for p in self.params:  # outside the active set (no gradient on the first step): never reduced, so never
            if id(p) not in self.bucket_of:  # left to accumulate across steps either
                p.grad = None

    def _on_grad(self, p):
        bi = self.bucket_of.get(id(p))
        if bi is None or self.suspended:
            return
        self.pending[bi] -= 1
        if self.capturing:  # the bucket's gradients are final at this point of the captured stream
            if self.pending[bi] == 0:
                self.events[bi].record(captured=True)
                self._recorded[bi] = True
            return
        if self.active is not None:
            while self.next_launch < len(self.buckets) and self.pending[self.next_launch] == 0:
                self._launch(self.next_launch)
                self.next_launch += 1

    def _launch(self, bi):
        flat = self.flats[bi]
        for p in self.buckets[bi]:  # gradients that are not the bucket's views (set to None, or missing)
            if not self._resident(p):
                v = self.views[id(p)]
                if p.grad is None:
                    v.zero_()
                else:
                    v.copy_(p.grad)
                    self.copies += 1
        work = dist.all_reduce(flat, group=self.group, async_op=True)
        self.works.append((bi, flat, work))

    def finish(self):
        """Wait for (and, on the first step, issue) every bucket's all-reduce; the rank mean is left in the
        buckets, which every active .grad views afterwards."""
        if self.active is None:
            # first step: learn which params get gradients (identical on every rank), rebuild, reduce now
            self.active = [p for p in self.params if p.grad is not None]
            self._build(self.active)
            self._make_flats()
            for bi in range(len(self.buckets)):
                self._launch(bi)
        else:
            while self.next_launch < len(self.buckets):
                self._launch(self.next_launch)
                self.next_launch += 1
        inv = 1.0 / self.world
        for bi, flat, work in self.works:
            work.wait()
            flat.mul_(inv)
            for p in self.buckets[bi]:
                if not self._resident(p):
                    p.grad = self.views[id(p)]
        self._reset()

    # ---- captured steps ----------------------------------------------------------------------------
    def begin_capture(self):
        """Before capturing a step that ends with the buckets' gradients (after a finish(): the active set and
        the flat buffers exist): bucket completions inside the capture record one external event each."""
        assert self.flats is not None, "begin_capture() after the first finish()"
        self.events = [_graph_event() for _ in self.buckets]
        self._recorded = [False] * len(self.buckets)
        self._reset()
        self.capturing = True

    def end_capture(self):
        """Inside the capture, after the backward: a bucket left open by a gradient that did not arrive (a branch
        not taken in the captured step) records its event here, where every gradient of the step is final."""
        for bi, ev in enumerate(self.events):
            if not self._recorded[bi]:
                ev.record(captured=True)
        self.capturing = False
        self._reset()

    def finish_replay(self, events=None):
        """After a replay of a step captured between begin_capture() and end_capture(): every bucket's all-reduce
        in index order on a side stream, each behind its event, so a bucket is reduced as soon as the replay has
        produced it; then the current stream waits for them and the rank mean is scaled in.  events: the ones that
        graph's capture recorded (StepGraph keeps them; a later capture with this reducer makes new ones)."""
        events = self.events if events is None else events
        if self._side is None:
            self._side = torch.cuda.Stream()
        works = []
        with torch.cuda.stream(self._side):
            for bi, flat in enumerate(self.flats):
                events[bi].wait(self._side)
                works.append((flat, dist.all_reduce(flat, group=self.group, async_op=True)))
        inv = 1.0 / self.world
        for flat, work in works:
            work.wait()  # the current stream waits for the collective (and the side stream's position)
            flat.mul_(inv)
        torch.cuda.current_stream().wait_stream(self._side)
