"""Shape-stable batches: one captured step graph for a stream of ragged batches.

Everything the host decides in a PDVC training step depends on the batch's event counts and caption lengths
(pdvc.py `_caption_rows`, criterion.py `static_pairs`, LSTM_DSA.py `caption_steps`), so a step graph captured for
one batch (pdvc/step_graph.py) fits only batches with the same counts -- real data (data/video_dataset.py:15-149)
never repeats them.  A capacity-padded batch fixes every shape the graph sees:

  * events: the padded targets are `events` wide for every video (matcher.padded_targets(capacity=...)); the
    matching runs on the device with the true per-video counts, and the pairs of phantom targets are masked out
    of every loss (criterion.video_losses);
  * caption rows: each decoder layer's block holds `rows` rows -- the batch's sum(E_v) real rows (layer-major,
    video-major, as the unpadded batch orders them) then phantom rows, whose token row is all zero (cap_mask 0:
    loss 0, gradients 0) and which count for no video in the per-(layer, video) means;
  * caption steps: the recurrence runs `words - 1` steps for every batch (the reference stops each video's loop
    at its first all-zero token column, LSTM_DSA.py:103-104: the steps past it are masked in the loss, so the
    result is the same).

The row bookkeeping (which query, caption and video each row has) is recomputed on the host per batch --
numpy over the counts -- and copied into the captured index buffers by StepGraph.load, with the features, masks,
token rows and targets.  `pad_to_capacity(dt, events, rows, words)` turns a collated batch (data.collate or the
reference's collate_fn) into such a batch; the unpadded batch and its padded form give the same losses and
gradients (tests/test_gpu_batch.py).
"""
import numpy as np
import torch

from . import hostio


def _rows_per_layer(counts, rows_cap):
    tot = int(sum(counts))
    if rows_cap is None:
        return tot, tot
    if tot > rows_cap:
        raise ValueError(f"batch has {tot} caption rows per decoder layer, capacity {rows_cap}")
    return tot, int(rows_cap)


def caption_layout(counts, Ld, N, Q, blocks, rows_cap=None, events_cap=None, steps=None):
    """Host bookkeeping of the caption rows of every (decoder layer, video, event), layer-major (pdvc.py
    `_caption_rows`).  counts: events per video; blocks: the matching block of each layer (LazyIndices.block);
    rows_cap: rows per layer block (None: exactly sum(counts), no phantom rows).
    steps: each video's caption step count (its teacher-forced loop length, LSTM_DSA.py:103-104), or None.  Without
    it the rows of a layer are video-major.  With it (and Ld <= 2) the rows of each layer are ordered by their video's
    steps so that the rows still running at any step form ONE contiguous range (step_ranges): layer 0 by ascending
    steps with its phantom rows first, layer 1 by descending steps with its phantom rows last -- the live rows of step
    t are the last a_t of layer 0 and the first a_t of layer 1.
    Returns numpy arrays of length Ld * rows: problem p, rank k, hs base row, caption row base, video, layer,
    valid (0 for phantom rows); last_sel: the last layer's rows in video-major order (phantom rows after); the
    per-video CSR of the real rows (start, rows) and its largest per-video row count (a bound from events_cap for a
    capacity-padded batch)."""
    counts = [int(c) for c in counts]
    tot, R = _rows_per_layer(counts, rows_cap)
    cap_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    vid_real = np.repeat(np.arange(N, dtype=np.int64), counts)
    rank_real = np.arange(tot, dtype=np.int64) - cap_off[vid_real]
    pad = R - tot
    ordered = steps is not None and Ld <= 2
    if ordered:
        st = np.asarray(steps, np.int64)[vid_real]
    parts = {k: [] for k in ("p", "k", "base", "cap", "vid", "lay", "valid")}
    pos_real = []  # per layer: global position of the real rows, in video-major order
    for l_id in range(Ld):
        b = int(blocks[l_id])
        asc = ordered and Ld == 2 and l_id == 0
        if ordered:
            perm = np.argsort(st if asc else -st, kind="stable")
        else:
            perm = np.arange(tot, dtype=np.int64)
        vr, rk = vid_real[perm], rank_real[perm]
        real = {"p": b * N + vr, "k": rk, "base": (l_id * N + vr) * Q, "cap": cap_off[vr], "vid": vr,
                "lay": np.full(tot, l_id, np.int64), "valid": np.ones(tot, np.int64)}
        # a phantom row reads caption row `tot` (an all-zero row of the padded cap_tensor) and rank 0 of the
        # layer's first problem; its target offset is multiplied by valid = 0
        phantom = {"p": np.full(pad, b * N, np.int64), "k": np.zeros(pad, np.int64),
                   "base": np.full(pad, l_id * N * Q, np.int64), "cap": np.full(pad, tot, np.int64),
                   "vid": np.zeros(pad, np.int64), "lay": np.full(pad, l_id, np.int64),
                   "valid": np.zeros(pad, np.int64)}
        first, second = (phantom, real) if asc else (real, phantom)
        for k in parts:
            parts[k] += [first[k], second[k]]
        where = np.empty(tot, np.int64)
        where[perm] = l_id * R + (pad if asc else 0) + np.arange(tot, dtype=np.int64)
        pos_real.append(where)
    out = {k: np.concatenate(v) if v else np.zeros(0, np.int64) for k, v in parts.items()}
    if Ld:
        lp = (Ld - 1) * R + tot + np.arange(pad, dtype=np.int64)  # the last layer's phantom rows come last
        out["last_sel"] = np.concatenate([pos_real[-1], lp])
    else:
        out["last_sel"] = np.zeros(0, np.int64)
    # per-video CSR of the real rows (the caption value gradient sums each video's rows in one pass)
    rows_of_video = [np.concatenate([pos_real[l_id][cap_off[v]:cap_off[v + 1]] for l_id in range(Ld)])
                     if counts[v] else np.zeros(0, np.int64) for v in range(N)]
    start = np.concatenate([[0], np.cumsum([len(r) for r in rows_of_video])]).astype(np.int64)
    flat = np.concatenate(rows_of_video) if rows_of_video else np.zeros(0, np.int64)
    if rows_cap is not None:  # a fixed-size buffer: the real rows, then zeros
        flat = np.concatenate([flat, np.zeros(Ld * R - len(flat), np.int64)])
    out["vr_start"], out["vr_rows"] = start, flat
    out["max_rows"] = Ld * (int(events_cap) if events_cap is not None else max(counts, default=0))
    out["rows_per_layer"], out["real_rows"] = R, tot
    out["ordered"] = ordered
    return out


def live_rows(counts, steps, n_steps):
    """Real caption rows per decoder layer still running at each step t < n_steps: sum of counts[v] over the
    videos with steps[v] > t."""
    c = np.asarray(counts, np.int64)
    s = np.asarray(steps, np.int64)
    return [int(c[s > t].sum()) for t in range(n_steps)]


def step_ranges(live, Ld, R):
    """(start, count) of the rows of each step for a caption_layout(..., steps=...) ordering: the live rows of
    Ld = 2 are [R - a_t, R + a_t), of Ld = 1 [0, a_t)."""
    live = [int(a) for a in live]
    if any(b > a for a, b in zip(live, live[1:])) or any(a < 0 or a > R for a in live):
        raise ValueError("step_ranges: live rows must be non-increasing and within the layer's rows")
    if Ld == 2:
        return tuple((R - a, 2 * a) for a in live)
    if Ld == 1:
        return tuple((0, a) for a in live)
    raise ValueError("step ranges need 1 or 2 decoder layers")


def pad_to_capacity(dt, events, rows, words, tokens=None, alive=None):
    """A collated batch (host tensors) padded to fixed shapes: every caption token row `words` wide, `rows + 1`
    caption rows (the real ones first, then all-zero rows; `rows` >= the batch's sum of events), `events` targets
    per video in the padded targets (to_device builds them), and dt["capacity"] recording them.  tokens: the
    loss-carrying caption tokens per decoder layer the stream's batches may hold (>= this batch's sum of
    cap_mask[:, 1:], pdvc/caption_tokens.py); the logit projection runs over that many token rows.  None: no
    packing (every (row, step) position).  alive: per step t < words - 1, the caption rows per decoder layer the
    stream's batches may still run at step t (>= live_rows of this batch); the recurrence then runs each step over
    that many rows per layer (pdvc.py `_caption_rows`).  None: every row runs every step."""
    cap = dt["cap_tensor"]
    tot, K = cap.shape
    counts = [len(t["labels"]) for t in dt["video_target"]]
    if tot != sum(counts):
        raise ValueError("pad_to_capacity: cap_tensor rows differ from the events of the targets")
    if K > words:
        raise ValueError(f"pad_to_capacity: captions {K} tokens wide, capacity {words}")
    if max(counts, default=0) > events:
        raise ValueError(f"pad_to_capacity: a video has {max(counts)} events, capacity {events}")
    if tot > rows:
        raise ValueError(f"pad_to_capacity: {tot} caption rows, capacity {rows}")
    if tokens is None:
        tokens = rows * (words - 1)
    have = int(dt["cap_mask"][:, 1:words].sum())
    if have > tokens:
        raise ValueError(f"pad_to_capacity: {have} caption tokens, capacity {tokens}")
    out = dict(dt)
    c = torch.zeros(rows + 1, words, dtype=cap.dtype)
    c[:tot, :K] = cap
    m = torch.zeros(rows + 1, words, dtype=dt["cap_mask"].dtype)
    m[:tot, :K] = dt["cap_mask"]
    out["cap_tensor"], out["cap_mask"] = c, m
    for k in ("cap_length", "gt_gather_idx"):  # per-caption vectors
        if k in dt:
            v = torch.zeros(rows + 1, dtype=dt[k].dtype)
            v[:tot] = dt[k]
            out[k] = v
    if "gt_boxes" in dt:
        gb = torch.zeros(dt["gt_boxes"].shape[0], events, 2, dtype=dt["gt_boxes"].dtype)
        gb[:, :dt["gt_boxes"].shape[1]] = dt["gt_boxes"]
        out["gt_boxes"] = gb
        out["gt_boxes_mask"] = (gb != 0).sum(2) > 0
    if alive is not None:
        alive = tuple(int(a) for a in alive)
        if len(alive) != words - 1:
            raise ValueError(f"pad_to_capacity: alive needs {words - 1} steps, got {len(alive)}")
        if any(b > a for a, b in zip(alive, alive[1:])) or min(alive, default=0) < 0:
            # each step's rows must be nested in the previous step's (CaptionDecodeFunction reads step t - 1's
            # state for every row of step t): a row entering a range late would read state never written
            raise ValueError("pad_to_capacity: alive must be non-increasing and non-negative")
        from .CaptioningHead.LSTM_DSA import caption_steps
        o, steps = 0, []
        for c_ in counts:
            steps.append(caption_steps(cap[o:o + c_]) if c_ else 0)
            o += c_
        have = live_rows(counts, steps, words - 1)
        if any(h > a for h, a in zip(have, alive)) or max(alive, default=0) > rows:
            raise ValueError("pad_to_capacity: live caption rows exceed the alive capacity")
    out["capacity"] = {"events": int(events), "rows": int(rows), "words": int(words), "tokens": int(tokens),
                       "alive": alive}
    return out


_DEVICE_KEYS = ("p", "k", "base", "cap", "vid", "lay", "valid", "last_sel", "vr_start", "vr_rows")


def caption_layout_to_device(lay, device):
    """The layout's index arrays as device tensors (one host->device copy), plus its host facts."""
    ts = hostio.pack_to_device([lay[k] for k in _DEVICE_KEYS], device)
    out = dict(zip(_DEVICE_KEYS, ts))
    out["max_rows"], out["rows_per_layer"], out["real_rows"] = lay["max_rows"], lay["rows_per_layer"], lay["real_rows"]
    out["rows_host"] = list(zip(lay["lay"].tolist(), lay["vid"].tolist()))
    out["last_sel_host"] = lay["last_sel"].tolist()
    out["ordered"] = lay.get("ordered", False)
    return out


def refresh_caption_layout(cached, lay):
    """Copy a new batch's layout (same capacity) into the device tensors of a cached one (StepGraph.load)."""
    for k in _DEVICE_KEYS:
        src = torch.from_numpy(np.ascontiguousarray(lay[k]))
        dst = cached[k]
        if tuple(src.shape) != tuple(dst.shape):
            raise ValueError(f"caption layout {k}: {tuple(src.shape)} vs captured {tuple(dst.shape)}")
        # pinned and asynchronous: queued behind the previous replay, which still reads dst (the caching host
        # allocator keeps the pinned block until the copy has run)
        dst.copy_(src.to(dst.dtype).pin_memory(), non_blocking=True)
    cached["real_rows"] = lay["real_rows"]
    cached["rows_host"] = list(zip(lay["lay"].tolist(), lay["vid"].tolist()))
    cached["last_sel_host"] = lay["last_sel"].tolist()
