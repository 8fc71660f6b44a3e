"""Deterministic, name-keyed parameter fill and synthetic-input builders shared by the golden
fixture generator (make_golden.py, which drives the *reference* model) and the parity tests (which
drive ours).  Weights are a pure function of (parameter name, shape), so fixtures never have to
store multi-megabyte state dicts: both sides fill identical weights into identically named params.
"""
import zlib

import numpy as np


def param_array(name, shape, scale=None):
    """Uniform(-s, s) with s = scale or 1/sqrt(fan_in); seeded by crc32(name)."""
    rng = np.random.RandomState(zlib.crc32(name.encode()) & 0x7FFFFFFF)
    shape = tuple(int(s) for s in shape)
    if scale is None:
        fan_in = shape[-1] if len(shape) > 1 else max(shape[0], 1)
        scale = 1.0 / np.sqrt(fan_in)
    if name.endswith("level_embed"):
        scale = 1.0
    if "norm" in name and name.endswith("weight"):
        return (1.0 + 0.1 * rng.uniform(-1, 1, size=shape)).astype(np.float32)
    return rng.uniform(-scale, scale, size=shape).astype(np.float32)


def fill_module(module, overrides=None):
    """Fill every parameter of a torch module in-place from param_array (torch imported lazily)."""
    import torch
    overrides = overrides or {}
    with torch.no_grad():
        for name, p in module.named_parameters():
            scale = None
            for key, s in overrides.items():
                if key in name:
                    scale = s
            p.copy_(torch.from_numpy(param_array(name, p.shape, scale)))


def synthetic_video_batch(n_videos, T, C, n_events, n_words, vocab, duration=120.0, seed=0):
    """Inputs in the reference collate_fn format (data/video_dataset.py:15-149, `batch` tuples):
    (feature (T,C), gt_featstamps, labels, captions, gt_raw_timestamps, raw_duration, raw_caption, key).
    Captions are [0] + randint(1, vocab) * n_words + [0] (0 = BOS/EOS), SURVEY.md section 8(d)."""
    rng = np.random.RandomState(seed)
    batch = []
    for v in range(n_videos):
        feat = rng.randn(T, C).astype(np.float32)
        ne = n_events[v] if isinstance(n_events, (list, tuple)) else n_events
        ts = np.sort(rng.uniform(0, duration, size=(ne, 2)), axis=1)
        # guarantee a non-degenerate length for every event
        ts[:, 1] = np.maximum(ts[:, 1], ts[:, 0] + 1.0)
        ts = np.minimum(ts, duration)
        nw = n_words[v] if isinstance(n_words, (list, tuple)) else n_words
        caps = []
        for e in range(ne):
            w = max(1, nw - (e % 3))  # ragged caption lengths
            caps.append(np.array([0] + list(rng.randint(1, vocab, size=w)) + [0], dtype=np.int64))
        featstamps = [[t[0] / duration * T, t[1] / duration * T] for t in ts]
        batch.append((feat, featstamps, [0] * ne, caps, [list(t) for t in ts], duration,
                      ["w"] * ne, f"v_{seed}_{v}"))
    return batch


def batch_items(seed=21, C=32, vocab=29):
    """Three videos in the reference collate_fn tuple format (data/video_dataset.py:15-149) with different
    event counts (2, 3, 5), caption lengths and durations; video 1 has 12 frames, so in a batch of 16-frame
    videos its mask is padded (False) over the last 4 frames."""
    rng = np.random.RandomState(seed)
    spec = [(16, [5, 2], 120.0), (12, [3, 6, 4], 90.0), (16, [6, 3, 1, 5, 4], 150.0)]
    items = []
    for v, (Tv, words, dur) in enumerate(spec):
        feat = rng.randn(Tv, C).astype(np.float32)
        ne = len(words)
        ts = np.sort(rng.uniform(0, dur, size=(ne, 2)), axis=1)
        ts[:, 1] = np.minimum(np.maximum(ts[:, 1], ts[:, 0] + 1.0), dur)
        caps = [np.array([0] + list(rng.randint(1, vocab, size=w)) + [0], dtype=np.int64) for w in words]
        stamps = [[t[0] / dur * Tv, t[1] / dur * Tv] for t in ts]
        items.append((feat, stamps, [0] * ne, caps, [list(t) for t in ts], dur, ["w"] * ne, f"b3_{v}"))
    return items


def dp_items(vocab=29):
    """Four videos for the data-parallel equivalence test: batch_items' three plus a fourth 16-frame video;
    split over 2 ranks as [0, 1] and [2, 3], every rank's batch pads to the union's 16 frames."""
    return batch_items(seed=21, vocab=vocab) + batch_items(seed=22, vocab=vocab)[2:]
