"""Input contract of PDVC.forward: the `dt` dict of the reference collate_fn
(data/video_dataset.py:15-149), plus synthetic videos of the BASELINE shapes.

`collate(batch)` builds the same keys from per-video tuples
(feature (T,C), gt_featstamps, labels, captions, gt_raw_timestamps, raw_duration, raw_caption, key);
`synthetic_videos(...)` makes such tuples: features ~ N(0,1), E events with sorted uniform timestamps in
[0, duration), labels 0, captions [0] + randint(1, vocab) * w + [0].  `to_device` moves a dt to the GPU
and keeps a host copy of the caption tokens (the caption loop length is decided on the host).
"""
from itertools import chain

import numpy as np
import torch


def collate(batch):
    B = len(batch)
    feats, _stamps, labels, captions, raw_ts, durations, _raw_caps, keys = zip(*batch)
    C = feats[0].shape[1]
    T = max(f.shape[0] for f in feats)
    max_cap = max(chain(*[[len(c) for c in caps] for caps in captions]))
    n_caps = sum(len(c) for c in captions)
    max_ev = max(len(c) for c in captions)
    video = torch.zeros(B, T, C)
    length = torch.zeros(B, 3)
    vmask = torch.zeros(B, T, dtype=torch.bool)
    cap = torch.zeros(n_caps, max_cap, dtype=torch.long)
    cap_len = torch.zeros(n_caps, dtype=torch.long)
    cap_mask = torch.zeros(n_caps, max_cap, dtype=torch.bool)
    gather = torch.zeros(n_caps, dtype=torch.long)
    gt_boxes = torch.zeros(B, max_ev, 2)
    row = 0
    targets = []
    for v in range(B):
        n = feats[v].shape[0]
        ne = len(raw_ts[v])
        video[v, :n] = torch.from_numpy(np.asarray(feats[v], dtype=np.float32))
        length[v] = torch.tensor([float(n), float(durations[v]), float(ne)])
        vmask[v, :n] = True
        gather[row:row + ne] = v
        boxes = torch.tensor([[(t[1] + t[0]) / (2 * durations[v]), (t[1] - t[0]) / durations[v]]
                              for t in raw_ts[v]]).float()
        gt_boxes[v, :ne] = boxes
        for e, c in enumerate(captions[v]):
            cap_len[row + e] = len(c)
            cap[row + e, :len(c)] = torch.from_numpy(np.asarray(c, dtype=np.int64))
            cap_mask[row + e, :len(c)] = True
        row += ne
        targets.append({"boxes": boxes, "labels": torch.tensor(labels[v]).long(), "masks": None,
                        "image_id": keys[v]})
    return {"video_tensor": video, "video_length": length, "video_mask": vmask, "video_key": list(keys),
            # host-side fact of the batch: no padded frame anywhere (the kernels then skip the padding mask)
            "video_mask_all_valid": bool(vmask.all()),
            "video_target": targets, "gt_featstamps": list(chain(*_stamps)), "gt_timestamp": list(raw_ts),
            "gt_gather_idx": gather, "gt_boxes": gt_boxes, "gt_boxes_mask": (gt_boxes != 0).sum(2) > 0,
            "cap_tensor": cap, "cap_length": cap_len, "cap_mask": cap_mask, "cap_raw": list(_raw_caps)}


def synthetic_videos(n_videos, T, C, n_events, n_words, vocab, duration=120.0, seed=0):
    rng = np.random.RandomState(seed)
    out = []
    for v in range(n_videos):
        feat = rng.standard_normal((T, C)).astype(np.float32)
        ts = np.sort(rng.uniform(0, duration, size=(n_events, 2)), axis=1)
        ts[:, 1] = np.minimum(np.maximum(ts[:, 1], ts[:, 0] + 1.0), duration)
        caps = [np.array([0] + list(rng.randint(1, vocab, size=n_words)) + [0], dtype=np.int64)
                for _ in range(n_events)]
        stamps = [[t[0] / duration * T, t[1] / duration * T] for t in ts]
        out.append((feat, stamps, [0] * n_events, caps, [list(t) for t in ts], duration, ["w"] * n_events,
                    f"syn_{seed}_{v}"))
    return out


def to_device(dt, device):
    out = {}
    for k, v in dt.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.to(device, non_blocking=True)
        elif k == "video_target":
            out[k] = [{kk: (vv.to(device) if isinstance(vv, torch.Tensor) else vv) for kk, vv in t.items()}
                      for t in v]
        else:
            out[k] = v
    out["cap_tensor_cpu"] = dt["cap_tensor"].clone()
    out["cap_mask_cpu"] = dt["cap_mask"].clone()  # the caption token count (pdvc/caption_tokens.py)
    from .matcher import padded_targets
    cap = dt.get("capacity")  # a capacity-padded batch (pdvc/batch_layout.py): targets padded to its event capacity
    out["video_target_padded"] = padded_targets(dt["video_target"], device,
                                                None if cap is None else cap["events"])  # from the host copies
    return out
