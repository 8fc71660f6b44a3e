"""Host logic of capacity-padded batches (pdvc/batch_layout.py), CPU only: the caption-row layout against the
per-row loop it replaced (pdvc.py `_caption_rows` up to round 2), phantom rows, pad_to_capacity, and the
criterion's static pairs at a capacity."""
import numpy as np
import pytest
import torch

from pdvc.batch_layout import caption_layout, pad_to_capacity


def legacy_rows(counts, Ld, N, Q, blocks):
    """The round-2 loop: for every layer, video and event: (problem, rank, hs base, caption base, video, layer)."""
    cap_off = [0]
    for g in counts:
        cap_off.append(cap_off[-1] + g)
    rows, r_p, r_k, r_base, r_cap = [], [], [], [], []
    for l_id in range(Ld):
        for v in range(N):
            for k in range(counts[v]):
                rows.append((l_id, v))
                r_p.append(blocks[l_id] * N + v)
                r_k.append(k)
                r_base.append((l_id * N + v) * Q)
                r_cap.append(cap_off[v])
    by_video = [[] for _ in range(N)]
    for i, r in enumerate(rows):
        by_video[r[1]].append(i)
    start = [0]
    for v in range(N):
        start.append(start[-1] + len(by_video[v]))
    flat = [i for v in range(N) for i in by_video[v]]
    return rows, r_p, r_k, r_base, r_cap, start, flat, max((len(b) for b in by_video), default=0)


@pytest.mark.parametrize("counts", [[2, 3, 5], [1], [4, 0, 7, 1], [3] * 9])
@pytest.mark.parametrize("Ld", [1, 2, 3])
def test_exact_layout_equals_the_row_loop(counts, Ld):
    N, Q = len(counts), 10
    blocks = [(l + 1) % Ld for l in range(Ld)]  # aux layers 1.., the last layer block 0 (criterion.forward)
    rows, r_p, r_k, r_base, r_cap, start, flat, mx = legacy_rows(counts, Ld, N, Q, blocks)
    lay = caption_layout(counts, Ld, N, Q, blocks)
    assert lay["p"].tolist() == r_p and lay["k"].tolist() == r_k
    assert lay["base"].tolist() == r_base and lay["cap"].tolist() == r_cap
    assert list(zip(lay["lay"].tolist(), lay["vid"].tolist())) == rows
    assert lay["vr_start"].tolist() == start and lay["vr_rows"].tolist() == flat and lay["max_rows"] == mx
    assert lay["valid"].tolist() == [1] * len(rows)
    assert lay["last_sel"].tolist() == [i for i, r in enumerate(rows) if r[0] == Ld - 1]


@pytest.mark.parametrize("counts,cap", [([2, 3, 5], 12), ([1, 1], 5), ([4, 0, 7, 1], 16)])
def test_capacity_layout_keeps_the_real_rows_and_adds_phantoms(counts, cap):
    N, Q, Ld = len(counts), 10, 2
    blocks = [1, 0]
    ex = caption_layout(counts, Ld, N, Q, blocks)
    lay = caption_layout(counts, Ld, N, Q, blocks, rows_cap=cap, events_cap=max(counts) + 2)
    tot = sum(counts)
    for l_id in range(Ld):
        real = slice(l_id * cap, l_id * cap + tot)
        phantom = slice(l_id * cap + tot, (l_id + 1) * cap)
        for k in ("p", "k", "base", "cap", "vid", "lay"):
            assert lay[k][real].tolist() == ex[k][l_id * tot:(l_id + 1) * tot].tolist(), k
        assert (lay["valid"][real] == 1).all() and (lay["valid"][phantom] == 0).all()
        assert (lay["cap"][phantom] == tot).all(), "phantom rows read the all-zero caption row"
        assert (lay["lay"][phantom] == l_id).all()
    assert lay["last_sel"].tolist() == list(range((Ld - 1) * cap, Ld * cap))
    # the CSR lists exactly the real rows, video by video, at their capacity positions
    n_real = int(lay["vr_start"][-1])
    assert n_real == Ld * tot and len(lay["vr_rows"]) == Ld * cap
    real_rows = sorted(lay["vr_rows"][:n_real].tolist())
    assert real_rows == sorted(i for i in range(Ld * cap) if lay["valid"][i])
    assert lay["max_rows"] == Ld * (max(counts) + 2)
    with pytest.raises(ValueError):
        caption_layout(counts, Ld, N, Q, blocks, rows_cap=tot - 1)


def test_pad_to_capacity():
    from pdvc.data import collate, synthetic_videos
    dt = collate(synthetic_videos(3, 16, 8, 4, 5, 30, seed=1))
    p = pad_to_capacity(dt, events=6, rows=20, words=11)
    assert p["cap_tensor"].shape == (21, 11) and p["cap_mask"].shape == (21, 11)
    tot, K = dt["cap_tensor"].shape
    assert torch.equal(p["cap_tensor"][:tot, :K], dt["cap_tensor"]) and not p["cap_tensor"][tot:].any()
    assert not p["cap_tensor"][:, K:].any() and not p["cap_mask"][tot:].any()
    assert p["gt_boxes"].shape == (3, 6, 2) and p["capacity"] == {"events": 6, "rows": 20, "words": 11, "tokens": 200, "alive": None}
    for bad in (dict(events=3, rows=20, words=11), dict(events=6, rows=11, words=11),
                dict(events=6, rows=20, words=K - 1)):
        with pytest.raises(ValueError):
            pad_to_capacity(dt, **bad)


def test_static_pairs_at_capacity():
    from pdvc.criterion import static_pairs
    sizes = [2, 0, 3]
    pt = {"sizes": sizes, "sizes_long": torch.tensor(sizes), "capacity": 4}
    pp, pk, nm, emax = static_pairs(pt)
    assert emax == 4 and pp.tolist() == [0] * 4 + [1] * 4 + [2] * 4 and pk.tolist() == list(range(4)) * 3
    valid = (pk < nm[pp]).tolist()
    assert valid == [True, True, False, False] + [False] * 4 + [True, True, True, False]


@pytest.mark.parametrize("Ld,rows_cap", [(2, None), (2, 40), (1, None), (1, 33)])
def test_step_ordered_layout_keeps_live_rows_contiguous(Ld, rows_cap):
    """caption_layout(..., steps=...): the same rows as the video-major layout, reordered so that the rows of the
    videos still running at each step are exactly step_ranges' range; last_sel lists the last layer video-major and
    the CSR still names each video's rows."""
    from pdvc.batch_layout import caption_layout, live_rows, step_ranges
    rng = np.random.RandomState(3)
    N, Q = 7, 20
    counts = [int(c) for c in rng.randint(0, 6, N)]
    steps = [int(s) for s in rng.randint(1, 12, N)]
    steps[2] = 0 if counts[2] else steps[2]
    blocks = list(range(Ld))
    plain = caption_layout(counts, Ld, N, Q, blocks, rows_cap=rows_cap)
    lay = caption_layout(counts, Ld, N, Q, blocks, rows_cap=rows_cap, steps=steps)
    R = lay["rows_per_layer"]
    key = lambda L, i: tuple(int(L[k][i]) for k in ("p", "k", "base", "cap", "vid", "lay", "valid"))
    assert sorted(key(lay, i) for i in range(Ld * R)) == sorted(key(plain, i) for i in range(Ld * R))
    n = max(steps)
    live = live_rows(counts, steps, n)
    for t, (s0, c) in enumerate(step_ranges(live, Ld, R)):
        running = {i for i in range(Ld * R) if lay["valid"][i] and steps[lay["vid"][i]] > t}
        assert running == set(range(s0, s0 + c)), f"step {t}"
    # the last layer's rows, video-major, as the unordered layout lists them
    assert [key(lay, i) for i in lay["last_sel"]] == [key(plain, i) for i in plain["last_sel"]]
    for v in range(N):
        rows = lay["vr_rows"][lay["vr_start"][v]:lay["vr_start"][v + 1]]
        assert sorted(int(lay["vid"][r]) for r in rows) == [v] * (Ld * counts[v])
        assert all(lay["valid"][r] for r in rows)


def test_step_ordered_last_layer_is_a_permutation_not_a_range():
    """with steps [9, 5, 7] and phantom rows, layer 1 (descending steps) puts video 0 first, so
    last_sel = [16, 18, 17, 19..31] -- first/last/length look contiguous but the order is not video-major.  The
    row selection must then gather, and contiguous_range must say so."""
    from pdvc.pdvc import contiguous_range
    counts, Ld, N, Q = [1, 1, 1], 2, 3, 10
    lay = caption_layout(counts, Ld, N, Q, [1, 0], rows_cap=16, events_cap=1, steps=[9, 5, 7])
    sel = lay["last_sel"].tolist()
    assert sel[:3] == [16, 18, 17] and sel[3:] == list(range(19, 32))
    assert sel[-1] - sel[0] + 1 == len(sel)  # the old test's condition holds ...
    assert contiguous_range(sel) is None  # ... but the rows are not in order
    # the gathered rows are video-major: row sel[i] of the layout belongs to video i for the real rows
    vids = lay["vid"][sel[:3]].tolist()
    assert vids == [0, 1, 2]
    assert contiguous_range(list(range(5, 9))) == (5, 4) and contiguous_range([]) is None


def test_alive_capacity_must_be_non_increasing():
    """CaptionDecodeFunction needs each step's rows nested in the previous step's."""
    from pdvc.batch_layout import step_ranges
    dt = {"cap_tensor": torch.tensor([[1, 5, 6, 0], [1, 7, 0, 0]]), "cap_mask": torch.tensor([[1, 1, 1, 0],
                                                                                               [1, 1, 0, 0]]),
          "video_target": [{"labels": torch.zeros(1)}, {"labels": torch.zeros(1)}]}
    with pytest.raises(ValueError, match="non-increasing"):
        pad_to_capacity(dt, events=2, rows=4, words=4, alive=(2, 3, 1))
    out = pad_to_capacity(dt, events=2, rows=4, words=4, alive=(3, 2, 1))
    assert out["capacity"]["alive"] == (3, 2, 1)
    with pytest.raises(ValueError, match="non-increasing"):
        step_ranges([2, 4, 1], 2, 8)
    assert step_ranges([4, 2, 0], 2, 8) == ((4, 8), (6, 4), (8, 0))
