"""CPU: host-side model surface -- build() from the reference cfg files, state_dict names/shapes identical to
the reference (strict checkpoint loading, train.py:116), weight_dict, option parsing; plus the criterion and
matcher host logic on synthetic tensors.  No kernels are launched."""
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
PKG = os.path.join(os.path.dirname(HERE), "dense-video-captioning_amd")


def load(name):
    return np.load(os.path.join(G, name + ".npz"), allow_pickle=False)


def build_cpu(cfg, **over):
    import opts
    from pdvc.pdvc import build
    args = opts.parse_opts(["--cfg_path", cfg, "--device", "cpu"], cfg_root=PKG, **over)
    return build(args)


def test_full_size_state_dict_matches_reference():
    ref = load("state_dict_anet_tsp_c768_q100")
    model, criterion, post = build_cpu("cfgs/anet_tsp_pdvc.yml", feature_dim=768, num_queries=100)
    sd = model.state_dict()
    assert list(sd.keys()) == [str(k) for k in ref["keys"]]
    assert [",".join(str(s) for s in v.shape) for v in sd.values()] == [str(s) for s in ref["shapes"]]
    assert [n for n, _ in model.named_parameters()] == [str(n) for n in ref["param_names"]]
    assert sum(p.numel() for p in model.parameters()) == int(ref["n_params"])
    assert list(criterion.weight_dict.keys()) == [str(k) for k in ref["weight_dict_keys"]]
    assert list(criterion.weight_dict.values()) == ref["weight_dict_vals"].tolist()
    assert "bbox" in post


@pytest.mark.parametrize("case", ["pdvc_small_anet", "pdvc_small_yc2_3l"])
def test_small_state_dicts_match_reference(case):
    import ast
    d = load(case)
    kv, cfg = {}, None
    for s in d["args"]:
        k, v = str(s).split("=", 1)
        if k == "cfg":
            cfg = ast.literal_eval(v)
        else:
            kv[k] = ast.literal_eval(v)
    model, _, _ = build_cpu(cfg, **kv)
    assert list(model.state_dict().keys()) == [str(k) for k in d["state_keys"]]


def test_yaml_chain_and_overrides():
    import opts
    a = opts.parse_opts(["--cfg_path", "cfgs/yc2_newModel_sound.yml"], cfg_root=PKG)
    assert a.id == "yc2_newModel_sound" and a.dec_layers == 3 and a.enc_layers == 3
    assert a.feature_dim == 768 and a.caption_decoder_type == "standard" and a.cap_nheads == 1
    assert a.with_box_refine == 1 and a.att_hid_size == 512 and a.max_eseq_length == 20
    b = opts.parse_opts(["--cfg_path", "cfgs/yc2_tsn_pdvc.yml"], cfg_root=PKG)
    assert b.feature_dim == 3072 and b.num_queries == 100 and b.vocab_size == 1607


def test_sampling_offset_bias_init():
    from pdvc.ops.modules import MSDeformAttn, MSDeformAttnCap
    m = MSDeformAttn(512, 4, 8, 4)
    b = m.sampling_offsets.bias.view(8, 4, 4)
    # head 0 points along +x: offsets 1,2,3,4; head 4 along -x
    assert torch.allclose(b[0, 0], torch.tensor([1., 2., 3., 4.]))
    assert torch.allclose(b[4, 0], torch.tensor([-1., -2., -3., -4.]))
    c = MSDeformAttnCap(512, 4, 1, 4)
    assert torch.allclose(c.sampling_offsets.bias.view(1, 4, 4)[0, 0], torch.tensor([-1.5, -0.5, 0.5, 1.5]))


def test_caption_steps_rule():
    from pdvc.CaptioningHead.LSTM_DSA import caption_steps
    cap = torch.tensor([[0, 5, 6, 0, 0, 0], [0, 7, 0, 0, 0, 0]])
    assert caption_steps(cap) == 3  # first all-zero column after 0 is column 3
    assert caption_steps(torch.tensor([[0, 1, 2, 3, 4, 0]])) == 5


def test_matcher_solves_like_scipy():
    from scipy.optimize import linear_sum_assignment
    from pdvc.matcher import HungarianMatcher
    m = HungarianMatcher(cost_class=2, cost_bbox=0, cost_giou=4)
    torch.manual_seed(0)
    logits = torch.randn(2, 10, 1)
    boxes = torch.rand(2, 10, 2) * 0.5 + 0.1
    targets = [{"labels": torch.zeros(3, dtype=torch.long), "boxes": torch.rand(3, 2) * 0.4 + 0.1},
               {"labels": torch.zeros(2, dtype=torch.long), "boxes": torch.rand(2, 2) * 0.4 + 0.1}]
    idx, _ = m({"pred_logits": logits, "pred_boxes": boxes}, targets)
    for v, (i, j) in enumerate(idx):
        c = m.cost_blocks(logits, boxes, targets)[v].numpy()
        ei, ej = linear_sum_assignment(c)
        assert i.tolist() == ei.tolist() and j.tolist() == ej.tolist()


def test_criterion_device_matching_path_equals_host_path(monkeypatch):
    """The device-matching bookkeeping of SetCriterion (static pairs, LazyIndices, per-layer means) gives the
    host path's losses and indices; the GPU solver is stood in for by scipy here (its own parity test is
    tests/test_gpu_lsap.py)."""
    import types
    import numpy as np
    from scipy.optimize import linear_sum_assignment
    from pdvc.criterion import SetCriterion
    from pdvc.matcher import DeviceMatching, HungarianMatcher, padded_targets

    def fake_solve_device(costs, sizes, sizes_dev):
        P, Q, E = costs.shape
        q = torch.zeros((P, max(E, 1)), dtype=torch.int64)
        t = torch.zeros_like(q)
        for p_, e in enumerate(sizes):
            i, j = linear_sum_assignment(costs[p_, :, :e].numpy())
            q[p_, :e] = torch.from_numpy(i)
            t[p_, :e] = torch.from_numpy(j)
        return DeviceMatching(q, t, list(sizes))

    monkeypatch.setattr(HungarianMatcher, "solve_device", staticmethod(fake_solve_device))
    torch.manual_seed(0)
    N, Q, Ld = 5, 20, 3
    targets = []
    for v in range(N):
        e = 1 + v % 4
        c = torch.rand(e) * 0.8 + 0.1
        targets.append({"labels": torch.zeros(e, dtype=torch.long),
                        "boxes": torch.stack([c, torch.rand(e) * 0.2 + 0.05], -1)})
    opt = types.SimpleNamespace(lloss_gau_mask=1, lloss_beta=1)
    weight = {"loss_ce": 2, "loss_bbox": 0, "loss_giou": 4, "loss_counter": 0.5}
    crit = SetCriterion(1, HungarianMatcher(2, 0, 4), weight, ["labels", "boxes"], opt=opt)

    def outputs():
        g = torch.Generator().manual_seed(1)
        layers = [{"pred_logits": torch.randn(N, Q, 1, generator=g), "pred_boxes": torch.rand(N, Q, 2, generator=g),
                   "pred_count": torch.randn(N, 11, generator=g)} for _ in range(Ld)]
        out = dict(layers[0])
        out["aux_outputs"] = layers[1:]
        return out

    res = {}
    for dev_match in (False, True):
        crit.device_matching = dev_match
        losses, last, aux = crit(outputs(), targets, padded_targets(targets, "cpu"))
        res[dev_match] = (losses, [list(last[0])] + [list(a[0]) for a in aux])
    lh, ih = res[False]
    ld, idd = res[True]
    assert set(lh) == set(ld)
    for k in lh:
        assert torch.allclose(lh[k], ld[k], rtol=1e-6, atol=1e-7, equal_nan=True), k
    for a, b in zip(ih, idd):
        for (i1, j1), (i2, j2) in zip(a, b):
            assert i1.tolist() == i2.tolist() and j1.tolist() == j2.tolist()
