"""The reference's CPU deformable-attention path, restated in torch -- the CPU BASELINE that bench.py times.

TEST / BASELINE INFRASTRUCTURE ONLY: used by tests/ (pinned against the reference's own border fixtures) and
by bench.py's cpu_baseline leg.  The product package never imports it.

`ms_deform_attn_core_cpu` follows ms_deform_attn_core_pytorch (pdvc/ops/functions/ms_deform_attn_func.py:
41-68) operation for operation: split value per level, grid = 2*loc - 1, per level F.grid_sample(bilinear,
padding_mode='border', align_corners=False) on (N*M, D, H, W), stack over levels, weight by the attention
and sum over (level, point).  Autograd supplies the backward, as in the reference's CPU run.

`time_call_set` times the per-video call set BASELINE.md specifies: enc_layers x (Lq = S) + dec_layers x
(Lq = Q) calls, each forward + backward, M = 8, D = 64, L = 4, P = 4, fp32, N = 1 (the reference trains one
video at a time), with torch using every CPU this process may run on -- capped by OMP_NUM_THREADS when the
environment sets it (a GPU box exposes the whole machine's CPUs but grants a 16-CPU share and sets it); 3
warm-up runs, then the median of `runs` timed runs.
"""
import os
import statistics
import time

import torch
import torch.nn.functional as F


def ms_deform_attn_core_cpu(value, value_spatial_shapes, sampling_locations, attention_weights,
                            return_value=False):
    N, S, M, D = value.shape
    _, Lq, M, L, P, _ = sampling_locations.shape
    sizes = [int(h) * int(w) for h, w in value_spatial_shapes]
    value_list = value.split(sizes, dim=1)
    grids = 2 * sampling_locations - 1
    samples = []
    for lid, (h, w) in enumerate(value_spatial_shapes):
        v = value_list[lid].flatten(2).transpose(1, 2).reshape(N * M, D, int(h), int(w))
        g = grids[:, :, :, lid].transpose(1, 2).flatten(0, 1)
        samples.append(F.grid_sample(v, g, mode="bilinear", padding_mode="border", align_corners=False))
    attn = attention_weights.transpose(1, 2).reshape(N * M, 1, Lq, L * P)
    if return_value:
        return torch.stack(samples, dim=-2)
    out = (torch.stack(samples, dim=-2).flatten(-2) * attn).sum(-1).view(N, M * D, Lq)
    return out.transpose(1, 2).contiguous()


def cpu_info():
    """(model name, physical cores, logical CPUs usable by this process)."""
    model, phys = "unknown", set()
    try:
        with open("/proc/cpuinfo") as f:
            cur = {}
            for line in f:
                if ":" in line:
                    k, v = (s.strip() for s in line.split(":", 1))
                    cur[k] = v
                    if k == "model name":
                        model = v
                elif cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
            if cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return model, len(phys) or None, usable


def time_call_set(T=512, Q=100, enc_layers=2, dec_layers=2, runs=20, warmup=3, threads=None, seed=0):
    """Median seconds of one video's MSDeformAttn call set (fwd+bwd) on the CPU, and the settings used."""
    model, phys, usable = cpu_info()
    if threads is None:
        threads = usable
        if os.environ.get("OMP_NUM_THREADS", "").isdigit():
            threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    torch.set_num_threads(threads)
    M, D, L, P = 8, 64, 4, 4
    T_l = [T // (2 ** i) for i in range(L)]
    S = sum(T_l)
    shapes = [(1, t) for t in T_l]
    g = torch.Generator().manual_seed(seed)
    calls = []
    for Lq in [S] * enc_layers + [Q] * dec_layers:
        value = torch.randn(1, S, M, D, generator=g)
        locx = torch.rand(1, Lq, M, L, P, generator=g)
        loc = torch.stack([locx, torch.full_like(locx, 0.5)], -1)
        attn = torch.rand(1, Lq, M, L, P, generator=g)
        attn = attn / attn.sum((-1, -2), keepdim=True)
        gout = torch.randn(1, Lq, M * D, generator=g)
        calls.append((value, loc, attn, gout))

    def one_video():
        for value, loc, attn, gout in calls:
            v, lo, a = (x.clone().requires_grad_(True) for x in (value, loc, attn))
            ms_deform_attn_core_cpu(v, shapes, lo, a).backward(gout)

    for _ in range(warmup):
        one_video()
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        one_video()
        times.append(time.perf_counter() - t0)
    return statistics.median(times), {"cpu_model": model, "physical_cores": phys, "usable_cpus": usable,
                                      "threads": threads, "runs": runs, "warmup": warmup, "T": T, "Q": Q,
                                      "calls": f"{enc_layers} x Lq={S} + {dec_layers} x Lq={Q}"}
