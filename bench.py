#!/usr/bin/env python
"""PDVC training-step throughput on MI355X: videos/sec fwd+bwd (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --videos-per-gpu B]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N rank processes itself (launch_ranks:
one per GPU, RCCL); under torchrun it is one of them.  Either way the world size must equal --gpus.

Workload (BASELINE.json metric config): cfgs/anet_tsp_pdvc.yml with C=768 features, T=512 frames
(4 levels: 512/256/128/64 -> S=960), Q=100 queries, 2 encoder + 2 decoder layers, vocab 5748, E=4 events of
13 words per video; synthetic inputs already resident in HBM; random-init weights.
One step = the reference's training iteration (train.py:181-187) over B videos per GPU: forward, losses,
backward, RCCL gradient all-reduce (N>1), grad-norm clip (100) and the AdamW step.  Dropout is active.
Weak scaling: B videos per GPU at every N; value = all ranks' videos / max-over-ranks time.

--workload yc2_tsp_bf16 measures BASELINE.json configs[1] instead: cfgs/yc2_tsp_pdvc.yml, T=256, C=768, Q=100,
E=8 events of 9 words, with every GEMM on bf16 operands and fp32 accumulation (pdvc/precision.py); its line
carries dtype "bf16" and the GEMM roofline against the bf16 MFMA peak.  --workload yc2_newmodel measures
BASELINE.json configs[3]: cfgs/yc2_newModel_sound.yml, NewModel = the dual-modality MHA front-end (T=512 clip
and sound features, 768-d, 32 heads; csrc/seqattn.hip) in front of a 3+3-layer PDVC, E=8 events of 9 words,
fp32.  --workload anet_c3d measures configs[4], the long-video stress config (cfgs/anet_c3d_pdvc.yml: T=1024,
C=500 C3D features, Q=300 queries, 2+2 layers, 512 videos per GPU).  The default (no flags) is the headline fp32
line.
"""
import argparse
import glob
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "dense-video-captioning_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
F32_MFMA_PEAK_TFS = 157.3  # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md: no xf32 on gfx950)
BF16_MFMA_PEAK_TFS = 2500.0  # MI355X dense BF16 matrix peak (MI355X_MICROARCH.md; the 5 PF figure is 2:1 sparse)
GEMM_KERNEL = re.compile(r"^Cijk_|gemm|Gemm")  # hipBLASLt / rocBLAS (Tensile) kernels, pdvc_gemm_f32, gemm3
GEMM3_KERNEL = re.compile(r"gemm3|split_planes_kernel|slab_sum_kernel")  # the in-tree split-bf16 GEMM family
# the two benchmarked workloads: the metric's headline config, and BASELINE.json configs[1] in bf16
WORKLOADS = {
    "anet_tsp": dict(cfg="cfgs/anet_tsp_pdvc.yml", T=512, C=768, Q=100, events=4, words=13, precision="fp32",
                     metric="videos/sec fwd+bwd (PDVC, T=512 C=768 L=4 Q=100) at 1/2/4/8 MI355X"),
    "yc2_tsp_bf16": dict(cfg="cfgs/yc2_tsp_pdvc.yml", T=256, C=768, Q=100, events=8, words=9, precision="bf16",
                         metric="videos/sec fwd+bwd (PDVC yc2_tsp_pdvc, T=256 C=768 L=4 Q=100, bf16) on 1 MI355X"),
    "anet_c3d": dict(cfg="cfgs/anet_c3d_pdvc.yml", T=1024, C=500, Q=300, events=4, words=13, precision="fp32",
                     videos_per_gpu=512,
                     metric="videos/sec fwd+bwd (PDVC anet_c3d_pdvc long-video stress, T=1024 C=500 L=4 Q=300) per "
                            "MI355X, DDP"),
    "yc2_newmodel": dict(cfg="cfgs/yc2_newModel_sound.yml", T=512, C=768, Q=100, events=8, words=9,
                         precision="fp32", frontend=True, videos_per_gpu=512,
                         metric="videos/sec fwd+bwd (NewModel yc2_newModel_sound: MHA front-end + PDVC, T=512 "
                                "C=768 3+3 layers Q=100) on 1 MI355X"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--videos-per-gpu", type=int, default=None,
                   help="default: 1024 (512 for yc2_newmodel and anet_c3d)")
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="anet_tsp",
                   help="anet_tsp: the metric's config (fp32, the reference's precision); yc2_tsp_bf16: "
                        "BASELINE.json configs[1] (T=256, bf16 GEMMs, pdvc/precision.py); yc2_newmodel: configs[3] "
                        "(MHA front-end + 3+3-layer PDVC, T=512); anet_c3d: configs[4] (T=1024, C=500, Q=300)")
    for k in ("T", "C", "Q", "events", "words"):
        p.add_argument(f"--{k}", type=int, default=None, help="override the workload's value")
    p.add_argument("--cfg", default=None)
    p.add_argument("--precision", choices=["fp32", "bf16"], default=None)
    p.add_argument("--mode", choices=["train", "eval"], default="train",
                   help="eval: the reference's evaluation pass instead (eval_utils.py:178 -> PDVC.forward(eval_mode="
                        "True): greedy captions of every query, then PostProcess) -- videos/s, not the headline")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-dropin", action="store_true", help="skip the drop-in operator's timing (profiling runs)")
    p.add_argument("--dist-backend", default=None, help="torch.distributed backend (default: nccl = RCCL on GPUs)")
    p.add_argument("--same-device", action="store_true",
                   help="rehearsal on a 1-GPU box: every rank on cuda:0 (use with --dist-backend gloo)")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="budget of the secondary C-oracle CPU figure")
    p.add_argument("--kernel-report", action="store_true", help="print per-kernel event timings to stderr")
    p.add_argument("--graph", choices=["step", "trunk", "none"], default="step",
                   help="step: forward+losses+backward replayed as one captured hipGraph (pdvc/step_graph.py); "
                        "trunk: only the static-shape trunk graphed (base encoder .. heads); none: eager")
    p.add_argument("--gemm", choices=["hip", "torch"], default=None,
                   help="projection GEMMs on pdvc_gemm_f32 (hip) or torch/hipBLASLt (default: PDVC_GEMM or torch)")
    p.add_argument("--no-gemm-roofline", action="store_true",
                   help="skip the profiled eager step that prices the projection GEMMs against the MFMA peak")
    p.add_argument("--gemm-table", choices=["auto", "off"], default="auto",
                   help="auto: library GEMMs use the pre-tuned solution table (pdvc/gemm_tuning.py) when present")
    p.add_argument("--stream", choices=["fixed", "ragged"], default="fixed",
                   help="fixed: one synthetic batch, E events x W words per video, replayed every step (the metric's "
                        "config); ragged: a seeded stream of distinct batches -- events per video drawn from the "
                        "ActivityNet count distribution, caption lengths from 2 to 28 words -- one per step, padded to "
                        "fixed capacities (pdvc/batch_layout.py) so one captured step graph serves them all")
    p.add_argument("--stream-batches", type=int, default=4, help="distinct batches of the ragged stream")
    a = p.parse_args()
    a.frontend = None
    for k, v in WORKLOADS[a.workload].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    a.frontend = bool(a.frontend)
    if a.videos_per_gpu is None:
        a.videos_per_gpu = 1024
    return a


def build_model(a, device):
    """(args, model, criterion); with the front-end (yc2_newmodel) the model is NewModel behind PDVC's calling
    convention (pdvc/newmodel.py NewModelStep)."""
    import opts
    from pdvc.pdvc import build
    args = opts.parse_opts(["--cfg_path", a.cfg, "--device", "cuda"], cfg_root=PKG, feature_dim=a.C,
                           num_queries=a.Q, frame_embedding_num=a.T)
    if a.frontend:
        from pdvc.newmodel import NewModelStep, build_newmodel
        nm, criterion, _ = build_newmodel(args)
        return args, NewModelStep(nm).to(device), criterion
    model, criterion, _ = build(args)
    return args, model.to(device), criterion


def add_sound(a, dt, device, seed):
    """The front-end's second input (per-clip sound features, HuBERT-sized 768-d), synthetic like the clips."""
    if a.frontend:
        g = torch.Generator(device="cpu").manual_seed(seed)
        dt["sound_tensor"] = torch.randn(dt["video_tensor"].shape[0], a.T, 768, generator=g).to(device)
    return dt


def msda_alg_bytes(meta, kind):
    """Algorithmic HBM bytes of one MSDA launch, e = 4 (fp32):
    fwd = N*S*M*D*e + N*Lq*M*L*P*(8+4) + N*Lq*M*D*e;  bwd = 3*N*S*M*D*e + N*Lq*M*D*e + 2*N*Lq*M*L*P*(8+4)."""
    N, Lq, S, M, D, NS = meta
    e = 4
    if kind == "fwd":
        return N * S * M * D * e + N * Lq * M * NS * 12 + N * Lq * M * D * e
    return 3 * N * S * M * D * e + N * Lq * M * D * e + 2 * N * Lq * M * NS * 12


class GemmFlops:
    """Counts 2*m*n*k of every aten GEMM (mm, addmm, addmm_, _addmm_activation, bmm, baddbmm and their out=
    forms) issued while active, backward included (a TorchDispatchMode is carried into autograd's threads).
    torch.utils.flop_counter misses the in-place and fused-activation forms the step uses."""

    def __enter__(self):
        from torch.utils._python_dispatch import TorchDispatchMode
        aten = torch.ops.aten
        packets = {aten.mm, aten.addmm, aten.addmm_, aten._addmm_activation, aten.bmm, aten.baddbmm}
        outer = self
        self.flops = 0

        class _Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                if func.overloadpacket in packets:
                    ts = [t for t in args if isinstance(t, torch.Tensor)]
                    a, b = ts[-2], ts[-1]
                    batch = a.shape[0] if a.dim() == 3 else 1
                    outer.flops += 2 * batch * a.shape[-2] * a.shape[-1] * b.shape[-1]
                return func(*args, **(kwargs or {}))

        self._mode = _Mode()
        self._mode.__enter__()
        from pdvc.ops.functions import gemm3
        self._g3 = gemm3.FLOPS[0]
        return self

    def __exit__(self, *exc):
        self._mode.__exit__(*exc)
        from pdvc.ops.functions import gemm3
        self.gemm3_flops = gemm3.FLOPS[0] - self._g3  # products on the in-tree kernels (not aten ops)
        self.flops += self.gemm3_flops
        return False


def gemm_roofline(flop_step, timed_step, precision, graphed):
    """MFMA roofline of the projection / FFN / LSTM / logit GEMMs on the TIMED path: their useful flops
    (GemmFlops over one eager step: 2mnk per GEMM, forward and backward; precision-independent)
    over the device time of the GEMM kernels (hipBLASLt / rocBLAS Tensile "Cijk_*", pdvc_gemm) in one profiled
    step of the timed kind -- a hipGraph replay when the bench replays graphs."""
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with GemmFlops() as fc:
        flop_step()
    torch.cuda.synchronize()
    flops = fc.flops
    g3_flops = getattr(fc, "gemm3_flops", 0)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        timed_step()
        torch.cuda.synchronize()
    gemm_us, cast_us, launches, total_us, g3_us, g3_launches = 0.0, 0.0, 0, 0.0, 0.0, 0
    for e in prof.key_averages():
        dt = e.device_time_total
        total_us += dt
        if GEMM3_KERNEL.search(e.key):
            g3_us += dt
            g3_launches += e.count
        if GEMM_KERNEL.search(e.key) or GEMM3_KERNEL.search(e.key):
            gemm_us += dt
            launches += e.count
        elif precision == "bf16" and "copy" in e.key.lower() and "bfloat16" in e.key.lower():
            cast_us += dt
    if gemm_us <= 0:
        return None
    peak = BF16_MFMA_PEAK_TFS if precision == "bf16" else F32_MFMA_PEAK_TFS
    ach = flops / (gemm_us * 1e-6) / 1e12
    r = {"kernel": "projection / FFN / LSTM / logit GEMMs (hipBLASLt, " +
                   ("bf16 operands, fp32 accumulation)" if precision == "bf16" else "fp32, tuned table)"),
         "bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak, "traffic": None,
         "gemm_kernel_launches_per_step": launches, "gflop_per_step": flops / 1e9,
         "gemm_device_ms_per_step": gemm_us / 1e3, "profiled_device_ms_per_step": total_us / 1e3,
         "timing": ("kernel device time in 1 profiled hipGraph replay of the step" if graphed else
                    "kernel device time in 1 profiled eager step") + "; flops: 2mnk of every aten GEMM of 1 eager step (GemmFlops)"}
    if precision == "bf16":
        r["bf16_cast_ms_per_step"] = cast_us / 1e3
    if g3_flops and g3_us > 0:
        # the in-tree kernels (csrc/gemm3.hip): fp32 products as six bf16 MFMA terms each -- priced on the bf16 matrix
        # peak with the EXECUTED flops (6 x 2mnk); the fp32-equivalent rate beside the fp32 matrix peak
        from pdvc.ops.functions.gemm3 import EXECUTED_PER_ALGORITHMIC as X
        alg = g3_flops / (g3_us * 1e-6) / 1e12
        lib_us, lib_flops = gemm_us - g3_us, flops - g3_flops
        r["gemm3"] = {"kernel": "gemm3p_kernel / gemm3_kernel (in-tree fp32 GEMM, exact 3-term bf16 split, six MFMA "
                                "products, fp32 accumulation)", "bound": "mfma", "achieved": X * alg,
                      "peak": BF16_MFMA_PEAK_TFS, "unit": "TFLOP/s (bf16 MFMA, executed)",
                      "frac": X * alg / BF16_MFMA_PEAK_TFS, "fp32_equivalent_tfs": alg,
                      "fp32_equivalent_vs_fp32_peak": alg / F32_MFMA_PEAK_TFS, "gflop_per_step": g3_flops / 1e9,
                      "device_ms_per_step": g3_us / 1e3, "launches_per_step": g3_launches}
        if lib_us > 0:
            r["library"] = {"kernel": "hipBLASLt / rocBLAS (fp32, tuned table)", "achieved": lib_flops / (lib_us * 1e-6) / 1e12,
                            "peak": F32_MFMA_PEAK_TFS, "frac": lib_flops / (lib_us * 1e-6) / 1e12 / F32_MFMA_PEAK_TFS,
                            "gflop_per_step": lib_flops / 1e9, "device_ms_per_step": lib_us / 1e3,
                            "launches_per_step": launches - g3_launches}
        r["kernel"] = ("projection / FFN / LSTM / logit GEMMs: in-tree gemm3 (split-bf16 MFMA) for the encoder-scale "
                       "products, hipBLASLt fp32 for the rest")
    # above the executed peak: the profiler saw only part of the kernels (another tracer attached, e.g. rocprofv3
    # around the bench) -- not a measurement.  (The all-GEMMs `frac` is priced on the f32-input peak and legitimately
    # exceeds 1 when gemm3 runs the products on the bf16 matrix cores; gemm3's own frac is on the executed bf16 peak.)
    if ("gemm3" in r and r["gemm3"]["frac"] > 1.0) or (precision == "bf16" and r["frac"] > 1.0):
        log("gemm roofline: the profiled kernel times are incomplete (another profiler attached?); not reported")
        return None
    return r


def cpu_baseline(a, enc_layers=2, dec_layers=2):
    """The reference's CPU deformable-attention path timed on this host: a torch restatement of
    ms_deform_attn_core_pytorch (pdvc/ops/functions/ms_deform_attn_func.py:41-68, grid_sample border; pinned to
    the reference's fixtures by tests/test_oracle.py) over one video's call set -- enc_layers x Lq=S + dec_layers
    x Lq=Q, forward + backward, M=8 D=64 L=4 P=4 fp32 -- with every CPU this process may use; 3 warm-ups, median
    of 20 runs."""
    from oracle.torch_core import time_call_set
    med, info = time_call_set(T=a.T, Q=a.Q, enc_layers=enc_layers, dec_layers=dec_layers, runs=20, warmup=3)
    return {"value": 1.0 / med, "unit": "videos/s", "cores": info["threads"], "kind": "port",
            "cpu_model": info["cpu_model"], "physical_cores": info["physical_cores"],
            "usable_cpus": info["usable_cpus"], "ms_per_video": 1e3 * med,
            "threads_note": (f"torch threads = min(usable CPUs {info['usable_cpus']}, OMP_NUM_THREADS "
                             f"{os.environ.get('OMP_NUM_THREADS', 'unset')}): the GPU pool grants each job a CPU share "
                             "and sets OMP_NUM_THREADS to it (16 for one GPU); the affinity mask still lists the "
                             "whole host, whose other CPUs serve other jobs, so more threads would oversubscribe "
                             "the share rather than add cores"),
            "sample": f"median of {info['runs']} runs (after {info['warmup']} warm-ups) of one video's MSDeformAttn "
                      f"call set ({info['calls']}), fwd+bwd, T={a.T}, M=8, D=64, L=4, P=4, fp32, "
                      f"torch.set_num_threads({info['threads']}): oracle/torch_core.py (grid_sample, border)"}


def cpu_baseline_c(a, budget_s, enc_layers=2, dec_layers=2):
    """Secondary CPU figure: the single-threaded C restatement of the CUDA op (oracle/msda_oracle.c, zero
    padding), whole videos of the same call set until budget_s is spent."""
    from oracle import oracle as O
    T_l = [a.T // (2 ** i) for i in range(4)]
    S = sum(T_l)
    M, D, L, P = 8, 64, 4, 4
    rng = np.random.RandomState(0)
    loc_fn = lambda Lq: np.stack([rng.uniform(0, 1, (1, Lq, M, L, P)), np.full((1, Lq, M, L, P), 0.5)], -1)
    shapes = np.stack([np.ones(4, np.int64), np.asarray(T_l, np.int64)], -1)
    lsi = np.concatenate([[0], np.cumsum(T_l)[:-1]]).astype(np.int64)
    value = rng.randn(1, S, M, D).astype(np.float32)
    calls = [S] * enc_layers + [a.Q] * dec_layers
    inputs = []
    for Lq in calls:
        at = rng.uniform(size=(1, Lq, M, L, P)).astype(np.float32)
        inputs.append((loc_fn(Lq).astype(np.float32), at / at.sum((-1, -2), keepdims=True),
                       rng.randn(1, Lq, M * D).astype(np.float32)))
    O.msda_forward(value, shapes, lsi, inputs[-1][0], inputs[-1][1])  # load/compile
    videos, t0 = 0, time.perf_counter()
    while True:
        for loc, at, g in inputs:
            O.msda_forward(value, shapes, lsi, loc, at)
            O.msda_backward(value, shapes, lsi, loc, at, g)
        videos += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": videos / el, "unit": "videos/s", "cores": 1, "kind": "port",
            "sample": f"{videos} video(s) x MSDA fwd+bwd call set ({enc_layers} x Lq={S} + {dec_layers} x Lq={a.Q}), T={a.T}, fp32, "
                      f"oracle/msda_oracle.c (zeros), single thread, {el:.1f} s"}


def ragged_items(n_videos, T, C, vocab, seed, duration=120.0):
    """One batch of a ragged stream in the collate tuple format: per video the event count drawn from the
    ActivityNet train distribution (criterion.COUNTER_CLASS_RATE, 2..27 events, mean 3.7), each caption's word count
    from a gamma law of mean 13.5 clipped to [2, 28] (the reference's translate() keeps at most max_caption_len - 2
    = 28 words, data/video_dataset.py:161-168)."""
    from pdvc.criterion import COUNTER_CLASS_RATE
    rng = np.random.RandomState(seed)
    rate = np.asarray(COUNTER_CLASS_RATE, np.float64)
    rate = rate / rate.sum()
    out = []
    for v in range(n_videos):
        ne = int(rng.choice(len(rate), p=rate))
        feat = rng.standard_normal((T, C)).astype(np.float32)
        ts = np.sort(rng.uniform(0, duration, size=(ne, 2)), axis=1)
        ts[:, 1] = np.minimum(np.maximum(ts[:, 1], ts[:, 0] + 1.0), duration)
        words = np.clip(np.round(rng.gamma(5.0, 13.5 / 5.0, size=ne)), 2, 28).astype(int)
        caps = [np.array([0] + list(rng.randint(1, vocab, size=w)) + [0], dtype=np.int64) for w in words]
        stamps = [[t[0] / duration * T, t[1] / duration * T] for t in ts]
        out.append((feat, stamps, [0] * ne, caps, [list(t) for t in ts], duration, ["w"] * ne, f"rag_{seed}_{v}"))
    return out


def ragged_stream(a, B, vocab, device, rank, padded):
    """`a.stream_batches` distinct ragged batches resident in HBM, capacity-padded when `padded` (the graph path):
    capacities = 27 events per video, the stream's largest caption-row count rounded up to 128, 30 tokens per
    caption, the stream's largest count of loss-carrying caption words rounded up to 256 (the packed logit
    projection, pdvc/caption_tokens.py), and per step the stream's largest count of caption rows still in their
    video's loop, rounded up to 64 (the recurrence's row ranges, pdvc.py `_caption_rows`)."""
    from pdvc.batch_layout import pad_to_capacity
    from pdvc.data import collate, to_device
    raw = [collate(ragged_items(B, a.T, a.C, vocab, seed=5000 + 97 * rank + i)) for i in range(a.stream_batches)]
    from pdvc.batch_layout import live_rows
    from pdvc.pdvc import video_steps
    rows = max(int(d["cap_tensor"].shape[0]) for d in raw)
    tokens = max(int(d["cap_mask"][:, 1:30].sum()) for d in raw)  # loss-carrying words (pdvc/caption_tokens.py)
    # caption rows per decoder layer still in their video's loop at each step (the recurrence's row ranges)
    lives = [live_rows([len(t["labels"]) for t in d["video_target"]],
                       video_steps(d["cap_tensor"], [len(t["labels"]) for t in d["video_target"]]), 29) for d in raw]
    alive = [max(x[t] for x in lives) for t in range(29)]
    alive = [min((a + 63) // 64 * 64, (rows + 127) // 128 * 128) for a in alive]
    caps = dict(events=27, rows=(rows + 127) // 128 * 128, words=30, tokens=(tokens + 255) // 256 * 256, alive=alive)
    stats = {"events_per_video_mean": float(np.mean([len(t["labels"]) for d in raw for t in d["video_target"]])),
             "caption_rows_per_batch": [int(d["cap_tensor"].shape[0]) for d in raw],
             "words_per_caption_mean": float(np.mean([float(m.sum()) - 2 for d in raw for m in d["cap_mask"]])),
             "capacity": caps if padded else None}
    out = [to_device(pad_to_capacity(d, **caps) if padded else d, device) for d in raw]
    return out, stats


def dropin_msda(T, videos=256, reps=10):
    """The drop-in operator MultiScaleDeformableAttention (what a stock MSDeformAttn module calls, vision.cpp:13-16)
    at PDVC's lifted pyramid (spatial_shapes [[1, T_l]], y = 0.5), encoder (Lq = S) and decoder (Lq = 100) shapes,
    M = 8, D = 64, fp32: per-launch forward / backward time (HIP events on the launching stream, median of `reps`
    after 3 warm-ups) and the section 8(d) algorithmic bytes per launch over it."""
    import MultiScaleDeformableAttention as MSDA
    dev = torch.device("cuda")
    T_l = [T // (2 ** i) for i in range(4)]
    S, M, D, L, P = sum(T_l), 8, 64, 4, 4
    shapes = torch.tensor([[1, t] for t in T_l], dtype=torch.int64, device=dev)
    lsi = torch.tensor([0] + list(np.cumsum(T_l)[:-1]), dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    value = torch.randn(videos, S, M, D, device=dev, generator=g)
    res = {"op": "MultiScaleDeformableAttention.ms_deform_attn_forward / _backward (1-D fast path: whole-pyramid "
                 "kernels at the encoder shape, L2-gather kernels at the decoder shape)",
           "videos": videos, "timing": f"HIP events, median of {reps} launches after 3 warm-ups"}
    for name, Lq in (("encoder", S), ("decoder", 100)):
        x = torch.rand(videos, Lq, M, L, P, device=dev, generator=g)
        loc = torch.stack([x, torch.full_like(x, 0.5)], -1).contiguous()
        attn = torch.rand(videos, Lq, M, L, P, device=dev, generator=g)
        attn = (attn / attn.sum((-1, -2), keepdim=True)).contiguous()
        gout = torch.randn(videos, Lq, M * D, device=dev, generator=g)
        t = {}
        for kind, fn in (("fwd", lambda: MSDA.ms_deform_attn_forward(value, shapes, lsi, loc, attn, 64)),
                         ("bwd", lambda: MSDA.ms_deform_attn_backward(value, shapes, lsi, loc, attn, gout, 64))):
            for _ in range(3):
                fn()
            ms = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ms.append(e0.elapsed_time(e1))
            med = float(np.median(ms))
            nbytes = msda_alg_bytes((videos, Lq, S, M, D, L * P), kind)
            t[kind] = {"avg_launch_us": 1e3 * med, "alg_bytes_per_launch": nbytes,
                       "achieved_gbs": nbytes / (med * 1e-3) / 1e9, "frac_hbm": nbytes / (med * 1e-3) / 1e9 / HBM_PEAK_GBS}
        res[name] = t
        del x, loc, attn, gout
    del value
    torch.cuda.empty_cache()
    return res


def latest_profile(suffix):
    """The newest profiles/r*_<suffix> file, or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_" + suffix)))
    return files[-1] if files else None


def pmc_bytes(kernel, workload):
    """avg HBM bytes per launch of a kernel from the workload's PMC file (tools/pmc_traffic.py), and its path."""
    f = latest_profile(f"{kernel}_traffic_{workload}.json")
    if not f:
        return None, None
    with open(f) as fh:
        return json.load(fh).get("avg_bytes_per_launch"), os.path.relpath(f, ROOT)


def log(msg):
    """Progress on stderr (a long GPU run that prints nothing for minutes is taken to be hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def freeze_gc():
    """After warm-up, before the timed steps: the objects alive then (model, buffers, captured graphs) moved out of
    Python's collector generations (gc.freeze), so a full collection during the timed steps walks only the steps' own
    garbage -- unfrozen, the eval line paid 70-110 ms for each such collection (2 of 12 steps,
    profiles/r06_eval_gc_freeze_ab.txt).  PDVC_GC_FREEZE=0 leaves the collector as it is."""
    if os.environ.get("PDVC_GC_FREEZE", "1") != "0":
        import gc
        gc.collect()
        gc.freeze()


def eval_main(a):
    """Evaluation throughput: forward with greedy captions for all Q queries (LSTM_DSA.py:118-186, the loop stops
    when every row has finished: tested on the device, read back a few steps late, the decode cut at the reference's
    exit step) + PostProcess (pdvc.py:493-546, captions detokenised on the host on a worker thread while the next
    batch is queued; drained inside the timed region).  Eager: the decode's length is data-dependent.  One GPU."""
    import types
    from pdvc.data import synthetic_videos, collate, to_device
    from data.video_dataset import Translator
    device = torch.device("cuda:0")
    torch.cuda.set_device(device)
    torch.manual_seed(0)
    args, model, criterion = build_model(a, device)
    model.eval()
    post = __import__("pdvc.pdvc", fromlist=["PostProcess"]).PostProcess(args)
    B = a.videos_per_gpu
    vocab = args.vocab_size + 1
    dt = add_sound(a, to_device(collate(synthetic_videos(B, a.T, a.C, a.events, a.words, vocab, seed=1000)), device),
                   device, 2000)
    tr = Translator.from_vocab({str(i): f"w{i}" for i in range(1, vocab)})
    loader = types.SimpleNamespace(dataset=types.SimpleNamespace(translator=tr))
    steps_seen = []

    def step():
        with torch.no_grad():
            out, _ = model(dt, criterion, "queries", eval_mode=True)
            res = post(out, dt["video_length"][:, 1], loader)
        steps_seen.append(out["seq"].shape[-1] if len(out["seq"]) else 0)
        return res

    # PostProcess's host half runs on a worker thread (pdvc.py DeferredRow) while this thread queues the next batch;
    # a short GIL switch interval keeps the queueing thread from waiting a whole default interval (5 ms) for it
    sys.setswitchinterval(float(os.environ.get("PDVC_EVAL_SWITCH_INTERVAL", "0.0005")))
    log(f"eval: {B} videos, warm-up")
    for _ in range(a.warmup):
        step()
    post.drain()
    torch.cuda.synchronize()
    freeze_gc()
    # every step timed on its own: host wall time (the greedy loop checks for finished rows on the host once per
    # decode step, LSTM_DSA.py:172-179) beside the device time between two events on the step's stream, so a slow
    # step is attributed to the host (wall >> device) or to the device
    walls, devs = [], []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        w0 = time.perf_counter()
        e0.record()
        step()
        e1.record()
        torch.cuda.synchronize()
        walls.append(1e3 * (time.perf_counter() - w0))
        devs.append(e0.elapsed_time(e1))
    post.drain()  # the last steps' deferred host halves (captions) are part of the timed work
    el = time.perf_counter() - t0
    ws, ds = sorted(walls), sorted(devs)
    med = ws[len(ws) // 2] if len(ws) % 2 else 0.5 * (ws[len(ws) // 2 - 1] + ws[len(ws) // 2])
    dmed = ds[len(ds) // 2] if len(ds) % 2 else 0.5 * (ds[len(ds) // 2 - 1] + ds[len(ds) // 2])
    result = {"metric": "videos/sec eval (PDVC forward + greedy captions of all queries + PostProcess, "
                        f"T={a.T} C={a.C} Q={a.Q}) on 1 MI355X",
              "value": a.steps * B / el, "unit": "videos/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
              "ms_per_step": 1e3 * el / a.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
              "dtype": "f32", "data": "synthetic",
              "per_step": {"median_videos_per_s": 1e3 * B / med, "wall_ms": {"median": med, "min": ws[0], "max": ws[-1]},
                           "device_ms": {"median": dmed, "min": ds[0], "max": ds[-1]},
                           "host_ms_median": med - dmed, "wall_ms_all": [round(w, 2) for w in walls],
                           "device_ms_all": [round(d, 2) for d in devs]},
              "config": {"workload": f"{os.path.basename(a.cfg)[:-4]} eval: {B} videos x {a.Q} queries, greedy "
                                     f"decoding up to max_caption_len {args.max_caption_len} + 1 steps, random-init "
                                     f"weights (decode length {steps_seen[-1]} steps)",
                         "videos_per_gpu": B, "global_batch": B, "seq_len": a.T, "parallelism": "dp1"}}
    print(json.dumps(result), flush=True)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a, script=None, argv=None):
    """`bench.py --gpus N` without a launcher: start N rank processes of this same command line, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (torchrun's contract; RCCL unless --dist-backend),
    and return the exit status.  Runs before anything touches the GPU (the children are started, not exec'd).  Rank 0
    prints the one JSON line; if any rank fails the others are stopped (by PID) and the status is non-zero."""
    import subprocess
    if not a.same_device:
        have = torch.cuda.device_count()  # does not initialise the GPU on this image
        if have < a.gpus:
            print(f"bench.py: --gpus {a.gpus} but {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
        cmd = [sys.executable, script or os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None else argv)
        procs.append(subprocess.Popen(cmd, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    log(f"launched {a.gpus} rank processes (pids {[p.pid for p in procs]}), master port {port}")
    status = 0
    live = {r: p for r, p in enumerate(procs)}
    # an overall bound (a rank stuck in a collective must not hang the launcher): PDVC_LAUNCH_TIMEOUT seconds
    limit = time.time() + float(os.environ.get("PDVC_LAUNCH_TIMEOUT", "3600"))
    deadline = None  # set once a rank failed: the others get 20 s after SIGTERM, then SIGKILL
    while live:
        # poll only the rank processes (a waitpid(-1) would also reap children this process did not start); the
        # first failing rank seen sets the job's status, not a peer that then lost its collective connection
        exited = [(r, p.poll()) for r, p in list(live.items())]
        exited = [(r, rc) for r, rc in exited if rc is not None]
        for r, rc in exited:
            live.pop(r)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                log(f"rank {r} (pid {procs[r].pid}) exited with {rc}: stopping the other ranks")
                for q in live.values():
                    q.terminate()
                deadline = time.time() + 20
        if not live:
            break
        now = time.time()
        if deadline is None and now > limit:
            log(f"ranks still running after PDVC_LAUNCH_TIMEOUT: stopping them")
            status = 124
            for q in live.values():
                q.terminate()
            deadline = now + 20
        if deadline is not None and now > deadline:
            for q in live.values():
                q.kill()
            deadline = float("inf")
        time.sleep(0.1)
    return status


def main():
    a = parse()
    if a.mode == "eval" and a.gpus > 1:
        raise SystemExit("bench.py --mode eval measures one GPU")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    if a.mode == "eval":
        return eval_main(a)
    from pdvc.distributed import GradAllReducer, broadcast_parameters, init_distributed
    from pdvc import _native
    from pdvc.data import synthetic_videos, collate, to_device
    import importlib
    _lin = importlib.import_module("pdvc.ops.functions.linear")
    if a.gemm:
        _lin.BACKEND = a.gemm
    rank, world, local = init_distributed(a.dist_backend)
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the initialised world size is {world}")
    device = torch.device("cuda:0" if a.same_device else f"cuda:{local}")
    torch.cuda.set_device(device)
    from pdvc import gemm_tuning
    tuned = a.gemm_table == "auto" and gemm_tuning.enable(tag=f"_r{rank}")
    torch.manual_seed(0)
    np.random.seed(0)
    args, model, criterion = build_model(a, device)
    model.train()
    if world > 1:
        broadcast_parameters(model)
    params = [p for p in model.parameters() if p.requires_grad]
    reducer = GradAllReducer(params) if world > 1 else None
    # the reference's AdamW (train.py) as torch's fused single-kernel implementation (same update rule)
    opt = torch.optim.AdamW(params, lr=args.lr, weight_decay=args.weight_decay, fused=True)
    B = a.videos_per_gpu
    vocab = args.vocab_size + 1
    stream, stream_stats = None, None
    if a.stream == "ragged":
        if a.frontend:
            raise SystemExit("--stream ragged: PDVC workloads only")
        stream, stream_stats = ragged_stream(a, B, vocab, device, rank, padded=a.graph == "step")
        dt = stream[0]
    else:
        dt = add_sound(a, to_device(collate(synthetic_videos(B, a.T, a.C, a.events, a.words, vocab,
                                                             seed=1000 + rank)), device), device, 2000 + rank)
    cur = [dt]  # the batch the eager step runs on (the ragged stream advances it)
    wd = criterion.weight_dict
    from pdvc.precision import bf16_matmul
    bf16 = a.precision == "bf16"
    step_no = [0]

    def next_batch():
        if stream is not None:
            cur[0] = stream[step_no[0] % len(stream)]
            step_no[0] += 1
        return cur[0]

    def fwd_bwd():
        out, loss = model(cur[0], criterion, "queries")
        total = sum(loss[k] * wd[k] for k in loss.keys() if k in wd)
        if reducer is not None:
            reducer.zero_grad()  # bucket-resident gradients (pdvc/distributed.py): one fill per bucket
        else:
            opt.zero_grad(set_to_none=True)
        total.backward()
        return total

    def eager_step():
        next_batch()
        with bf16_matmul(bf16):
            total = fwd_bwd()
        if reducer is not None:
            reducer.finish()
        torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
        opt.step()
        return total

    step = eager_step
    sg = None
    if a.graph == "trunk":
        model.enable_graph(dt)  # capture base encoder -> encoder -> decoder -> heads, fwd and bwd
    elif a.graph == "step":
        from pdvc.step_graph import StepGraph
        with bf16_matmul(bf16):  # the bf16 mode reroutes the GEMMs once, at capture
            sg = StepGraph(model, criterion, dt, reducer=reducer)  # forward + losses + backward, one hipGraph

        dbg = os.environ.get("PDVC_DEBUG_SYNC") == "1"

        def step():  # the graph leaves the gradients in place (and averaged over ranks by its reducer)
            if stream is not None:  # the stream's next batch into the captured inputs (same capacities)
                sg.load(next_batch())
            total = sg.replay()
            if dbg:
                torch.cuda.synchronize()
                print("debug: replay ok", file=sys.stderr, flush=True)
            torch.nn.utils.clip_grad_norm_(params, args.grad_clip)
            if dbg:
                torch.cuda.synchronize()
                print("debug: clip ok", file=sys.stderr, flush=True)
            opt.step()
            if dbg:
                torch.cuda.synchronize()
                print("debug: adam ok", file=sys.stderr, flush=True)
            return total
    log(f"{B} videos/GPU, {world} rank(s): warm-up")
    for _ in range(a.warmup):
        step()
    freeze_gc()
    log("timed steps")
    names = ["pdvc_msda1d_forward_f32", "pdvc_msda1d_backward_ex_f32", "pdvc_cap_gather_forward_f32",
             "pdvc_cap_gather_backward_f32", "pdvc_cap_gather_backward2_f32", "pdvc_cap_softattn_forward_f32", "pdvc_cap_softattn_backward_f32",
             "pdvc_softattn_forward_f32", "pdvc_seq_attention_forward_f32",
             "pdvc_seq_attention_backward_f32",
             # the bf16 mode's forms of the encoder's MSDA launches (also writing the bf16 GEMM operands)
             "pdvc_msda1d_forward_f32_bf16out", "pdvc_msda1d_backward_ex_f32_bf16out"]
    graphed = a.graph != "none"
    timer = _native.KernelTimer(names)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if not graphed:
        _native.TIMER = timer  # eager: HIP events around every launch of the timed steps themselves
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    _native.TIMER = None
    if world > 1:
        dist.barrier()
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    timing_note = "HIP events around every launch in the timed steps"
    if graphed:
        # the timed steps replay the kernels inside a hipGraph, where no event can bracket one launch:
        # time them in 2 untimed eager steps at the same shapes right after (same kernels, same data sizes)
        model.__dict__.pop("_graphed_trunk", None)
        _native.TIMER = timer
        for _ in range(2):
            eager_step()
        torch.cuda.synchronize()
        _native.TIMER = None
        timing_note = ("HIP events around every launch in 2 eager steps right after the timed (hipGraph) steps, "
                       "same shapes; step wall time excludes them")
        if stream is not None:
            timing_note += " (eager steps on the capacity-padded batches)"
    ks = timer.summary()
    for base in ("pdvc_msda1d_forward_f32", "pdvc_msda1d_backward_ex_f32"):  # one entry per MSDA pass, either form
        extra = ks.pop(base + "_bf16out", None)
        if extra:
            d = ks.setdefault(base, {"launches": 0, "ms": 0.0, "metas": [], "launch_ms": []})
            for k in ("launches", "ms"):
                d[k] += extra[k]
            d["metas"] += extra["metas"]
            d["launch_ms"] += extra["launch_ms"]
    log("GEMM roofline step")
    groof = None if a.no_gemm_roofline else gemm_roofline(fwd_bwd, step, a.precision, graphed)
    dropin = None
    if rank == 0 and not a.frontend and stream is None and not a.no_dropin:
        log("drop-in operator timing")
        dropin = dropin_msda(a.T)
    videos = a.steps * B * world
    result = {
        "metric": WORKLOADS[a.workload]["metric"],
        "value": videos / el, "unit": "videos/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": 1000.0 * el / a.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16" if bf16 else "f32", "data": "synthetic",
        "config": {"workload": f"{os.path.basename(a.cfg)[:-4]} training step (fwd+loss+bwd" + ("+allreduce" if world > 1 else "") + "+AdamW): " +
                               ("dual-modality MHA front-end (clips + sound, 768-d, 32 heads) + " if a.frontend
                                else "") +
                               f"T={a.T} C={a.C} L=4 Q={a.Q} {args.enc_layers} enc/{args.dec_layers} dec layers, " +
                               (f"E={a.events} events x {a.words} words" if stream is None else
                                f"ragged stream of {len(stream)} distinct batches (events per video from the "
                                f"ActivityNet count distribution, 2-28 words per caption), a new batch every step" +
                                (" loaded into the captured graph" if a.graph == "step" else "")) +
                               f", vocab {vocab}, dropout on" +
                               (", GEMMs on bf16 operands with fp32 accumulation, fp32 storage elsewhere" if bf16
                                else ", fp32 throughout"),
                   "videos_per_gpu": B, "global_batch": B * world, "seq_len": a.T,
                   "gemm": _lin.BACKEND + ("+tuned-table" if tuned else ""),
                   "peak_hbm_gb": round(torch.cuda.max_memory_reserved(device) / 2 ** 30, 1),
                   "graph": {"step": "fwd+loss+bwd as one hipGraph", "trunk": "trunk hipGraph",
                             "none": "eager"}[a.graph],
                   "parallelism": f"dp{world}"},
    }
    # roofline_gather: the fused MSDA forward (the north star's gather kernel; algorithmic bytes per launch / avg
    # launch time).  `roofline` is the dominant work, the GEMMs against the MFMA peak of the precision in use
    def msda_split(kname, kind):
        """(encoder, decoder) launch groups of one MSDA entry point: (launches, avg us, avg algorithmic bytes);
        an encoder launch has Lq == S (self-attention over the pyramid), a decoder launch Lq = Q queries."""
        k = ks.get(kname)
        if not k or not k["launches"] or len(k.get("launch_ms", [])) != len(k["metas"]):
            return None, None
        out = []
        for enc in (True, False):
            sel = [(ms, m) for ms, m in zip(k["launch_ms"], k["metas"]) if (m[1] == m[2]) == enc]
            if not sel:
                out.append(None)
                continue
            ms = sum(x for x, _ in sel) / len(sel)
            by = sum(msda_alg_bytes(m, kind) for _, m in sel) / len(sel)
            out.append({"launches": len(sel), "avg_launch_us": ms * 1e3, "alg_bytes_per_launch": by,
                        "achieved": by / (ms * 1e-3) / 1e9, "frac": by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS})
        return out[0], out[1]

    # roofline_gather: the fused MSDA forward of the encoder's self-attention (the north star's gather kernel, the
    # pyramid kernel): algorithmic bytes per launch / avg launch time; the decoder's launches (Q = 100 queries,
    # msda1d_fwd_buf_kernel) beside it.  `roofline` is the dominant work, the GEMMs against the MFMA peak
    enc, dec = msda_split("pdvc_msda1d_forward_f32", "fwd")
    # the encoder's kernels at this pyramid (msda1d.hip's dispatch: whole-pyramid staging while level 0 fits one
    # 512-row phase, two row windows of level 0 up to 1024 rows)
    T0 = a.T
    fwd_k, bwdq_k = (("msda1d_fwd_pyr2", "msda1d_bwd_query_pyr") if T0 <= 512 else
                     ("msda1d_fwd_win", "msda1d_bwd_query_dot"))
    if enc is not None:
        # PMC passes of the same workload (tools/pmc_workload.sh -> tools/pmc_traffic.py): HBM bytes per launch
        traffic, tsrc = pmc_bytes(fwd_k if T0 > 512 else "msda1d_fwd_pyr", a.workload)
        result["roofline_gather"] = dict(
            {"kernel": f"{fwd_k}_kernel (fused MSDeformAttn forward, encoder self-attention, Lq = S)",
             "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": traffic, "traffic_source": tsrc,
             "timing": timing_note}, **enc)
        if dec is not None:
            dt_, ds_ = pmc_bytes("msda1d_fwd_buf", a.workload)
            result["roofline_gather"]["decoder"] = dict({"kernel": "msda1d_fwd_buf_kernel (decoder cross-attention, "
                                                         "Lq = Q)", "traffic": dt_, "traffic_source": ds_}, **dec)
    enc, dec = msda_split("pdvc_msda1d_backward_ex_f32", "bwd")  # query-side + value-side kernels per launch
    if enc is not None:
        tq, sq = pmc_bytes(bwdq_k, a.workload)
        tv, sv = pmc_bytes("msda1d_bwd_value_enc", a.workload)
        result["roofline_gather_bwd"] = dict(
            {"kernel": f"{bwdq_k}_kernel + msda1d_bwd_value_kernel (fused MSDeformAttn backward, encoder "
                       "self-attention)", "bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "traffic": (tq + tv) if (tq is not None and tv is not None) else None,
             "traffic_source": [sq, sv] if sq else None, "timing": timing_note}, **enc)
        if dec is not None:
            result["roofline_gather_bwd"]["decoder"] = dict(
                {"kernel": "msda1d_bwd_query_dot_kernel + msda1d_bwd_value_kernel (decoder cross-attention)"}, **dec)
    if a.frontend and ks.get("pdvc_seq_attention_forward_f32", {}).get("launches"):
        # front-end attention core (csrc/seqattn.hip): 4*T*T*E flops per video forward (scores + P.V over all
        # heads), 10*T*T*E backward (scores recomputed, dP, dQ, dK, dV), against the fp32 MFMA peak
        E = 768
        fl = 4.0 * B * a.T * a.T * E
        r = {"kernel": "seqattn_fwd_kernel / seqattn_bwd_dq+dkv kernels (front-end MHA core, fp32 MFMA)",
             "bound": "mfma", "peak": F32_MFMA_PEAK_TFS, "unit": "TFLOP/s", "timing": timing_note}
        for n, key, f in (("pdvc_seq_attention_forward_f32", "forward", fl),
                          ("pdvc_seq_attention_backward_f32", "backward", 2.5 * fl)):
            k = ks.get(n)
            if k and k["launches"]:
                avg_ms = k["ms"] / k["launches"]
                r[key] = {"avg_launch_us": 1e3 * avg_ms, "achieved": f / (avg_ms * 1e-3) / 1e12,
                          "frac": f / (avg_ms * 1e-3) / 1e12 / F32_MFMA_PEAK_TFS, "gflop_per_launch": f / 1e9}
        result["roofline_frontend_attention"] = r
    if groof is not None:  # the dominant kernels (~70% of the step's device time): `roofline` proper
        groof["share_of_step"] = groof["gemm_device_ms_per_step"] / (1e3 * el / a.steps)
        gfile = latest_profile(f"gemm_traffic_{a.workload}.json")
        if gfile and B == WORKLOADS[a.workload].get("videos_per_gpu", 1024):  # PMC passes of an eager step at the
            # workload's default batch (tools/pmc_workload.sh -> tools/pmc_gemm.py)
            with open(gfile) as f:
                g = json.load(f)
            groof["traffic"] = g.get("bytes_per_step")
            groof["traffic_unit"] = "HBM bytes per step, every library GEMM launch (eager step)"
            groof["traffic_source"] = os.path.relpath(gfile, ROOT)
        g3 = groof.get("gemm3")
        if g3 is not None:
            # the dominant kernel family is the in-tree split-bf16 GEMM: `roofline` prices it -- algorithmic fp32
            # flops (2mnk) over its device time, against the ceiling of the six-product scheme on the bf16 matrix
            # cores (dense bf16 peak / 6); the fp32-input MFMA peak (157.3) and the whole GEMM mix ride beside it
            g3file = latest_profile(f"gemm3_traffic_{a.workload}.json")
            traffic = None
            if g3file and B == WORKLOADS[a.workload].get("videos_per_gpu", 1024):
                with open(g3file) as f:
                    traffic = json.load(f).get("bytes_per_step")
            from pdvc.ops.functions.gemm3 import EXECUTED_PER_ALGORITHMIC as X
            top = {"kernel": g3["kernel"], "bound": "mfma", "achieved": g3["fp32_equivalent_tfs"],
                   "peak": BF16_MFMA_PEAK_TFS / X, "unit": "TFLOP/s", "frac": g3["fp32_equivalent_tfs"] * X / BF16_MFMA_PEAK_TFS,
                   "traffic": traffic, "traffic_unit": "HBM bytes per step over every gemm3 launch (PMC, eager step)",
                   "traffic_source": os.path.relpath(g3file, ROOT) if traffic is not None else None,
                   "peak_note": f"dense bf16 MFMA peak {BF16_MFMA_PEAK_TFS:.0f} / {X} bf16 products per fp32 product; "
                                f"the f32-input MFMA peak is {F32_MFMA_PEAK_TFS} (achieved / that = "
                                f"{g3['fp32_equivalent_tfs'] / F32_MFMA_PEAK_TFS:.3f})",
                   "gflop_per_step": g3["gflop_per_step"], "device_ms_per_step": g3["device_ms_per_step"],
                   "launches_per_step": g3["launches_per_step"], "timing": groof.get("timing"),
                   "all_gemms": {k: v for k, v in groof.items() if k not in ("gemm3", "timing")}}
            result["roofline"] = top
        else:
            result["roofline"] = groof
    elif "roofline_gather" in result:
        result["roofline"] = result["roofline_gather"]
    if dropin is not None:
        result["dropin_msda"] = dropin
    if stream_stats is not None:
        result["config"]["stream"] = stream_stats
    if sg is not None:  # the replayed step's launches (graph nodes by type, after the memset-node rewrite)
        result["config"]["graph_nodes_per_replay"] = dict(getattr(sg, "node_counts", {}),
                                                          memsets_rewritten=getattr(sg, "memsets_replaced", None))
    ksteps = 2 if graphed else a.steps
    result["kernels"] = {n: {"launches": v["launches"], "avg_us": 1e3 * v["ms"] / max(v["launches"], 1),
                             "share_of_step": v["ms"] / ksteps / (1e3 * el / a.steps)} for n, v in ks.items()}
    # the north-star comparison, like for like: MSDeformAttn fwd+bwd (the fused 1-D kernels, encoder + decoder
    # calls) per step on the GPU, from the HIP-event timings above, as videos/s against the CPU figure
    msda_ms = sum(ks[n]["ms"] for n in ("pdvc_msda1d_forward_f32", "pdvc_msda1d_backward_ex_f32") if n in ks) / ksteps
    if msda_ms > 0:
        result["msda_gpu"] = {"ms_per_step": msda_ms, "videos_per_s": B / (msda_ms * 1e-3) * world,
                              "what": "fused MSDeformAttn forward + backward kernels of every encoder and decoder "
                                      "layer, HIP events, per step of B videos per GPU"}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        log("CPU baseline (reference core, torch)")
        result["cpu_baseline"] = cpu_baseline(a, args.enc_layers, args.dec_layers)
        log("CPU baseline (C oracle)")
        result["cpu_baseline_c_oracle"] = cpu_baseline_c(a, a.cpu_seconds, args.enc_layers, args.dec_layers)
        if "msda_gpu" in result:
            result["msda_gpu"]["vs_cpu_baseline"] = result["msda_gpu"]["videos_per_s"] / result["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
