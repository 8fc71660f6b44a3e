"""PDVC model assembly for MI355X (reference: pdvc/pdvc.py:35-604).

`build(args) -> (model, criterion, {'bbox': PostProcess})` and `PDVC.forward(dt, criterion,
transformer_input_type, eval_mode=False) -> (out, loss)` keep the reference's contract and state_dict.
Batches of N videos are supported (the reference asserts N == 1 in its caption head): every loss entry is
the mean over videos of the reference's batch-1 value, all matched captions of all decoder layers and
videos are decoded in one recurrence, and all Hungarian matchings share one device->host copy.
"""
import copy
import math
import os
import threading
import time

import torch
import torch.nn.functional as F
from torch import nn

from . import box_ops, hostio
from .base_encoder import build_base_encoder
from .ops.functions import linear as _lin
from .ops.functions.linear import dense, multi_dense
from .ops.functions.boxref import box_refine
from .CaptioningHead import build_captioner
from .CaptioningHead.LSTM_DSA import caption_steps
from .criterion import SetCriterion
from .deformable_transformer import build_deforamble_transformer
from .batch_layout import caption_layout, caption_layout_to_device, live_rows, step_ranges
from .caption_tokens import DeferredLogprobs, LazyProbs, RowSelect, pack_tokens, token_count
from .matcher import LazyIndices, build_matcher


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def decide_two_stage(transformer_input_type, dt, criterion):
    """misc/utils.py:31-49.  'gt_proposals' (the cfgs/*_gt.yml runs): the ground-truth segments dt['gt_boxes']
    (N, Emax, 2) become the decoder's queries and reference points, their mask dt['gt_boxes_mask'] the query mask;
    the caption cost leaves the matcher and the length / class / box / GIoU losses get weight 0 -- on the
    criterion object itself, as the reference does (a later 'queries' call keeps those weights) -- and the
    decoder's iterative refinement is off."""
    if transformer_input_type == "gt_proposals":
        criterion.matcher.cost_caption = 0
        for q_k in ("loss_length", "loss_ce", "loss_bbox", "loss_giou"):
            for key in criterion.weight_dict.keys():
                if q_k in key:
                    criterion.weight_dict[key] = 0
        return True, True, dt["gt_boxes"], dt["gt_boxes_mask"]
    if transformer_input_type == "queries":
        return False, False, None, None
    raise ValueError(f"Wrong value of transformer_input_type, got {transformer_input_type}")


# PDVC_CAP_DEFERRED=0: per-step float atomics for the caption value gradient (A/B switch)
_CAP_DEFERRED = os.environ.get("PDVC_CAP_DEFERRED", "1") != "0"
# caption log-probabilities and the loss's target gather in one HIP pass each way (csrc/logprob.hip);
# PDVC_STEP_RANGES=0: every caption row runs every step of the recurrence (no per-video stop, no row ordering)
_STEP_RANGES = os.environ.get("PDVC_STEP_RANGES", "1") != "0"


def video_steps(cap_cpu, counts):
    """Each video's caption step count (LSTM_DSA.py:103-104: its loop stops at the first all-zero token column of its
    captions), from the host copy of cap_tensor; 0 for a video without captions."""
    out, o = [], 0
    for c in counts:
        out.append(caption_steps(cap_cpu[o:o + c]) if c else 0)
        o += c
    return out


# PDVC_TOKENS_PACKED=0: the logit GEMM and log-softmax over every (row, step) position, not the packed valid tokens
_TOKENS_PACKED = os.environ.get("PDVC_TOKENS_PACKED", "1") != "0"


def _cap_mask_cpu(dt):
    """The host copy of cap_mask (data.to_device keeps one; else one device->host copy)."""
    m = dt.get("cap_mask_cpu")
    if m is None:
        m = dt["cap_mask"].detach().cpu()
        dt["cap_mask_cpu"] = m
    return m


# PDVC_LOGPROB_FUSED=0 keeps torch's log_softmax + gather (same-box A/B)
_LOGPROB_FUSED = os.environ.get("PDVC_LOGPROB_FUSED", "1") != "0"


def _video_csr(rows, N):
    """Host CSR of the caption rows of each video (rows: tuples whose [1] is the video): (start (N+1,),
    row indices grouped by video, largest row count of a video)."""
    by_video = [[] for _ in range(N)]
    for i, r in enumerate(rows):
        by_video[r[1]].append(i)
    start = [0]
    for v in range(N):
        start.append(start[-1] + len(by_video[v]))
    flat = [i for v in range(N) for i in by_video[v]]
    return start, flat, max((len(b) for b in by_video), default=0)


class MLP(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))

    def forward(self, x):
        # nn.Linear parameters (state_dict unchanged) through `dense`: ReLU fused, split-K weight gradients
        for i, layer in enumerate(self.layers):
            x = dense(x, layer.weight, layer.bias, relu=i < self.num_layers - 1)
        return x


class _TrunkModule(nn.Module):
    """PDVC.trunk as a module whose parameters are exactly the trunk's (for make_graphed_callables)."""

    def __init__(self, pdvc):
        super().__init__()
        self.base_encoder = pdvc.base_encoder
        self.transformer = pdvc.transformer
        self.query_embed = pdvc.query_embed
        self.class_head = pdvc.class_head
        self.count_head = pdvc.count_head
        self.bbox_head = pdvc.bbox_head
        object.__setattr__(self, "_pdvc", pdvc)

    def forward(self, vf, video_mask, duration):
        return self._pdvc.trunk(vf, video_mask, duration)


def _masked_query_max(hs_l, query_mask):
    """The count head's max over queries (pdvc.py:169-172) over the valid queries only: a batch of videos with
    different proposal counts pads the shorter ones (the reference runs one video, every query valid)."""
    if query_mask is None:
        return hs_l
    return hs_l.masked_fill(~query_mask[..., None], float("-inf"))



def contiguous_range(sel):
    """(start, length) when the row list `sel` is exactly start, start + 1, ..., start + length - 1, else None: the
    last decoder layer's caption rows can then be a narrow view instead of a gather (a permutation
    of a contiguous block is not such a range)."""
    if not sel:
        return None
    s0 = int(sel[0])
    return (s0, len(sel)) if list(sel) == list(range(s0, s0 + len(sel))) else None

class PDVC(nn.Module):
    def __init__(self, base_encoder, transformer, captioner, num_classes, num_queries, num_feature_levels,
                 aux_loss=True, with_box_refine=False, opt=None, translator=None):
        super().__init__()
        self.opt = opt
        self.base_encoder = base_encoder
        self.transformer = transformer
        self.caption_head = captioner
        hidden_dim = transformer.d_model
        self.query_embed = nn.Embedding(num_queries, hidden_dim * 2)
        self.class_head = nn.Linear(hidden_dim, num_classes)
        self.count_head = nn.Linear(hidden_dim, opt.max_eseq_length + 1)
        self.bbox_head = MLP(hidden_dim, hidden_dim, 2, 3)
        self.num_feature_levels = num_feature_levels
        self.aux_loss = aux_loss
        self.with_box_refine = with_box_refine
        self.share_caption_head = opt.share_caption_head
        prior_prob = 0.01
        self.class_head.bias.data = torch.ones(num_classes) * -math.log((1 - prior_prob) / prior_prob)
        nn.init.constant_(self.bbox_head.layers[-1].weight.data, 0)
        nn.init.constant_(self.bbox_head.layers[-1].bias.data, 0)
        num_pred = transformer.decoder.num_layers
        if self.share_caption_head:
            self.caption_head = nn.ModuleList([self.caption_head for _ in range(num_pred)])
        else:
            self.caption_head = _get_clones(self.caption_head, num_pred)
        if with_box_refine:
            self.class_head = _get_clones(self.class_head, num_pred)
            self.count_head = _get_clones(self.count_head, num_pred)
            self.bbox_head = _get_clones(self.bbox_head, num_pred)
            nn.init.constant_(self.bbox_head[0].layers[-1].bias.data[1:], -2)
            self.transformer.decoder.bbox_head = self.bbox_head
        else:
            nn.init.constant_(self.bbox_head.layers[-1].bias.data[1:], -2)
            self.class_head = nn.ModuleList([self.class_head for _ in range(num_pred)])
            self.count_head = nn.ModuleList([self.count_head for _ in range(num_pred)])
            self.bbox_head = nn.ModuleList([self.bbox_head for _ in range(num_pred)])
            self.transformer.decoder.bbox_head = None
        self.translator = translator
        self.disable_mid_caption_heads = opt.disable_mid_caption_heads

    # ------------------------------------------------------------------------------------------------
    def trunk(self, vf, video_mask, duration, proposals=None, proposals_mask=None):
        """The static-shape part of PDVC.forward (pdvc/pdvc.py:123-150 in the reference): base encoder,
        deformable encoder, decoder with iterative refinement and the per-layer class/count/box heads.
        Tensors in, tensors out, no host synchronisation: it can be captured as one hipGraph forward and
        one backward (enable_graph).  With proposals (the 'gt_proposals' input, pdvc.py:141-143): the decoder's
        queries come from the proposals (prepare_decoder_input_proposal), the refinement is off and the boxes
        are the proposals."""
        mask = ~video_mask
        N = vf.shape[0]
        srcs, masks, pos = self.base_encoder(vf, mask, duration)
        tr = self.transformer
        src_flatten, temporal_shapes, lsi, valid_ratios, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(
            srcs, masks, pos)
        level_T = tr.last_level_T
        # no padded frame in the batch (a host-side fact, dt["video_mask_all_valid"]): the all-False padding mask
        # changes nothing, so the kernels get none and skip its per-corner byte loads
        kmask = None if self.__dict__.get("_no_padding", False) else mask_flatten
        memory = tr.forward_encoder(src_flatten, level_T, lsi, valid_ratios, lvl_pos, kmask)
        _HOST_GATE.set()  # the encoder's GEMMs queued: a deferred PostProcess host half may take the GIL now
        self._project_memory(memory)
        two_stage = proposals is not None
        if two_stage:
            init_reference, tgt, reference_points, query_embed = tr.prepare_decoder_input_proposal(proposals)
        else:
            query_embed = self.query_embed.weight
            proposals_mask = torch.ones(N, query_embed.shape[0], device=query_embed.device).bool()
            init_reference, tgt, reference_points, query_embed = tr.prepare_decoder_input_query(memory, query_embed)
        hs, inter_references = tr.forward_decoder(tgt, reference_points, memory, level_T, lsi, valid_ratios,
                                                  query_embed, kmask, proposals_mask, two_stage)
        side = tr.decoder.__dict__.pop("_side", None)
        if os.environ.get("PDVC_HEAD_SIDE", "1") == "0":  # A/B switch: heads on hs[l], box MLP evaluated again
            side = None
        classes, counts, coords = self._layer_heads(hs, init_reference, inter_references, two_stage, side,
                                                    proposals_mask if two_stage else None)
        return (memory, mask_flatten, temporal_shapes, lsi, valid_ratios, proposals_mask, hs, init_reference,
                inter_references, torch.stack(classes), torch.stack(counts), torch.stack(coords))

    def _project_memory(self, memory):
        """The value projections of every consumer of the encoder memory (each decoder layer's cross-attention
        and the shared caption head) as one autograd node, attached to `memory` for the consumers to pick up:
        their input gradients then accumulate in GEMM epilogues instead of autograd adds over (N, S, d)."""
        if not (memory.is_cuda and memory.dtype == torch.float32 and _lin.BACKEND != "hip"):
            return
        if os.environ.get("PDVC_FUSED_MEMORY_PROJ") == "0":  # A/B switch
            return
        users = [layer.cross_attn.value_proj for layer in self.transformer.decoder.layers]
        if self.share_caption_head:
            att = getattr(getattr(self.caption_head[0], "core", None), "deformable_att", None)
            if att is not None:
                users.append(att.value_proj)
        vals = multi_dense(memory, users)
        memory._pdvc_values = {id(u): v for u, v in zip(users, vals)}

    def enable_graph(self, dt):
        """Capture trunk() for the shapes of `dt` (training mode) with torch.cuda.make_graphed_callables:
        later training forwards of the same shapes replay one forward graph and, inside backward(), one
        backward graph, instead of launching ~700 kernels from Python.  Dropout inside stays random per
        replay (graph-safe RNG; the HIP kernels draw their seeds on the device)."""
        sample = (dt["video_tensor"], dt["video_mask"], dt["video_length"][:, 1].contiguous())
        mod = _TrunkModule(self)
        # the padding decision is captured with the graph: take it from THIS batch, and key the replay on it
        no_padding = bool(dt.get("video_mask_all_valid", False))
        object.__setattr__(self, "_no_padding", no_padding)
        key = (tuple((tuple(t.shape), t.dtype) for t in sample), no_padding)
        from .precision import begin_capture
        from .step_graph import rewriting_graphs
        begin_capture()
        with rewriting_graphs():  # the captured memset nodes become kernel nodes (step_graph.replace_memsets)
            graphed = torch.cuda.make_graphed_callables(mod, sample, allow_unused_input=True)
        # kept outside the module registry: state_dict keys stay the reference's
        object.__setattr__(self, "_graph_key", key)
        object.__setattr__(self, "_graphed_trunk", graphed)

    def _run_trunk(self, dt, proposals=None, proposals_mask=None):
        args = (dt["video_tensor"], dt["video_mask"], dt["video_length"][:, 1].contiguous())
        if proposals is not None:  # the proposal-input trunk is not graphed on its own (StepGraph captures it whole)
            return self.trunk(*args, proposals=proposals, proposals_mask=proposals_mask)
        g = self.__dict__.get("_graphed_trunk")
        key = (tuple((tuple(t.shape), t.dtype) for t in args), bool(self.__dict__.get("_no_padding", False)))
        if g is not None and self.training and key == self._graph_key:
            return g(*args)  # same shapes and padding decision as the capture
        return self.trunk(*args)

    def forward(self, dt, criterion, transformer_input_type, eval_mode=False):
        two_stage, disable_refine, proposals, proposals_mask = decide_two_stage(transformer_input_type, dt,
                                                                                 criterion)
        object.__setattr__(self, "_no_padding", bool(dt.get("video_mask_all_valid", False)))
        (memory, mask_flatten, temporal_shapes, lsi, valid_ratios, proposals_mask, hs, init_reference,
         inter_references, classes, counts, coords) = self._run_trunk(dt, proposals if two_stage else None,
                                                                      proposals_mask if two_stage else None)
        others = {"memory": memory, "mask_flatten": None if self._no_padding else mask_flatten,
                  "spatial_shapes": temporal_shapes,
                  "level_T": self.transformer.last_level_T, "level_start_index": lsi, "valid_ratios": valid_ratios,
                  "proposals_mask": proposals_mask}
        heads = (list(classes.unbind(0)), list(counts.unbind(0)), list(coords.unbind(0)))
        if eval_mode or self.opt.caption_loss_coef == 0:
            return self.parallel_prediction_full(dt, criterion, hs, init_reference, inter_references, others,
                                                 disable_refine, heads)
        return self.parallel_prediction_matched(dt, criterion, hs, init_reference, inter_references, others,
                                                disable_refine, heads)

    def predict_event_num(self, counter, hs_lid, query_mask=None):
        return counter(torch.max(_masked_query_max(hs_lid, query_mask), dim=1, keepdim=False)[0])

    def _layer_heads(self, hs, init_reference, inter_references, disable_refine, side=None, query_mask=None):
        """Class / count / box heads of every decoder layer (pdvc.py:184-192, 245-253).  side = (per-layer outputs, the
        decoder's refinement bbox_head outputs or None) from DeformableTransformerDecoder.forward: the same values
        as hs[l] and bbox_head[l](hs[l]), without the select's backward and the repeated box MLP."""
        outs, boxes = side if side is not None else (None, None)
        classes, counts, coords = [], [], []
        for l_id in range(hs.shape[0]):
            hs_l = outs[l_id] if outs is not None else hs[l_id]
            reference = init_reference if l_id == 0 else inter_references[l_id - 1]
            ch = self.class_head[l_id]
            classes.append(dense(hs_l, ch.weight, ch.bias))  # 1-wide head: weight gradient as a column sum
            counts.append(self.predict_event_num(self.count_head[l_id], hs_l, query_mask))
            if disable_refine:  # the boxes are the references (pdvc.py:257-258); the box MLP's output is unused
                coords.append(reference)
            else:
                tmp = boxes[l_id] if boxes is not None else self.bbox_head[l_id](hs_l)
                coords.append(box_refine(tmp, reference))  # sigmoid(tmp + inverse_sigmoid(reference)), one pass
        return classes, counts, coords

    def _pack(self, classes, counts, coords, cap_probs, seqs, query_mask=None):
        all_out = {"pred_logits": torch.stack(classes), "pred_count": torch.stack(counts),
                   "pred_boxes": torch.stack(coords), "caption_probs": cap_probs, "seq": seqs}
        if query_mask is not None:  # 'gt_proposals': which proposal slots are real (the criterion masks the rest)
            all_out["query_mask"] = [query_mask] * len(classes)
        out = {k: v[-1] for k, v in all_out.items()}
        if self.aux_loss:
            ks, vs = list(zip(*all_out.items()))
            out["aux_outputs"] = [{ks[i]: vs[i][j] for i in range(len(ks))} for j in range(len(classes) - 1)]
        return out

    def _caption_rows(self, dt, hs, init_reference, inter_references, others, layer_indices):
        """Gather every matched (layer, video, event) row: features, references (valid-ratio scaled per level,
        pdvc/CaptioningHead/LSTM_DSA.py:66-70), token rows and the row bookkeeping."""
        Ld, N, Q, C = hs.shape
        dev = hs.device
        L = self.caption_head[0].core.n_levels
        vr = others["valid_ratios"][:, :L]  # (N, L)
        cap_tensor = dt["cap_tensor"]
        cap_cpu = dt.get("cap_tensor_cpu")
        if cap_cpu is None:
            cap_cpu = cap_tensor.detach().cpu()
        gt_counts = [len(t["labels"]) for t in dt["video_target"]]
        cap_off = [0]
        for g in gt_counts:
            cap_off.append(cap_off[-1] + g)
        Ld_last = Ld - 1
        cap = dt.get("capacity")
        if all(isinstance(ix, LazyIndices) for ix in layer_indices):
            # matching on the device: which rows exist is known from the target counts alone (every target is
            # matched); only the matched query and target of each row come from the device matching.  The row
            # bookkeeping is host numpy over the counts (batch_layout.caption_layout), copied to the device once per
            # batch and cached on dt -- a captured step graph re-uses the device tensors, and StepGraph.load
            # refreshes them for a new batch of a capacity-padded stream
            m = layer_indices[0].matching
            blocks = tuple(ix.block for ix in layer_indices)
            key = ("_caption_rows", Ld, N, Q, blocks)
            if key not in dt:
                # rows ordered by their video's step count, so that every step of the recurrence runs over one
                # contiguous range of the rows still in their video's loop (ranged_steps); a capacity-padded batch
                # needs the stream's live-row capacities for that (pad_to_capacity(alive=...))
                ranged = _STEP_RANGES and Ld <= 2 and (cap is None or cap.get("alive") is not None)
                vsteps = video_steps(cap_cpu, gt_counts) if ranged else None
                lay = caption_layout(gt_counts, Ld, N, Q, blocks, None if cap is None else cap["rows"],
                                     None if cap is None else cap["events"], steps=vsteps)
                Lc = caption_layout_to_device(lay, dev)
                if ranged:
                    n_dec = cap["words"] - 1 if cap is not None else max(vsteps, default=0)
                    live = tuple(cap["alive"]) if cap is not None else live_rows(gt_counts, vsteps, n_dec)
                    host = step_ranges(live, Ld, Lc["rows_per_layer"])
                    if any(c < Ld * Lc["rows_per_layer"] for _, c in host):  # (every row at every step: no ranges)
                        Lc["step_ranges"] = (host, hostio.pack_to_device([[v for r in host for v in r]], dev)[0]
                                             .to(torch.int32))
                dt[key] = Lc
            Lc = dt[key]
            rp, rk, rb, rc, row_video = Lc["p"], Lc["k"], Lc["base"], Lc["cap"], Lc["vid"]
            lay_t, vid, last_sel_d, vr_start_d, vr_rows_d = Lc["lay"], Lc["vid"], Lc["last_sel"], Lc["vr_start"], \
                Lc["vr_rows"]
            max_rows, Rl = Lc["max_rows"], Lc["rows_per_layer"]
            flat_idx = rb + m.queries[rp, rk]
            cap_rows = rc + m.targets[rp, rk] * Lc["valid"]
            rows = Lc["rows_host"]  # (layer, video) per row, phantom rows (layer, 0): rd1 and n_last below
            last_sel = Lc["last_sel_host"]
            # a step-ordered layout permutes the last layer's rows per batch; a captured step graph keeps whatever
            # view it was captured with, so such a layout always gathers (never a narrow view)
            ordered_layout = bool(Lc.get("ordered"))
            ranges = Lc.get("step_ranges")
            row_valid = Lc["valid"] if cap is not None else None
            lay = lay_t
        else:
            row_valid = None
            ranges = None
            ordered_layout = False
            rows = []  # (layer, video, flat_hs_index, cap_row)
            for l_id, indices in enumerate(layer_indices):
                for v, (qi, gi) in enumerate(indices):
                    for q, g in zip(qi.tolist(), gi.tolist()):
                        rows.append((l_id, v, (l_id * N + v) * Q + q, cap_off[v] + g))
            # layer-0 rows first: their reference is 1-d
            rows.sort(key=lambda r: (0 if r[0] == 0 else 1))
            last_sel = [i for i, r in enumerate(rows) if r[0] == Ld_last]
            # every per-row index array in ONE asynchronous host->device copy
            vr_start, vr_rows, max_rows = _video_csr(rows, N)
            flat_idx, cap_rows, row_video, lay, vid, last_sel_d, vr_start_d, vr_rows_d = hostio.pack_to_device(
                [[r[2] for r in rows], [r[3] for r in rows], [r[1] for r in rows], [r[0] for r in rows],
                 [r[1] for r in rows], last_sel, vr_start, vr_rows], dev)
        row_video = row_video.to(torch.int32)
        rd1 = sum(1 for r in rows if r[0] == 0 and init_reference.shape[-1] == 1)
        hs_rows = hs.reshape(Ld * N * Q, C).index_select(0, flat_idx)
        refs = []
        for l_id in range(Ld):
            reference = init_reference if l_id == 0 else inter_references[l_id - 1]
            if reference.shape[-1] == 2:
                ref = reference[:, :, None] * torch.stack([vr, vr], -1)[:, None]
            else:
                ref = reference[:, :, None] * vr[:, None, :, None]
                ref = torch.cat([ref, torch.zeros_like(ref)], -1)
            refs.append(ref)
        ref_all = torch.stack(refs).reshape(Ld * N * Q, L, 2)
        ref_rows = ref_all.index_select(0, flat_idx)
        if cap is not None:  # every video's loop runs the capacity's steps (the steps past a video's end are masked)
            steps_v = [cap["words"] - 1] * N
        else:
            steps_v = [caption_steps(cap_cpu[cap_off[v]:cap_off[v + 1]]) for v in range(N)]
        video_csr = (vr_start_d.to(torch.int32), vr_rows_d.to(torch.int32), max_rows)
        # the last layer's rows are one contiguous block in video-major order (rows are layer-major): its outputs
        # are views, not copies.  With the step-ordered layout last_sel is a permutation of its block (layer 1 in
        # descending step count), so the test is element by element, not first/last/length
        last_range = contiguous_range(last_sel) if not ordered_layout else None
        return dict(rows=rows, hs_rows=hs_rows, ref_rows=ref_rows.contiguous(), rd1=rd1, row_video=row_video,
                    cap_rows=cap_rows, lay=lay, vid=vid, last_sel=last_sel_d, last_range=last_range, steps_v=steps_v,
                    video_csr=video_csr, row_valid=row_valid, step_ranges=ranges)

    def parallel_prediction_matched(self, dt, criterion, hs, init_reference, inter_references, others,
                                    disable_refine, heads=None):
        classes, counts, coords = heads if heads is not None else self._layer_heads(hs, init_reference,
                                                                                    inter_references, disable_refine)
        N, Q = hs.shape[1], hs.shape[2]
        zero_probs = {"cap_prob_train": torch.zeros(1, device=hs.device),
                      "cap_prob_eval": torch.zeros(N, Q, 3, device=hs.device)}
        zero_seq = torch.zeros(N, Q, 3, device=hs.device)
        qmask = others["proposals_mask"] if disable_refine else None
        out = self._pack(classes, counts, coords, [zero_probs] * len(classes), [zero_seq] * len(classes), qmask)
        if not self.aux_loss:
            raise NotImplementedError("aux_loss=False is not supported")
        loss, last_indices, aux_indices = criterion(out, dt["video_target"], dt.get("video_target_padded"))
        Ld = hs.shape[0]
        layer_indices = [aux_indices[l][0] for l in range(Ld - 1)] + [last_indices[0]]
        R = self._caption_rows(dt, hs, init_reference, inter_references, others, layer_indices)
        n_steps = max(R["steps_v"]) if R["steps_v"] else 0
        seq_rows = dt["cap_tensor"].index_select(0, R["cap_rows"])
        cap_mask_rows = dt["cap_mask"].index_select(0, R["cap_rows"])
        tokens = None
        if _LOGPROB_FUSED and _TOKENS_PACKED and n_steps > 0:
            # the logit GEMM and log-softmax over the loss-carrying tokens only (pdvc/caption_tokens.py): capacity =
            # the batch's token count (a capacity-padded stream: its fixed token capacity); no packing when every
            # (row, step) position carries the loss
            cap_tok = (dt.get("capacity") or {}).get("tokens")
            per_layer = cap_tok if cap_tok is not None else token_count(_cap_mask_cpu(dt), n_steps)
            capacity = Ld * int(per_layer)
            if capacity < seq_rows.shape[0] * n_steps:
                tokens = pack_tokens(cap_mask_rows[:, 1:n_steps + 1] > 0, capacity)
        if self.share_caption_head:
            logprobs = self.caption_head[0].decode_teacher_forced(
                R["hs_rows"], R["ref_rows"], R["rd1"], R["row_video"], others["memory"], others["mask_flatten"],
                others["level_T"], seq_rows, n_steps,
                video_csr=R["video_csr"] if _CAP_DEFERRED else None,
                pick_target=seq_rows[:, 1:] if _LOGPROB_FUSED else None, tokens=tokens,
                step_ranges=R["step_ranges"])
        else:
            raise NotImplementedError("share_caption_head=0 is not supported on the batched caption path")
        if _LOGPROB_FUSED:
            logprobs, picked = logprobs
            cap_loss = self.caption_head[0].build_loss_picked(picked, cap_mask_rows[:, 1:].float())
        else:
            cap_loss = self.caption_head[0].build_loss(logprobs, seq_rows[:, 1:], cap_mask_rows[:, 1:].float())
        # per (layer, video) mean over events, then mean over videos (= the reference's batch-1 losses)
        rows = R["rows"]
        key = R["lay"] * N + R["vid"]
        ones = torch.ones_like(cap_loss)
        if R["row_valid"] is not None:  # phantom rows of a capacity-padded batch count for no video
            ones = R["row_valid"].to(cap_loss.dtype)
            cap_loss = cap_loss * ones
        sums = torch.zeros(Ld * N, device=hs.device, dtype=cap_loss.dtype).index_add_(0, key, cap_loss)
        cnts = torch.zeros(Ld * N, device=hs.device, dtype=cap_loss.dtype).index_add_(0, key, ones)
        per = (sums / cnts.clamp(min=1)).view(Ld, N).mean(1)
        for l_id in range(Ld):
            k = "loss_caption" if l_id == Ld - 1 else f"loss_caption_{l_id}"
            loss[k] = per[l_id]
        last_sel = R["last_sel"]
        last_v = [r[1] for r in rows if r[0] == Ld - 1]
        n_last = max([R["steps_v"][v] for v in last_v], default=0)
        if dt.get("capacity") is not None:
            n_last = n_steps
        if isinstance(logprobs, DeferredLogprobs):  # packed tokens: materialised on first read
            probs = LazyProbs(cap_prob_train=logprobs.select(
                tuple(R["last_range"]) if R["last_range"] is not None else last_sel, n_last))
        else:
            if R["last_range"] is not None:
                probs = {"cap_prob_train": logprobs.narrow(0, R["last_range"][0], R["last_range"][1])[:, :n_last]}
            else:  # a gather of the last layer's rows: formed only if read
                probs = LazyProbs(cap_prob_train=RowSelect(logprobs, last_sel, n_last))
        out.update({"caption_probs": probs, "seq": seq_rows.index_select(0, last_sel)})
        return out, loss

    def parallel_prediction_full(self, dt, criterion, hs, init_reference, inter_references, others,
                                 disable_refine, heads=None):
        classes, counts, coords = heads if heads is not None else self._layer_heads(hs, init_reference,
                                                                                    inter_references, disable_refine)
        Ld, N, Q, C = hs.shape
        probs, seqs = [], []
        for l_id in range(Ld):
            if l_id != Ld - 1:
                probs.append({"cap_prob_train": torch.zeros(1, device=hs.device),
                              "cap_prob_eval": torch.zeros(N, Q, 3, device=hs.device)})
                seqs.append(torch.zeros(N, Q, 3, device=hs.device))
                continue
            reference = init_reference if l_id == 0 else inter_references[l_id - 1]
            head = self.caption_head[l_id]
            L = head.core.n_levels
            vr = others["valid_ratios"][:, :L]
            if reference.shape[-1] == 2:
                ref = reference[:, :, None] * torch.stack([vr, vr], -1)[:, None]
                rd1 = 0
            else:
                ref = reference[:, :, None] * vr[:, None, :, None]
                ref = torch.cat([ref, torch.zeros_like(ref)], -1)
                rd1 = N * Q
            row_video = torch.arange(N, device=hs.device, dtype=torch.int32).repeat_interleave(Q)
            seq, lp = head.decode_greedy(hs[l_id].reshape(N * Q, C), ref.reshape(N * Q, L, 2).contiguous(), rd1,
                                         row_video, others["memory"], others["mask_flatten"], others["level_T"])
            if seq is None:
                probs.append({"cap_prob_eval": []})
                seqs.append([])
            else:
                probs.append({"cap_prob_eval": lp.reshape(N, Q, -1)})
                seqs.append(seq.reshape(N, Q, -1))
        out = self._pack(classes, counts, coords, probs, seqs, others["proposals_mask"] if disable_refine else None)
        loss, last_indices, aux_indices = criterion(out, dt["video_target"], dt.get("video_target_padded"))
        return out, loss


_POOL = []
_PENDING = []
# A deferred PostProcess host half (Python work, the GIL) waits behind this gate until the next batch's forward has
# queued its encoder (trunk), so that it does not compete with the launches of a step whose device queue is still
# empty; drain() and a DeferredRow read open it, and a 0.25 s timeout bounds the wait when no forward follows.
_HOST_GATE = threading.Event()
_HOST_GATE.set()
_GATED = os.environ.get("PDVC_POST_GATE", "1") != "0"


def _host_pool():
    if not _POOL:
        import concurrent.futures
        _POOL.append(concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="pdvc-postprocess"))
    return _POOL[0]


def _host_captions(ev, host_scores, host_seq, tr, N, Q):
    """The host half of PostProcess: the ranked tokens detokenised (Translator.rtranslate, data/video_dataset.py:
    172-180) and the caption scores as per-video lists.  ev: the event behind the device -> pinned copies."""
    if ev is not None:
        ev.synchronize()
        _HOST_GATE.wait(0.25)
    host_seq = host_seq.numpy().astype("int")
    if hasattr(tr, "rtranslate_batch"):  # data.video_dataset.Translator: one vectorised pass
        flat = tr.rtranslate_batch(host_seq.reshape(N * Q, -1), yield_every=2048 if ev is not None else 0)
        caps = [flat[b * Q:(b + 1) * Q] for b in range(N)]
    else:
        caps = [[tr.rtranslate(s) for s in vid] for vid in host_seq]
    if ev is not None:
        time.sleep(0)
    return caps, host_scores.numpy().tolist()


class DeferredRow:
    """One video's captions (part 0) or caption scores (part 1) of a deferred PostProcess host half: a read-only list
    that waits for the worker on first use."""

    def __init__(self, fut, part, b):
        self._fut, self._part, self._b = fut, part, b

    def value(self):
        if not self._fut.done():
            _HOST_GATE.set()
        return self._fut.result()[self._part][self._b]

    def __len__(self):
        return len(self.value())

    def __getitem__(self, i):
        return self.value()[i]

    def __iter__(self):
        return iter(self.value())

    def __eq__(self, other):
        return list(self.value()) == (other.value() if isinstance(other, DeferredRow) else list(other))

    def __repr__(self):
        return repr(self.value())

    def __array__(self, dtype=None, copy=None):
        import numpy as np
        return np.asarray(self.value(), dtype=dtype)


class PostProcess(nn.Module):
    """Eval outputs of a batch -> one result dict per video, in the reference's format (pdvc/pdvc.py:493-546).

    Everything numeric is computed for the whole batch on the device, ranked per video by detection score:
      scores        sigmoid(pred_logits) over the (query, class) grid, descending (top-k with k = Q);
      query_id      the query of each ranked entry, labels its class;
      boxes         (centre, length) -> (start, end), clamped to [0, 1], times the video's duration,
                    gathered in ranked order (`raw_boxes` is the same tensor, as in the reference);
      caption_scores  sum of the greedy tokens' log-probabilities over tokens > 0, in ranked order;
      pred_seq_len  argmax of the count head, at least 1.
    The caption scores and tokens reach the host in one copy; captions are detokenised there by the
    loader's translator (`loader.dataset.translator.rtranslate`, data/video_dataset.py:172-180)."""

    def __init__(self, opt, defer_host=None):
        super().__init__()
        self.opt = opt
        # the captions' host half on a worker thread (DeferredRow results; PostProcess.drain() waits for all)
        self.defer_host = os.environ.get("PDVC_POST_DEFER", "1") != "0" if defer_host is None else bool(defer_host)

    @staticmethod
    def drain():
        """Wait for every deferred host half (captions, caption scores) queued so far; re-raise its error."""
        _HOST_GATE.set()
        while _PENDING:
            _PENDING.pop(0).result()

    @torch.no_grad()
    def forward(self, outputs, target_sizes, loader):
        logits = outputs["pred_logits"]
        N, Q, K = logits.shape
        if len(target_sizes) != N:
            raise ValueError(f"PostProcess: {len(target_sizes)} durations for {N} videos")
        scores, ranked = logits.sigmoid().reshape(N, Q * K).topk(Q, dim=1)
        query_id = torch.div(ranked, K, rounding_mode="floor")
        labels = ranked - query_id * K
        se = box_ops.box_cl_to_xy(outputs["pred_boxes"]).clamp(0, 1)
        boxes = se.gather(1, query_id[..., None].expand(N, Q, 2)) * target_sizes.to(se.dtype)[:, None, None]
        seq_len = outputs["pred_count"].argmax(dim=-1).clamp(min=1)
        seq = outputs["seq"]
        if len(seq):
            cap_scores = (outputs["caption_probs"]["cap_prob_eval"] * (seq > 0)).sum(2).gather(1, query_id)
            seq_ranked = seq.gather(1, query_id[..., None].expand(N, Q, seq.shape[2]))
            tr = loader.dataset.translator
            if self.defer_host and seq.is_cuda:
                # the host half (captions detokenised, scores as lists) runs on a worker thread behind an event on
                # the device copies, while the caller queues its next batch: the device does not idle through it
                hs = torch.empty(cap_scores.shape, dtype=torch.float64, pin_memory=True)
                hq = torch.empty(seq_ranked.shape, dtype=torch.long, pin_memory=True)
                hs.copy_(cap_scores.double(), non_blocking=True)
                hq.copy_(seq_ranked, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                if _GATED:
                    _HOST_GATE.clear()
                fut = _host_pool().submit(_host_captions, ev, hs, hq, tr, N, Q)
                _PENDING.append(fut)
                caps = [DeferredRow(fut, 0, b) for b in range(N)]
                cap_scores = [DeferredRow(fut, 1, b) for b in range(N)]
            else:
                caps, cap_scores = _host_captions(None, cap_scores.double().cpu(), seq_ranked.cpu(), tr, N, Q)
        else:  # no caption decoded (every query finished at once)
            cap_scores = [[-1e5] * Q for _ in range(N)]
            caps = [[""] * Q for _ in range(N)]
        # per-video views by unbind (one call per tensor; indexing each video's slice cost ~5 us a view)
        sc, lb, bx, qi = scores.unbind(0), labels.unbind(0), boxes.unbind(0), query_id.unbind(0)
        ts, sl = target_sizes.unbind(0), seq_len.unbind(0)
        return [{"scores": sc[b], "labels": lb[b], "boxes": bx[b], "raw_boxes": bx[b], "captions": caps[b],
                 "caption_scores": cap_scores[b], "query_id": qi[b], "vid_duration": ts[b], "pred_seq_len": sl[b]}
                for b in range(N)]


def build(args):
    device = torch.device(args.device)
    base_encoder = build_base_encoder(args)
    transformer = build_deforamble_transformer(args)
    captioner = build_captioner(args)
    model = PDVC(base_encoder, transformer, captioner, num_classes=args.num_classes, num_queries=args.num_queries,
                 num_feature_levels=args.num_feature_levels, aux_loss=args.aux_loss,
                 with_box_refine=args.with_box_refine, opt=args)
    matcher = build_matcher(args)
    weight_dict = {"loss_ce": args.cls_loss_coef, "loss_bbox": args.bbox_loss_coef,
                   "loss_giou": args.giou_loss_coef, "loss_counter": args.count_loss_coef,
                   "loss_caption": args.caption_loss_coef}
    if args.aux_loss:
        aux = {}
        for i in range(args.dec_layers - 1):
            aux.update({k + f"_{i}": v for k, v in weight_dict.items()})
        weight_dict.update(aux)
    criterion = SetCriterion(args.num_classes, matcher, weight_dict, ["labels", "boxes", "cardinality"],
                             focal_alpha=args.focal_alpha, focal_gamma=args.focal_gamma, opt=args)
    criterion.to(device)
    return model, criterion, {"bbox": PostProcess(args)}
