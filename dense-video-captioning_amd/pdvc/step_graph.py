"""The whole PDVC training forward + losses + backward as ONE captured hipGraph.

The reference's training iteration (train.py:181-187: `model(dt, criterion, ...)`, weighted loss sum,
`backward()`) launches ~1700 kernels per step from Python at PDVC's shapes; the host, not the GPU, then
sets the pace.  Every host decision of the step depends only on the batch's shapes and event/caption counts
(level lengths, matched rows, caption steps), the set matching runs on the GPU (pdvc_lsap_f32), and no
kernel needs a host read-back, so the step is captured once per batch shape and replayed:

    sg = StepGraph(model, criterion, dt)   # warm-up + capture (dt tensors become the graph's inputs)
    sg.load(dt_next)                       # copy a same-shape batch into the captured inputs (optional)
    total = sg.replay()                    # forward + losses + backward; param.grad hold the new gradients

Dropout stays random per replay (torch's graph-safe Philox offsets; the HIP kernels draw their seeds on the
device).  Gradients live in the graph's memory pool: do not set them to None between replays (the optimizer
step and grad clipping run eagerly on them).  A GradAllReducer (data parallel) is suspended while capturing;
call its finish() after each replay to average the gradients over ranks.
"""
import torch


class StepGraph:
    def __init__(self, model, criterion, dt, transformer_input_type="queries", warmup=2, reducer=None):
        self.model, self.criterion, self.dt, self.tit = model, criterion, dt, transformer_input_type
        self.wd = criterion.weight_dict
        self.reducer = reducer
        # host-side facts of the batch, made once here (they would be host round trips inside the capture)
        if "video_target_padded" not in dt:
            from .matcher import padded_targets
            dt["video_target_padded"] = padded_targets(dt["video_target"], dt["video_tensor"].device)
        if "cap_tensor_cpu" not in dt:
            dt["cap_tensor_cpu"] = dt["cap_tensor"].detach().cpu()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: lazy init, allocator pools, cached host->device bookkeeping
            for _ in range(warmup):
                model.zero_grad(set_to_none=True)
                self._forward_backward()
                if reducer is not None:
                    reducer.finish()
        torch.cuda.current_stream().wait_stream(side)
        model.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        if reducer is not None:
            reducer.suspended = True
        try:
            with torch.cuda.graph(self.graph):
                self.total, self.losses = self._forward_backward()
        finally:
            if reducer is not None:
                reducer.suspended = False

    def _forward_backward(self):
        out, loss = self.model(self.dt, self.criterion, self.tit)
        total = sum(loss[k] * self.wd[k] for k in loss.keys() if k in self.wd)
        total.backward()
        return total, loss

    def load(self, dt):
        """Copy a batch of the captured shapes (same event and caption counts) into the graph's inputs."""
        if bool(dt.get("video_mask_all_valid", False)) != bool(self.dt.get("video_mask_all_valid", False)):
            raise ValueError("StepGraph.load: the batch's padding (video_mask_all_valid) differs from the captured "
                             "batch's; capture a graph for it")
        for k, v in dt.items():
            dst = self.dt.get(k)
            if isinstance(v, torch.Tensor) and isinstance(dst, torch.Tensor) and dst.device.type == "cuda":
                if dst.shape != v.shape:
                    raise ValueError(f"StepGraph.load: {k} has shape {tuple(v.shape)}, captured {tuple(dst.shape)}")
                dst.copy_(v, non_blocking=True)

    def replay(self):
        self.graph.replay()
        if self.reducer is not None:
            self.reducer.finish()
        return self.total
