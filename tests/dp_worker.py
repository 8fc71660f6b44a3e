"""One rank of the data-parallel equivalence test (tests/test_gpu_dp.py), launched as a fresh process:
    python tests/dp_worker.py RANK WORLD PORT OUT.npz MODE     (MODE: eager | graph)
Builds the toy PDVC of the pdvc_batch3_anet fixture, takes its share of weights.dp_items() (2 videos per
rank), runs one training step through GradAllReducer (gloo; every rank on cuda:0) and saves the reduced
gradients.  MODE graph: the step is a StepGraph replay (the bench path), reducer.finish() after it."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "dense-video-captioning_amd"), ROOT, HERE, os.path.join(HERE, "golden")):
    sys.path.insert(0, p)


def main():
    rank, world, port, out, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
    import numpy as np
    import torch
    import torch.distributed as dist
    import weights as W
    import test_gpu_model as TM
    from pdvc.data import collate, to_device
    from pdvc.distributed import GradAllReducer, broadcast_parameters, init_distributed
    init_distributed("gloo")
    torch.cuda.set_device(0)
    d = TM.load("pdvc_batch3_anet")
    model, criterion = TM.build_filled(d)
    model.train()
    broadcast_parameters(model)
    items = W.dp_items()
    share = len(items) // world
    dt = to_device(collate(items[rank * share:(rank + 1) * share]), "cuda")
    params = [p for p in model.parameters() if p.requires_grad]
    reducer = GradAllReducer(params, bucket_mb=4.0)
    wd = criterion.weight_dict
    if mode == "graph":
        from pdvc.step_graph import StepGraph
        sg = StepGraph(model, criterion, dt, reducer=reducer)
        sg.replay()
        sg.replay()
        overlap = sg.overlap
        event_nodes = int(sg.node_counts.get("event_record", 0))
    else:
        model.zero_grad(set_to_none=True)
        _, loss = model(dt, criterion, "queries")
        sum(loss[k] * wd[k] for k in loss.keys() if k in wd).backward()
        reducer.finish()
        overlap = False
        event_nodes = 0
    torch.cuda.synchronize()
    res = {}
    for n, p in model.named_parameters():
        if p.grad is None:
            res["none." + n] = np.zeros(0)
        else:
            res["grad." + n] = p.grad.detach().cpu().numpy()
    res["n_buckets"] = np.asarray(len(reducer.buckets))
    res["overlap"] = np.asarray(int(overlap))
    res["event_nodes"] = np.asarray(event_nodes)  # graph mode: one event-record node per bucket in the replayed graph  # graph mode: the all-reduces queued behind the capture's events
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
