"""A rank process for tests/test_bench_launcher.py: what bench.py's launch_ranks starts, minus the model.
    python tests/launch_probe.py [--fail-rank R]
Initialises torch.distributed from the launcher's environment (gloo), all-reduces its rank, and rank 0 prints one
JSON line; --fail-rank R makes rank R exit with status 3 before the collective (the others then block in it)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "dense-video-captioning_amd"))


def main():
    import torch
    import torch.distributed as dist
    from pdvc.distributed import init_distributed
    fail = int(sys.argv[sys.argv.index("--fail-rank") + 1]) if "--fail-rank" in sys.argv else -1
    rank, world, local = init_distributed("gloo")
    if rank == fail:
        sys.exit(3)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world": world, "sum_of_ranks": float(t.item()), "local_rank": local,
                          "master_addr": os.environ["MASTER_ADDR"]}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
