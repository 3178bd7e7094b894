"""Stand-in rank program for tests/test_bench.py::test_launch_ranks_spawns_world2:
started by bench.launch_ranks through torch.distributed.run, it joins a gloo
group, checks the torchrun environment and all-gathers the ranks' shard counts
of a global batch (bench.plan, strong scaling), then rank 0 writes them out."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

out_path, G = sys.argv[1], int(sys.argv[2])
world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1"
dist.init_process_group("gloo")
a = bench.parse(["--gpus", str(world), "--global-batch", str(G)])
pl = bench.plan(a, world, rank)
t = torch.tensor([rank, pl["start"], pl["count"], pl["cap"]], dtype=torch.int64)
parts = [torch.empty_like(t) for _ in range(world)]
dist.all_gather(parts, t)
if rank == 0:
    json.dump({"world": world, "shards": [p.tolist() for p in parts]}, open(out_path, "w"))
dist.destroy_process_group()
