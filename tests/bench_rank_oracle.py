"""One rank of the CPU rehearsal of bench.py's multi-GPU launch path
(tests/test_bench_launch.py): started by bench.relaunch_ranks through
torch.distributed.run exactly like `bench.py --gpus N`, it checks the rank
environment with bench.rank_env, joins a gloo group and runs its strip of the
world on the CPU oracle through the same StripWorld / DistTransport host path
bench.py drives over RCCL.  Test infrastructure only (it loads the oracle)."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from avida_amd import tiles  # noqa: E402
import tile_util as tu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gpus", type=int, required=True)
ap.add_argument("--updates", type=int, default=12)
ap.add_argument("--out", required=True)
args = ap.parse_args()
rank, world, local = bench.rank_env(args.gpus)
dist.init_process_group("gloo")
assert dist.get_world_size() == world == args.gpus
X, Y = 32, 32
b, t = tu.make_tile("oracle", os.path.join(HERE, "golden"), X, Y, world, rank)
sw = tiles.StripWorld([t], tiles.DistTransport(dist))
births = 0
for _ in range(args.updates):
    sw.update()
    births += tu.tile_stats(b).births
s, o, f = b.states(0, X * (Y // world), 512)
torch.save({"states": bytes(s), "ops": o, "flags": f, "births": births},
           os.path.join(args.out, f"rank{rank}.pt"))
tot = torch.tensor([births], dtype=torch.int64)
dist.all_reduce(tot)
if rank == 0:
    print(json.dumps({"ranks": dist.get_world_size(), "local_rank": local, "births": int(tot.item())}),
          flush=True)
dist.destroy_process_group()
