"""Probe: can two ranks share one GPU over RCCL (backend "nccl")?  Each rank
all-reduces and exchanges (batch_isend_irecv) a small device tensor; prints
one JSON line per rank.  usage: timeout -k 10 90 python tools/rccl_probe.py"""
import json
import os
import socket
import sys


def rank_main(rank, world, port):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    out = {"rank": rank}
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((4,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["all_reduce"] = x.tolist()
        s, r = torch.full((8,), rank, dtype=torch.uint8, device="cuda"), torch.zeros(8, dtype=torch.uint8, device="cuda")
        peer = 1 - rank
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, r, peer)]):
            w.wait()
        torch.cuda.synchronize()
        out["p2p"] = r.tolist()
        out["ok"] = True
        dist.destroy_process_group()
    except Exception as e:          # noqa: BLE001 -- the probe reports whatever RCCL says
        out["ok"] = False
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(rank_main, args=(2, port), nprocs=2, join=True)
    sys.exit(0)
