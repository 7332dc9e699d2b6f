"""The product's strips across processes: two ranks, each
holding a HIP strip of one torus on the box's one GPU, run the tiled update
through tiles.StripWorld with a torch.distributed transport -- the host path
bench.py --gpus N drives over RCCL -- and must equal the untiled oracle world,
every cell and every resource amount.

RCCL refuses two ranks on one device, so the transport is "gloo" with the
device buffers staged through host tensors (tiles.StagedTransport); the
kernels, the halo / record buffers and their packing are the multi-GPU
path's own.  This closes the gap between the oracle-only gloo test
(tests/test_tiles.py) and the one-process loopback HIP strips
(tests/test_parity_gpu.py)."""
import os
import socket

import pytest
import torch

import tile_util as tu

pytestmark = pytest.mark.gpu
CAP = 512
X, Y, U = 64, 64, 30


def _env(golden, env_kind):
    if env_kind == "bench":              # configs[4]'s environment (bench.py --env resources)
        import bench
        from avida_amd import files
        return files.parse_environment(bench.resource_env_text(X, Y))
    return tu.resource_env(golden) if env_kind == "tile" else None


def _rank_main(rank, world_size, golden, port, out_dir, env_kind):
    import torch.distributed as dist
    from avida_amd import tiles
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    b, t = tu.make_tile("gpu", golden, X, Y, world_size, rank, device="cuda", env=_env(golden, env_kind))
    sw = tiles.StripWorld([t], tiles.StagedTransport(dist))
    sent = births = 0
    for _ in range(U):
        sw.update()
        torch.cuda.synchronize()
        sent += tu.records_sent(t)
        births += tu.tile_stats(b).births
    per = X * (Y // world_size)
    s, o, f = b.states(0, per, CAP)
    res = b.resources(spatial=True) if env_kind else None
    torch.save({"states": bytes(s), "ops": o, "flags": f, "births": births, "sent": sent, "res": res},
               os.path.join(out_dir, f"rank{rank}.pt"))
    b.close()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("env_kind", [None, "bench"])
def test_gpu_strips_two_processes_equal_untiled_oracle(golden, tmp_path, env_kind):
    import torch.multiprocessing as mp
    from avida_amd import capi
    import parity_util as pu
    T = 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_rank_main, args=(T, golden, port, str(tmp_path), env_kind), nprocs=T, join=True)
    ref, _ = tu.single("oracle", golden, X, Y, U, env=_env(golden, env_kind))
    a, oa, fa = ref.states(0, X * Y, CAP)
    per = X * Y // T
    if env_kind:
        lv, grids = ref.resources(spatial=True)
    sent = 0
    for k in range(T):
        d = torch.load(os.path.join(tmp_path, f"rank{k}.pt"), weights_only=True)
        s = (capi.AvgpuCpuState * per).from_buffer_copy(d["states"])
        lo = k * per
        bad = pu.diff_states(a[lo:lo + per], s, oa[lo * CAP:(lo + per) * CAP], d["ops"],
                             fa[lo * CAP:(lo + per) * CAP], d["flags"], CAP)
        assert not bad, f"rank {k}: {len(bad)} mismatches, first {bad[:3]}"
        sent += d["sent"]
        if env_kind:
            tl, tg = d["res"]
            for r in range(len(lv)):
                if any(grids[r]):
                    assert tg[r] == grids[r][lo:lo + per], (k, r)
                else:
                    assert tl[r] == lv[r], (k, r)
    assert sent > 0, "no offspring crossed a strip edge"
