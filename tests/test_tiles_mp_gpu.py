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
(tests/test_parity_gpu.py).  With four ranks every strip has two distinct
neighbours (rank k - 1 above, k + 1 below, the torus closing 3 -> 0), so the
up and down halves of every exchange travel to different processes; the
transport counts its collective rounds per batch step (1 all-gather of the
partials, 6 halo exchanges, 1 record exchange: 8)."""
import os
import socket

import pytest
import torch

import tile_util as tu

pytestmark = pytest.mark.gpu
CAP = 512
X, U = 64, 30


def _env(golden, env_kind, Y):
    if env_kind == "bench":              # configs[4]'s environment (bench.py --env resources)
        import bench
        from avida_amd import files
        return files.parse_environment(bench.resource_env_text(X, Y))
    return tu.resource_env(golden) if env_kind == "tile" else None


class _Counting:
    """a transport that counts the collective rounds it is asked for"""

    def __init__(self, tr):
        self.tr, self.rounds = tr, 0

    def __getattr__(self, name):
        fn = getattr(self.tr, name)
        if name in ("all_gather", "exchange", "exchange_start", "all_reduce_sum"):
            def counted(*a, **k):
                self.rounds += 1
                return fn(*a, **k)
            return counted
        return fn


def _rank_main(rank, world_size, golden, port, out_dir, env_kind, Y):
    import torch.distributed as dist
    from avida_amd import tiles
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    b, t = tu.make_tile("gpu", golden, X, Y, world_size, rank, device="cuda", env=_env(golden, env_kind, Y))
    tr = _Counting(tiles.StagedTransport(dist))
    sw = tiles.StripWorld([t], tr)
    sent = births = steps = 0
    for _ in range(U):
        sw.update()
        torch.cuda.synchronize()
        sent += tu.records_sent(t)
        st = tu.tile_stats(b)
        births += st.births
        steps += st.sub_steps
    per = X * (Y // world_size)
    s, o, f = b.states(0, per, CAP)
    res = b.resources(spatial=True) if env_kind else None
    torch.save({"states": bytes(s), "ops": o, "flags": f, "births": births, "sent": sent, "res": res,
                "rounds": tr.rounds, "steps": steps},
               os.path.join(out_dir, f"rank{rank}.pt"))
    b.close()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("env_kind,T,Y", [(None, 2, 64), ("bench", 2, 64), (None, 4, 128), ("bench", 4, 128)])
def test_gpu_strips_processes_equal_untiled_oracle(golden, tmp_path, env_kind, T, Y):
    import torch.multiprocessing as mp
    from avida_amd import capi
    import parity_util as pu
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_rank_main, args=(T, golden, port, str(tmp_path), env_kind, Y), nprocs=T, join=True)
    ref, _ = tu.single("oracle", golden, X, Y, U, env=_env(golden, env_kind, Y))
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
        # per batch step: the partials' all-gather, 6 halo exchanges, the
        # record exchange
        if not env_kind:
            assert d["rounds"] == 8 * d["steps"], (d["rounds"], d["steps"])
        if env_kind:
            tl, tg = d["res"]
            for r in range(len(lv)):
                if any(grids[r]):
                    assert tg[r] == grids[r][lo:lo + per], (k, r)
                else:
                    assert tl[r] == lv[r], (k, r)
    assert sent > 0, "no offspring crossed a strip edge"
