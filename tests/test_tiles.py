"""Strip tiles on the CPU oracle: the tiled update (include/avida_gpu.h
"strip tiles", avida_amd/tiles.py) must reproduce the untiled world cell for
cell -- in one process (loopback) and across 2 gloo ranks (DistTransport, the
host path bench.py drives over RCCL)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from avida_amd import capi, tiles
import parity_util as pu
import tile_util as tu

CAP = 512


def _compare(single_b, tile_bs, n, T):
    a, oa, fa = single_b.states(0, n, CAP)
    per = n // T
    for k, b in enumerate(tile_bs):
        s, o, f = b.states(0, per, CAP)
        lo = k * per
        sub = (a[lo:lo + per], s, oa[lo * CAP:(lo + per) * CAP], o, fa[lo * CAP:(lo + per) * CAP], f)
        bad = pu.diff_states(*sub, CAP)
        assert not bad, f"tile {k}: {len(bad)} mismatches, first {bad[:3]}"


@pytest.mark.parametrize("T,geometry", [(2, 2), (4, 2), (2, 1)])
def test_oracle_tiles_loopback_equal_single_world(golden, T, geometry):
    X, Y, U = 32, 32, 30
    ref, rstats = tu.single("oracle", golden, X, Y, U, geometry=geometry)
    pairs = [tu.make_tile("oracle", golden, X, Y, T, k, geometry=geometry) for k in range(T)]
    world = tiles.StripWorld([t for _, t in pairs], tiles.LoopbackTransport())
    sent = 0
    for u in range(U):
        world.update()
        sent += sum(tu.records_sent(t) for _, t in pairs)
        tot = [tu.tile_stats(b) for b, _ in pairs]
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped"):
            assert sum(getattr(s, f) for s in tot) == getattr(rstats[u], f), (u, f)
    _compare(ref, [b for b, _ in pairs], X * Y, T)
    assert sent > 0, "no offspring crossed a strip edge: the test exercised nothing"


def _rank_main(rank, world_size, golden, port, out_dir, with_res, staged=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    X, Y, U = 32, 32, 20
    env = tu.resource_env(golden) if with_res else None
    b, t = tu.make_tile("oracle", golden, X, Y, world_size, rank, env=env)
    sw = tiles.StripWorld([t], (tiles.StagedTransport if staged else tiles.DistTransport)(dist))
    births = 0
    for _ in range(U):
        sw.update()
        births += tu.tile_stats(b).births
    s, o, f = b.states(0, b.cfg.world_x * (Y // world_size), CAP)
    res = b.resources(spatial=True) if with_res else None
    torch.save({"states": bytes(s), "ops": o, "flags": f, "births": births, "res": res},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("with_res,staged", [(False, False), (True, False), (True, True)])
def test_oracle_tiles_gloo_two_ranks(golden, tmp_path, with_res, staged):
    X, Y, U, T = 32, 32, 20, 2
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank_main, args=(T, golden, port, str(tmp_path), with_res, staged), nprocs=T, join=True)
    env = tu.resource_env(golden) if with_res else None
    ref, _ = tu.single("oracle", golden, X, Y, U, env=env)
    a, oa, fa = ref.states(0, X * Y, CAP)
    per = X * Y // T
    if with_res:
        lv, grids = ref.resources(spatial=True)
    for k in range(T):
        d = torch.load(os.path.join(tmp_path, f"rank{k}.pt"), weights_only=True)
        s = (capi.AvgpuCpuState * per).from_buffer_copy(d["states"])
        lo = k * per
        bad = pu.diff_states(a[lo:lo + per], s, oa[lo * CAP:(lo + per) * CAP], d["ops"],
                             fa[lo * CAP:(lo + per) * CAP], d["flags"], CAP)
        assert not bad, f"rank {k}: {bad[:3]}"
        if with_res:
            tl, tg = d["res"]
            assert tg[0] == grids[0][lo:lo + per] and tg[1] == grids[1][lo:lo + per]
            assert tl[2] == lv[2]


def test_tile_validation(golden):
    b, _ = tu.single("oracle", golden, 32, 32, 0)
    with pytest.raises(RuntimeError):
        tiles.Tile(b.lib, b.p, b.h, 0, 1, "cpu")        # the whole world is not a strip: no buffers
    iset, env, cfg, _ = tu.setup(golden, 24, 32)
    import oracle_lib as ol
    odd = ol.Backend("oracle", cfg, iset, env, ncells=24 * 5)   # 120 cells: not whole merit blocks
    with pytest.raises(RuntimeError):
        tiles.Tile(odd.lib, odd.p, odd.h, 0, 2, "cpu")


def resource_grids_match(single_res, tile_bs, T, X, Y):
    """per-cell spatial amounts of every strip == the untiled world's rows;
    global pools identical everywhere"""
    lv, grids = single_res
    per = X * Y // T
    for k, b in enumerate(tile_bs):
        tl, tg = b.resources(spatial=True)
        for r in range(len(lv)):
            if any(grids[r]):
                assert tg[r] == grids[r][k * per:(k + 1) * per], (k, r)
            else:
                assert tl[r] == lv[r], (k, r, tl[r], lv[r])


@pytest.mark.parametrize("T,geometry", [(2, 2), (4, 2), (4, 1)])
def test_oracle_tiles_with_resources(golden, T, geometry):
    """Resources on strips (BASELINE config 5): spatial grids whose inflow box,
    CELL list and diffusion/gravity flows cross strip edges, and a consumed
    global pool settled by an all-reduce; strips == the untiled world."""
    X, Y, U = 32, 32, 25
    env = tu.resource_env(golden)
    per_update = []
    ref, rstats = tu.single("oracle", golden, X, Y, U, geometry=geometry, env=env,
                            on_update=lambda u, b: per_update.append(b.resources(spatial=True)))
    pairs = [tu.make_tile("oracle", golden, X, Y, T, k, geometry=geometry, env=env) for k in range(T)]
    assert all(t.has_res_rows for _, t in pairs)
    world = tiles.StripWorld([t for _, t in pairs], tiles.LoopbackTransport())
    for u in range(U):
        world.update()
        tot = [tu.tile_stats(b) for b, _ in pairs]
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides"):
            assert sum(getattr(s, f) for s in tot) == getattr(rstats[u], f), (u, f)
        resource_grids_match(per_update[u], [b for b, _ in pairs], T, X, Y)
    _compare(ref, [b for b, _ in pairs], X * Y, T)
    lv = per_update[-1][0]
    assert lv[2] < per_update[0][0][2] + 1e9 and lv[0] > 0 and lv[1] > 0
