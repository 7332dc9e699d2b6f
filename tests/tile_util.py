"""Strip-tile harness shared by the CPU (oracle, loopback + gloo) and GPU
tile tests: one global world run untiled and as T row strips must agree cell
for cell (DESIGN.md "Multi-GPU")."""
from __future__ import annotations

import os

from avida_amd import capi, files, tiles
import oracle_lib as ol
import parity_util as pu


def setup(golden, X, Y, seed=7, geometry=2, overrides=None):
    ov = {"WORLD_X": X, "WORLD_Y": Y, "WORLD_GEOMETRY": geometry}
    ov.update(overrides or {})
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=seed)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    # a dense world of ancestor point mutants: births land on occupied cells
    # and cross strip edges from the first updates on
    genomes = pu.mutants_of(anc, iset, X * Y, rate=0.01, seed=seed)
    return iset, env, cfg, genomes


def make_tile(kind, golden, X, Y, T, k, seed=7, geometry=2, device="cpu", overrides=None, arena=0):
    """Backend + Tile for strip k of T (rows [k*Y/T, (k+1)*Y/T))."""
    iset, env, cfg, genomes = setup(golden, X, Y, seed, geometry, overrides)
    rows = Y // T
    b = ol.Backend(kind, cfg, iset, env, ncells=rows * X)
    if kind != "oracle":
        import torch
        b.lib.avgpu_set_stream(b.h, C_void(torch.cuda.current_stream().cuda_stream))
    t = tiles.Tile(b.lib, b.p, b.h, k * rows, T, device, arena)
    b.set_orgs(0, genomes[k * rows * X:(k + 1) * rows * X], deterministic=False)
    return b, t


def C_void(p):
    import ctypes
    return ctypes.c_void_p(p)


def single(kind, golden, X, Y, updates, seed=7, geometry=2, overrides=None):
    iset, env, cfg, genomes = setup(golden, X, Y, seed, geometry, overrides)
    b = ol.Backend(kind, cfg, iset, env, ncells=X * Y)
    b.set_orgs(0, genomes, deterministic=False)
    stats = [b.run_update() for _ in range(updates)]
    return b, stats


def tile_stats(b):
    st = capi.AvgpuUpdateStats()
    b._call("get_stats", b.h, st)
    return st


def records_sent(tile):
    """halo birth records packed by this tile in the last update (both directions)"""
    import torch
    return sum(int(tile.rec_send[d][:4].cpu().view(torch.int32)[0]) for d in range(2))
