"""Strip-tile harness shared by the CPU (oracle, loopback + gloo) and GPU
tile tests: one global world run untiled and as T row strips must agree cell
for cell (DESIGN.md "Multi-GPU")."""
from __future__ import annotations

import os

from avida_amd import capi, files, tiles
import oracle_lib as ol
import parity_util as pu


def resource_env(golden):
    """spatial_res_100u's environment reshaped so every resource path crosses
    strip edges: a torus ResA with diffusion and gravity whose inflow box spans
    rows 6..27, a grid ResB with flows and CELL cells on rows 15..16, and the
    AND reaction drawing on the global pool ResGlobal"""
    import copy
    env = copy.deepcopy(files.read_environment(os.path.join(golden, "spatial_res_100u", "environment.cfg")))
    a, b, g = env.resources
    a.geometry, a.xdiffuse, a.ydiffuse, a.xgravity, a.ygravity = 2, 1.0, 0.5, 0.2, -0.3
    a.inflow_x1, a.inflow_x2, a.inflow_y1, a.inflow_y2 = 20, 35, 6, 27     # wraps in x
    a.outflow_x1, a.outflow_x2, a.outflow_y1, a.outflow_y2 = 0, 31, 30, 33  # wraps in y
    b.xdiffuse, b.ydiffuse, b.xgravity, b.ygravity = 0.3, 1.0, -0.4, 0.25
    for c in env.cells:
        c.cell += 15 * 32 - 40                                              # cells 480..499
    env[2].resource, env[2].max_fraction, env[2].max_number = 3, 0.01, 5.0
    return env


def setup(golden, X, Y, seed=7, geometry=2, overrides=None, env=None):
    ov = {"WORLD_X": X, "WORLD_Y": Y, "WORLD_GEOMETRY": geometry}
    ov.update(overrides or {})
    iset, env0, cfg = pu.load_env(golden, overrides=ov, seed=seed)
    env = env if env is not None else env0
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    # a dense world of ancestor point mutants: births land on occupied cells
    # and cross strip edges from the first updates on
    genomes = pu.mutants_of(anc, iset, X * Y, rate=0.01, seed=seed)
    if env is not env0:
        # resource worlds: mutants of two task-performing genomes (the
        # spatial_res_100u inject sequence: NOT, NAND; resources_9r's 9task.org),
        # so consumption crosses strips too
        legacy = files.read_instset(os.path.join(golden, "resources_9r", "instset-heads.cfg"))
        to_iset = lambda g: bytes(iset.op_of_name(legacy.names[o]) for o in g)
        seqs = [legacy.parse_sequence("rucavcqgfcqapqeccthzscpcccpqcxaqnccxxbcgdutycasvab"),
                files.read_org(os.path.join(golden, "resources_9r", "9task.org"), legacy)]
        half = [pu.mutants_of(to_iset(g), iset, X * Y // 2, rate=0.005, seed=seed + i) for i, g in enumerate(seqs)]
        genomes = [g for pair in zip(*half) for g in pair]
    return iset, env, cfg, genomes


def make_tile(kind, golden, X, Y, T, k, seed=7, geometry=2, device="cpu", overrides=None, arena=0, env=None):
    """Backend + Tile for strip k of T (rows [k*Y/T, (k+1)*Y/T))."""
    iset, env, cfg, genomes = setup(golden, X, Y, seed, geometry, overrides, env)
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


def single(kind, golden, X, Y, updates, seed=7, geometry=2, overrides=None, env=None, on_update=None):
    iset, env, cfg, genomes = setup(golden, X, Y, seed, geometry, overrides, env)
    b = ol.Backend(kind, cfg, iset, env, ncells=X * Y)
    b.set_orgs(0, genomes, deterministic=False)
    stats = []
    for u in range(updates):
        stats.append(b.run_update())
        if on_update:
            on_update(u, b)
    return b, stats


def tile_stats(b):
    st = capi.AvgpuUpdateStats()
    b._call("get_stats", b.h, st)
    return st


def records_sent(tile):
    """halo birth records packed by this tile in the last update (both directions)"""
    import torch
    return sum(int(tile.rec_send[d][:4].cpu().view(torch.int32)[0]) for d in range(2))
