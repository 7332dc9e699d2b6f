"""BIRTH_METHOD 4 (POSITION_OFFSPRING_FULL_SOUP_RANDOM,
main/cPopulation.cc:5297-5310): an offspring goes to a cell drawn from the
whole world -- with PREFER_EMPTY, FindRandEmptyCell (:5650-5668), uniform
among the empty cells, or any cell once the world is full; without it,
GetUInt(size), redrawn while it is the parent and ALLOW_PARENT is 0
(oracle soup_target, world.hip place_pick_one).  In the batch step the empty
cells are those empty at the step's end that the placement round has not
taken.

KAT: one ancestor about to divide in an otherwise empty 9x9 grid; over many
seeds its offspring lands in every part of the grid, a neighbour about as
often as 8 of the 80 empty cells predict, never in the parent's cell.  World:
a 32x32 grid grown from 12 mutants until it is full, GPU == oracle bit for
bit under every PREFER_EMPTY / ALLOW_PARENT combination.  The serial world
(the reference's schedule) places soup births with FindRandEmptyCell on the
reference's persistent empty-cell array (oracle serial_soup, interp.hip
k_serial_update): GPU == oracle, and the batch world's growth is compared
with it over many seeds (two-sample tests)."""
import ctypes as C
import multiprocessing
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

CAP = capi.MAX_GENOME
OV = {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0, "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0}


def _about_to_divide(golden, ov):
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=5)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.step(0, 1, uniform=388, mode=capi.MODE_FROZEN)
    st, ops, fl = b.states(0, 1, CAP)
    b.close()
    return st[0], ops, fl


def _child_cell(golden, seed, x=9, prefer_empty=1):
    ov = dict(OV, WORLD_X=x, WORLD_Y=x, BIRTH_METHOD=4, PREFER_EMPTY=prefer_empty, WORLD_GEOMETRY=1)
    s0, ops0, fl0 = _about_to_divide(golden, ov)
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=seed)
    n = x * x
    centre = (x // 2) * x + x // 2
    b = ol.Backend("oracle", cfg, iset, env, ncells=n)
    st, ops, fl = b.states(0, n, CAP)
    st[centre] = s0
    st[centre].rng_key_lo = (0x9E3779B9 * seed) & 0xFFFFFFFF     # a parent stream per seed
    st[centre].rng_key_hi = (0x85EBCA6B * seed + 17) & 0xFFFFFFFF
    ops = bytearray(ops)
    fl = bytearray(fl)
    ops[centre * CAP:(centre + 1) * CAP] = ops0[:CAP]
    fl[centre * CAP:(centre + 1) * CAP] = fl0[:CAP]
    o = (C.c_uint8 * len(ops)).from_buffer(ops)
    f = (C.c_uint8 * len(fl)).from_buffer(fl)
    b._call("set_states", b.h, 0, n, st, o, f, CAP)
    s = b.run_update()
    after, _, _ = b.states(0, n, CAP)
    b.close()
    assert s.births == 1, s.births
    kids = [c for c in range(n) if after[c].generation == 1 and after[c].num_divides == 0]
    assert len(kids) == 1, kids
    return kids[0], centre


def test_soup_random_kat(golden):
    x = 9
    cells = []
    for seed in range(1, 161):
        c, centre = _child_cell(golden, seed, x)
        assert c != centre
        cells.append(c)
    centre = (x // 2) * x + x // 2
    near = {centre + dy * x + dx for dy in (-1, 0, 1) for dx in (-1, 0, 1)} - {centre}
    frac_near = sum(c in near for c in cells) / len(cells)
    # 8 of the 80 empty cells: 0.10 expected; a neighbour-only method gives 1.0
    assert 0.02 <= frac_near <= 0.22, frac_near
    rows = {c // x for c in cells}
    cols = {c % x for c in cells}
    assert rows == set(range(x)) and cols == set(range(x))
    assert len(set(cells)) >= 55


def test_soup_refused_where_unbuilt(golden):
    """strip tiles refuse BIRTH_METHOD 4 (a soup birth may land in any
    strip); the library refuses BIRTH_METHOD 6 and beyond"""
    ov = dict(OV, WORLD_X=8, WORLD_Y=8, BIRTH_METHOD=4)
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=3)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend("oracle", cfg, iset, env, ncells=64)
    b.set_orgs(0, [anc] * 4, deterministic=False)
    with pytest.raises(RuntimeError):
        b._call("set_tile", b.h, C.c_int64(0), C.c_int64(1 << 20))
    b.close()
    lib = capi.load_product()
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"BIRTH_METHOD": 4}))
    assert lib.avgpu_check_cfg(C.byref(c)) == 0
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"BIRTH_METHOD": 6}))
    assert lib.avgpu_check_cfg(C.byref(c)) == -5


def _grow_pair(golden, prefer_empty, allow_parent):
    ov = {"WORLD_X": 32, "WORLD_Y": 32, "BIRTH_METHOD": 4, "PREFER_EMPTY": prefer_empty,
          "ALLOW_PARENT": allow_parent}
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=43)
    n = cfg.world_x * cfg.world_y
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    g = pu.mutants_of(anc, iset, 12, rate=0.02, seed=5)
    return iset, env, cfg, n, g


def test_soup_world_fills_oracle(golden):
    """the oracle world grows from 12 organisms to a full grid (soup births
    need no empty neighbour, so the growth is not a front)"""
    iset, env, cfg, n, g = _grow_pair(golden, 1, 0)
    b = ol.Backend("oracle", cfg, iset, env, ncells=n)
    b.set_orgs(0, g, deterministic=False)
    full = None
    for upd in range(120):
        s = b.run_update()
        if full is None and s.num_organisms == n:
            full = upd
    b.close()
    assert full is not None and full < 110, full


@pytest.mark.gpu
@pytest.mark.parametrize("prefer_empty,allow_parent", [(1, 0), (1, 1), (0, 0), (0, 1)])
def test_soup_world_gpu(golden, prefer_empty, allow_parent):
    """12 mutants in a 32x32 grid, 130 updates (the grid fills, then births
    replace organisms anywhere): every update's counters, then every cell,
    field and digest, GPU world == oracle world"""
    iset, env, cfg, n, g = _grow_pair(golden, prefer_empty, allow_parent)
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(0, g, deterministic=False)
    births = 0
    for upd in range(130):
        so, sg = orc.run_update(), gpu.run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten", "births_cancelled"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        births += so.births
    assert births > 500
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
    nbad, cells = pu.compare_digests(orc.digests(), gpu.digests())
    assert nbad == 0, cells


def _serial_pair(golden, prefer_empty, allow_parent, side=16, seed=29):
    ov = {"WORLD_X": side, "WORLD_Y": side, "BIRTH_METHOD": 4, "PREFER_EMPTY": prefer_empty,
          "ALLOW_PARENT": allow_parent}
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=seed)
    n = cfg.world_x * cfg.world_y
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    g = pu.mutants_of(anc, iset, 6, rate=0.02, seed=7)
    return iset, env, cfg, n, g


@pytest.mark.gpu
@pytest.mark.parametrize("prefer_empty,allow_parent", [(1, 0), (1, 1), (0, 0), (0, 1)])
def test_soup_serial_world_gpu(golden, prefer_empty, allow_parent):
    """the serial world with soup births, 6 mutants on a 16x16 grid, 90
    updates (it fills; then FindRandEmptyCell sees a full world): every
    update's counters, then every cell and field, GPU == oracle"""
    iset, env, cfg, n, g = _serial_pair(golden, prefer_empty, allow_parent)
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(0, g, deterministic=False)
    births = 0
    for upd in range(90):
        so, sg = orc.run_serial_update(), gpu.run_serial_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        births += so.births
    assert births > 150
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"


def _growth(args):
    """organisms at updates 10, 20, ..., 100 of one seed (a worker process)"""
    root, seed, serial = args
    for p in (root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import oracle_lib as olw
    import parity_util as puw
    from avida_amd import files as fw
    golden = os.path.join(root, "tests", "golden")
    ov = {"WORLD_X": 32, "WORLD_Y": 32, "BIRTH_METHOD": 4, "PREFER_EMPTY": 1, "ALLOW_PARENT": 1}
    iset, env, cfg = puw.load_env(golden, overrides=ov, seed=seed)
    anc = fw.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = olw.Backend("oracle", cfg, iset, env, ncells=1024)
    b.set_orgs(0, [anc] * 8, deterministic=False)
    out = []
    for u in range(100):
        s = b.run_serial_update() if serial else b.run_update()
        if u % 10 == 9:
            out.append(s.num_organisms)
    b.close()
    return out


def test_soup_batch_growth_matches_serial():
    """8 ancestors on a 32x32 grid with soup births, 40 seeds per world: the
    batch world's population at updates 50..100 against the serial world's
    (the reference's schedule), Welch t and KS two-sample tests, Bonferroni at
    a family-wise 0.01 (measured with 48 seeds: means within 0.3 sd of the
    serial world's at every printed update)."""
    from scipy import stats
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    seeds = range(1, 41)
    with ProcessPoolExecutor(8, mp_context=multiprocessing.get_context("forkserver")) as ex:
        ser = np.array(list(ex.map(_growth, [(root, s, True) for s in seeds])))
        bat = np.array(list(ex.map(_growth, [(root, s + 1000, False) for s in seeds])))
    cols = range(4, 10)                  # updates 50, 60, ..., 100
    alpha = 0.01 / (2 * len(cols))
    for k in cols:
        pt = stats.ttest_ind(bat[:, k], ser[:, k], equal_var=False).pvalue
        pk = stats.ks_2samp(bat[:, k], ser[:, k]).pvalue
        assert pt > alpha and pk > alpha, (10 * (k + 1), bat[:, k].mean(), ser[:, k].mean(), pt, pk)
    assert ser[:, -1].mean() > 300
