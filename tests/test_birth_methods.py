"""BIRTH_METHOD 1 (PositionAge) and 2 (PositionMerit): with no empty
neighbour the offspring replaces the neighbour -- or, with ALLOW_PARENT, the
parent -- of the largest phenotype age (updates since birth or the last
divide; cPhenotype::IncAge in UpdateOrganismStats, main/cPopulation.cc:6021,
reset by DivideReset, main/cPhenotype.cc:950) or the largest age / merit
(cOrganism::CalcMeritRatio, main/cOrganism.cc:703-708); ties are drawn
(main/cPopulation.cc:5385-5413, :5416-5470).

KAT: a 5x5 torus full of ancestors; the centre organism is the ancestor one
instruction before its first h-divide (its FROZEN state after 388
instructions), its eight neighbours get chosen ages (and merits) through
avgpu_set_states; one update later the offspring must sit in the neighbour
the method names.  World: a full 32x32 grid, GPU == oracle bit for bit with
the age field in every state and digest."""
import ctypes as C
import os

import numpy as np
import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

CAP = capi.MAX_GENOME
X = 5
CENTRE = 2 * X + 2
NB = {"NW": 1 * X + 1, "N": 1 * X + 2, "NE": 1 * X + 3, "W": 2 * X + 1, "E": 2 * X + 3,
      "SW": 3 * X + 1, "S": 3 * X + 2, "SE": 3 * X + 3}
OV = {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0, "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0}


def _about_to_divide(kind, golden, ov):
    """(state, ops, flags) of the ancestor one instruction before its h-divide"""
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=5)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend(kind, cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.step(0, 1, uniform=388, mode=capi.MODE_FROZEN)
    st, ops, fl = b.states(0, 1, CAP)
    assert st[0].num_divides == 0 and ops[st[0].head[0]] == iset.op_of_name("h-divide")
    b.close()
    return st[0], ops, fl


def _kat(kind, golden, method, ages, merits, allow_parent=1):
    ov = dict(OV, WORLD_X=X, WORLD_Y=X, BIRTH_METHOD=method, ALLOW_PARENT=allow_parent)
    s0, ops0, fl0 = _about_to_divide(kind, golden, ov)
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=5)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    n = X * X
    b = ol.Backend(kind, cfg, iset, env, ncells=n)
    b.set_orgs(0, [anc] * n, merits=[100.0] * n, deterministic=False)
    st, ops, fl = b.states(0, n, CAP)
    st[CENTRE] = s0
    ops = bytearray(ops)
    fl = bytearray(fl)
    ops[CENTRE * CAP:(CENTRE + 1) * CAP] = ops0[:CAP]
    fl[CENTRE * CAP:(CENTRE + 1) * CAP] = fl0[:CAP]
    for name, c in NB.items():
        st[c].age = ages.get(name, 3)
        st[c].merit = merits.get(name, 100.0)
    o = (C.c_uint8 * len(ops)).from_buffer(ops)
    f = (C.c_uint8 * len(fl)).from_buffer(fl)
    b._call("set_states", b.h, 0, n, st, o, f, CAP)
    s = b.run_update()
    after, _, _ = b.states(0, n, CAP)
    b.close()
    assert s.births == 1, s.births
    return [c for c in range(n) if after[c].generation == 1 and after[c].num_divides == 0]


@pytest.mark.parametrize("kind", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_position_age_kat(golden, kind):
    # NE is the oldest neighbour: the offspring lands there
    assert _kat(kind, golden, 1, {"NE": 7}, {}) == [NB["NE"]]
    # two oldest: one of them (a draw)
    assert _kat(kind, golden, 1, {"W": 9, "S": 9}, {})[0] in (NB["W"], NB["S"])


@pytest.mark.parametrize("kind", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_position_merit_kat(golden, kind):
    # age / merit: NE 7 / 100 = 0.07 loses to SW 3 / 10 = 0.3
    assert _kat(kind, golden, 2, {"NE": 7}, {"SW": 10.0}) == [NB["SW"]]


def _full_grid_pair(golden, method, allow_parent):
    ov = {"WORLD_X": 32, "WORLD_Y": 32, "BIRTH_METHOD": method, "ALLOW_PARENT": allow_parent}
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=41)
    n = cfg.world_x * cfg.world_y
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    g = pu.mutants_of(anc, iset, n, rate=0.02, seed=3)
    return iset, env, cfg, n, g


def test_birth_methods_refused_where_unbuilt(golden):
    """the serial world and strip tiles refuse BIRTH_METHOD 1 / 2 (their
    placement has no age / merit of the ghost rows); PREFER_EMPTY 0 with
    them is refused by the library (the reference reads the organism of an
    empty cell)"""
    iset, env, cfg, n, g = _full_grid_pair(golden, 1, 1)
    b = ol.Backend("oracle", cfg, iset, env, ncells=n)
    b.set_orgs(0, g[:10], deterministic=False)
    with pytest.raises(RuntimeError):
        b.run_serial_update()
    lib = capi.load_product()
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"BIRTH_METHOD": 2, "PREFER_EMPTY": 0}))
    assert lib.avgpu_check_cfg(C.byref(c)) == -5
    for m in (1, 2):
        c = capi.cfg_from_avida(files.read_avida_cfg(None, {"BIRTH_METHOD": m}))
        assert lib.avgpu_check_cfg(C.byref(c)) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("method,allow_parent", [(1, 1), (1, 0), (2, 1), (2, 0)])
def test_birth_methods_full_grid_gpu(golden, method, allow_parent):
    """A full 32x32 grid of ancestor mutants, 60 updates: every birth
    replaces an organism chosen by age (1) or age / merit (2); every update's
    counters equal, then every cell, field (age included) and digest, GPU
    world == oracle world."""
    iset, env, cfg, n, g = _full_grid_pair(golden, method, allow_parent)
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(0, g, deterministic=False)
    births = 0
    for upd in range(60):
        so, sg = orc.run_update(), gpu.run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten", "births_cancelled"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        births += so.births
    assert births > 200
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
    assert len({a[c].age for c in range(n)}) > 3
    nbad, cells = pu.compare_digests(orc.digests(), gpu.digests())
    assert nbad == 0, cells
