"""BIRTH_METHOD 5 (POSITION_OFFSPRING_FULL_SOUP_ELDEST,
main/cPopulation.cc:5312-5319) in the serial world (the reference's own
schedule): an offspring takes the cell of the reaper queue's rear entry
(PopRear; without ALLOW_PARENT the parent's is pushed back to the rear and
the next one taken), and ActivateOrganism pushes every newborn's cell at the
front (:1358-1361); deaths leave the queue alone (oracle serial_eldest,
interp.hip k_serial_update).  The queue starts as the reference's Setup
order (cells 0..N-1, :343-347) followed by the living cells in ascending
order (their injections).  The batch world and strips refuse the method.

KAT: one ancestor about to divide in an otherwise empty 9x9 grid -- its
offspring lands in cell 0 (the queue's rear), or in cell 1 when the parent
sits in cell 0 without ALLOW_PARENT.  World: 6 mutants on a 16x16 grid, 90
serial updates, GPU == oracle."""
import ctypes as C
import os

import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu
from test_birth_soup import _about_to_divide

CAP = capi.MAX_GENOME
OV = {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0, "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0}


def _serial_child(kind, golden, parent_cell, allow_parent, x=9):
    ov = dict(OV, WORLD_X=x, WORLD_Y=x, BIRTH_METHOD=5, ALLOW_PARENT=allow_parent, WORLD_GEOMETRY=1)
    s0, ops0, fl0 = _about_to_divide(golden, ov)
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=3)
    n = x * x
    b = ol.Backend(kind, cfg, iset, env, ncells=n)
    st, ops, fl = b.states(0, n, CAP)
    st[parent_cell] = s0
    ops = bytearray(ops)
    fl = bytearray(fl)
    ops[parent_cell * CAP:(parent_cell + 1) * CAP] = ops0[:CAP]
    fl[parent_cell * CAP:(parent_cell + 1) * CAP] = fl0[:CAP]
    o = (C.c_uint8 * len(ops)).from_buffer(ops)
    f = (C.c_uint8 * len(fl)).from_buffer(fl)
    b._call("set_states", b.h, 0, n, st, o, f, CAP)
    s = b.run_serial_update()
    after, _, _ = b.states(0, n, CAP)
    b.close()
    assert s.births == 1, s.births
    kids = [c for c in range(n) if after[c].generation == 1 and after[c].num_divides == 0]
    assert len(kids) == 1, kids
    return kids[0]


@pytest.mark.parametrize("kind", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_eldest_kat(golden, kind):
    assert _serial_child(kind, golden, 40, 1) == 0
    assert _serial_child(kind, golden, 40, 0) == 0
    assert _serial_child(kind, golden, 0, 0) == 1      # the parent's cell is skipped (pushed back)
    assert _serial_child(kind, golden, 0, 1) == 0      # ALLOW_PARENT: the parent is replaced


def test_eldest_refused_on_batch_and_strips(golden):
    ov = dict(OV, WORLD_X=8, WORLD_Y=8, BIRTH_METHOD=5)
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=3)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend("oracle", cfg, iset, env, ncells=64)
    b.set_orgs(0, [anc] * 4, deterministic=False)
    with pytest.raises(RuntimeError):
        b.run_update()
    with pytest.raises(RuntimeError):
        b._call("set_tile", b.h, C.c_int64(0), C.c_int64(1 << 20))
    b.run_serial_update()
    b.close()
    lib = capi.load_product()
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"BIRTH_METHOD": 5}))
    assert lib.avgpu_check_cfg(C.byref(c)) == 0
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"BIRTH_METHOD": 6}))
    assert lib.avgpu_check_cfg(C.byref(c)) == -5


@pytest.mark.gpu
@pytest.mark.parametrize("allow_parent", [0, 1])
def test_eldest_serial_world_gpu(golden, allow_parent):
    """6 mutants on a 16x16 grid, 90 serial updates with the reaper queue:
    every update's counters, then every cell and field, GPU == oracle"""
    ov = {"WORLD_X": 16, "WORLD_Y": 16, "BIRTH_METHOD": 5, "ALLOW_PARENT": allow_parent}
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=31)
    n = cfg.world_x * cfg.world_y
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    g = pu.mutants_of(anc, iset, 6, rate=0.02, seed=7)
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
    assert births > 80
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
