"""Checkpoint / resume and mid-run injection of the serial world (ADVICE r5:
the reaper queue and the soup's empty_cell_id_array are persistent state).

avida_amd/checkpoint.py saves the serial world's own state with the
organisms' (avgpu_get_serial_state: the scheduler's and the context stream's
positions, speculative credits and deaths, connection-list rotations,
BIRTH_METHOD 4's empty_cell_id_array, BIRTH_METHOD 5's reaper queue), so a
restored serial world continues bit for bit like the one that never stopped;
an injection after the queue exists maintains it as the reference's
InjectGenome + ActivateOrganism do (main/cPopulation.cc:6964-6968,
:1358-1361).  Worlds: 16 x 16, eight ancestors spread over the grid, so that
births land in empty cells (soup draws) and replace organisms (reaper pops)."""
import os

import pytest

from avida_amd import files
import oracle_lib as ol
import parity_util as pu
import test_checkpoint as tc

X = Y = 16
N = X * Y
SEEDS = {4: 11, 5: 13, 0: 17}


def _world(kind, golden, bm, seed=None):
    ov = {"WORLD_X": X, "WORLD_Y": Y, "BIRTH_METHOD": bm, "ALLOW_PARENT": 1}
    if bm == 4:
        ov["PREFER_EMPTY"] = 1
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=SEEDS[bm] if seed is None else seed)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend(kind, cfg, iset, env, ncells=N)
    for k in range(8):
        b.set_orgs(k * 37 % N, [anc], deterministic=False)
    b.anc = anc
    return b


def _run(b, n):
    return [b.run_serial_update() for _ in range(n)]


def _same(a, b):
    tc.compare(a, b, N)


def _stats_equal(sa, sb):
    for x, y in zip(sa, sb):
        for f in ("update", "num_organisms", "insts_executed", "births", "deaths", "cum_insts_executed"):
            assert getattr(x, f) == getattr(y, f), f


def _resume(kind_a, kind_b, golden, bm, tmp_path, u1=30, u2=25):
    a = _world(kind_a, golden, bm)
    _run(a, u1)
    path = os.path.join(tmp_path, "s.npz")
    a.checkpoint(path)
    b = _world(kind_b, golden, bm, seed=99)
    b.restore(path)
    _same(a, b)
    _stats_equal(_run(a, u2), _run(b, u2))
    _same(a, b)
    a.close()
    b.close()


@pytest.mark.parametrize("bm", [4, 5, 0])
def test_oracle_serial_resume(golden, tmp_path, bm):
    _resume("oracle", "oracle", golden, bm, tmp_path)


def _inject(b, cells):
    for c in cells:
        b.set_orgs(c, [b.anc], deterministic=False)


@pytest.mark.parametrize("bm", [5, 4])
def test_oracle_serial_injection_then_resume(golden, tmp_path, bm):
    """an injection after the first serial updates (into living and empty
    cells), then a checkpoint: the restored world continues like the original"""
    a = _world("oracle", golden, bm)
    _run(a, 25)
    _inject(a, [0, 1, 100, 200, 255])
    _run(a, 5)
    path = os.path.join(tmp_path, "i.npz")
    a.checkpoint(path)
    b = _world("oracle", golden, bm, seed=7)
    b.restore(path)
    _stats_equal(_run(a, 20), _run(b, 20))
    _same(a, b)


def test_reaper_queue_injection_oracle(golden):
    """the queue after an injection: an occupied cell's entry taken out (the
    first from the front), the cell pushed at the front"""
    import ctypes as C
    import numpy as np
    from avida_amd import capi
    a = _world("oracle", golden, 5)
    _run(a, 20)

    def queue():
        st = capi.AvgpuSerialState()
        q = np.zeros(2 * N + 64, dtype=np.int32)
        a._call("get_serial_state", a.h, C.byref(st), None, None, None, q.ctypes.data_as(C.c_void_p), len(q))
        return list(q[:st.reaper_len])

    q0 = queue()
    alive = {c for c in range(N) if a.states(c, 1, 8)[0][0].alive}
    c_live = min(alive)
    c_dead = min(set(range(N)) - alive)
    _inject(a, [c_live])
    q1 = queue()
    front = len(q0) - 1 - q0[::-1].index(c_live)         # its newest entry
    assert q1 == q0[:front] + q0[front + 1:] + [c_live]
    _inject(a, [c_dead])
    assert queue() == q1 + [c_dead]


@pytest.mark.gpu
@pytest.mark.parametrize("bm", [4, 5])
def test_gpu_serial_resume_and_injection(golden, tmp_path, bm):
    """the GPU serial world: resumed from the oracle's checkpoint and from its
    own, and injected into mid-run, the oracle's world bit for bit"""
    _resume("oracle", "gpu", golden, bm, tmp_path)
    _resume("gpu", "gpu", golden, bm, tmp_path)
    o, g = _world("oracle", golden, bm), _world("gpu", golden, bm)
    _stats_equal(_run(o, 25), _run(g, 25))
    _inject(o, [0, 1, 100, 200, 255])
    _inject(g, [0, 1, 100, 200, 255])
    _stats_equal(_run(o, 20), _run(g, 20))
    _same(o, g)
