"""Scheduler weights near DBL_MAX: each weight is capped at 2^990
(oracle / device sched_weight), so the sums of the scheduler's tree over a
world stay finite and a world holding a few merits near DBL_MAX still hands
out its AVE_TIME_SLICE x N picks (uncapped, the tree's root was inf: every
node's p = x / inf drew nothing)."""
import os

import pytest

from avida_amd import files
import oracle_lib as ol
import parity_util as pu

X = Y = 8


def _world(kind, golden):
    iset, env, cfg = pu.load_env(golden, overrides={"WORLD_X": X, "WORLD_Y": Y}, seed=3)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend(kind, cfg, iset, env, ncells=X * Y)
    merits = [1.5e308 if c % 16 == 0 else 100.0 for c in range(X * Y)]
    b.set_orgs(0, [anc] * (X * Y), merits=merits)
    return b


def _check(b):
    st = b.run_update()
    n = st.num_organisms
    assert n == X * Y
    # the huge-merit organisms take (nearly) every pick between them
    assert st.insts_executed >= 0.9 * b.cfg.ave_time_slice * n, st.insts_executed
    return st


def test_huge_merits_oracle(golden):
    _check(_world("oracle", golden))


@pytest.mark.gpu
def test_huge_merits_gpu(golden):
    o, g = _world("oracle", golden), _world("gpu", golden)
    so, sg = _check(o), _check(g)
    assert (so.insts_executed, so.births) == (sg.insts_executed, sg.births)
    assert (o.digests() == g.digests()).all()
