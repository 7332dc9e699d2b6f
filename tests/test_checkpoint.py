"""Checkpoint / resume (avida_amd/checkpoint.py over avgpu_get_states /
avgpu_set_states / avgpu_set_clock / avgpu_set_resources): a world saved
after U1 updates and restored into a fresh world continues bit for bit like
the world that never stopped -- organisms, statistics and resources."""
import os

import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu
import tile_util as tu

CAP = 512


def _world(kind, golden, env_kind, X=32, Y=32, seed=5):
    if env_kind == "logic9":
        iset, env, cfg = pu.load_env(golden, overrides={"WORLD_X": X, "WORLD_Y": Y}, seed=seed)
        anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
        genomes = pu.mutants_of(anc, iset, X * Y // 2, rate=0.01, seed=seed)
    else:
        env = tu.resource_env(golden)
        iset, _, cfg, genomes = tu.setup(golden, X, Y, seed=seed, env=env)
        genomes = genomes[:X * Y // 2]
    b = ol.Backend(kind, cfg, iset, env, ncells=X * Y)
    b.set_orgs(0, genomes, deterministic=False)
    return b


def compare(a, b, n):
    sa, oa, fa = a.states(0, n, CAP)
    sb, ob, fb = b.states(0, n, CAP)
    bad = pu.diff_states(sa, sb, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:3]}"
    if a.nres:
        assert a.resources(spatial=True) == b.resources(spatial=True)


def resume_case(kind_a, kind_b, golden, env_kind, tmp_path, u1=20, u2=15):
    n = 32 * 32
    a = _world(kind_a, golden, env_kind)
    for _ in range(u1):
        a.run_update()
    path = os.path.join(tmp_path, "w.npz")
    a.checkpoint(path)
    b = _world(kind_b, golden, env_kind, seed=99)        # different seed: everything comes from the file
    last = b.restore(path)
    assert last.update == u1 - 1
    compare(a, b, n)
    for _ in range(u2):
        sa, sb = a.run_update(), b.run_update()
        for f in ("update", "num_organisms", "insts_executed", "births", "deaths", "cum_insts_executed",
                  "cum_births"):
            assert getattr(sa, f) == getattr(sb, f), f
        assert list(sa.task_orgs) == list(sb.task_orgs)
        # the statistics' double sums reduce in a different order on the two
        # backends (the organisms' merits themselves are compared bit for bit)
        if kind_a == kind_b:
            assert sa.sum_merit == sb.sum_merit
        else:
            assert sa.sum_merit == pytest.approx(sb.sum_merit, rel=1e-12)
    compare(a, b, n)


@pytest.mark.parametrize("env_kind", ["logic9", "resources"])
def test_oracle_checkpoint_resume(golden, tmp_path, env_kind):
    resume_case("oracle", "oracle", golden, env_kind, tmp_path)
