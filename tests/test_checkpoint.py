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


def test_older_checkpoint_formats_load(golden, tmp_path):
    """A checkpoint written before round 4 (stats without births_cancelled /
    seed, or round 6's sub-step predictor and pick carry) and round 5 (state records without `age`) loads: the missing
    fields are zero -- the world's configured seed stays, every organism's
    age is 0 -- and the world continues."""
    import ctypes as C
    import numpy as np
    n = 32 * 32
    a = _world("oracle", golden, "logic9")
    for _ in range(10):
        a.run_update()
    path = os.path.join(tmp_path, "w.npz")
    a.checkpoint(path)
    z = dict(np.load(path, allow_pickle=False))
    size = C.sizeof(capi.AvgpuCpuState)
    off = capi.AvgpuCpuState.age.offset
    raw = z["states"].tobytes()
    old = b"".join(raw[k * size:k * size + off] + raw[k * size + off + 8:(k + 1) * size] for k in range(n))
    z["states"] = np.frombuffer(old, dtype=np.uint8)
    z["stats"] = z["stats"][:capi.AvgpuUpdateStats.births_cancelled.offset]   # no births_cancelled, seed, ...
    for k in ("version", "state_size", "stats_size"):
        z.pop(k)
    old_path = os.path.join(tmp_path, "old.npz")
    np.savez_compressed(old_path, **z)
    b = _world("oracle", golden, "logic9", seed=5)
    last = b.restore(old_path)
    assert last.update == 9 and last.seed == 0 and last.births_cancelled == 0
    st, _, _ = b.states(0, n, CAP)
    assert all(st[i].age == 0 for i in range(n))
    sa, _, _ = a.states(0, n, CAP)
    assert [sa[i].merit for i in range(n)] == [st[i].merit for i in range(n)]
    for _ in range(5):
        b.run_update()
    assert b.run_update().num_organisms > 0
