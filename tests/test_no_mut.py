"""NO_MUT_INSTS (cHardwareCPU::checkNoMutList, cpu/cHardwareCPU.cc:797-810):
an h-copy whose read instruction's symbol is listed draws its copy mutation
but keeps the instruction (:7144), and a uniform copy mutation leaves a listed
write-head instruction (doUniformCopyMutation, cpu/cHardwareBase.cc:597-612).

Known answers on the oracle: with every site mutated on copy
(COPY_MUT_PROB 1), the first offspring keeps exactly the sites whose
instruction is listed and (with the whole instruction set listed) equals its
parent; the same with COPY_UNIFORM_PROB 1.  On the GPU: a mutating world with
a partial list equals the oracle's, every cell."""
import os

import pytest

from avida_amd import files
import oracle_lib as ol
import parity_util as pu

X = Y = 5


def _first_offspring(golden, ov):
    iset, env, cfg = pu.load_env(golden, overrides=dict({"WORLD_X": X, "WORLD_Y": Y, "DIVIDE_INS_PROB": 0.0,
                                                         "DIVIDE_DEL_PROB": 0.0, "DIVIDE_MUT_PROB": 0.0}, **ov),
                                 seed=3)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend("oracle", cfg, iset, env, ncells=X * Y)
    b.set_orgs(12, [anc])
    for _ in range(40):
        if b.run_update().births:
            break
    st, ops, _ = b.states(0, X * Y, 512)
    kids = [c for c in range(X * Y) if c != 12 and st[c].alive]
    assert kids, "no offspring"
    c = kids[0]
    return anc, bytes(ops[c * 512:c * 512 + st[c].genome_length]), iset


def test_copy_mutation_keeps_listed_instructions(golden):
    iset = files.read_instset(os.path.join(golden, "instset-heads.cfg"))
    every = "".join(iset.symbol(i) for i in range(len(iset.names)))
    anc, kid, _ = _first_offspring(golden, {"COPY_MUT_PROB": 1.0, "NO_MUT_INSTS": every})
    assert kid == anc
    anc, kid, _ = _first_offspring(golden, {"COPY_MUT_PROB": 1.0})
    assert kid != anc and len(kid) == len(anc)
    # a partial list: the listed sites survive every copy mutation
    keep = {iset.names.index("h-copy"), iset.names.index("nop-C")}
    anc, kid, _ = _first_offspring(golden, {"COPY_MUT_PROB": 1.0,
                                            "NO_MUT_INSTS": "".join(iset.symbol(o) for o in keep)})
    assert len(kid) == len(anc)
    assert all(k == a for k, a in zip(kid, anc) if a in keep)
    assert any(k != a for k, a in zip(kid, anc) if a not in keep)


def test_uniform_copy_mutation_keeps_listed_instructions(golden):
    iset = files.read_instset(os.path.join(golden, "instset-heads.cfg"))
    every = "".join(iset.symbol(i) for i in range(len(iset.names)))
    anc, kid, _ = _first_offspring(golden, {"COPY_UNIFORM_PROB": 1.0, "NO_MUT_INSTS": every})
    assert kid == anc
    anc, kid, _ = _first_offspring(golden, {"COPY_UNIFORM_PROB": 1.0})
    assert kid != anc


@pytest.mark.gpu
@pytest.mark.parametrize("ov", [{"COPY_MUT_PROB": 0.05}, {"COPY_MUT_PROB": 0.02, "COPY_UNIFORM_PROB": 0.02,
                                                          "COPY_INS_PROB": 0.01, "COPY_DEL_PROB": 0.01}])
def test_no_mut_world_gpu_equals_oracle(golden, ov):
    ov = dict(ov, WORLD_X=24, WORLD_Y=24, NO_MUT_INSTS="cdhk")
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=11)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    o = ol.Backend("oracle", cfg, iset, env, ncells=24 * 24)
    g = ol.Backend("gpu", cfg, iset, env, ncells=24 * 24)
    for b in (o, g):
        b.set_orgs(0, [anc] * 64, deterministic=False)
    births = 0
    for _ in range(60):
        so, sg = o.run_update(), g.run_update()
        assert (so.births, so.insts_executed) == (sg.births, sg.insts_executed)
        births += so.births
    assert (o.digests() == g.digests()).all()
    assert births > 0
