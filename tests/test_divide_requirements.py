"""cOrganism::Divide_CheckViable's task / reaction requirements
(main/cOrganism.cc:788-919): REQUIRED_TASK (unless IMMUNITY_TASK was done),
REQUIRED_REACTION (unless IMMUNITY_REACTION), MAX_UNIQUE_TASK_COUNT and
REQUIRE_SINGLE_REACTION fail an h-divide that lacks them.

Known answers, on the test CPU (cTestCPU, the oracle) over the first 600 of
the reference's detail-recalc genomes, whose unconstrained results are the
reference's own file (tests/test_oracle_golden.py): under a requirement every genome that
divides meets it at its divide, and every genome whose unconstrained divide
met it divides exactly as before (the check has no side effect).  The
ancestor, which performs no task, never reproduces when a task or a reaction
is required.  On the GPU: the test CPU over the same genomes and a mutating
world of the evolved population, the oracle's bit for bit."""
import os

import pytest

from avida_amd import files
import oracle_lib as ol
import parity_util as pu

# (the genomes perform nand, orn, andn and nor; library index = logic-9 order)
KNOBS = [
    {"REQUIRED_TASK": 3},                              # orn
    {"REQUIRED_TASK": 3, "IMMUNITY_TASK": 6},          # orn, unless nor
    {"REQUIRED_REACTION": 5},                          # the andn reaction
    {"REQUIRED_REACTION": 5, "IMMUNITY_REACTION": 1},  # andn, unless nand
    {"MAX_UNIQUE_TASK_COUNT": 2},
    {"REQUIRE_SINGLE_REACTION": 1},
]


def _genomes(golden, iset):
    _, rows = files.parse_detail_dat(os.path.join(golden, "detail-recalc.dat"))
    return [iset.parse_sequence(r[8]) for r in rows[:600]]


def _meets(ov, tasks):
    """the requirement, from a divide's task counts (reaction i = task i in the
    logic-9 environment)"""
    if "REQUIRED_TASK" in ov:
        return tasks[ov["REQUIRED_TASK"]] > 0 or ("IMMUNITY_TASK" in ov and tasks[ov["IMMUNITY_TASK"]] > 0)
    if "REQUIRED_REACTION" in ov:
        return tasks[ov["REQUIRED_REACTION"]] > 0 or ("IMMUNITY_REACTION" in ov and
                                                     tasks[ov["IMMUNITY_REACTION"]] > 0)
    if "MAX_UNIQUE_TASK_COUNT" in ov:
        return sum(t > 0 for t in tasks) <= ov["MAX_UNIQUE_TASK_COUNT"]
    return any(t > 0 for t in tasks)


def _key(r):
    return (r.divided, r.gestation_time, r.copied_size, r.executed_size, r.merit, list(r.task_count)[:9])


@pytest.mark.parametrize("ov", KNOBS)
def test_test_cpu_requirement_known_answers(golden, ov):
    iset, env, cfg0 = pu.load_env(golden, "instset-classic.cfg")
    _, _, cfg = pu.load_env(golden, "instset-classic.cfg", overrides=ov)
    genomes = _genomes(golden, iset)
    free = ol.Backend("oracle", cfg0, iset, env, ncells=16).test_genomes(genomes)
    req = ol.Backend("oracle", cfg, iset, env, ncells=16).test_genomes(genomes)
    n_same = n_div = 0
    for (rf, _, _), (rr, _, _) in zip(free, req):
        tf = list(rf.task_count)[:9]
        if rr.divided:
            n_div += 1
            assert _meets(ov, list(rr.task_count)[:9])
        if rf.divided and _meets(ov, tf):
            assert _key(rr) == _key(rf)
            n_same += 1
    assert n_same > 0 and n_div > 0


@pytest.mark.parametrize("ov", [{"REQUIRED_TASK": 0}, {"REQUIRE_SINGLE_REACTION": 1}, {"REQUIRED_REACTION": 0}])
def test_taskless_ancestor_never_reproduces(golden, ov):
    iset, env, cfg = pu.load_env(golden, overrides=dict(ov, WORLD_X=6, WORLD_Y=6))
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend("oracle", cfg, iset, env, ncells=36)
    b.set_orgs(0, [anc] * 4)
    assert sum(b.run_update().births for _ in range(40)) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("ov", KNOBS)
def test_requirements_gpu_equals_oracle(golden, ov):
    iset, env, cfg = pu.load_env(golden, "instset-classic.cfg", overrides=ov)
    genomes = _genomes(golden, iset)
    o = ol.Backend("oracle", cfg, iset, env, ncells=16).test_genomes(genomes)
    g = ol.Backend("gpu", cfg, iset, env, ncells=16).test_genomes(genomes)
    assert [_key(r) for r, _, _ in o] == [_key(r) for r, _, _ in g]
    # a mutating world of those genomes under the requirement (detail-50000.pop's
    # organisms all perform the nine tasks)
    ovw = dict(ov, WORLD_X=40, WORLD_Y=40)
    iset, env, cfg = pu.load_env(golden, "instset-classic.cfg", overrides=ovw, seed=23)
    pop = (genomes * 3)[:1600]
    wo = ol.Backend("oracle", cfg, iset, env, ncells=1600)
    wg = ol.Backend("gpu", cfg, iset, env, ncells=1600)
    for b in (wo, wg):
        b.set_orgs(0, pop, deterministic=False)
    births = 0
    for _ in range(25):
        so, sg = wo.run_update(), wg.run_update()
        assert (so.births, so.insts_executed, so.divides) == (sg.births, sg.insts_executed, sg.divides)
        births += so.births
    assert (wo.digests() == wg.digests()).all()
    assert births > 0
