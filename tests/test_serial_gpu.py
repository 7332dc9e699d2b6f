"""The serial world (avgpu_run_serial_updates): the
reference's own update schedule -- a merit-weighted pick of one organism per
step from the scheduler's stream, ProcessStepSpeculative's run-ahead,
offspring placed at once (main/cPopulation.cc:5698-5788, :621-952) -- run by
the product's interpreter on the GPU, against the oracle's restatement of the
same loop (oracle/oracle.cc orc_run_serial_updates): every update's
statistics and, at the end, every cell and every field bit for bit."""
import os

import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

pytestmark = pytest.mark.gpu
CAP = capi.MAX_GENOME
# integer statistics bit for bit; the double sums over organisms within 1e-12
# relative (the statistics kernels and the oracle add in different orders)
INT_FIELDS = ("num_organisms", "insts_executed", "births", "births_dropped", "deaths", "divides",
              "cum_insts_executed", "cum_births")
SUM_FIELDS = ("sum_merit", "sum_fitness", "sum_gestation", "sum_mem_size")


def _compare_states(orc, gpu, n):
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"


def _run(orc, gpu, updates):
    last = None
    for u in range(updates):
        so = orc.run_serial_update()
        sg = gpu.run_serial_update()
        for f in INT_FIELDS:
            assert getattr(so, f) == getattr(sg, f), (u, f, getattr(so, f), getattr(sg, f))
        for f in SUM_FIELDS:
            a, b = getattr(so, f), getattr(sg, f)
            assert abs(a - b) <= 1e-12 * max(1.0, abs(a)), (u, f, a, b)
        last = so
    return last


def test_serial_world_from_ancestor(golden):
    """One ancestor on a 60x60 torus, default mutation rates, 120 serial
    updates: the colony grows through thousands of immediate placements."""
    iset, env, cfg = pu.load_env(golden, seed=101)
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    center = (cfg.world_y // 2) * cfg.world_x + cfg.world_x // 2
    for b in (orc, gpu):
        b.set_orgs(center, [anc], deterministic=False)
    last = _run(orc, gpu, 200)
    _compare_states(orc, gpu, n)
    assert last.num_organisms > 20 and last.births > 0


def test_serial_world_dense_population(golden):
    """The bench's evolved logic-9 population (detail-50000.pop, classic
    instset) filling a 60x60 torus, with the divide slip, uniform and
    per-site (DIV_MUT_PROB, PARENT_MUT_PROB) and Poisson mutations on as well: 4 serial updates (~430k picks)."""
    iset, env, cfg = pu.load_env(golden, "instset-classic.cfg", seed=5,
                                 overrides={"DIVIDE_SLIP_PROB": 0.05, "DIVIDE_UNIFORM_PROB": 0.02,
                                            "DIV_MUT_PROB": 0.005, "PARENT_MUT_PROB": 0.002,
                                            "DIVIDE_POISSON_MUT_MEAN": 0.5,
                                            "DIVIDE_POISSON_INS_MEAN": 0.2,
                                            "DIVIDE_POISSON_DEL_MEAN": 0.2,
                                            "DIV_INS_PROB": 0.002, "DIV_DEL_PROB": 0.002,
                                            "DIV_UNIFORM_PROB": 0.002, "DIV_SLIP_PROB": 0.0005})
    n = cfg.world_x * cfg.world_y
    genomes = pu.pop_genomes(golden, iset)[:n]
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(0, genomes, deterministic=False)
    _run(orc, gpu, 4)
    _compare_states(orc, gpu, n)


def test_serial_world_refuses_recorded_streams(golden):
    iset, env, cfg = pu.load_env(golden, seed=3)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=cfg.world_x * cfg.world_y)
    import numpy as np
    n = cfg.world_x * cfg.world_y
    gpu.set_rng_mode(capi.RNG_RECORDED, np.full(16, 0.5), np.zeros(n, dtype=np.int64))
    with pytest.raises(RuntimeError, match="counter streams"):
        gpu.run_serial_update()
