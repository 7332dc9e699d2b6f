"""GPU parity: the HIP interpreter (through the C-ABI) against the CPU oracle
and the reference's golden vectors.  Integer/byte state must match bit for bit;
doubles (merit, bonus, fitness) must match exactly too, because both sides
perform the same IEEE operations without contraction."""
import os

import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

pytestmark = pytest.mark.gpu
CAP = capi.MAX_GENOME


def _pair(golden, n, instset="instset-heads.cfg", overrides=None, seed=7):
    iset, env, cfg = pu.load_env(golden, instset, overrides, seed)
    return (ol.Backend("oracle", cfg, iset, env, ncells=n),
            ol.Backend("gpu", cfg, iset, env, ncells=n), iset)


def _run_compare(orc, gpu, n, chunks, mode=capi.MODE_FROZEN):
    for budget in chunks:
        orc.step(0, n, uniform=budget, mode=mode)
        gpu.step(0, n, uniform=budget, mode=mode)
        a, oa, fa = orc.states(0, n, CAP)
        b, ob, fb = gpu.states(0, n, CAP)
        bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
        assert not bad, f"{len(bad)} mismatches after budget {budget}: {bad[:5]}"


def test_test_cpu_detail_recalc_on_gpu(golden):
    """All 1794 golden genomes recalculated by the GPU test-CPU path."""
    iset, env, cfg = pu.load_env(golden, "instset-classic.cfg")
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=16)
    fmt, rows = files.parse_detail_dat(os.path.join(golden, "detail-recalc.dat"))
    genomes = [iset.parse_sequence(r[8]) for r in rows]
    res = ol.recalculate(gpu, genomes)
    bad = []
    for row, (r, flags, viable) in zip(rows, res):
        got = [int(viable), r.copied_size, r.executed_size, "%g" % r.merit, r.gestation_time,
               flags, [int(x) for x in list(r.task_count)[:9]]]
        exp = [int(row[10]), int(row[11]), int(row[12]), "%g" % float(row[13]), int(row[15]),
               row[19], [int(x) for x in row[20:29]]]
        if got != exp:
            bad.append((row[0], exp, got))
    assert not bad, f"{len(bad)} mismatches: {bad[:3]}"


@pytest.mark.parametrize("death", [0, 2])
def test_frozen_population_config2(golden, death):
    """BASELINE config 2: frozen 3600-organism population, mutations off,
    10^4 instructions per organism; per-lane state compared after every chunk."""
    iset_c = files.read_instset(os.path.join(golden, "instset-classic.cfg"))
    genomes = pu.pop_genomes(golden, iset_c)
    anc = files.read_org(os.path.join(golden, "default-heads.org"),
                         files.read_instset(os.path.join(golden, "instset-heads.cfg")))
    # the ancestor re-expressed in classic op codes
    heads = files.read_instset(os.path.join(golden, "instset-heads.cfg"))
    anc_c = bytes(iset_c.op_of_name(heads.names[o]) for o in anc)
    genomes = genomes[:3599] + [anc_c]
    n = len(genomes)
    assert n == 3600
    ov = {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0, "DIVIDE_DEL_PROB": 0.0,
          "DEATH_METHOD": death}
    orc, gpu, iset = _pair(golden, n, "instset-classic.cfg", ov)
    orc.set_orgs(0, genomes, deterministic=False)
    gpu.set_orgs(0, genomes, deterministic=False)
    _run_compare(orc, gpu, n, [1, 29, 970, 3000, 6000])


def test_random_genomes_fuzz(golden):
    """Random genomes 8..2048 sites (all LDS size classes, spills, faults)."""
    orc, gpu, iset = _pair(golden, 512, overrides={"DEATH_METHOD": 0})
    g = pu.random_genomes(iset, 384, 8, 300, seed=11) + pu.random_genomes(iset, 128, 300, 2048, seed=12)
    orc.set_orgs(0, g, deterministic=False)
    gpu.set_orgs(0, g, deterministic=False)
    _run_compare(orc, gpu, len(g), [1, 7, 500, 1500])


def test_ancestor_mutants_fuzz(golden):
    """Point mutants of the ancestor with copy mutations ON (FROZEN mode draws
    copy mutations from the per-organism counter stream on both sides)."""
    orc, gpu, iset = _pair(golden, 1024, overrides={"DEATH_METHOD": 0, "COPY_MUT_PROB": 0.02})
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    g = pu.mutants_of(anc, iset, 1024, rate=0.03, seed=5)
    orc.set_orgs(0, g, deterministic=False)
    gpu.set_orgs(0, g, deterministic=False)
    _run_compare(orc, gpu, len(g), [250, 750, 2000])


@pytest.mark.timeout(900)
def test_world_updates_bit_exact(golden):
    """BASELINE.json configs[0] at its stated length: the default avida.cfg
    world (60x60 torus, heads_default, logic-9, default mutation rates), the
    default-heads ancestor injected once, 1000 full batch-synchronous updates
    (allot, interpret with copy/divide mutations, time-ordered placement,
    activation): every update's counters equal, then GPU world == oracle
    world, every cell, every field, and the cell digests."""
    iset, env, cfg = pu.load_env(golden, seed=101)
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    center = (cfg.world_y // 2) * cfg.world_x + cfg.world_x // 2
    for b in (orc, gpu):
        b.set_orgs(center, [anc], deterministic=False)
    for upd in range(1000):
        so = orc.run_update()
        sg = gpu.run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten", "births_cancelled", "cum_insts_executed", "cum_births"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        assert list(so.task_orgs) == list(sg.task_orgs), upd
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
    nbad, cells = pu.compare_digests(orc.digests(0, n), gpu.digests(0, n))
    assert nbad == 0, f"{nbad} cell digests differ, first {cells}"
    assert so.num_organisms > 3000 and so.update == 999
    assert gpu.counters(cumulative=1)[capi.CNT_BAD_RECORD] == 0


def test_lazy_statistics_equal_eager(golden):
    """An update run with out == NULL skips the statistics reduction (the bench
    regime); the counts still reach the running sums (folded in by the next
    update's counter reset) and avgpu_get_stats reduces on demand: the same
    world run lazily equals the world run with statistics every update --
    stats, per-update and cumulative counters, every cell."""
    import ctypes as C
    iset, env, cfg = pu.load_env(golden, seed=101)
    n = cfg.world_x * cfg.world_y
    eager = ol.Backend("gpu", cfg, iset, env, ncells=n)
    lazy = ol.Backend("gpu", cfg, iset, env, ncells=n)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    for b in (eager, lazy):
        b.set_orgs(n // 2 + 30, [anc], deterministic=False)
    fields = [f for f, _ in capi.AvgpuUpdateStats._fields_]

    def vals(st):
        return [list(v) if hasattr(v, "__len__") else v for v in (getattr(st, f) for f in fields)]

    for upd in range(120):
        se = eager.run_update()
        lazy._call("run_update", lazy.h, None)
        if upd % 7 == 6 or upd > 110:
            sl = capi.AvgpuUpdateStats()
            lazy._call("get_stats", lazy.h, C.byref(sl))
            assert vals(se) == vals(sl), upd
            assert eager.counters(1) == lazy.counters(1), upd
            assert eager.counters(0) == lazy.counters(0), upd
        elif upd % 5 == 0:
            assert eager.counters(1) == lazy.counters(1), upd      # shards still pending
    assert se.num_organisms > 100 and se.cum_births > 100
    assert (eager.digests() == lazy.digests()).all()


@pytest.mark.parametrize("T,geometry", [(2, 2), (4, 2), (2, 1)])
def test_gpu_strip_tiles_equal_single_world(golden, T, geometry):
    """Multi-GPU row on one GPU: T strips of one 64x64 world run
    through the halo protocol (avida_amd/tiles.py, in-process loopback
    transport) equal the untiled oracle world, every cell, every field."""
    import torch
    from avida_amd import tiles
    import tile_util as tu
    X, Y, U = 64, 64, 40
    ref, rstats = tu.single("oracle", golden, X, Y, U, geometry=geometry)
    pairs = [tu.make_tile("gpu", golden, X, Y, T, k, geometry=geometry, device="cuda")
             for k in range(T)]
    world = tiles.StripWorld([t for _, t in pairs], tiles.LoopbackTransport())
    sent = 0
    for u in range(U):
        world.update()
        torch.cuda.synchronize()
        sent += sum(tu.records_sent(t) for _, t in pairs)
        tot = [tu.tile_stats(b) for b, _ in pairs]
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten"):
            assert sum(getattr(s, f) for s in tot) == getattr(rstats[u], f), (u, f)
    a, oa, fa = ref.states(0, X * Y, CAP)
    per = X * Y // T
    for k, (b, _) in enumerate(pairs):
        s, o, f = b.states(0, per, CAP)
        lo = k * per
        bad = pu.diff_states(a[lo:lo + per], s, oa[lo * CAP:(lo + per) * CAP], o,
                             fa[lo * CAP:(lo + per) * CAP], f, CAP)
        assert not bad, f"tile {k}: {len(bad)} mismatches, first {bad[:3]}"
    assert sent > 0


def _resource_env(golden, variant):
    """spatial_res_100u's environment (variant "flow": diffusion and gravity on,
    a torus ResA and a grid ResB, so FlowAll runs) or resources_9r's nine
    consumed global pools"""
    import copy
    if variant == "bench":
        import bench
        return files.parse_environment(bench.resource_env_text(48, 40)), \
            files.read_instset(os.path.join(golden, "resources_9r", "instset-heads.cfg")).parse_sequence(
                "rucavcqgfcqapqeccthzscpcccpqcxaqnccxxbcgdutycasvab")
    if variant == "9r":
        d = os.path.join(golden, "resources_9r")
        return files.read_environment(os.path.join(d, "environment.9resource")), \
            files.read_org(os.path.join(d, "9task.org"),
                           files.read_instset(os.path.join(d, "instset-heads.cfg")))
    env = files.read_environment(os.path.join(golden, "spatial_res_100u", "environment.cfg"))
    if variant in ("flow", "diffuse"):
        env = copy.deepcopy(env)
        a, b = env.resources[0], env.resources[1]
        a.geometry, a.xdiffuse, a.ydiffuse, a.xgravity, a.ygravity = 2, 1.0, 0.5, 0.2, -0.1
        a.inflow_x1, a.inflow_x2, a.inflow_y1, a.inflow_y2 = 40, 50, 45, 52    # box wraps the torus
        b.xdiffuse, b.ydiffuse, b.xgravity, b.ygravity = 0.3, 1.0, -0.4, 0.25
        if variant == "diffuse":     # zero gravity (one axis of ResB only)
            a.xgravity = a.ygravity = 0.0
            b.xgravity = 0.0
            # the global pool first (resource index != spatial slot), drawn on by AND
            order = [2, 0, 1]
            env.resources[:] = [env.resources[i] for i in order]
            for r in env:
                if r.resource:
                    r.resource = 1 + order.index(r.resource - 1)
            for c in env.cells:
                c.resource = order.index(c.resource)
            env[2].resource, env[2].max_fraction, env[2].max_number = 1, 0.01, 5.0
    iset = files.read_instset(os.path.join(golden, "resources_9r", "instset-heads.cfg"))
    return env, iset.parse_sequence("rucavcqgfcqapqeccthzscpcccpqcxaqnccxxbcgdutycasvab")


@pytest.mark.parametrize("variant", ["spatial", "flow", "diffuse", "9r", "bench"])
def test_world_updates_resources_bit_exact(golden, variant):
    """Updates with environment resources (the environment around the
    path): spatial grids, CELL lists, diffusion/gravity flows and consumed
    global pools; GPU world == oracle world, every cell, every field, and every
    resource level and per-cell amount bit for bit."""
    env, anc = _resource_env(golden, variant)
    iset = files.read_instset(os.path.join(golden, "resources_9r", "instset-heads.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": 48, "WORLD_Y": 40}), seed=23)
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(0, [anc] * 200, [100.0] * 200, deterministic=False)
    for upd in range(60):
        so = orc.run_update()
        sg = gpu.run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        lo, go = orc.resources(spatial=True)
        lg, gg = gpu.resources(spatial=True)
        assert lo == lg, (upd, lo, lg)
        assert go == gg, upd
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
    assert so.num_organisms > 200


@pytest.mark.parametrize("shape", [(130, 37), (5, 7), (63, 18), (2, 33), (124, 16)])
def test_resource_step_world_shapes(golden, shape):
    """k_res_step's windows (62 written columns x 16 rows a wave, the rim lanes
    wrapping mod WORLD_X): worlds narrower than a window, a last window that
    wraps, row counts off the band size, a torus and a grid resource with
    diffusion and gravity -- every level and per-cell amount == the oracle's
    after every update."""
    env, anc = _resource_env(golden, "flow")
    iset = files.read_instset(os.path.join(golden, "resources_9r", "instset-heads.cfg"))
    X, Y = shape
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": X, "WORLD_Y": Y}), seed=29)
    n = X * Y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    k = min(60, n // 2)
    for b in (orc, gpu):
        b.set_orgs(0, [anc] * k, [100.0] * k, deterministic=False)
    for upd in range(25):
        so, sg = orc.run_update(), gpu.run_update()
        assert (so.num_organisms, so.insts_executed, so.births) == (sg.num_organisms, sg.insts_executed, sg.births)
        lo, go = orc.resources(spatial=True)
        lg, gg = gpu.resources(spatial=True)
        assert lo == lg, (upd, lo, lg)
        assert go == gg, upd
    assert (orc.digests() == gpu.digests()).all()


@pytest.mark.parametrize("variant", ["logic9", "9r"])
def test_world_subupdates_bit_exact(golden, variant):
    """sub_updates = 3 (DESIGN.md 5 "Sub-updates": an update's picks in three
    batch steps, the scheduler weights re-read before each, resources stepped
    once per update, global consumption settled after each step): GPU world ==
    oracle world, every update's counters (summed over the steps), every
    resource level, then every cell, field and digest."""
    if variant == "logic9":
        iset, env, cfg = pu.load_env(golden, seed=31)
        anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
        orgs, merits, updates = [anc], None, 400
    else:
        env, anc = _resource_env(golden, variant)
        iset = files.read_instset(os.path.join(golden, "resources_9r", "instset-heads.cfg"))
        cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": 48, "WORLD_Y": 40}), seed=23)
        orgs, merits, updates = [anc] * 200, [100.0] * 200, 60
    cfg.sub_updates = 3
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(0 if merits else n // 2 + cfg.world_x // 2, orgs, merits, deterministic=False)
    for upd in range(updates):
        so = orc.run_update()
        sg = gpu.run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten", "births_cancelled", "cum_insts_executed", "cum_births", "slices"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        assert list(so.task_orgs) == list(sg.task_orgs), upd
        if variant != "logic9":
            assert orc.resources(spatial=True) == gpu.resources(spatial=True), upd
    # the update's picks are UD = AVE_TIME_SLICE x N split over the steps
    assert so.num_organisms > 100
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
    nbad, cells = pu.compare_digests(orc.digests(0, n), gpu.digests(0, n))
    assert nbad == 0, f"{nbad} cell digests differ, first {cells}"
    assert gpu.counters(cumulative=1)[capi.CNT_BAD_RECORD] == 0


@pytest.mark.parametrize("T,geometry,env_kind", [(2, 2, "tile"), (4, 1, "tile"), (4, 2, "bench")])
def test_gpu_strip_tiles_with_resources(golden, T, geometry, env_kind):
    """Config 5's path on one GPU: T strips with spatial resources (flows,
    inflow box and CELL list across strip edges, edge rows exchanged) and a
    consumed global pool (consumption all-reduced) == the untiled oracle world:
    organisms, per-cell amounts and pool levels bit for bit, every update."""
    import torch
    from avida_amd import tiles
    import tile_util as tu
    from test_tiles import resource_grids_match
    X, Y, U = 64, 64, 30
    if env_kind == "bench":          # configs[4]'s environment (bench.py --env resources)
        import bench
        env = files.parse_environment(bench.resource_env_text(X, Y))
    else:
        env = tu.resource_env(golden)
    per_update = []
    ref, rstats = tu.single("oracle", golden, X, Y, U, geometry=geometry, env=env,
                            on_update=lambda u, b: per_update.append(b.resources(spatial=True)))
    pairs = [tu.make_tile("gpu", golden, X, Y, T, k, geometry=geometry, device="cuda", env=env)
             for k in range(T)]
    world = tiles.StripWorld([t for _, t in pairs], tiles.LoopbackTransport())
    for u in range(U):
        world.update()
        torch.cuda.synchronize()
        tot = [tu.tile_stats(b) for b, _ in pairs]
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides"):
            assert sum(getattr(s, f) for s in tot) == getattr(rstats[u], f), (u, f)
        resource_grids_match(per_update[u], [b for b, _ in pairs], T, X, Y)
    a, oa, fa = ref.states(0, X * Y, CAP)
    per = X * Y // T
    for k, (b, _) in enumerate(pairs):
        s, o, f = b.states(0, per, CAP)
        lo = k * per
        bad = pu.diff_states(a[lo:lo + per], s, oa[lo * CAP:(lo + per) * CAP], o,
                             fa[lo * CAP:(lo + per) * CAP], f, CAP)
        assert not bad, f"tile {k}: {len(bad)} mismatches, first {bad[:3]}"


@pytest.mark.parametrize("kinds", [("gpu", "gpu"), ("gpu", "oracle"), ("oracle", "gpu")])
@pytest.mark.parametrize("env_kind", ["logic9", "resources"])
def test_checkpoint_resume_across_backends(golden, tmp_path, kinds, env_kind):
    """A checkpoint written by one backend and restored into the other (or the
    same) continues bit for bit like the world that never stopped."""
    from test_checkpoint import resume_case
    resume_case(kinds[0], kinds[1], golden, env_kind, tmp_path)


def test_driver_gpu_equals_oracle(golden, tmp_path):
    """avida_amd/driver.py on the GPU (ProductWorld) and on the oracle over the
    spatial_res_100u config: the data files agree (count with its genotype
    columns, tasks, resource, dominant exactly: the census is equal; averages to print precision -- their sums reduce in another order)."""
    from avida_amd import driver
    cfgdir = os.path.join(golden, "spatial_res_100u", "config")
    g, o = tmp_path / "gpu", tmp_path / "oracle"
    dg = driver.Driver(cfgdir, str(g))
    assert dg.run() == 100
    dg.world.close()
    driver.Driver(cfgdir, str(o), make_world=lambda cfg, iset, env: ol.Backend("oracle", cfg, iset, env)).run()

    def rows(p):
        return [l.split() for l in open(p) if l.strip() and not l.startswith("#")]
    for name in ("count.dat", "tasks.dat", "resource.dat", "dominant.dat"):
        assert rows(g / name) == rows(o / name), name
    for name in ("average.dat", "time.dat"):
        for a, b in zip(rows(g / name), rows(o / name)):
            assert [float(x) for x in a] == pytest.approx([float(x) for x in b], rel=1e-5), name


def test_trace_every_instruction(golden):
    """Per-instruction traces (avida_amd/trace.py, the reference tracer's
    PrintStatus at cpu/cHardwareCPU.cc:956): 192 organisms -- ancestor mutants
    and evolved detail-50000 genotypes -- single-stepped 600 times with copy
    and divide mutations on; GPU state == oracle state before every one of the
    600 instructions (no divergence can hide between chunk boundaries), and the
    PrintStatus texts agree."""
    from avida_amd import trace
    iset, env, cfg = pu.load_env(golden, overrides={"COPY_MUT_PROB": 0.02, "DIVIDE_MUT_PROB": 0.05,
                                                    "DEATH_METHOD": 0})
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    iset_c = files.read_instset(os.path.join(golden, "instset-classic.cfg"))
    pop = [bytes(iset.op_of_name(iset_c.names[o]) for o in g) for g in pu.pop_genomes(golden, iset_c)[::40][:96]]
    g = pu.mutants_of(anc, iset, 96, rate=0.02, seed=4) + pop
    n = len(g)
    orc, gpu = (ol.Backend(k, cfg, iset, env, ncells=n) for k in ("oracle", "gpu"))
    for b in (orc, gpu):
        b.set_orgs(0, g, deterministic=False)
    for step in range(600):
        a, oa, fa = orc.states(0, n, 512)
        s, os_, fs = gpu.states(0, n, 512)
        nbad, rep = pu.diff_states_np(a, s, oa, os_, fa, fs, 512)
        assert nbad == 0, f"before instruction {step + 1}: {nbad} organisms differ {rep[:3]}"
        if step % 150 == 0:
            for i in range(0, n, 17):
                assert trace.status_text(a[i], oa[i * 512:(i + 1) * 512], iset) == \
                    trace.status_text(s[i], os_[i * 512:(i + 1) * 512], iset)
        orc.step(0, n, uniform=1, mode=capi.MODE_FROZEN)
        gpu.step(0, n, uniform=1, mode=capi.MODE_FROZEN)
    assert sum(a[i].num_divides for i in range(n)) > 0


@pytest.mark.parametrize("allow_parent", [0, 1])
def test_birth_method3_full_grid(golden, allow_parent):
    """BIRTH_METHOD 3 (an empty neighbour, else the parent's cell without a
    draw; cPopulation::PositionOffspring, main/cPopulation.cc:5407) on a full
    grid: with ALLOW_PARENT 0 the offspring is never placed and the parent
    lives (ActivateOffspring :706-713, BS_NO_CELL, counted as dropped); with
    ALLOW_PARENT 1 it replaces its parent.  Every update's counters equal,
    then every cell and digest, GPU world == oracle world."""
    ov = {"WORLD_X": 32, "WORLD_Y": 32, "BIRTH_METHOD": 3, "ALLOW_PARENT": allow_parent}
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=29)
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    for b in (orc, gpu):
        b.set_orgs(0, [anc] * n, deterministic=False)
    dropped = births = 0
    for upd in range(40):
        so, sg = orc.run_update(), gpu.run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten", "births_cancelled"):
            assert getattr(so, f) == getattr(sg, f), (upd, f, getattr(so, f), getattr(sg, f))
        dropped += so.births_dropped
        births += so.births
    if allow_parent:
        assert births > 0 and dropped == 0
    else:
        assert dropped > 0 and births == 0   # the grid stays full of the ancestors
    a, oa, fa = orc.states(0, n, CAP)
    b, ob, fb = gpu.states(0, n, CAP)
    bad = pu.diff_states(a, b, oa, ob, fa, fb, CAP)
    assert not bad, f"{len(bad)} mismatches: {bad[:5]}"
    assert gpu.counters(cumulative=1)[capi.CNT_BAD_RECORD] == 0
