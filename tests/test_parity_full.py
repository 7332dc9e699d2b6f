"""Full-size GPU parity at BASELINE.json's own configurations.

* configs[2]: the bench's 1024x1024 logic-9 world (every cell seeded from the
  detail-50000.pop genotype pool exactly as bench.build_world does, default
  mutation rates, births on) run on the GPU and on the oracle for 14 updates --
  two lock-step birth waves (updates 5 and 12: ~0.5M births each, most of them
  onto occupied cells) included.  Every update the counters must agree and
  every cell's state digest (avgpu_state_digests: registers, heads, stacks,
  label, phenotype, RNG position, tape with flags) must be equal.
* configs[3] geometry on one GPU: the 4096x4096 world as 8 row strips of
  4096x512 through the halo protocol (loopback transport) equals the untiled
  4096x4096 GPU world for 8 updates (the first birth wave crosses every strip
  edge), and the untiled GPU world equals the oracle after 2 updates.
"""
import ctypes as C
import os

import numpy as np
import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

pytestmark = pytest.mark.gpu


def _bench_seed(golden, X, Y):
    """cfg, instset, env and the per-cell (blob, lens, merits) of bench.build_world"""
    import bench
    iset, pool = bench._pool(golden)
    env = files.read_environment(os.path.join(golden, "environment-logic9.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": X, "WORLD_Y": Y}), seed=101)
    n = X * Y
    idx = (np.arange(n, dtype=np.uint64) * np.uint64(2654435761)) % np.uint64(len(pool))
    idx = idx.astype(np.int64)
    gen = np.empty(len(pool), dtype=object)
    gen[:] = [g for g, _ in pool]
    glen = np.array([len(g) for g, _ in pool], dtype=np.int32)
    gmer = np.array([m for _, m in pool], dtype=np.float64)
    return cfg, iset, env, idx, gen, glen, gmer


def _seed(backend, first, idx, gen, glen, gmer):
    blob = b"".join(gen[idx].tolist())
    backend.set_orgs_np(first, blob, glen[idx], gmer[idx], deterministic=False)


def _assert_digests(a, b, what, ba=None, bb=None, first=0):
    nbad, cells = pu.compare_digests(a, b, first)
    if nbad and ba is not None:
        report = []
        for c in cells[:3]:
            sa, oa, fa = ba.states(c, 1)
            sb, ob, fb = bb.states(c, 1)
            m = sa[0].mem_size
            report.append((c, [k for k in pu.STATE_FIELDS
                               if pu.state_tuple(sa[0])[k] != pu.state_tuple(sb[0])[k]]
                           + (["mem_ops"] if oa[:m] != ob[:m] else [])
                           + (["mem_flags"] if fa[:m] != fb[:m] else [])))
        cells = report
    assert nbad == 0, f"{what}: {nbad} cells differ, first {cells}"


STAT_FIELDS = ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
               "births_overwritten")


@pytest.mark.timeout(900)
def test_config2_full_world_bit_exact(golden):
    X = Y = 1024
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(golden, X, Y)
    orc = ol.Backend("oracle", cfg, iset, env, ncells=X * Y)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=X * Y)
    for b in (orc, gpu):
        _seed(b, 0, idx, gen, glen, gmer)
    _assert_digests(orc.digests(), gpu.digests(), "seeded world", orc, gpu)
    births = 0
    for u in range(14):
        so, sg = orc.run_update(), gpu.run_update()
        for f in STAT_FIELDS:
            assert getattr(so, f) == getattr(sg, f), (u, f, getattr(so, f), getattr(sg, f))
        births += sg.births
        _assert_digests(orc.digests(), gpu.digests(), f"update {u}", orc, gpu)
    assert births > 500_000 and sg.num_organisms > 1_000_000


@pytest.mark.timeout(1100)
def test_config3_geometry_strips_equal_untiled(golden):
    import torch
    from avida_amd import tiles
    X = Y = 4096
    T = 8
    rows = Y // T
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(golden, X, Y)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    full = ol.Backend("gpu", cfg, iset, env, ncells=X * Y)
    full.lib.avgpu_set_stream(full.h, stream)
    _seed(full, 0, idx, gen, glen, gmer)
    strips = []
    for k in range(T):
        b = ol.Backend("gpu", cfg, iset, env, ncells=X * rows)
        b.lib.avgpu_set_stream(b.h, stream)
        t = tiles.Tile(b.lib, b.p, b.h, k * rows, T, "cuda")
        sl = slice(k * rows * X, (k + 1) * rows * X)
        _seed(b, 0, idx[sl], gen, glen, gmer)
        strips.append((b, t))
    world = tiles.StripWorld([t for _, t in strips], tiles.LoopbackTransport())

    def strip_digests():
        return np.concatenate([b.digests() for b, _ in strips])

    # the oracle at this size for the first 2 updates
    orc = ol.Backend("oracle", cfg, iset, env, ncells=X * Y)
    _seed(orc, 0, idx, gen, glen, gmer)
    sent = births = 0
    for u in range(8):
        sf = full.run_update()
        births += sf.births
        world.update()
        torch.cuda.synchronize()
        sent += sum(int(t.rec_send[d][:4].cpu().view(torch.int32)[0]) for _, t in strips for d in range(2))
        st = []
        for b, _ in strips:
            s = capi.AvgpuUpdateStats()
            b._call("get_stats", b.h, s)
            st.append(s)
        for f in STAT_FIELDS:
            assert sum(getattr(s, f) for s in st) == getattr(sf, f), (u, f)
        df = full.digests()
        _assert_digests(df, strip_digests(), f"strips, update {u}")
        if orc is not None:
            so = orc.run_update()
            for f in STAT_FIELDS:
                assert getattr(so, f) == getattr(sf, f), (u, f, getattr(so, f), getattr(sf, f))
            _assert_digests(orc.digests(), df, f"oracle, update {u}", orc, full)
            if u == 1:
                orc.close()
                orc = None
    assert sent > 0, "no offspring crossed a strip edge"
    assert births > 1_000_000


def _resources_np(b, nres, n):
    """(levels, grids [nres][n]) of a backend as numpy arrays"""
    lv = np.zeros(max(1, nres))
    gr = np.zeros(max(1, nres * n))
    b._call("get_resources", b.h, lv.ctypes.data_as(C.POINTER(C.c_double)),
            gr.ctypes.data_as(C.POINTER(C.c_double)))
    return lv[:nres], gr[:nres * n].reshape(nres, n)


def _transfer(src, dst, n, chunk=1 << 16):
    """every cell's state + tape of backend src into backend dst (set_states),
    chunk by chunk, then the genotype keys and the update clock"""
    cap = 1
    for lo in range(0, n, chunk):
        st = (capi.AvgpuCpuState * min(chunk, n - lo))()
        src._call("get_states", src.h, lo, len(st), st, None, None, 0)
        cap = max([cap] + [st[i].mem_size for i in range(len(st))])
    for lo in range(0, n, chunk):
        cnt = min(chunk, n - lo)
        st = (capi.AvgpuCpuState * cnt)()
        ops = (C.c_uint8 * (cnt * cap))()
        fl = (C.c_uint8 * (cnt * cap))()
        src._call("get_states", src.h, lo, cnt, st, ops, fl, cap)
        dst._call("set_states", dst.h, lo, cnt, st, ops, fl, cap)
    gk = np.ascontiguousarray(src.census()["genotype_key"], dtype=np.uint64)
    dst._call("set_genotype_keys", dst.h, 0, n, gk.ctypes.data_as(C.c_void_p))
    stats = capi.AvgpuUpdateStats()
    src._call("get_stats", src.h, C.byref(stats))
    dst._call("set_clock", dst.h, C.byref(stats))
    return cap


@pytest.mark.timeout(900)
def test_config2_bench_regime_bit_exact(golden):
    """Parity in the regime bench.py times (VERDICT r2 'next' #1): the
    configs[2] world run on the GPU for bench.py's 150 burn-in updates -- an
    aged world with size-class spills, list classes running beside class 0
    on the aux streams, sorted windows -- is checkpointed cell by cell
    (avgpu_get_states) into the oracle; both then run 3 more updates and
    every counter and every cell digest must agree.  Every birth is placed
    (births_dropped == 0: no queue overflow, no oversize offspring)."""
    import bench
    X = Y = 1024
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(golden, X, Y)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=X * Y)
    _seed(gpu, 0, idx, gen, glen, gmer)
    spills = 0
    for u in range(bench.BURN_IN + bench.WARMUP):
        s = gpu.run_update()
        spills += gpu.counters()[capi.CNT_SPILLS]
        assert s.births_dropped == 0, (u, s.births_dropped)
    assert spills > 1000                         # the aged world spills out of class 0
    orc = ol.Backend("oracle", cfg, iset, env, ncells=X * Y)
    cap = _transfer(gpu, orc, X * Y)
    _assert_digests(orc.digests(), gpu.digests(), "restored world", orc, gpu)
    for u in range(3):
        so, sg = orc.run_update(), gpu.run_update()
        for f in STAT_FIELDS:
            assert getattr(so, f) == getattr(sg, f), (u, f, getattr(so, f), getattr(sg, f))
        assert sg.births_dropped == 0 and sg.births > 10_000 and sg.births_overwritten > 0
        _assert_digests(orc.digests(), gpu.digests(), f"bench regime, update {bench.BURN_IN + bench.WARMUP + u}", orc, gpu)
    assert cap > 320                             # organisms beyond class 0's slots took part
    assert gpu.counters(cumulative=1)[capi.CNT_BAD_RECORD] == 0   # no guarded field ever out of range


@pytest.mark.timeout(1100)
def test_config4_bench_regime_bit_exact(golden):
    """configs[4] at its own workload: bench.py --env
    resources -- the 1024x1024 world with one diffusing spatial torus resource
    per logic-9 reaction (inflow / outflow everywhere, diffusion 1) -- run on
    the GPU for the bench's burn-in + warmup updates, then checkpointed cell by
    cell AND resource grid by grid into the oracle; both run 3 more updates
    and every counter, every cell digest, every resource level and every
    per-cell amount must agree bit for bit."""
    import bench
    X = Y = 1024
    n = X * Y
    cfg, iset, _, idx, gen, glen, gmer = _bench_seed(golden, X, Y)
    env = files.parse_environment(bench.resource_env_text(X, Y))
    nres = len(env.resources)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    _seed(gpu, 0, idx, gen, glen, gmer)
    for u in range(bench.BURN_IN + bench.WARMUP):
        s = gpu.run_update()
        assert s.births_dropped == 0, (u, s.births_dropped)
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    _transfer(gpu, orc, n)
    lv, gr = _resources_np(gpu, nres, n)
    orc._call("set_resources", orc.h, lv.ctypes.data_as(C.POINTER(C.c_double)),
              np.ascontiguousarray(gr).ctypes.data_as(C.POINTER(C.c_double)))
    _assert_digests(orc.digests(), gpu.digests(), "restored world", orc, gpu)
    for u in range(3):
        so, sg = orc.run_update(), gpu.run_update()
        for f in STAT_FIELDS:
            assert getattr(so, f) == getattr(sg, f), (u, f, getattr(so, f), getattr(sg, f))
        assert list(so.task_orgs) == list(sg.task_orgs), u
        assert sg.births_dropped == 0 and sg.births > 10_000
        _assert_digests(orc.digests(), gpu.digests(), f"configs[4] bench regime, update {u}", orc, gpu)
        lo, go = _resources_np(orc, nres, n)
        lg, gg = _resources_np(gpu, nres, n)
        assert np.array_equal(lo, lg), (u, lo, lg)
        bad = np.argwhere(go != gg)
        assert len(bad) == 0, f"update {u}: {len(bad)} resource cells differ, first {bad[:3].tolist()}"
    assert gr.sum() > 0 and gpu.counters(cumulative=1)[capi.CNT_BAD_RECORD] == 0
