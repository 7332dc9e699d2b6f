"""Run-to-run determinism of the GPU world.

The same seeded world -- the bench's evolved population on a 512x256 torus,
default mutation rates, births on, the last 20 of its 40 updates run as
bench.py runs them (no statistics, no host sync) -- run twice from scratch on
the GPU must leave every cell digest equal.  Results are designed not to
depend on the order in which waves, atomics or streams complete
(per-organism RNG streams, placement by priority), so
any difference is a race or a hazard in hand-written code.  (The unpadded
16-byte asm store of round 3, DESIGN.md section 7, showed in the C++ host
driver's world -- test_host_driver.py, tools/gpu/determinism.sh -- but not in
this one: such hazards are timing-dependent, so the two checks run side by
side.)
"""
import pytest

from avida_amd import capi
import oracle_lib as ol
import parity_util as pu
from test_parity_full import _bench_seed, _seed

pytestmark = pytest.mark.gpu


def _run(golden, X, Y, updates, lazy):
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(golden, X, Y)
    b = ol.Backend("gpu", cfg, iset, env, ncells=X * Y)
    _seed(b, 0, idx, gen, glen, gmer)
    stats = [b.run_update() for _ in range(updates - lazy)]
    for _ in range(lazy):           # as bench.py runs them: no statistics, no host sync
        b._call("run_update", b.h, None)
    stats.append(b.run_update())
    d = b.digests(0, X * Y)
    bad = b.counters(cumulative=1)[capi.CNT_BAD_RECORD]
    b.close()
    assert bad == 0, f"{bad} record / cell fields out of range (AVGPU_CNT_BAD_RECORD)"
    return d, stats


@pytest.mark.timeout(600)
def test_gpu_world_run_to_run_identical(golden):
    X, Y = 512, 256
    d1, s1 = _run(golden, X, Y, 40, 20)
    d2, s2 = _run(golden, X, Y, 40, 20)
    for u, (a, b) in enumerate(zip(s1, s2)):
        for f in ("num_organisms", "insts_executed", "births", "divides", "births_overwritten"):
            assert getattr(a, f) == getattr(b, f), (u, f, getattr(a, f), getattr(b, f))
    assert sum(s.births for s in s1) > 0
    nbad, cells = pu.compare_digests(d1, d2)
    assert nbad == 0, f"{nbad} cells differ between two runs, first {cells}"
