"""Stream ordering of the C-ABI's host calls: every copy an
API call makes runs on the world's own (non-blocking) stream and is complete
on return (capi.hip COPY_SYNC / SET_SYNC), so calls issued right behind
updates that are still queued -- avgpu_run_update(w, NULL) returns before its
kernels finish -- see the world those updates leave, and the next update sees
what the call wrote: avgpu_kill, avgpu_get_resources / avgpu_set_resources,
avgpu_test_genomes, avgpu_set_rng_mode (recorded, then counter streams) and
avgpu_set_serial_streams, each right behind queued updates.  The same sequence on the oracle (synchronous by
construction) is the expected result, bit for bit: organisms, resources and
the test CPU's results."""
import ctypes as C
import os

import numpy as np
import pytest

from avida_amd import capi, files
import test_checkpoint as tc


def _queue(b, n):
    for _ in range(n):
        if b.kind == "oracle":
            b.run_update()
        else:
            rc = b.lib.avgpu_run_update(b.h, None)      # queued: no statistics, no sync
            assert rc == 0, b.lib.avgpu_last_error().decode()


def _set_resources(b, levels, grids):
    n = b.ncells
    lv = (C.c_double * max(1, len(levels)))(*levels)
    sp = (C.c_double * max(1, len(grids) * n))(*[v for g in grids for v in g])
    b._call("set_resources", b.h, lv, sp)


def _sequence(b, golden):
    _queue(b, 3)
    for c in (5, 17, 200, 513):
        b.kill(c)                                  # read-modify-write of the cell's control word
    levels, grids = b.resources(spatial=True)
    _set_resources(b, [0.5 * v for v in levels], [[0.5 * v for v in g] for g in grids])
    _queue(b, 2)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), b.instset)
    tests = b.test_genomes([anc, anc[:40] + anc[41:]])   # the test CPU's own world, its tables copied
    _queue(b, 2)
    # per-organism recorded streams set right behind queued updates, then back
    # to the counter streams
    rnd = np.random.default_rng(5).random(40000)
    b.set_rng_mode(capi.RNG_RECORDED, rnd, np.arange(b.ncells, dtype=np.int64) * 37)
    _queue(b, 2)
    b.set_rng_mode(capi.RNG_COUNTER)
    _queue(b, 1)
    # the serial world's two recorded streams, set behind a queued update
    b._sched = np.ascontiguousarray(np.random.default_rng(6).random(60000))
    b._ctx = np.ascontiguousarray(np.random.default_rng(7).random(60000))
    b._call("set_serial_streams", b.h, b._sched.ctypes.data_as(C.c_void_p), len(b._sched),
            b._ctx.ctypes.data_as(C.c_void_p), len(b._ctx))
    b.run_serial_update()
    _queue(b, 2)
    st = b.run_update()
    return tests, st


@pytest.mark.gpu
def test_calls_behind_queued_updates_match_oracle(golden):
    o = tc._world("oracle", golden, "resources")
    g = tc._world("gpu", golden, "resources")
    to, so = _sequence(o, golden)
    tg, sg = _sequence(g, golden)
    for (ro, fo, co), (rg, fg, cg) in zip(to, tg):
        assert (ro.divided, ro.gestation_time, ro.merit, ro.copied_size) == \
               (rg.divided, rg.gestation_time, rg.merit, rg.copied_size)
        assert fo == fg and co == cg
    for f in ("update", "num_organisms", "insts_executed", "births", "deaths", "cum_insts_executed"):
        assert getattr(so, f) == getattr(sg, f), f
    tc.compare(o, g, o.ncells)
    o.close()
    g.close()
