"""Seed runs of heads_midrun_30u for the statistical tests (test
infrastructure): the reference's config directory (LoadPopulation of the
evolved detail-50000.pop, the bench's own population) through the
Avida2Driver restatement (avida_amd/driver.py), recording the printed task
counts and the average.dat merit, gestation time and fitness at updates 5,
10, ..., 30, for one of the worlds:

* "serial" -- the oracle's serial world (the reference's own schedule);
* "batchK" -- the batch world with avgpu_cfg.sub_updates = K (0: the
              product's adaptive default), on the oracle.
"""
from __future__ import annotations

import functools
import multiprocessing
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
GOLDEN = os.path.join(ROOT, "tests", "golden")
CFG = os.path.join(GOLDEN, "heads_midrun_30u", "config")
U = [5, 10, 15, 20, 25, 30]
COLS = [f"task{t}" for t in range(9)] + ["merit", "gestation", "fitness"]


def rows(path):
    return {int(l.split()[0]): [float(x) for x in l.split()[1:]] for l in open(path)
            if l.strip() and not l.startswith("#")}


def run_seed(kind, seed):
    """printed columns [6][12] of one seed"""
    from avida_amd import driver
    import oracle_lib as ol
    serial = kind == "serial"

    class Rec(ol.Backend):
        def run_update(self):
            return self.run_serial_update() if serial else ol.Backend.run_update(self)

    def mk(c, i, e):
        if not serial:
            c.sub_updates = int(kind[5:])
        return Rec("oracle", c, i, e)
    with tempfile.TemporaryDirectory() as d:
        drv = driver.Driver(CFG, d, make_world=mk, seed=seed)
        assert drv.run() == 30
        drv.world.close()
        t, a = rows(os.path.join(d, "tasks.dat")), rows(os.path.join(d, "average.dat"))
    return [t[u] + a[u][:3] for u in U]


def _one(args):
    return run_seed(*args)


@functools.lru_cache(maxsize=None)
def runs(kind, nseeds, workers=8):
    """seeds 1..nseeds: printed [n][6][12] (oracle worlds, forkserver workers)"""
    args = [(kind, s) for s in range(1, nseeds + 1)]
    with ProcessPoolExecutor(workers, mp_context=multiprocessing.get_context("forkserver")) as ex:
        out = list(ex.map(_one, args, chunksize=2))
    return np.array(out, dtype=float)


def two_sample_tests(a, b, cols=range(len(COLS))):
    """Welch t and KS per printed update and column: [(name, p)]"""
    from scipy import stats
    out = []
    for j, u in enumerate(U):
        for c in cols:
            x, y = a[:, j, c], b[:, j, c]
            if np.all(x == x[0]) and np.all(y == x[0]):
                continue
            out.append((f"{COLS[c]} at update {u} (Welch)", float(stats.ttest_ind(x, y, equal_var=False).pvalue)))
            out.append((f"{COLS[c]} at update {u} (KS)", float(stats.ks_2samp(x, y).pvalue)))
    return out
