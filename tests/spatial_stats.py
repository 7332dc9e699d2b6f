"""Seed runs of spatial_res_100u for the statistical tests (test
infrastructure): the reference's config directory through the Avida2Driver
restatement (avida_amd/driver.py), recording

* the Or-organism count after EVERY update (task discovery), and
* the printed columns of tasks.dat (Not, Nand, OrNot, Or) and resource.dat
  (ResA, ResB) at updates 10, 20, ..., 100,

for one of the worlds:

* "serial"   -- the oracle's serial world: the reference's own schedule (a
                merit-weighted pick per instruction, speculative run-ahead,
                births placed inside the divide);
* "batchK"   -- the batch world with avgpu_cfg.sub_updates = K (K = 0: the
                product's default, adaptive batch steps), on
                the oracle;
* "gpuK"     -- the same batch world on the GPU (libavida_gpu.so).

Also recorded: average.dat's merit, gestation time and fitness at the printed
updates.
"""
from __future__ import annotations

import functools
import multiprocessing
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
GOLDEN = os.path.join(ROOT, "tests", "golden")
CFG = os.path.join(GOLDEN, "spatial_res_100u", "config")
OR = 4                         # task_orgs / tasks.dat column of Or
PRINTED = list(range(10, 101, 10))
TASKS = (0, 1, 3, 4)          # tasks.dat columns Not, Nand, OrNot, Or
RES = (0, 1)                  # resource.dat columns ResA, ResB
NAMES = ("Not", "Nand", "OrNot", "Or", "ResA", "ResB")


def rows(path):
    return {int(l.split()[0]): [float(x) for x in l.split()[1:]] for l in open(path)
            if l.strip() and not l.startswith("#")}


def reference():
    """the reference's run: printed columns [update][6]"""
    t = rows(os.path.join(GOLDEN, "spatial_res_100u", "tasks.dat"))
    r = rows(os.path.join(GOLDEN, "spatial_res_100u", "resource.dat"))
    return np.array([[t[u][c] for c in TASKS] + [r[u][c] for c in RES] for u in PRINTED])


def _make(kind):
    from avida_amd import driver
    import oracle_lib as ol

    serial = kind == "serial"
    gpu = kind.startswith("gpu")
    k = 1 if serial else int(kind[3:] if gpu else kind[5:])

    def wrap(base):
        class Rec(base):
            def run_update(self):
                st = self.run_serial_update() if serial else base.run_update(self)
                self.trace.append(int(st.task_orgs[OR]))
                return st
        return Rec

    def mk(c, i, e):
        c.sub_updates = k
        b = wrap(driver.ProductWorld)(c, i, e) if gpu else wrap(ol.Backend)("oracle", c, i, e)
        b.trace = []
        return b
    return mk


AVG = (0, 1, 2)                # average.dat columns Merit, Gestation Time, Fitness
AVG_NAMES = ("merit", "gestation", "fitness")


def run_seed(kind, seed):
    """(Or count after each update 0..100, printed columns [10][6],
    average.dat columns [10][3])"""
    from avida_amd import driver
    with tempfile.TemporaryDirectory() as d:
        drv = driver.Driver(CFG, d, make_world=_make(kind), seed=seed)
        assert drv.run() == 100
        tr = list(drv.world.trace)
        drv.world.close()
        t, r = rows(os.path.join(d, "tasks.dat")), rows(os.path.join(d, "resource.dat"))
        a = rows(os.path.join(d, "average.dat"))
    return (tr, [[t[u][c] for c in TASKS] + [r[u][c] for c in RES] for u in PRINTED],
            [[a[u][c] for c in AVG] for u in PRINTED])


def _one(args):
    return run_seed(*args)


def runs(kind, nseeds, workers=8):
    """seeds 1..nseeds of a world: (traces [n][101], printed [n][10][6])"""
    tr, pr, _ = _runs(kind, nseeds, workers)
    return tr, pr


def average_runs(kind, nseeds, workers=8):
    """seeds 1..nseeds: (traces [n][101], average.dat columns [n][10][3])"""
    tr, _, av = _runs(kind, nseeds, workers)
    return tr, av


@functools.lru_cache(maxsize=None)
def _runs(kind, nseeds, workers=8):
    """seeds 1..nseeds of a world: (traces, printed, averages).
    Oracle worlds run in the workers of a fork server (a fresh process: no
    GPU context is inherited), GPU worlds in threads of this process (each
    world has its own HIP stream)."""
    args = [(kind, s) for s in range(1, nseeds + 1)]
    if kind.startswith("gpu"):
        with ThreadPoolExecutor(4) as ex:
            out = list(ex.map(_one, args))
    else:
        with ProcessPoolExecutor(workers, mp_context=multiprocessing.get_context("forkserver")) as ex:
            out = list(ex.map(_one, args, chunksize=8))
    return (np.array([o[0] for o in out]), np.array([o[1] for o in out], dtype=float),
            np.array([o[2] for o in out], dtype=float))


def discovery(traces):
    """first update with an Or organism per seed (inf: none by update 100)"""
    return np.array([next((u for u, v in enumerate(t) if v > 0), np.inf) for t in traces])


DISCOVERY_BY = (20, 30, 50, 100)


def discovery_tests(a_tr, b_tr):
    """two-sample tests of task discovery between two worlds: Fisher's exact
    test on the fraction of seeds with Or by updates 20 / 30 / 50 / 100, and a
    two-sample KS test of the Or count at update 50.  Returns [(name, p)]."""
    from scipy import stats
    da, db = discovery(a_tr), discovery(b_tr)
    out = []
    for u in DISCOVERY_BY:
        t = [[int((da <= u).sum()), int((da > u).sum())], [int((db <= u).sum()), int((db > u).sum())]]
        out.append((f"Or by update {u}: {t}", float(stats.fisher_exact(t)[1])))
    out.append(("Or at update 50 (KS)", float(stats.ks_2samp(a_tr[:, 50], b_tr[:, 50]).pvalue)))
    return out


def trajectory_tests(a_pr, b_pr):
    """two-sample KS test of every printed column at every printed update:
    [(name, p)] (60 tests)"""
    from scipy import stats
    out = []
    for j, u in enumerate(PRINTED):
        for c, name in enumerate(NAMES):
            x, y = a_pr[:, j, c], b_pr[:, j, c]
            p = 1.0 if (np.all(x == x[0]) and np.all(y == x[0])) else float(stats.ks_2samp(x, y).pvalue)
            out.append((f"{name} at update {u}", p))
    return out


def average_tests(a_av, b_av):
    """Welch t and two-sample KS of average.dat's merit, gestation time and
    fitness at every printed update: [(name, p)] (60 tests)"""
    from scipy import stats
    out = []
    for j, u in enumerate(PRINTED):
        for c, name in enumerate(AVG_NAMES):
            x, y = a_av[:, j, c], b_av[:, j, c]
            if np.all(x == x[0]) and np.all(y == x[0]):
                out += [(f"{name} at update {u} (Welch)", 1.0), (f"{name} at update {u} (KS)", 1.0)]
                continue
            out.append((f"{name} at update {u} (Welch)", float(stats.ttest_ind(x, y, equal_var=False).pvalue)))
            out.append((f"{name} at update {u} (KS)", float(stats.ks_2samp(x, y).pvalue)))
    return out


def effect_sizes(a_pr, b_pr):
    """Cohen's d of every printed column at every printed update [10][6]
    (pooled sd floored at 0.5)"""
    sd = np.sqrt((a_pr.var(0, ddof=1) + b_pr.var(0, ddof=1)) / 2)
    return (a_pr.mean(0) - b_pr.mean(0)) / np.maximum(sd, 0.5)


def mid_ranks(ref, pr):
    """the reference's mid-rank in the seeds' distribution [10][6]"""
    return (pr < ref[None]).mean(0) + 0.5 * (pr == ref[None]).mean(0)
