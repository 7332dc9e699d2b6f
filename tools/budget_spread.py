"""Lane efficiency of budget-sorted class-0 windows (diagnostic): the oracle's
batch world seeded like bench.py (evolved population, X x Y), burned in, then
the last allotment's budgets cut into SORT_WIN-cell windows, each sorted by
budget (descending, budgets >= CAP in one bucket as k_window_count does) and
dealt to 64-lane waves: efficiency = sum(budget) / sum(64 x wave maximum).
Also the same for the round-3 rule floor(lambda) + Bernoulli on the same
merits, for comparison.  usage: python tools/budget_spread.py [X Y burn CAP]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_lib as ol  # noqa: E402
from test_parity_full import _bench_seed, _seed  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def efficiency(b, cap, win=2048):
    tot = waves = 0
    for w0 in range(0, len(b), win):
        v = b[w0:w0 + win]
        key = np.minimum(v, cap)
        order = np.lexsort((-v, -key))       # within a capped bucket the order is free; best case
        s = v[order]
        s = s[s > 0]
        for k in range(0, len(s), 64):
            tot += s[k:k + 64].sum()
            waves += 64 * s[k:k + 64].max()
    return tot / waves


def main():
    X, Y, burn = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 256, 60)))
    cap = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(GOLDEN, X, Y)
    b = ol.Backend("oracle", cfg, iset, env, ncells=X * Y)
    _seed(b, 0, idx, gen, glen, gmer)
    for _ in range(burn):
        b.run_update()
    bud = (C.c_int32 * (X * Y))()
    b.lib.orc_last_budgets.argtypes = [C.c_void_p, C.c_void_p]
    b.lib.orc_last_budgets(b.h, bud)
    bud = np.array(bud, dtype=np.int64)
    st, _, _ = b.states(0, X * Y)
    merit = np.array([st[i].merit if st[i].alive else 0.0 for i in range(X * Y)])
    lam = 30 * (merit > 0).sum() * merit / merit.sum()
    rng = np.random.default_rng(1)
    old = np.floor(lam).astype(np.int64) + (rng.random(len(lam)) < lam - np.floor(lam))
    pct = np.percentile(bud[bud > 0], [10, 50, 90, 99, 99.9])
    print(f"budgets>0: {int((bud > 0).sum())}  percentiles 10/50/90/99/99.9: {pct}  max {bud.max()}")
    for win in (2048, 4096, 8192, 16384):
        print(f"window {win:5d}: lane efficiency multinomial {efficiency(bud, cap, win):.4f}, "
              f"floor+Bernoulli {efficiency(old, cap, win):.4f}")
    b.close()


if __name__ == "__main__":
    main()
