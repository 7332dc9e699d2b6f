"""Measure the batch model's gap on heads_midrun_30u (diagnostic): the oracle's
batch world -- bit-identical to the GPU batch world (tests/test_parity_gpu.py)
-- over many seeds through the Avida2Driver restatement; per printed update
and column: the reference's value, the seed mean and sd, and how far apart
they are in sd and in relative terms.
usage: python tools/midrun_gap.py [seeds] [workers]"""
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def one(seed):
    from avida_amd import driver
    import oracle_lib as ol
    import test_statistical_midrun as tm
    cfg = os.path.join(GOLDEN, "heads_midrun_30u", "config")
    with tempfile.TemporaryDirectory() as d:
        drv = driver.Driver(cfg, d, make_world=lambda c, i, e: ol.Backend("oracle", c, i, e), seed=seed)
        assert drv.run() == 30
        drv.world.close()
        t, a = tm._rows(os.path.join(d, "tasks.dat")), tm._rows(os.path.join(d, "average.dat"))
        return [t[u] + a[u][:3] for u in tm.U]


def main():
    import test_statistical_midrun as tm
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    with ProcessPoolExecutor(workers) as ex:
        rows = list(ex.map(one, range(1, seeds + 1)))
    ref = tm._ref(GOLDEN)
    print("update column reference mean sd (ref-mean)/sd rel_gap")
    for k, u in enumerate(tm.U):
        v = np.array([r[k] for r in rows])
        m, sd = v.mean(0), v.std(0, ddof=1)
        for j, name in enumerate(tm.COLS):
            z = (ref[u][j] - m[j]) / sd[j] if sd[j] > 0 else float("nan")
            rel = (ref[u][j] - m[j]) / max(abs(ref[u][j]), 1e-12)
            print(f"{u:3d} {name:10s} {ref[u][j]:12.5g} {m[j]:12.5g} {sd[j]:10.4g} {z:7.2f} {rel:+.4f}")


if __name__ == "__main__":
    main()
