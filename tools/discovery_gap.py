"""Task-discovery gap between the batch world and the serial world on
spatial_res_100u (diagnostic).  Both run on the oracle
(the batch world is bit-identical to the GPU's, tests/test_parity_gpu.py; the
serial world is the reference's schedule) through the
Avida2Driver restatement, with the Or-organism count recorded after EVERY
update.  Prints, per world: the fraction of seeds with Or by updates
10/20/30/50/100, Or at update 50 quantiles, and two-proportion z / Fisher p
for batch vs serial.

usage: python tools/discovery_gap.py [seeds] [workers] [variant ...]
variants: batch, batchK (K sub-updates), serial (default batch serial); env AVGPU_ORC_* knobs pass through."""
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
OR = 4
CHECK = (10, 20, 30, 50, 100)
PRINTED = list(range(10, 101, 10))
TASKS = (0, 1, 3, 4)          # tasks.dat columns Not, Nand, OrNot, Or
RES = (0, 1)                  # resource.dat columns ResA, ResB
NAMES = ("Not", "Nand", "OrNot", "Or", "ResA", "ResB")


def run_seed(args):
    kind, seed = args
    from avida_amd import driver
    import oracle_lib as ol

    class Rec(ol.Backend):
        serial = kind == "serial"

        def run_update(self):
            st = self.run_serial_update() if self.serial else ol.Backend.run_update(self)
            self.trace.append(int(st.task_orgs[OR]))
            return st

    def mk(c, i, e):
        if kind.startswith("batch") and kind != "batch":
            c.sub_updates = int(kind[5:])      # batchK: K sub-updates per update
        b = Rec("oracle", c, i, e)
        b.trace = []
        return b

    cfg = os.path.join(GOLDEN, "spatial_res_100u", "config")
    with tempfile.TemporaryDirectory() as d:
        drv = driver.Driver(cfg, d, make_world=mk, seed=seed)
        assert drv.run() == 100
        tr = drv.world.trace
        drv.world.close()
        t, r = _rows(os.path.join(d, "tasks.dat")), _rows(os.path.join(d, "resource.dat"))
    printed = [[t[u][c] for c in TASKS] + [r[u][c] for c in RES] for u in PRINTED]
    return tr, printed


def _rows(path):
    return {int(l.split()[0]): [float(x) for x in l.split()[1:]] for l in open(path)
            if l.strip() and not l.startswith("#")}


def discovery(traces):
    """first update with an Or organism (inf: none)"""
    return np.array([next((u for u, v in enumerate(t) if v > 0), np.inf) for t in traces])


def collect(kind, seeds, workers):
    with ProcessPoolExecutor(workers) as ex:
        out = list(ex.map(run_seed, [(kind, s) for s in seeds]))
    return np.array([o[0] for o in out]), np.array([o[1] for o in out])


def summary(name, tr):
    d = discovery(tr)
    frac = {u: float(np.mean(d <= u)) for u in CHECK}
    q = np.quantile(tr[:, 50], [0.5, 0.9, 0.95, 0.99])
    print(f"{name:10s} n={len(tr)} Or-by " + " ".join(f"u{u}:{frac[u]:.3f}" for u in CHECK)
          + f"  Or@50 q50/90/95/99 {q.round(1).tolist()}  mean {tr[:, 50].mean():.2f}")
    return d


def main():
    from scipy import stats
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    kinds = sys.argv[3:] or ["batch", "serial"]
    both = {k: collect(k, range(1, seeds + 1), workers) for k in kinds}
    res = {k: v[0] for k, v in both.items()}
    pr = {k: v[1] for k, v in both.items()}
    ds = {k: summary(k, v) for k, v in res.items()}
    ref_t = _rows(os.path.join(GOLDEN, "spatial_res_100u", "tasks.dat"))
    ref_r = _rows(os.path.join(GOLDEN, "spatial_res_100u", "resource.dat"))
    for k, v in pr.items():
        print(f"{k}: reference percentile in the seeds (mid-rank) per printed update")
        for j, u in enumerate(PRINTED):
            ref = [ref_t[u][c] for c in TASKS] + [ref_r[u][c] for c in RES]
            pc = [(np.mean(v[:, j, c] < ref[c]) + 0.5 * np.mean(v[:, j, c] == ref[c])) for c in range(6)]
            print(f"  u{u:3d} " + " ".join(f"{NAMES[c]}={ref[c]:g}@{pc[c]:.3f}" for c in range(6)))
    for k in [k for k in pr if k.startswith("batch") and "serial" in pr]:
        worst = sorted((stats.ks_2samp(pr[k][:, j, c], pr["serial"][:, j, c]).pvalue, PRINTED[j], NAMES[c])
                       for j in range(len(PRINTED)) for c in range(6))[:4]
        print(f"{k} printed columns: smallest KS p vs serial", [(float(p), u, n) for p, u, n in worst])
        a, b = ds[k], ds["serial"]
        for u in CHECK:
            t = [[int((a <= u).sum()), int((a > u).sum())], [int((b <= u).sum()), int((b > u).sum())]]
            print(f"  u{u}: fisher p={stats.fisher_exact(t)[1]:.4f} table={t}")
        print("  Or@50 KS p=%.4f" % stats.ks_2samp(res[k][:, 50], res["serial"][:, 50]).pvalue)
    out = os.environ.get("DISCOVERY_OUT")
    if out:
        np.savez(out, **res, **{k + "_printed": v for k, v in pr.items()})


if __name__ == "__main__":
    main()
