"""Task-discovery statistics on resources_9r: for each
task and each threshold T in (10, 50, 100), the first printed update at which
T organisms do it -- 27 crossing updates of the reference
(tests/golden/resources_9r/tasks.dat; the 9task ancestor does all nine
tasks) -- must lie inside the 2.5-97.5 % quantiles of the seeds' crossing
updates.  Run over 32 seeds on the GPU batch world (the metric's world) and
on the oracle (bit-identical to it, tests/test_parity_gpu.py).

spatial_res_100u's discovery statistics (Or, two-sample against the serial
world) are in test_statistical_spatial.py.
"""
import os

import numpy as np
import pytest

from avida_amd import capi, files
import oracle_lib as ol

SEEDS = range(1, 33)
U = list(range(0, 101, 10))
THRESHOLDS = (10, 50, 100)


def _rows(path):
    return {int(l.split()[0]): [float(x) for x in l.split()[1:]] for l in open(path)
            if l.strip() and not l.startswith("#")}


def _first(series, pred):
    """first printed update whose value satisfies pred (inf: none)"""
    return next((float(u) for u, v in series if pred(v)), float("inf"))


def _inside(name, ref, samples):
    s = np.asarray(samples, dtype=float)
    lo, hi = np.quantile(s, 0.025, method="inverted_cdf"), np.quantile(s, 0.975, method="inverted_cdf")
    assert lo <= ref <= hi, f"{name}: reference {ref} outside the seeds' [{lo}, {hi}] ({sorted(s)})"


def resources_crossings(golden, kind):
    d = os.path.join(golden, "resources_9r")
    iset = files.read_instset(os.path.join(d, "instset-heads.cfg"))
    env = files.read_environment(os.path.join(d, "environment.9resource"))
    anc = files.read_org(os.path.join(d, "9task.org"), iset)
    runs = []
    for seed in SEEDS:
        cfg = capi.cfg_from_avida(files.read_avida_cfg(None), seed=seed)
        b = ol.Backend(kind, cfg, iset, env)
        b.set_orgs(0, [anc], deterministic=False)
        traj = []
        for u in range(101):
            st = b.run_update()
            if u % 10 == 0:
                traj.append((u, list(st.task_orgs)[:9]))
        b.close()
        runs.append(traj)
    ref = _rows(os.path.join(d, "tasks.dat"))
    checked = 0
    for t in range(9):
        for T in THRESHOLDS:
            want = _first([(u, ref[u][t]) for u in U], lambda v: v >= T)
            got = [_first([(u, row[t]) for u, row in traj], lambda v: v >= T) for traj in runs]
            _inside(f"task {t} reaches {T}", want, got)
            checked += 1
    assert checked == 27


def test_discovery_resources_9r_oracle(golden):
    resources_crossings(golden, "oracle")


@pytest.mark.gpu
def test_discovery_resources_9r_gpu(golden):
    resources_crossings(golden, "gpu")
