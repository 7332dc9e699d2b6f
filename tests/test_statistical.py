"""Free-running evolution against the reference's own runs, in distribution.

The reference's RNG (Apto AvidaRNG) and scheduler are absent and
this path runs batch-synchronous updates with per-organism counter streams
(DESIGN.md sections 4-5), so a free-running world can agree with the reference
only statistically.  The expected data files of two reference tests are one
seed each; these tests run the CPU oracle (which the GPU world equals bit for
bit, tests/test_parity_gpu.py) over SEEDS seeds and require the reference's
values to lie inside the seed distribution:

    |reference - mean| <= 3 * max(sd, SD_FLOOR)      (TOLERANCE, per quantity)

at every printed update.  SD_FLOOR keeps the early, deterministic updates
(sd 0) from demanding more than exact agreement +- 1.5.

* heads_default_100u (tests/golden/heads_default_100u, from
  avida-core/tests/heads_default_100u/expected/data): the default-heads
  ancestor alone in a 60x60 logic-9 world, seed 101, 100 updates --
  organisms (count.dat), average generation (time.dat), average merit,
  gestation time and fitness (average.dat) and the task organisms
  (tasks.dat: none are discovered in 100 updates).
* resources_9r (tests/golden/resources_9r): the 9task ancestor with nine
  global pools, 100 updates -- organisms, average generation and the nine
  task-organism counts (tasks.dat; offspring carry their parent's
  last-gestation task counts, cPhenotype::SetupOffspring main/cPhenotype.cc:447).
"""
import os

import numpy as np

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

SEEDS = range(1, 41)
TOLERANCE = 3.0
SD_FLOOR = 0.5


def _dat(path):
    rows = {}
    for line in open(path):
        if line.startswith("#") or not line.strip():
            continue
        t = line.split()
        rows[int(t[0])] = [float(x) for x in t[1:]]
    return rows


def _run(make, updates=101):
    """per seed: {update: (orgs, ave_generation, ave merit, ave gestation, ave fitness, task_orgs[9])}"""
    out = []
    for seed in SEEDS:
        b, anc = make(seed)
        b.set_orgs(0, [anc], deterministic=False)
        traj = {}
        for u in range(updates):
            st = b.run_update()
            if u % 10 == 0:
                n = max(1, st.num_organisms)
                traj[u] = (st.num_organisms, st.ave_generation, st.sum_merit / n, st.sum_gestation / n,
                           st.sum_fitness / n, list(st.task_orgs)[:9])
        b.close()
        out.append(traj)
    return out


def _check(name, ref, samples):
    samples = np.asarray(samples, dtype=float)
    mean, sd = samples.mean(), samples.std()
    assert abs(ref - mean) <= TOLERANCE * max(sd, SD_FLOOR), \
        f"{name}: reference {ref} vs seeds mean {mean:.3f} sd {sd:.3f}"


def test_heads_default_100u_in_distribution(golden):
    d = os.path.join(golden, "heads_default_100u")

    def make(seed):
        iset, env, cfg = pu.load_env(golden, seed=seed)
        return ol.Backend("oracle", cfg, iset, env), files.read_org(os.path.join(golden, "default-heads.org"), iset)

    runs = _run(make)
    count, time_, avg, tasks = (_dat(os.path.join(d, f)) for f in ("count.dat", "time.dat", "average.dat",
                                                                    "tasks.dat"))
    for u in range(0, 101, 10):
        _check(f"organisms@{u}", count[u][1], [r[u][0] for r in runs])
        _check(f"generation@{u}", time_[u][1], [r[u][1] for r in runs])
        for t in range(9):
            _check(f"task{t}@{u}", tasks[u][t], [r[u][5][t] for r in runs])
    for u in (60, 80, 100):   # once the population has diversified
        _check(f"merit@{u}", avg[u][0], [r[u][2] for r in runs])
        _check(f"gestation@{u}", avg[u][1], [r[u][3] for r in runs])
        _check(f"fitness@{u}", avg[u][2], [r[u][4] for r in runs])


def test_resources_9r_in_distribution(golden):
    d = os.path.join(golden, "resources_9r")
    iset = files.read_instset(os.path.join(d, "instset-heads.cfg"))
    env = files.read_environment(os.path.join(d, "environment.9resource"))
    anc = files.read_org(os.path.join(d, "9task.org"), iset)

    def make(seed):
        cfg = capi.cfg_from_avida(files.read_avida_cfg(None), seed=seed)
        return ol.Backend("oracle", cfg, iset, env), anc

    runs = _run(make)
    count, time_, tasks = (_dat(os.path.join(d, f)) for f in ("count.dat", "time.dat", "tasks.dat"))
    for u in range(0, 101, 10):
        _check(f"organisms@{u}", count[u][1], [r[u][0] for r in runs])
        _check(f"generation@{u}", time_[u][1], [r[u][1] for r in runs])
        for t in range(9):
            _check(f"task{t}@{u}", tasks[u][t], [r[u][5][t] for r in runs])
