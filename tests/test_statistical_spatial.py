"""Statistical parity on spatial_res_100u (north star:
"task-discovery times and fitness trajectories within stated statistical
tolerance of the reference over many seeds").

The reference's config directory (the classic ancestor injected into all 100
cells of a 10x10 grid at update 0, two spatial resources, a CELL list, a
global pool) runs through the Avida2Driver restatement over 1024 seeds per
world (tests/spatial_stats.py).  The reference's expected data are ONE run,
so the product's world is compared with the world that has the reference's
own semantics -- the serial world (a merit-weighted pick per instruction,
speculative run-ahead, births placed inside the divide) -- by
two-sample tests, Bonferroni-corrected at a family-wise alpha of 0.01.

The product's world is the batch world at its default, avgpu_cfg.sub_updates
= 0: each batch step's newborns run their share of the
step's remaining picks after placement (a replaced organism's consumption
after the birth given back, the picks beyond what it had left carried into
the next update), and an update takes more batch steps the more its sub-step
predictor expects the total weight to move or the more organisms it expects
to divide in one quarter of it (the lock-step start of the 100 ancestors) -- the bench's own
world runs the same code and takes one step per update (bench.py
batch_steps_per_update).  No effect-size carve-out, no update excluded:

* task discovery: Fisher's exact test on the fraction of seeds with an Or
  organism by updates 20 / 30 / 50 / 100 and a KS test of the Or count at
  update 50 (5 tests);
* the whole printed trajectory: Not, Nand, OrNot, Or organisms and the ResA,
  ResB totals at updates 10..100, KS per column and update (60 tests);
* average.dat's merit, gestation time and fitness at updates 10..100, Welch
  t and KS per column and update (60 tests);
* the reference's run itself lies inside the central 99.5 % of the serial
  world's and the product world's seeds (mid-rank in [0.0025, 0.9975]) at
  every printed update and column (60 checks, strongly correlated within the
  run): an early, strong Or sweep, around the 97th percentile.

Measured (1024 seeds, this build; tools/piece_stats.py): smallest
trajectory / discovery p 0.0126 (ResA at update 10; threshold 0.01 / 65 =
1.5e-4), largest |Cohen's d| 0.12; the reference run's mid-ranks 0.012 ..
0.996.  The GPU batch world is the oracle's bit for bit (checked
per seed below), so its statistics are these.
"""
import numpy as np
import pytest

import spatial_stats as ss

N = 1024          # oracle seeds per world
ALPHA = 0.01      # family-wise
PRODUCT = "batch0"


def _assert_two_sample(results, tag):
    thr = ALPHA / len(results)
    bad = [(n, p) for n, p in results if p <= thr]
    assert not bad, f"{tag}: p <= {thr:.2e}: {bad}"


def test_discovery_and_trajectory_product_vs_serial_oracle():
    b_tr, b_pr = ss.runs(PRODUCT, N)
    s_tr, s_pr = ss.runs("serial", N)
    _assert_two_sample(ss.trajectory_tests(b_pr, s_pr) + ss.discovery_tests(b_tr, s_tr), "product world")
    # both regimes occur in both worlds (the process is bimodal)
    for tr in (b_tr, s_tr):
        d = ss.discovery(tr)
        assert 0.05 < np.mean(np.isfinite(d)) < 0.95
    assert np.abs(ss.effect_sizes(b_pr, s_pr)).max() <= 0.15


def test_merit_gestation_fitness_product_vs_serial_oracle():
    _, b_av = ss.average_runs(PRODUCT, N)
    _, s_av = ss.average_runs("serial", N)
    _assert_two_sample(ss.average_tests(b_av, s_av), "average.dat")


def test_reference_run_inside_seed_distribution():
    ref = ss.reference()
    for kind in ("serial", PRODUCT):
        mr = ss.mid_ranks(ref, ss.runs(kind, N)[1])
        assert mr.min() >= 0.0025 and mr.max() <= 0.9975, (kind, mr.round(4))


def _gpu_equals_oracle(kind, n):
    g_tr, g_pr = ss.runs(kind, n)
    o_tr, o_pr = ss.runs("batch" + kind[3:], N)
    assert np.array_equal(g_tr, o_tr[:n]), "GPU batch world != oracle batch world (Or per update)"
    assert np.array_equal(g_pr, o_pr[:n]), "GPU batch world != oracle batch world (printed columns)"
    return g_tr, g_pr


@pytest.mark.gpu
def test_product_world_gpu():
    """the product's world on the GPU, 128 seeds: the oracle's, seed for seed
    (every update's Or count, every printed column), and the two-sample tests
    against the serial world"""
    g_tr, g_pr = _gpu_equals_oracle("gpu0", 128)
    s_tr, s_pr = ss.runs("serial", N)
    _assert_two_sample(ss.discovery_tests(g_tr, s_tr) + ss.trajectory_tests(g_pr, s_pr), "GPU product world")


@pytest.mark.gpu
def test_fixed_steps_gpu():
    """fixed batch steps (avgpu_cfg.sub_updates = 3) on the GPU, 32 seeds:
    the oracle's, seed for seed"""
    _gpu_equals_oracle("gpu3", 32)
