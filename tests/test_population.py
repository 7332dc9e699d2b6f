"""cPopulation::LoadPopulation / SavePopulation restated (avida_amd/population.py,
main/cPopulation.cc:6723-7000 / :6294-6500), pinned to the reference's own
population files: tests/golden/detail-100.spop (a structured save of
heads_default_100u at update 100) and detail-50000.pop (the genotype list
heads_midrun_30u loads)."""
import os

import pytest

from avida_amd import capi, files, population, systematics
import oracle_lib as ol
import parity_util as pu


def _world(golden, instset="instset-heads.cfg", backend="oracle", n=3600):
    iset = files.read_instset(os.path.join(golden, instset))
    env = files.read_environment(os.path.join(golden, "environment-logic9.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None), seed=5)
    return iset, ol.Backend(backend, cfg, iset, env, ncells=n)


def test_load_structured_spop(golden):
    """detail-100.spop: every organism at its saved cell, with its genotype's
    sequence, and merit scaled by gest_time / (gest_time - gest_offset)
    (:6948-6958); genotypes without merit take their test-CPU merit."""
    iset, b = _world(golden)
    path = os.path.join(golden, "detail-100.spop")
    gts = files.read_pop(path)
    placed = population.load_population(b, iset, path, 3600)
    assert placed == sum(g.num_cpus for g in gts)
    st, ops, _ = b.states(0, 3600, 2048)
    occupied = {c for g in gts for c in (g.cells or [])}
    for g in gts:
        seq = iset.parse_sequence(g.sequence)
        for i, c in enumerate(g.cells or []):
            assert ops[c * 2048:c * 2048 + len(seq)] == seq, (g.id, c)
            if g.merit > 0:
                remain = g.gest_time - g.gest_offset[i]
                exp = g.merit * (g.gest_time / remain) if remain > 0 and g.gest_time > 0 else g.merit
                assert st[c].merit == pytest.approx(exp, rel=1e-12), (g.id, c)
    g1 = next(g for g in gts if g.id == 1)         # the ancestor: merit 97, gest 389, offset 388
    assert st[g1.cells[0]].merit == pytest.approx(97 * 389 / 1)
    gz = next(g for g in gts if g.id == 25)        # merit 0 in the file: test-CPU merit
    assert st[gz.cells[0]].merit >= 0
    assert all(st[c].alive == (c in occupied) for c in range(3600))


def test_load_pop_list_descending_ids(golden):
    """detail-50000.pop (no cells column): organisms fill cells 0, 1, ... in
    descending genotype-id order (sTmpGenotype::operator<, :6683)."""
    iset, b = _world(golden, "instset-classic.cfg")
    path = os.path.join(golden, "detail-50000.pop")
    gts = sorted(files.read_pop(path), key=lambda g: -g.id)
    n = population.load_population(b, iset, path, 3600)
    assert n == 3599
    st, ops, _ = b.states(0, 3600, 512)
    cell = 0
    for g in gts[:20]:
        seq = iset.parse_sequence(g.sequence)
        for _ in range(g.num_cpus):
            assert ops[cell * 512:cell * 512 + len(seq)] == seq
            if g.merit > 0:
                assert st[cell].merit == g.merit
            else:                       # merit 0 in the file: test-CPU merit (GetTestMerit)
                assert st[cell].merit > 0
            cell += 1
    assert st[3599].alive == 0


def test_save_load_roundtrip(golden, tmp_path):
    """SavePopulation of a running world, loaded into a fresh one: the same
    genotypes in the same cells; the file's columns follow the reference's
    structured save (detail-100.spop's #format line)."""
    iset, b = _world(golden)
    population.load_population(b, iset, os.path.join(golden, "detail-100.spop"), 3600)
    for _ in range(15):
        b.run_update()
    arb = systematics.GenotypeArbiter()
    arb.update(b.census(), 115)
    out = tmp_path / "detail-115.spop"
    population.save_population(b, iset, arb, str(out), 115)
    ref_fmt = open(os.path.join(golden, "detail-100.spop")).readline(), \
        open(os.path.join(golden, "detail-100.spop")).readlines()[1]
    assert open(out).readlines()[1].split() == ref_fmt[1].split()
    saved = files.read_pop(str(out))
    assert sum(g.num_cpus for g in saved) == int((b.census()["genotype_key"] != 0).sum())
    _, b2 = _world(golden)
    population.load_population(b2, iset, str(out), 3600)
    c1, c2 = b.census(), b2.census()
    assert (c1["genotype_key"] != 0).sum() == (c2["genotype_key"] != 0).sum()
    # every saved organism is back at its cell with its genotype's birth genome
    same = (c1["genotype_key"] == c2["genotype_key"]) | (c1["genotype_key"] == 0)
    assert same.mean() > 0.95      # organisms that copied over their own first sites excepted


def test_load_with_offset_keeps_existing_population(golden):
    """LoadPopulation with a non-zero cellid_offset adds the file's organisms
    to the world: the clearing KillOrganism pass runs only at offset 0
    (main/cPopulation.cc:6731-6732).  Offset 0 clears the world first.
    detail-50000.pop (3599 organisms, no cells column) at offset 1 fills
    cells 1 .. 3599; the organism already in cell 0 survives."""
    iset, b = _world(golden, "instset-classic.cfg")
    path = os.path.join(golden, "detail-50000.pop")
    g0 = iset.parse_sequence(files.read_pop(path)[0].sequence)
    b.set_orgs(0, [g0], deterministic=False)
    placed = population.load_population(b, iset, path, 3600, cellid_offset=1)
    assert placed == 3599
    st, _, _ = b.states(0, 3600, 8)
    assert all(st[c].alive for c in range(3600))            # cell 0 kept its organism
    b.kill(5)
    population.load_population(b, iset, path, 3600, cellid_offset=0)
    st, _, _ = b.states(0, 3600, 8)
    assert all(st[c].alive for c in range(3599)) and not st[3599].alive   # cleared, then cells 0..3598
