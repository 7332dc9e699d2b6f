"""Genotype classification (avida_amd/systematics.py).

* The genome key: the oracle's (oracle/oracle.cc genome_key) equals the
  Python restatement on random genomes, and the census reports it for live
  cells only.
* GenotypeArbiter rules on hand-built censuses: ids in first-cell order,
  nameGenotype's per-size base-26 names (systematics/GenotypeArbiter.cc:
  482-497), threshold at THRESHOLD or best, removal at abundance 0, the
  dominant's tie rule.
* The driver writes dominant.dat and count.dat's genotype columns; on the
  reference's own configs the rows that do not depend on its RNG stream are
  the reference's (spatial_res_100u: update 0, "2 050-aaaaa" after the
  classic ancestor is replaced by 100 injected sequences;
  heads_default_100u: updates 0 and 10, before the first divide).
"""
import os
import shutil

import numpy as np
import pytest

from avida_amd import capi, driver, files, systematics
import oracle_lib as ol
import parity_util as pu


def _rows(path):
    return {int(l.split()[0]): l.split()[1:] for l in open(path) if l.strip() and not l.startswith("#")}


def _census(keys, gest=None, lens=None):
    c = np.zeros(len(keys), dtype=capi.CENSUS_DTYPE)
    c["genotype_key"] = keys
    c["genome_length"] = lens if lens is not None else 100
    if gest is not None:
        c["gestation_time"] = gest
    return c


def test_name_letters():
    assert systematics.name_letters(0) == "aaaaa"
    assert systematics.name_letters(4) == "aaaae"
    assert systematics.name_letters(26) == "aaaba"


def test_oracle_key_matches_restatement(golden):
    iset, env, cfg = pu.load_env(golden)
    b = ol.Backend("oracle", cfg, iset, env, ncells=64)
    gs = pu.random_genomes(iset, 40, lo=1, hi=300, seed=5)
    b.set_orgs(3, gs)
    c = b.census()
    assert (c["genotype_key"][:3] == 0).all() and (c["genotype_key"][43:] == 0).all()
    for i, g in enumerate(gs):
        codes = bytes(iset.handlers[op] for op in g)
        assert int(c["genotype_key"][3 + i]) == systematics.genome_key(codes)
        assert c["genome_length"][3 + i] == len(g)
    # equal genomes share a key, a one-site change does not
    b.set_orgs(50, [gs[0], gs[0][:-1] + bytes([(gs[0][-1] + 1) % len(iset.names)])])
    c = b.census()
    assert c["genotype_key"][50] == c["genotype_key"][3] != c["genotype_key"][51]


def test_checkpoint_keeps_genotype_keys(golden, tmp_path):
    """After 200 updates some organisms have copied into their own sites
    (their tape prefix is no longer the birth genome): the checkpoint
    carries the keys, so a restored world's census is the original's."""
    iset, env, cfg = pu.load_env(golden, seed=11)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    n = cfg.world_x * cfg.world_y
    o = ol.Backend("oracle", cfg, iset, env, ncells=n)
    o.set_orgs(n // 2 + cfg.world_x // 2, [anc], deterministic=False)
    for _ in range(200):
        o.run_update()
    c = o.census()
    o.checkpoint(str(tmp_path / "w.npz"))
    o2 = ol.Backend("oracle", cfg, iset, env, ncells=n)
    o2.restore(str(tmp_path / "w.npz"))
    assert (c["genotype_key"] != 0).sum() > 100 and np.array_equal(o2.census(), c)


def test_arbiter_rules():
    a = systematics.GenotypeArbiter(threshold=3)
    a.update(_census([7, 0, 0, 0]), 0)
    g7 = a.dominant()
    assert (g7.id, g7.name, g7.num_units) == (1, "100-aaaaa", 1)      # best -> threshold at once
    a.update(_census([7, 9, 9, 5], lens=[100, 100, 100, 99]), 1)
    # new ids in first-cell order: 9 (cell 1) before 5 (cell 3)
    assert a.active[9].id == 2 and a.active[5].id == 3
    assert a.dominant() is a.active[9]                                  # 2 units > 1
    assert a.active[9].name == "100-aaaab" and a.active[5].name == "099-no_name"
    assert (a.num_genotypes(), a.num_threshold()) == (3, 2)
    a.update(_census([5, 5, 5, 9]), 2)
    assert 7 not in a.active and a.num_genotypes() == 2
    assert a.active[5].name == "099-aaaaa" and a.dominant() is a.active[5]
    a.update(_census([5, 5, 9, 9]), 3)                                  # tie: the dominant stays
    assert a.dominant() is a.active[5]
    a.update(_census([7, 0, 0, 0]), 4)                                  # a returning genome: new genotype
    assert a.active[7].id == 4 and a.num_genotypes() == 1


def test_genotype_averages():
    a = systematics.GenotypeArbiter()
    c = _census([3, 3, 3], gest=[0, 389, 389])
    c["merit"] = [100.0, 97.0, 97.0]
    c["fitness"] = [0.0, 97.0 / 389, 97.0 / 389]
    c["copied_size"] = [100, 100, 100]
    a.update(c, 20)
    row = a.dominant_row(20)
    assert row[1:5] == [97.0, 389.0, 97.0 / 389, 1.0 / 389]
    assert row[5:10] == [100, 100.0, 0.0, 3, 0] and row[14:] == [1, "100-aaaaa"]
    a.update(_census([3]), 21)
    assert a.dominant_row(21)[1:5] == [0.0, 0.0, 0.0, 0.0] and a.dominant_row(21)[13] == systematics.DBL_MIN


def test_driver_dominant_spatial_res_100u(golden, tmp_path):
    ref = os.path.join(golden, "spatial_res_100u")
    d = driver.Driver(os.path.join(ref, "config"), str(tmp_path),
                      make_world=lambda cfg, iset, env: ol.Backend("oracle", cfg, iset, env))
    d.run()
    got, want = _rows(tmp_path / "dominant.dat"), _rows(os.path.join(ref, "dominant.dat"))
    hdr = lambda p: [l for l in open(p) if l.startswith("#")][2:]
    assert hdr(tmp_path / "dominant.dat") == hdr(os.path.join(ref, "dominant.dat"))
    assert sorted(got) == list(range(0, 101, 10))
    assert got[0] == want[0]                       # 0 0 0 0 0 50 0 0 100 ... 2 050-aaaaa
    cnt = _rows(tmp_path / "count.dat")
    assert cnt[0][2:4] == ["1", "1"]               # genotypes, threshold genotypes (reference: 1 1)
    for u in range(10, 101, 10):
        assert int(cnt[u][2]) > 1 and got[u][6] == "0"


def test_driver_dominant_heads_default_100u(golden, tmp_path):
    cfgdir = tmp_path / "config"
    cfgdir.mkdir()
    shutil.copy(os.path.join(golden, "heads_default_100u", "avida.cfg"), cfgdir / "avida.cfg")
    shutil.copy(os.path.join(golden, "instset-heads.cfg"), cfgdir / "instset-heads.cfg")
    shutil.copy(os.path.join(golden, "environment-logic9.cfg"), cfgdir / "environment.cfg")
    shutil.copy(os.path.join(golden, "default-heads.org"), cfgdir / "default-heads.org")
    (cfgdir / "events.cfg").write_text("u begin Inject default-heads.org\n"
                                       "u 0:10:end PrintDominantData\nu 0:10:end PrintCountData\n"
                                       "u 30 Exit\n")
    out = tmp_path / "data"
    d = driver.Driver(str(cfgdir), str(out),
                      make_world=lambda cfg, iset, env: ol.Backend("oracle", cfg, iset, env))
    d.run()
    got = _rows(out / "dominant.dat")
    want = _rows(os.path.join(golden, "heads_default_100u", "dominant.dat"))
    assert got[0] == want[0] and got[10] == want[10]     # ... 1 0 0 0 0 2.22507e-308 1 100-aaaaa
    assert got[20][4:6] == want[20][4:6] == ["100", "100"] and got[20][13:] == ["1", "100-aaaaa"]
    cnt, wcnt = _rows(out / "count.dat"), _rows(os.path.join(golden, "heads_default_100u", "count.dat"))
    assert cnt[0][:4] == wcnt[0][:4] and cnt[10][:4] == wcnt[10][:4]


@pytest.mark.gpu
def test_gpu_census_equals_oracle(golden, tmp_path):
    """Keys and phenotype rows of a free-running world after 200 updates:
    the device keys births in k_activate (wave-parallel), the oracle from
    its birth genomes; checkpoint restore re-keys from the tape."""
    import torch
    assert torch.cuda.is_available()
    iset, env, cfg = pu.load_env(golden, seed=11)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    for b in (orc, gpu):
        b.set_orgs(n // 2 + cfg.world_x // 2, [anc], deterministic=False)
    for _ in range(200):
        orc.run_update(), gpu.run_update()
    co, cg = orc.census(), gpu.census()
    assert (co["genotype_key"] != 0).sum() > 100
    for f in capi.CENSUS_DTYPE.names:
        assert np.array_equal(co[f], cg[f]), f
    ao, ag = systematics.GenotypeArbiter(), systematics.GenotypeArbiter()
    ao.update(co, 200), ag.update(cg, 200)
    assert ao.dominant_row(200) == ag.dominant_row(200)
    # a restored world takes the checkpoint's keys: same census
    gpu.checkpoint(str(tmp_path / "w.npz"))
    g2 = ol.Backend("gpu", cfg, iset, env, ncells=n)
    g2.restore(str(tmp_path / "w.npz"))
    assert np.array_equal(g2.census(), cg)
    for b in (orc, gpu, g2):
        b.close()
