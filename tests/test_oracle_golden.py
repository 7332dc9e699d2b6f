"""Pin the CPU oracle to the reference's own RNG-free golden vectors.

* tests/golden/detail-recalc.dat: avida-core/tests/_analyze_detail_all/expected/
  data/detail-recalc.dat -- analyze-mode RECALCULATE (cTestCPU, deterministic
  inputs, cleared mutation rates) of 1794 genotypes with the classic legacy
  instruction set and the logic-9 environment.  Every column the hot path
  determines is compared exactly: viable, copy_length, exe_length, merit,
  gest_time, fitness (to the file's printed precision), executed_flags and the
  nine task counts.
* the default-heads ancestor: gestation 389, 97 executed, 100 copied, merit 97,
  fitness 0.249357 (tests/heads_default_100u/expected/data/detail-100.spop:22).
"""
import os

import pytest

from avida_amd import capi, files
import oracle_lib as ol


def _backend(golden, instset_file):
    iset = files.read_instset(os.path.join(golden, instset_file))
    env = files.read_environment(os.path.join(golden, "environment-logic9.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None))
    return ol.Backend("oracle", cfg, iset, env, ncells=1), iset


def _fmt(x):
    # cDataFile prints doubles with the default ostream precision (6 significant)
    return "%g" % x


def test_detail_recalc_all_rows(golden):
    b, iset = _backend(golden, "instset-classic.cfg")
    fmt, rows = files.parse_detail_dat(os.path.join(golden, "detail-recalc.dat"))
    assert len(rows) == 1794
    genomes = [iset.parse_sequence(r[8]) for r in rows]
    res = ol.recalculate(b, genomes)
    bad = []
    for row, (r, flags, viable) in zip(rows, res):
        got = [int(viable), r.copied_size, r.executed_size, _fmt(r.merit), r.gestation_time,
               _fmt(r.fitness) if r.gestation_time else "0", flags,
               [int(x) for x in list(r.task_count)[:9]]]
        exp = [int(row[10]), int(row[11]), int(row[12]), _fmt(float(row[13])), int(row[15]),
               row[17] if row[17] != "0" else "0", row[19], [int(x) for x in row[20:29]]]
        if got != exp:
            bad.append((row[0], exp, got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:3]}"


def test_ancestor_heads_default(golden):
    b, iset = _backend(golden, "instset-heads.cfg")
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    assert len(anc) == 100
    (r, flags, child), = b.test_genomes([anc])
    assert r.divided and r.copy_true
    assert r.gestation_time == 389
    assert r.executed_size == 97
    assert r.copied_size == 100
    assert r.merit == 97.0
    assert _fmt(r.fitness) == "0.249357"
    # Appendix B: executed everywhere except sites 3, 95, 99
    assert [i for i, c in enumerate(flags) if c == "-"] == [3, 95, 99]
    # detail-100.spop:22 records the same phenotype for the world-run ancestor
    line = [l for l in open(os.path.join(golden, "detail-100.spop")) if l.startswith("1 div:ext")][0]
    toks = line.split()
    assert toks[6:10] == ["100", "97", "389", "0.249357"]


def test_ancestor_trace_prefix(golden):
    """Appendix B cycle-level KAT: h-alloc, h-search, mov-head, 85 nops, h-search."""
    b, iset = _backend(golden, "instset-heads.cfg")
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b.set_orgs(0, [anc])
    b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
    st, _, _ = b.states(0, 1)
    assert st[0].mem_size == 300 and st[0].reg[0] == 100       # h-alloc
    b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
    st, _, _ = b.states(0, 1)
    assert (st[0].reg[1], st[0].reg[2], st[0].head[3], st[0].head[0]) == (96, 2, 100, 4)
    b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
    st, _, _ = b.states(0, 1)
    assert st[0].head[2] == 100 and st[0].head[0] == 6          # mov-head nop-C -> WRITE
    b.step(0, 1, uniform=86, mode=capi.MODE_FROZEN)
    st, _, _ = b.states(0, 1)
    assert (st[0].reg[1], st[0].reg[2], st[0].head[3]) == (0, 0, 92)  # empty-label h-search
    b.step(0, 1, uniform=300, mode=capi.MODE_FROZEN)
    st, _, _ = b.states(0, 1)
    assert st[0].num_divides == 1 and st[0].gestation_time == 389


def test_state_digest_restatement(golden):
    """The oracle's per-cell state digest (the cross-check the full-size GPU
    parity tests use) equals its Python restatement on a stepped world, and
    is 0 only for never-occupied cells."""
    import parity_util as pu
    iset, env, cfg = pu.load_env(golden, overrides={"WORLD_X": 12, "WORLD_Y": 10}, seed=5)
    b = ol.Backend("oracle", cfg, iset, env, ncells=120)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b.set_orgs(0, pu.mutants_of(anc, iset, 100, rate=0.05, seed=3), deterministic=False)
    for _ in range(12):
        b.run_update()
    d = b.digests()
    st, ops, fl = b.states(0, 120, 2048)
    for i in range(120):
        exp = pu.digest_of(st[i], ops[i * 2048:(i + 1) * 2048], fl[i * 2048:(i + 1) * 2048], iset.handlers)
        assert int(d[i]) == exp, i
    assert (d[:100] != 0).all() and (d[100:] == 0).all() == (st[110].birth_length == 0)


def test_print_status_format(golden):
    """avida_amd.trace.status_text renders cHardwareCPU::PrintStatus
    (cpu/cHardwareCPU.cc:1111-1169) for the ancestor before its first and
    after 20 instructions (oracle state, SURVEY.md Appendix B prefix)."""
    from avida_amd import trace
    iset = files.read_instset(os.path.join(golden, "instset-heads.cfg"))
    env = files.read_environment(os.path.join(golden, "environment-logic9.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None))
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    st, ops, _ = b.states(0, 1)
    t0 = trace.status_text(st[0], ops, iset)
    assert t0.splitlines()[0] == "1 IP:0 (h-alloc)"
    assert t0.splitlines()[1] == "AX:0 [0x0]  BX:0 [0x0]  CX:0 [0x0]  "
    assert t0.splitlines()[3] == "* Stack 0:" + " Ox00000000" * 10
    assert t0.splitlines()[5].startswith("  Mem (100):  " + iset.to_sequence(anc[:5]))
    b.step(0, 1, uniform=1)
    st, ops, _ = b.states(0, 1)
    t1 = trace.status_text(st[0], ops, iset).splitlines()
    # h-alloc grew the memory to 300 and put its old size in AX
    assert t1[0].startswith("2 IP:1 (") and t1[1].startswith("AX:100 [0x64]")
    assert t1[5].startswith("  Mem (300):")


@pytest.mark.parametrize("allow_parent", [0, 1])
def test_birth_method3_full_grid_oracle(golden, allow_parent):
    """The oracle's BIRTH_METHOD 3 on a full 16x16 grid (no empty neighbour
    anywhere): ALLOW_PARENT 0 drops every offspring and the parents live
    (cPopulation::ActivateOffspring, main/cPopulation.cc:706-713); ALLOW_PARENT
    1 puts each offspring into its parent's cell (PositionOffspring :5407)."""
    import parity_util as pu
    ov = {"WORLD_X": 16, "WORLD_Y": 16, "BIRTH_METHOD": 3, "ALLOW_PARENT": allow_parent}
    iset, env, cfg = pu.load_env(golden, overrides=ov, seed=29)
    n = cfg.world_x * cfg.world_y
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    orc.set_orgs(0, [anc] * n, deterministic=False)
    dropped = births = 0
    for _ in range(30):
        s = orc.run_update()
        dropped += s.births_dropped
        births += s.births
        assert s.num_organisms == n and s.deaths == 0
    if allow_parent:
        assert births > 0 and dropped == 0
    else:
        assert dropped > 0 and births == 0
