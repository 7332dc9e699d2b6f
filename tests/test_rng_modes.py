"""Random streams (include/avida_gpu.h "random streams").

CPU: the oracle's RECORDED mode consumes the host's doubles with the
reference's Apto::RNG interface -- P(p) = u < p, GetUInt(n) = floor(u n),
GetRandomInst = the cOrderedWeightedIndex lookup of u * total weight -- in the
reference's call order (Divide_DoMutations: TestDivideSlip, -Mut, -Ins, -Del
always draw; cpu/cHardwareBase.cc:296-569, main/cMutationRates.h:119-128).
GPU: the device equals the oracle bit for bit with mutations on, fed from a
recorded stream (FROZEN traces of the configs[2] population) and with the
divide slip / uniform mutations in a world."""
import os

import ctypes as C

import numpy as np
import pytest

from avida_amd import capi, files
import oracle_lib as ol
import parity_util as pu

CAP = capi.MAX_GENOME


def _ancestor(golden, overrides):
    iset, env, cfg = pu.load_env(golden, overrides=overrides, seed=3)
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    return iset, env, cfg, anc


def test_recorded_draws_follow_reference_interface(golden):
    """Every h-copy mutates (COPY_MUT_PROB 1: P(1) = u < 1 always), every
    draw is u = 0.37: the ancestor's 100 copies each consume two doubles (the
    test, then GetRandomInst = the op whose cumulative weight first exceeds
    0.37 * total), the divide consumes slip, mut, ins, del tests (DIVIDE_MUT 0:
    no hit at u < 0) -- so the offspring is 100 copies of that op and the
    stream position after the first gestation is 2 * 100 + 4 (+ the line and
    instruction draws of an insertion hit when 0.37 < DIVIDE_INS_PROB)."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 1.0, "DIVIDE_INS_PROB": 0.5,
                                             "DIVIDE_DEL_PROB": 0.1, "DEATH_METHOD": 0})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    u = 0.37
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, u))
    st0, _, _ = b.states(0, 1, CAP)
    assert st0[0].rng_counter == 0
    # run until the first divide (one gestation: 389 instructions without mutations)
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, ops, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    # 100 h-copies x (P + GetRandomInst), then slip, mut, ins (hit: u < 0.5 ->
    # GetUInt(101), GetRandomInst), del (u >= 0.1: no hit)
    assert st[0].rng_counter == 2 * 100 + 1 + 1 + 1 + 2 + 1
    assert b.lib.orc_rec_exhausted() == 0


def test_recorded_draws_per_site_divide_mutations(golden):
    """DIV_MUT_PROB (cpu/cHardwareBase.cc:447-460) after the always-drawing
    slip / mut / ins / del tests: Binomial(100, 0.5) as one P(0.5) per site
    (u = 0.37 hits every time: 100 substitutions), then GetUInt(100) and
    GetRandomInst per substitution -- 4 + 100 + 2 * 100 draws at the first
    divide, with no copy-mutation draws at COPY_MUT_PROB 0 (they are skipped at
    a zero rate, main/cMutationRates.h:111)."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "DIV_MUT_PROB": 0.5,
                                             "DEATH_METHOD": 0})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, 0.37))
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, _, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    assert st[0].rng_counter == 4 + 100 + 2 * 100
    assert b.lib.orc_rec_exhausted() == 0


def test_recorded_draws_parent_mutations(golden):
    """PARENT_MUT_PROB (cpu/cHardwareBase.cc:508-520) on the parent's memory,
    cut to the divide point (Divide_Main :1803-1806): after the 4 always-drawing
    divide tests, Binomial(100, 0.5) as 100 P(0.5) draws (all hit at u = 0.37),
    then GetUInt(100) + GetRandomInst per substitution -- all of them on
    site 37, which becomes the op GetRandomInst(0.37) picks."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "PARENT_MUT_PROB": 0.5,
                                             "DEATH_METHOD": 0})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, 0.37))
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, ops, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    assert st[0].rng_counter == 4 + 100 + 2 * 100
    assert st[0].mem_size == 100
    # every GetUInt(100) at u = 0.37 picks site 37: only it changed
    assert [i for i in range(100) if ops[i] != anc[i]] == [37]


def test_recorded_draws_poisson_divide_mutations(golden):
    """DIVIDE_POISSON_{SLIP,MUT,INS,DEL}_MEAN = 1 (cpu/cHardwareBase.cc:318-320,
    :383-435): at u = 0.37 every Poisson count is 1 (0.37 >= exp(-1), then
    0.37^2 < exp(-1): two uniforms), each right after its one-shot test --
    slip 1 + 2 + (from, to) 2, mut 1 + 2 + (line, inst) 2, ins 1 + 2 + 2,
    del 1 + 2 + (line) 1 = 19 draws at the first divide."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0,
                                             "DIVIDE_POISSON_SLIP_MEAN": 1.0,
                                             "DIVIDE_POISSON_MUT_MEAN": 1.0,
                                             "DIVIDE_POISSON_INS_MEAN": 1.0,
                                             "DIVIDE_POISSON_DEL_MEAN": 1.0})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, 0.37))
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, _, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    assert st[0].rng_counter == 19
    assert b.lib.orc_rec_exhausted() == 0


def test_recorded_draws_per_site_ins_del_uniform_slip(golden):
    """DIV_SLIP_PROB, DIV_INS_PROB, DIV_DEL_PROB, DIV_UNIFORM_PROB = 0.5
    (cpu/cHardwareBase.cc:323-327, :463-503) at u = 0.37 on the 100-site
    ancestor: 1 slip test, 100 + 100 x 2 per-site slips (from = to = 37: no
    change), mut / ins / del tests 3, 100 + 100 insertion sites + 100
    instructions, 200 deletion tests of which 192 fit above the 8-site minimum
    (+192 sites), 8 uniform tests + 8 x 2 (op 19 < 26: a substitution) = 1020."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0,
                                             "DIV_SLIP_PROB": 0.5, "DIV_INS_PROB": 0.5,
                                             "DIV_DEL_PROB": 0.5, "DIV_UNIFORM_PROB": 0.5})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, 0.37))
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, _, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    assert st[0].rng_counter == 1 + 300 + 3 + 300 + 200 + 192 + 8 + 16
    assert b.lib.orc_rec_exhausted() == 0


def test_recorded_draws_translocations(golden):
    """DIVIDE_TRANS_PROB 0.5, DIVIDE_POISSON_TRANS_MEAN 1, DIV_TRANS_PROB 0.5
    (cpu/cHardwareBase.cc:331-343, doTransMutation :700-760) at u = 0.37: slip
    test 1, one-shot test 1 + (from, to, insertion site) 3, Poisson count 2 +
    3, 100 per-site tests + 100 x 3, mut / ins / del tests 3 = 413 draws."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0,
                                             "DIVIDE_TRANS_PROB": 0.5,
                                             "DIVIDE_POISSON_TRANS_MEAN": 1.0,
                                             "DIV_TRANS_PROB": 0.5})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, 0.37))
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, _, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    assert st[0].rng_counter == 1 + 1 + 3 + 2 + 3 + 100 + 300 + 3
    # TRANS_FILL_MODE 1 (scrambled) is on the path; an unknown mode and
    # SLIP_FILL_MODE 1 (nop-X) are refused by the library itself
    lib = capi.load_product()
    _, _, cfg1 = pu.load_env(golden, overrides={"DIVIDE_TRANS_PROB": 0.1, "TRANS_FILL_MODE": 1})
    assert lib.avgpu_check_cfg(C.byref(cfg1)) == 0
    _, _, cfg2 = pu.load_env(golden, overrides={"DIVIDE_TRANS_PROB": 0.1, "TRANS_FILL_MODE": 2})
    assert lib.avgpu_check_cfg(C.byref(cfg2)) == -5
    assert "TRANS_FILL_MODE" in lib.avgpu_last_error().decode()
    _, _, cfg3 = pu.load_env(golden, overrides={"DIVIDE_SLIP_PROB": 0.1, "SLIP_FILL_MODE": 1})
    assert lib.avgpu_check_cfg(C.byref(cfg3)) == -5
    assert "SLIP_FILL_MODE" in lib.avgpu_last_error().decode()


def test_recorded_draws_fill_modes(golden):
    """The data fills draw once per filled site, after from / to (/ ins_loc):
    SLIP_FILL_MODE 2 GetRandomInst, SLIP_FILL_MODE 3 and TRANS_FILL_MODE 1
    GetInt(L - i) (cpu/cHardwareBase.cc:636-665, :721-741).  At u = 0.37 on
    the 100-site ancestor: from = floor(0.37 * 101) = 37, to = 37 (L = 0, no
    fill) -- so the stream puts from = 60, to = 20 (L = 40) instead."""
    for ov, head, fills in [({"DIVIDE_SLIP_PROB": 1.0, "SLIP_FILL_MODE": 2}, [0.1, _u(60, 101), _u(20, 101)], 40),
                            ({"DIVIDE_SLIP_PROB": 1.0, "SLIP_FILL_MODE": 3}, [0.1, _u(60, 101), _u(20, 101)], 40),
                            ({"DIVIDE_TRANS_PROB": 1.0, "TRANS_FILL_MODE": 1},
                             [0.9, 0.1, _u(60, 101), _u(20, 101), _u(5, 101)], 40)]:
        iset, env, cfg, anc = _ancestor(golden, dict({"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                                      "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0}, **ov))
        b = ol.Backend("oracle", cfg, iset, env, ncells=1)
        b.set_orgs(0, [anc], deterministic=True)
        b.set_rng_mode(capi.RNG_RECORDED, np.array(head + [0.37] * 4000))
        for k in range(2000):
            b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
            st, _, _ = b.states(0, 1, CAP)
            if st[0].num_divides:
                break
        assert st[0].num_divides == 1
        assert st[0].rng_counter == len(head) + fills + 3, ov      # + mut / ins / del tests
        b.close()


def _scramble(draws):
    """the copied_so_far walk of doSlipMutation / doTransMutation
    (cpu/cHardwareBase.cc:652-664): each draw picks the draw-th index not
    taken yet"""
    free = list(range(len(draws)))
    return [free.pop(d) for d in draws]


def _fill_cases(anc, nops):
    """(overrides, stream, expected offspring), derived by hand from
    doSlipMutation / doTransMutation on the 100-site ancestor."""
    cases = []
    # slip from 30 to 25 (L = 5): child = a[:30] + fill + a[30:]
    codes = [5, 17, 0, 25, 9]
    cases.append(({"DIVIDE_SLIP_PROB": 1.0, "SLIP_FILL_MODE": 2},
                  [0.1, _u(30, 101), _u(25, 101)] + [_u(c, nops) for c in codes] + [0.9] * 3,
                  anc[:30] + bytes(codes) + anc[30:]))
    draws = [4, 0, 2, 0, 0]                  # -> indices 4, 0, 3, 1, 2
    assert _scramble(draws) == [4, 0, 3, 1, 2]
    cases.append(({"DIVIDE_SLIP_PROB": 1.0, "SLIP_FILL_MODE": 3},
                  [0.1, _u(30, 101), _u(25, 101)] + [_u(d, 5 - i) for i, d in enumerate(draws)] + [0.9] * 3,
                  anc[:30] + bytes(anc[25 + k] for k in [4, 0, 3, 1, 2]) + anc[30:]))
    # translocation from 30 to 10 (L = 20) inserted at 15, scrambled with every
    # draw 0 (indices in order): site 15 + i reads the sequence being filled at
    # 10 + i, which for i >= 5 is a site this fill already wrote -- the fill is
    # a[10:15] four times; then a[15:] after it
    cases.append(({"DIVIDE_TRANS_PROB": 1.0, "TRANS_FILL_MODE": 1},
                  [0.9, 0.1, _u(30, 101), _u(10, 101), _u(15, 101)] + [_u(0, 20 - i) for i in range(20)] + [0.9] * 3,
                  anc[:15] + anc[10:15] * 4 + anc[15:]))
    # scrambled without overlap: from 60 to 50 (L = 10) at 5
    draws = [9, 0, 7, 1, 5, 0, 3, 2, 1, 0]
    cases.append(({"DIVIDE_TRANS_PROB": 1.0, "TRANS_FILL_MODE": 1},
                  [0.9, 0.1, _u(60, 101), _u(50, 101), _u(5, 101)] + [_u(d, 10 - i) for i, d in enumerate(draws)]
                  + [0.9] * 3,
                  anc[:5] + bytes(anc[50 + k] for k in _scramble(draws)) + anc[5:]))
    return cases


@pytest.mark.parametrize("kind", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_fill_mode_offspring_content(golden, kind):
    """Offspring of recorded slips with SLIP_FILL_MODE 2 (random instructions)
    and 3 (scrambled), and of scrambled translocations (TRANS_FILL_MODE 1,
    including the read-back of sites the fill already wrote), against the
    hand derivations of _fill_cases."""
    iset = files.read_instset(os.path.join(golden, "instset-heads.cfg"))
    anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
    for ov, stream, want in _fill_cases(anc, len(iset.names)):
        child, parent, pos, _, _ = first_offspring(kind, golden, ov, stream)
        assert pos == len(stream), ov
        assert child == want, (ov, list(child), list(want))


def _u(k, n):
    """the recorded double that GetUInt(n) / GetInt(n) turns into k"""
    return (k + 0.5) / n


def first_offspring(kind, golden, overrides, stream, side=3):
    """Run a side x side world holding the default-heads ancestor in its
    centre cell, the ancestor drawing from `stream` (RECORDED), until the first
    birth; return (offspring op codes, parent op codes after the divide,
    stream position of the parent)."""
    iset, env, cfg, anc = _ancestor(golden, dict({"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                                  "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0,
                                                  "WORLD_X": side, "WORLD_Y": side}, **overrides))
    n = side * side
    c0 = n // 2
    b = ol.Backend(kind, cfg, iset, env, ncells=n)
    try:
        b.set_orgs(c0, [anc], deterministic=True)
        offs = np.zeros(n, dtype=np.int64)
        offs[:] = len(stream)                     # every other cell: an empty segment
        offs[c0] = 0
        b.set_rng_mode(capi.RNG_RECORDED, np.asarray(stream, dtype=np.float64), offsets=offs)
        for _ in range(40):
            s = b.run_update()
            if s.births + s.births_overwritten:
                break
        st, ops, _ = b.states(0, n, CAP)
        kids = [c for c in range(n) if c != c0 and st[c].alive]
        assert len(kids) == 1, kids
        k = kids[0]
        child = bytes(ops[k * CAP:k * CAP + st[k].birth_length])
        parent = bytes(ops[c0 * CAP:c0 * CAP + st[c0].mem_size])
        return child, parent, st[c0].rng_counter, iset, anc
    finally:
        b.close()


def _trans_cases():
    """doTransMutation (cpu/cHardwareBase.cc:700-760) on the 100-site
    ancestor, derived by hand: (from, to, ins_loc) -> offspring.
    from > to: copy[to, from) is inserted at ins_loc (g[:ins] = copy[:ins],
    g[ins:ins+L] = copy[to:from], then copy[ins:]); from < to: the size shrinks
    by to - from and g[ins:] = copy[ins + to - from:]."""
    def dup(a, f, t, i):
        return a[:i] + a[t:f] + a[i:]

    def cut(a, f, t, i):
        return a[:i] + a[i + (t - f):]
    return [((30, 10, 50), dup), ((10, 30, 40), cut), ((95, 2, 7), dup), ((3, 90, 5), cut)]


@pytest.mark.parametrize("kind", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_translocation_offspring_content(golden, kind):
    """Offspring of a recorded translocation, checked against the hand
    derivation: the divide draws TestDivideSlip, the one-shot
    TestDivideTrans hit, from, to (GetInt(size+1)), the insertion site
    (GetInt(size+1)), then the mut / ins / del tests."""
    for (f, t, i), make in _trans_cases():
        stream = [0.9, 0.1, _u(f, 101), _u(t, 101), _u(i, 101), 0.9, 0.9, 0.9]
        child, parent, pos, iset, anc = first_offspring(kind, golden, {"DIVIDE_TRANS_PROB": 1.0}, stream)
        assert pos == 8
        assert child == make(anc, f, t, i), (f, t, i)
        assert parent[:100] == anc          # (it may have re-allocated since)


def test_recorded_draws_parent_insertions_deletions(golden):
    """PARENT_INS_PROB / PARENT_DEL_PROB 0.5 (cpu/cHardwareBase.cc:523-565) at
    u = 0.37 on the 100-site ancestor: slip, mut, ins, del tests 4; 100
    insertion tests (all hit) + 100 sites + 100 instructions (the parent grows
    to 200); 200 deletion tests, capped at 200 - 8 = 192 deletions + 192 sites:
    696 draws, and the parent is left with the 8-site minimum."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "DEATH_METHOD": 0,
                                             "PARENT_INS_PROB": 0.5, "PARENT_DEL_PROB": 0.5})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(4096, 0.37))
    for k in range(2000):
        b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
        st, _, _ = b.states(0, 1, CAP)
        if st[0].num_divides:
            break
    assert st[0].num_divides == 1
    assert st[0].rng_counter == 4 + 300 + 200 + 192
    assert st[0].mem_size == 8
    assert b.lib.orc_rec_exhausted() == 0


def test_copy_mutation_draw_order(golden):
    """Inst_HeadCopy's copy mutations (cpu/cHardwareCPU.cc:7144-7161): per
    h-copy TestCopyMut, then TestCopyIns [+ GetRandomInst], TestCopyDel,
    TestCopyUniform [+ GetUInt(2n+1)], TestCopySlip [+ GetInt(size)], each
    drawing only at a non-zero rate.  At u = 0.37 with every rate 0.5 every
    test hits: a copy draws mut 2 + ins 2 + del 1 + uniform 2 + slip 2 = 9."""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.5, "COPY_INS_PROB": 0.5,
                                             "COPY_DEL_PROB": 0.5, "COPY_UNIFORM_PROB": 0.5,
                                             "COPY_SLIP_PROB": 0.5, "DEATH_METHOD": 0})
    b = ol.Backend("oracle", cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.full(100000, 0.37))
    # the ancestor's first h-copy is its 90th instruction (Appendix B of SURVEY.md)
    b.step(0, 1, uniform=89, mode=capi.MODE_FROZEN)
    st0, _, _ = b.states(0, 1, CAP)
    assert st0[0].rng_counter == 0
    b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
    st, ops, fl = b.states(0, 1, CAP)
    assert st[0].rng_counter == 9
    # ins then del at the write head cancel; the uniform draw floor(0.37 * 53)
    # = 19 < 26 substitutes op 19 in place; the slip moves the read head to
    # floor(0.37 * 300) = 111, then Advance -> 112; the write head advances
    assert st[0].mem_size == 300
    assert st[0].head[1] == 112 and st[0].head[2] == 101
    assert ops[100] == 19 and fl[100] & 1


def _slip_memory_expected(ops, fl, M, frm, to, fill, rand_code=None):
    """doSlipMutation on the whole memory (cpu/cHardwareBase.cc:621-694),
    restated independently of the oracle: (ops, flags) after the slip.  Only
    the instructions move; flags stay with positions (new positions: 0)."""
    copy = list(ops[:M])
    ins = frm - to
    Mn = M + ins
    new = copy[:min(M, Mn)] + [0] * max(0, Mn - M)
    for i in range(max(ins, 0)):
        new[frm + i] = copy[to + i] if fill == 0 else (2 if fill == 4 else rand_code(i))
    for i in range(max(ins, 0), M - to):
        new[frm + i] = copy[to + i]
    flags = list(fl[:min(M, Mn)]) + [0] * max(0, Mn - M)
    return new, flags


def _first_copy_state(kind, golden, stream, fill):
    """the ancestor (COPY_SLIP_PROB 0.5, SLIP_COPY_MODE 1, every other
    mutation off) just before its first h-copy (its 90th instruction, SURVEY.md
    Appendix B) and just after it, fed from `stream`"""
    iset, env, cfg, anc = _ancestor(golden, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                             "DIVIDE_DEL_PROB": 0.0, "COPY_SLIP_PROB": 0.5,
                                             "SLIP_COPY_MODE": 1, "SLIP_FILL_MODE": fill,
                                             "DEATH_METHOD": 0})
    b = ol.Backend(kind, cfg, iset, env, ncells=1)
    b.set_orgs(0, [anc], deterministic=True)
    b.set_rng_mode(capi.RNG_RECORDED, np.asarray(stream, dtype=np.float64))
    b.step(0, 1, uniform=89, mode=capi.MODE_FROZEN)
    before = b.states(0, 1, CAP)
    b.step(0, 1, uniform=1, mode=capi.MODE_FROZEN)
    after = b.states(0, 1, CAP)
    b.close()
    return iset, before, after


@pytest.mark.parametrize("kind", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("second,fill", [(0.37, 0), (0.1, 0), (0.1, 4), (0.0, 2)])
def test_copy_slip_memory_kat(golden, kind, second, fill):
    """SLIP_COPY_MODE 1 (cpu/cHardwareCPU.cc:785, :7157-7161): the copy slip
    is doSlipMutation of the whole memory at the write head.  The first
    h-copy of the ancestor (memory 300 after h-alloc, read head 0, write head
    100) with draws [0.37 (TestCopySlip hits), `second` (to = GetInt(301))]:
    0.37 -> to 111, a deletion of sites 100..110 (memory 289); 0.1 -> to 30,
    sites 30..99 duplicated at 100 (memory 370), SLIP_FILL_MODE 4 fills them
    with nop-C instead; 0.0 -> to 0, SLIP_FILL_MODE 2 draws one GetRandomInst
    per inserted site (memory 400).  Expected memory and flags restated in
    the test; then both heads advance (read 1, write 101)."""
    stream = [0.37, second] + [0.61] * 200
    iset, (st0, o0, f0), (st, o1, f1) = _first_copy_state(kind, golden, stream, fill)
    M = st0[0].mem_size
    assert M == 300 and st0[0].head[1] == 0 and st0[0].head[2] == 100
    ops, fl = list(o0[:M]), list(f0[:M])
    ops[100] = ops[0]                              # the copy itself (COPY_MUT 0)
    fl[100] |= 1                                   # copied flag (cpu/cHeadCPU SetFlagCopied)
    to = int(second * 301)
    # GetRandomInst of u = 0.61: the op whose cumulative redundancy first exceeds 0.61 * total
    cum = np.cumsum(iset.redundancy)
    rnd = int(np.searchsorted(cum, 0.61 * cum[-1], side="right"))
    want_ops, want_fl = _slip_memory_expected(ops, fl, M, 100, to, fill, lambda i: rnd)
    Mn = len(want_ops)
    assert st[0].mem_size == Mn == M + 100 - to
    assert list(o1[:Mn]) == want_ops
    assert [x & 1 for x in f1[:Mn]] == [x & 1 for x in want_fl]       # copied flags stay per position
    assert st[0].head[1] == 1 and st[0].head[2] == 101
    assert st[0].rng_counter == 2 + (100 - to if fill == 2 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("muts", ["copy", "all", "site", "poisson", "copyext"])
def test_recorded_stream_frozen_traces_gpu(golden, muts):
    """BASELINE configs[2] traces with mutations on, fed from one recorded
    stream: 3600 organisms of the detail-50000 population, each with its own
    segment, FROZEN mode (divide-mutation draws happen, the offspring is
    discarded); per-lane state equal after 1, 30, 1000, 4000 instructions."""
    iset_c = files.read_instset(os.path.join(golden, "instset-classic.cfg"))
    genomes = pu.pop_genomes(golden, iset_c)[:3600]
    ov = {"COPY_MUT_PROB": 0.02, "DIVIDE_INS_PROB": 0.05, "DIVIDE_DEL_PROB": 0.05, "DEATH_METHOD": 0}
    if muts == "all":
        ov.update({"DIVIDE_MUT_PROB": 0.1, "DIVIDE_SLIP_PROB": 0.05, "DIVIDE_UNIFORM_PROB": 0.05})
    if muts == "site":      # per-site divide substitutions: one draw per offspring site
        ov.update({"DIV_MUT_PROB": 0.02, "PARENT_MUT_PROB": 0.01, "DIV_INS_PROB": 0.005,
                   "DIV_DEL_PROB": 0.005, "DIV_UNIFORM_PROB": 0.005, "DIV_SLIP_PROB": 0.001,
                   "PARENT_INS_PROB": 0.005, "PARENT_DEL_PROB": 0.005})
    if muts == "copyext":   # copy insertions / deletions / uniform / slips (cpu/cHardwareCPU.cc:7153-7161)
        ov.update({"COPY_INS_PROB": 0.02, "COPY_DEL_PROB": 0.02, "COPY_UNIFORM_PROB": 0.01,
                   "COPY_SLIP_PROB": 0.005, "PARENT_MUT_PROB": 0.0})
    if muts == "poisson":
        ov.update({"DIVIDE_POISSON_SLIP_MEAN": 0.3, "DIVIDE_POISSON_MUT_MEAN": 1.5,
                   "DIVIDE_TRANS_PROB": 0.05, "DIVIDE_POISSON_TRANS_MEAN": 0.1,
                   "DIVIDE_POISSON_INS_MEAN": 0.8, "DIVIDE_POISSON_DEL_MEAN": 0.8})
    iset, env, cfg = pu.load_env(golden, "instset-classic.cfg", ov)
    n = len(genomes)
    rng = np.random.default_rng(42)
    per = {"site": 16000, "copyext": 24000}.get(muts, 4500)   # h-copy draws per copy at non-zero rates
    stream = rng.random(n * per)
    offsets = np.arange(n, dtype=np.int64) * per
    pair = [ol.Backend(k, cfg, iset, env, ncells=n) for k in ("oracle", "gpu")]
    for b in pair:
        b.set_orgs(0, genomes, deterministic=False)
        b.set_rng_mode(capi.RNG_RECORDED, stream, offsets)
    for budget in [1, 29, 970, 3000]:
        for b in pair:
            b.step(0, n, uniform=budget, mode=capi.MODE_FROZEN)
        a, oa, fa = pair[0].states(0, n, CAP)
        g, og, fg = pair[1].states(0, n, CAP)
        bad = pu.diff_states(a, g, oa, og, fa, fg, CAP)
        assert not bad, f"after {budget}: {len(bad)} mismatches {bad[:4]}"
    assert max(a[i].rng_counter for i in range(n)) > 10
    assert max(a[i].rng_counter for i in range(n)) < per    # no segment ran into the next one
    assert pair[1].counters()[capi.CNT_REC_EXHAUSTED] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("fill", [0, 2, 3, 4])
def test_divide_slip_uniform_world_gpu(golden, fill):
    """World updates with DIVIDE_SLIP_PROB (SLIP_FILL_MODE 0 duplication, 2
    random, 3 scrambled, 4 nop-C) and DIVIDE_UNIFORM_PROB on top of the default
    mutations (with 2 / 3 also Poisson and per-site slips and scrambled
    translocations): GPU world == oracle world, every cell digest, 120 updates."""
    ov = {"DIVIDE_SLIP_PROB": 0.1, "DIVIDE_UNIFORM_PROB": 0.1, "SLIP_FILL_MODE": fill,
          "WORLD_X": 48, "WORLD_Y": 48}
    if fill in (2, 3):
        ov.update({"DIVIDE_POISSON_SLIP_MEAN": 0.05, "DIV_SLIP_PROB": 0.0005,
                   "DIVIDE_TRANS_PROB": 0.05, "TRANS_FILL_MODE": 1})
    iset, env, cfg, anc = _ancestor(golden, ov)
    n = 48 * 48
    pair = [ol.Backend(k, cfg, iset, env, ncells=n) for k in ("oracle", "gpu")]
    g = pu.mutants_of(anc, iset, n // 4, rate=0.01, seed=9)
    for b in pair:
        b.set_orgs(0, g, deterministic=False)
    for u in range(120):
        so, sg = pair[0].run_update(), pair[1].run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten"):
            assert getattr(so, f) == getattr(sg, f), (u, f)
    nbad, cells = pu.compare_digests(pair[0].digests(), pair[1].digests())
    assert nbad == 0, cells
    lens = {pair[0].states(c, 1)[0][0].birth_length for c in range(0, n, 7)}
    assert len(lens) > 5      # slips changed genome lengths


@pytest.mark.gpu
@pytest.mark.parametrize("knob", ["DIV_MUT_PROB", "PARENT_MUT_PROB", "POISSON", "PER_SITE", "TRANS",
                                  "PARENT_INDEL"])
def test_per_site_divide_mutations_world_gpu(golden, knob):
    """World updates with DIV_MUT_PROB (per-site substitutions in the
    offspring, cpu/cHardwareBase.cc:447-460) or PARENT_MUT_PROB (in the
    parent, :508-520) on top of the default mutations: GPU world == oracle
    world, every cell digest, 120 updates; the substitution arena never fills.
    POISSON: the four DIVIDE_POISSON_*_MEAN knobs (:318-320, :383-435)."""
    ov = {knob: 0.02, "WORLD_X": 48, "WORLD_Y": 48}
    if knob == "PER_SITE":   # per-site insertions, deletions, uniform mutations, slips (:323-327, :463-503)
        ov = {"DIV_INS_PROB": 0.005, "DIV_DEL_PROB": 0.005, "DIV_UNIFORM_PROB": 0.005,
              "DIV_SLIP_PROB": 0.001, "WORLD_X": 48, "WORLD_Y": 48}
    if knob == "TRANS":      # translocations: one-shot, Poisson, per site (:331-343)
        ov = {"DIVIDE_TRANS_PROB": 0.1, "DIVIDE_POISSON_TRANS_MEAN": 0.1, "DIV_TRANS_PROB": 0.0005,
              "WORLD_X": 48, "WORLD_Y": 48}
    if knob == "PARENT_INDEL":   # per-site insertions / deletions in the parent (:523-565)
        ov = {"PARENT_INS_PROB": 0.01, "PARENT_DEL_PROB": 0.01, "PARENT_MUT_PROB": 0.005,
              "WORLD_X": 48, "WORLD_Y": 48}
    if knob == "POISSON":
        ov = {"DIVIDE_POISSON_SLIP_MEAN": 0.1, "DIVIDE_POISSON_MUT_MEAN": 1.0,
              "DIVIDE_POISSON_INS_MEAN": 0.5, "DIVIDE_POISSON_DEL_MEAN": 0.5,
              "WORLD_X": 48, "WORLD_Y": 48}
    iset, env, cfg, anc = _ancestor(golden, ov)
    n = 48 * 48
    pair = [ol.Backend(k, cfg, iset, env, ncells=n) for k in ("oracle", "gpu")]
    g = pu.mutants_of(anc, iset, n // 4, rate=0.01, seed=11)
    for b in pair:
        b.set_orgs(0, g, deterministic=False)
    births = 0
    for u in range(120):
        so, sg = pair[0].run_update(), pair[1].run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten"):
            assert getattr(so, f) == getattr(sg, f), (u, f)
        births += sg.births
        assert pair[1].counters()[capi.CNT_SUB_OVERFLOW] == 0
        assert pair[1].counters()[capi.CNT_MEM_CAP] == 0
    nbad, cells = pu.compare_digests(pair[0].digests(), pair[1].digests())
    assert nbad == 0, cells
    assert births > 500


@pytest.mark.gpu
@pytest.mark.parametrize("rec,slip_mode,fill", [(False, 0, 0), (True, 0, 0), (False, 1, 0), (True, 1, 2),
                                                (False, 1, 4)])
def test_copy_mutations_world_gpu(golden, rec, slip_mode, fill):
    """World updates with COPY_INS_PROB, COPY_DEL_PROB, COPY_UNIFORM_PROB and
    COPY_SLIP_PROB (cpu/cHardwareCPU.cc:7153-7161) on top of the default
    mutations: the memory grows and shrinks in the middle of h-copy, and a copy
    that would outgrow its LDS size class is rewound and spills to the next
    class.  GPU world == oracle world, every cell digest, 150 updates; rec:
    every organism of the seeded world draws from a recorded stream."""
    ov = {"COPY_INS_PROB": 0.03, "COPY_DEL_PROB": 0.02, "COPY_UNIFORM_PROB": 0.01,
          "COPY_SLIP_PROB": 0.005, "WORLD_X": 48, "WORLD_Y": 48,
          "SLIP_COPY_MODE": slip_mode, "SLIP_FILL_MODE": fill}   # mode 1: memory slips (cpu/cHardwareBase.cc:621)
    iset, env, cfg, anc = _ancestor(golden, ov)
    n = 48 * 48
    pair = [ol.Backend(k, cfg, iset, env, ncells=n) for k in ("oracle", "gpu")]
    g = pu.mutants_of(anc, iset, n // 4, rate=0.01, seed=13)
    if rec:
        per = 60000
        stream = np.random.default_rng(5).random(n * per)
        offsets = np.arange(n, dtype=np.int64) * per
    for b in pair:
        b.set_orgs(0, g, deterministic=False)
        if rec:
            b.set_rng_mode(capi.RNG_RECORDED, stream, offsets)
    births = 0
    for u in range(150):
        so, sg = pair[0].run_update(), pair[1].run_update()
        for f in ("num_organisms", "insts_executed", "births", "deaths", "divides", "births_dropped",
                  "births_overwritten"):
            assert getattr(so, f) == getattr(sg, f), (u, f)
        births += sg.births
    nbad, cells = pu.compare_digests(pair[0].digests(), pair[1].digests())
    assert nbad == 0, cells
    c = pair[1].counters(cumulative=1)
    assert births > 500
    assert c[capi.CNT_SPILLS] > 0          # copies rewound into the next size class
    assert slip_mode == 1 or c[capi.CNT_MEM_CAP] == 0
    lens = {pair[0].states(k, 1)[0][0].birth_length for k in range(0, n, 7)}
    assert len(lens) > 5
