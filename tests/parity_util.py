"""Helpers shared by the parity tests: build matched oracle/GPU backends and
compare organism state tuples field by field."""
from __future__ import annotations

import os
import random

from avida_amd import capi, files
import oracle_lib as ol

STATE_FIELDS = [n for n, _ in capi.AvgpuCpuState._fields_ if not n.startswith("pad")]


def state_tuple(s):
    out = {}
    for n in STATE_FIELDS:
        v = getattr(s, n)
        if hasattr(v, "__len__"):
            v = [list(x) if hasattr(x, "__len__") else x for x in v]
        out[n] = v
    return out


def diff_states(a, b, ops_a, ops_b, fl_a, fl_b, cap):
    """Return a list of (index, field, a, b) mismatches; memory compared up to mem_size."""
    bad = []
    for i in range(len(a)):
        if a[i].birth_length == 0 and b[i].birth_length == 0:
            continue   # never-occupied cell: no organism, nothing to compare
        ta, tb = state_tuple(a[i]), state_tuple(b[i])
        for k in STATE_FIELDS:
            if ta[k] != tb[k]:
                bad.append((i, k, ta[k], tb[k]))
        m = a[i].mem_size
        if m == b[i].mem_size:
            o = i * cap
            if ops_a[o:o + m] != ops_b[o:o + m]:
                bad.append((i, "mem_ops", None, None))
            if fl_a[o:o + m] != fl_b[o:o + m]:
                bad.append((i, "mem_flags", None, None))
    return bad


def load_env(golden, instset="instset-heads.cfg", overrides=None, seed=7):
    iset = files.read_instset(os.path.join(golden, instset))
    env = files.read_environment(os.path.join(golden, "environment-logic9.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, overrides or {}), seed=seed)
    return iset, env, cfg


def pop_genomes(golden, iset_classic):
    """BASELINE config 2: the 3599 organisms of heads_midrun_30u/config/detail-50000.pop
    (genotypes expanded by num_cpus, classic legacy instset) + the ancestor."""
    gs = files.read_pop(os.path.join(golden, "detail-50000.pop"))
    out = []
    for g in gs:
        seq = iset_classic.parse_sequence(g.sequence)
        out.extend([seq] * g.num_cpus)
    return out


def random_genomes(iset, n, lo=8, hi=400, seed=1):
    rnd = random.Random(seed)
    out = []
    for _ in range(n):
        L = rnd.randint(lo, hi)
        out.append(bytes(rnd.randrange(len(iset.names)) for _ in range(L)))
    return out


def mutants_of(seq, iset, n, rate=0.03, seed=2):
    """Point mutants of a viable genome: exercises copy loops, divides, labels."""
    rnd = random.Random(seed)
    out = []
    for _ in range(n):
        g = bytearray(seq)
        for i in range(len(g)):
            if rnd.random() < rate:
                g[i] = rnd.randrange(len(iset.names))
        out.append(bytes(g))
    return out
