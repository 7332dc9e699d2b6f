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


def diff_states_np(a, b, ops_a, ops_b, fl_a, fl_b, cap, first=0, limit=20):
    """diff_states for large worlds: raw struct bytes and memory images are
    compared with numpy, the field-by-field report only for mismatching cells
    (at most `limit`).  Returns (number of mismatching cells, report)."""
    import ctypes as C
    import numpy as np
    n = len(a)
    sz = C.sizeof(capi.AvgpuCpuState)
    ra = np.frombuffer(a, dtype=np.uint8).reshape(n, sz)
    rb = np.frombuffer(b, dtype=np.uint8).reshape(n, sz)
    bad = np.any(ra != rb, axis=1)
    msz = np.frombuffer(a, dtype=np.uint8).reshape(n, sz)[:, capi.AvgpuCpuState.mem_size.offset:
                                                            capi.AvgpuCpuState.mem_size.offset + 4]
    m = np.ascontiguousarray(msz).view(np.int32).reshape(n)
    keep = np.arange(cap)[None, :] < np.minimum(m, cap)[:, None]
    oa = np.frombuffer(ops_a, dtype=np.uint8).reshape(n, cap)
    ob = np.frombuffer(ops_b, dtype=np.uint8).reshape(n, cap)
    fa = np.frombuffer(fl_a, dtype=np.uint8).reshape(n, cap)
    fb = np.frombuffer(fl_b, dtype=np.uint8).reshape(n, cap)
    bad |= np.any((oa != ob) & keep, axis=1) | np.any((fa != fb) & keep, axis=1)
    idx = np.nonzero(bad)[0]
    report = []
    for i in idx[:limit]:
        i = int(i)
        ta, tb = state_tuple(a[i]), state_tuple(b[i])
        diffs = [k for k in STATE_FIELDS if ta[k] != tb[k]]
        report.append((first + i, diffs or ["memory"]))
    return len(idx), report


M64 = (1 << 64) - 1


def _mix(z):
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def digest_of(state, ops, flags, handlers):
    """Python restatement of the per-cell state digest (avida_amd/csrc/world.hip
    k_state_digest, oracle orc_state_digests) from one avgpu_get_states record
    and its memory (op codes, flags bit0 copied / bit2 executed)."""
    import ctypes as C
    import struct
    if state.birth_length == 0:
        return 0
    raw = bytes(C.string_at(C.addressof(state), C.sizeof(state)))
    h = 0x9E3779B97F4A7C15
    for k, (w,) in enumerate(struct.iter_unpack("<I", raw)):
        h = _mix(h ^ ((k << 32) | w))
    m = state.mem_size
    for k in range((m + 3) // 4):
        v = 0
        for j in range(4):
            q = 4 * k + j
            if q < m:
                b = (handlers[ops[q]] & 0x3F) | (0x40 if flags[q] & 1 else 0) | (0x80 if flags[q] & 4 else 0)
                v |= b << (8 * j)
        h = _mix(h ^ (((0x10000 + k) << 32) | v))
    return h


def compare_digests(da, db, first=0, limit=10):
    """(number of differing cells, first `limit` differing global cell ids)"""
    import numpy as np
    idx = np.nonzero(da != db)[0]
    return len(idx), [int(first + i) for i in idx[:limit]]
