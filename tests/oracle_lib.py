"""Test-infrastructure loader for the CPU oracle (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from avida_amd import capi, files

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

_lib = None


def load_oracle():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    lib = C.CDLL(ORACLE_SO)
    capi.bind_common(lib, "orc_")
    lib.orc_create.restype = C.c_void_p
    lib.orc_create.argtypes = [C.POINTER(capi.AvgpuCfg), C.c_int64]
    lib.orc_destroy.restype = None
    lib.orc_run_serial_updates.argtypes = [C.c_void_p, C.c_int, C.POINTER(capi.AvgpuUpdateStats)]
    lib.orc_rec_exhausted.restype = C.c_int64
    _lib = lib
    return lib


class Backend:
    """Uniform wrapper over the oracle (prefix orc_) and the product (avgpu_)."""

    def __init__(self, kind, cfg: capi.AvgpuCfg, instset: files.InstSet, reactions, ncells=0,
                 device=0):
        self.kind = kind
        if kind == "oracle":
            self.lib, self.p = load_oracle(), "orc_"
            self.h = self.lib.orc_create(C.byref(cfg), ncells)
        else:
            self.lib, self.p = capi.load_product(), "avgpu_"
            self.h = self.lib.avgpu_create(C.byref(cfg), device, ncells)
            if not self.h:
                raise RuntimeError(self.lib.avgpu_last_error().decode())
        self.cfg = cfg
        self.ncells = ncells or cfg.world_x * cfg.world_y
        self.instset = instset
        hid = (C.c_uint8 * len(instset.names))(*instset.handlers)
        red = (C.c_int32 * len(instset.names))(*instset.redundancy)
        self._call("load_instset", self.h, len(instset.names), hid, red)
        self.nres = 0
        if getattr(reactions, "resources", None):   # resources first: reactions name them
            self.load_resources(reactions)
        arr = capi.reactions_array(reactions)
        self._call("load_env", self.h, len(reactions), arr)

    def _call(self, name, *args):
        rc = getattr(self.lib, self.p + name)(*args)
        if rc is not None and rc < 0:
            msg = getattr(self.lib, self.p + "last_error")()
            raise RuntimeError(f"{self.p}{name}: {msg.decode() if msg else rc}")
        return rc

    def close(self):
        if self.h:
            getattr(self.lib, self.p + "destroy")(self.h)
            self.h = None

    def set_orgs(self, first, genomes, merits=None, inputs=None, deterministic=True):
        n = len(genomes)
        blob = b"".join(genomes)
        buf = (C.c_uint8 * max(1, len(blob))).from_buffer_copy(blob or b"\0")
        lens = (C.c_int32 * n)(*[len(g) for g in genomes])
        m = (C.c_double * n)(*(merits or [0.0] * n))
        inp = None
        if inputs is not None:
            flat = [v for t in inputs for v in t]
            inp = (C.c_int32 * len(flat))(*flat)
        self._call("set_orgs", self.h, first, n, buf, lens, m, inp, 1 if deterministic else 0)

    def set_orgs_np(self, first, blob, lens, merits=None, deterministic=False):
        """set_orgs for large worlds: genomes packed in `blob` (bytes), lens /
        merits numpy arrays"""
        import numpy as np
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        n = len(lens)
        buf = (C.c_uint8 * max(1, len(blob))).from_buffer_copy(blob or b"\0")
        m = None
        if merits is not None:
            merits = np.ascontiguousarray(merits, dtype=np.float64)
            m = merits.ctypes.data_as(C.POINTER(C.c_double))
        self._call("set_orgs", self.h, first, n, buf, lens.ctypes.data_as(C.POINTER(C.c_int32)), m, None,
                   1 if deterministic else 0)

    def kill(self, cell):
        self._call("kill", self.h, cell)

    def step(self, first, count, budget=None, uniform=0, mode=capi.MODE_FROZEN):
        b = None
        if budget is not None:
            b = (C.c_int32 * count)(*budget)
        self._call("step", self.h, first, count, b, uniform, mode)
        if self.kind != "oracle":
            self.lib.avgpu_sync(self.h)

    def states(self, first, count, cap=capi.MAX_GENOME):
        st = (capi.AvgpuCpuState * count)()
        ops = (C.c_uint8 * (count * cap))()
        fl = (C.c_uint8 * (count * cap))()
        self._call("get_states", self.h, first, count, st, ops, fl, cap)
        return st, bytes(ops), bytes(fl)

    def digests(self, first=0, count=None):
        """per-cell state digests (numpy uint64) of a cell range:
        avgpu_state_digests / orc_state_digests"""
        import numpy as np
        if count is None:
            count = self.ncells - first
        out = np.zeros(count, dtype=np.uint64)
        self._call("state_digests", self.h, first, count, out.ctypes.data_as(C.c_void_p))
        return out

    def set_rng_mode(self, mode, stream=None, offsets=None):
        """avgpu_set_rng_mode / orc_set_rng_mode: stream = numpy float64
        array (RECORDED), offsets = numpy int64 per cell or None"""
        import numpy as np
        sp, n, op = None, 0, None
        if stream is not None:
            self._rec = np.ascontiguousarray(stream, dtype=np.float64)
            sp, n = self._rec.ctypes.data_as(C.c_void_p), len(self._rec)
        if offsets is not None:
            self._off = np.ascontiguousarray(offsets, dtype=np.int64)
            op = self._off.ctypes.data_as(C.c_void_p)
        self._call("set_rng_mode", self.h, mode, sp, n, op)

    def counters(self, cumulative=0):
        """avgpu_counters of the last update, or summed over every update
        (cumulative=1) (product only)"""
        out = (C.c_int64 * capi.NUM_COUNTERS)()
        self._call("counters", self.h, cumulative, out, capi.NUM_COUNTERS)
        return list(out)

    def census(self, first=0, count=None):
        """avgpu_census rows (numpy, capi.CENSUS_DTYPE) of a cell range"""
        if count is None:
            count = self.ncells - first
        return capi.get_census(self.lib, self.p, self.h, first, count)

    def test_genomes(self, genomes, flags_cap=2049):
        n = len(genomes)
        blob = b"".join(genomes)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        lens = (C.c_int32 * n)(*[len(g) for g in genomes])
        res = (capi.AvgpuTestResult * n)()
        flags = C.create_string_buffer(n * flags_cap)
        off = (C.c_uint8 * (n * capi.MAX_GENOME))()
        self._call("test_genomes", self.h, n, buf, lens, res, flags, flags_cap, off)
        out = []
        raw = flags.raw
        offb = bytes(off)
        for i in range(n):
            r = res[i]
            f = raw[i * flags_cap:(i + 1) * flags_cap].split(b"\0", 1)[0].decode()
            child = offb[i * capi.MAX_GENOME:i * capi.MAX_GENOME + r.offspring_len]
            out.append((r, f, child))
        return out

    def load_resources(self, env):
        self.nres = len(env.resources)
        ra, ca = capi.resources_arrays(env.resources, env.cells)
        self._call("load_resources", self.h, len(env.resources), ra, len(env.cells), ca)

    def resources(self, spatial=False):
        """(levels, per-cell grids or None): avgpu_get_resources"""
        nres = self.nres
        n = self.ncells
        lv = (C.c_double * max(1, nres))()
        sp = (C.c_double * max(1, nres * n))() if spatial else None
        self._call("get_resources", self.h, lv, sp)
        grids = [list(sp[r * n:(r + 1) * n]) for r in range(nres)] if spatial else None
        return list(lv[:nres]), grids

    def checkpoint(self, path):
        from avida_amd import checkpoint
        checkpoint.save(self.lib, self.p, self.h, self.ncells, self.nres, path)

    def restore(self, path):
        from avida_amd import checkpoint
        return checkpoint.load(self.lib, self.p, self.h, path)

    def run_update(self):
        st = capi.AvgpuUpdateStats()
        self._call("run_update", self.h, C.byref(st))
        return st

    def run_serial_update(self):
        """one update of the serial world (reference schedule, births at once)"""
        st = capi.AvgpuUpdateStats()
        self._call("run_serial_updates", self.h, 1, C.byref(st))
        return st


def recalculate(backend: Backend, genomes, generations=3):
    """cTestCPU::TestGenome viability recursion (cpu/cTestCPU.cc:233-326) over a batch.

    Returns per genome (result_at_depth0, exec_flags, viable)."""
    first = backend.test_genomes(genomes)
    viable = [False] * len(genomes)
    # chains: genome index -> list of ancestors' genomes for case 3
    pending = []
    for i, (r, f, child) in enumerate(first):
        if not r.divided:
            continue
        if r.copy_true:
            viable[i] = True
        else:
            pending.append((i, [genomes[i]], child))
    depth = 1
    while pending and depth < generations:
        nxt = []
        res = backend.test_genomes([c for (_, _, c) in pending])
        for (i, anc, child), (r, f, grandchild) in zip(pending, res):
            if not r.divided:
                continue
            if r.copy_true:
                viable[i] = True
                continue
            anc2 = anc + [child]
            if any(grandchild == a for a in anc2):
                viable[i] = True
                continue
            nxt.append((i, anc2, grandchild))
        # case 3 at depth>0 checks the offspring of depth d against ancestors < d
        pending = nxt
        depth += 1
    return [(r, f, viable[i]) for i, (r, f, _) in enumerate(first)]


AVGPU_FLAGS_CAP = 2049
