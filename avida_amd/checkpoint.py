"""Checkpoint / resume of a world through the C-ABI.

The reference saves populations as genotype lists (`SavePopulation`,
main/cPopulation.cc:6294-6600) and restarts organisms from their genomes.
Here a checkpoint holds the whole architectural + phenotype state of every
cell (`avgpu_get_states`: registers, heads, stacks, labels, counters, RNG
stream position, tape with copied / executed flags), the update clock and
cumulative counters (`avgpu_get_stats`), and the resource levels and grids
(`avgpu_get_resources`), so a restored world continues bit for bit -- on the
same backend or the other one (product "avgpu_" or CPU oracle "orc_").

File: one `numpy.savez_compressed` archive (no pickles): `states` (raw
avgpu_cpu_state records), `tape` (one byte per site: op | copied << 6 |
executed << 7, `cap` bytes per cell), `stats` (raw avgpu_update_stats),
`levels` / `grids` (resources), `gkeys` (the census genotype keys of the
birth genomes, which the tape no longer holds once an organism copied into
its own sites; avgpu_set_genotype_keys), `serial` / `spec` / `face` /
`soup_perm` / `reaper` (the serial world's own state, avgpu_get_serial_state:
its two streams' positions, speculative credits, connection-list rotations,
BIRTH_METHOD 4's empty_cell_id_array and 5's reaper queue, rear first),
`version` and the byte sizes of the
two raw structures (`state_size`, `stats_size`).  A file from before a
structure grew (round 4 added births_cancelled and seed to the stats) loads
with the missing tail zeroed; a zero seed then leaves the world's configured
RANDOM_SEED in place (avgpu_set_clock).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import capi

VERSION = 4
# round 5 added `age` (+ a pad word) before cur_bonus: an older state record
# gets them inserted as zeros (age 0: as if every organism had just divided)
_AGE_OFF = capi.AvgpuCpuState.age.offset


def _call(lib, prefix, name, *args):
    rc = getattr(lib, prefix + name)(*args)
    if rc is not None and rc < 0:
        msg = getattr(lib, prefix + "last_error")()
        raise RuntimeError(f"{prefix}{name}: {msg.decode() if msg else rc}")
    return rc


def save(lib, prefix, handle, ncells, nres, path):
    """Write the world behind `handle` (ncells cells, nres resources) to `path`."""
    st = (capi.AvgpuCpuState * ncells)()
    _call(lib, prefix, "get_states", handle, 0, ncells, st, None, None, 0)
    cap = max([1] + [st[i].mem_size for i in range(ncells)])
    ops = (C.c_uint8 * (ncells * cap))()
    fl = (C.c_uint8 * (ncells * cap))()
    _call(lib, prefix, "get_states", handle, 0, ncells, st, ops, fl, cap)
    o = np.frombuffer(ops, dtype=np.uint8)
    f = np.frombuffer(fl, dtype=np.uint8)
    tape = (o & 0x3F) | ((f & 0x01) << 6) | (((f >> 2) & 0x01) << 7)
    stats = capi.AvgpuUpdateStats()
    _call(lib, prefix, "get_stats", handle, C.byref(stats))
    levels = np.zeros(max(1, nres))
    grids = np.zeros(max(1, nres * ncells))
    if nres:
        _call(lib, prefix, "get_resources", handle, levels.ctypes.data_as(C.POINTER(C.c_double)),
              grids.ctypes.data_as(C.POINTER(C.c_double)))
    gkeys = capi.get_census(lib, prefix, handle, 0, ncells)["genotype_key"]
    ser = capi.AvgpuSerialState()
    spec = np.zeros(ncells, dtype=np.int32)
    face = np.zeros(ncells, dtype=np.uint8)
    soup = np.zeros(ncells, dtype=np.int32)
    reaper = np.zeros(2 * ncells + 64, dtype=np.int32)
    _call(lib, prefix, "get_serial_state", handle, C.byref(ser), spec.ctypes.data_as(C.c_void_p),
          face.ctypes.data_as(C.c_void_p), soup.ctypes.data_as(C.c_void_p), reaper.ctypes.data_as(C.c_void_p),
          len(reaper))
    np.savez_compressed(path, states=np.frombuffer(st, dtype=np.uint8), tape=tape.astype(np.uint8), gkeys=gkeys,
                        serial=np.frombuffer(ser, dtype=np.uint8), spec=spec, face=face, soup_perm=soup,
                        reaper=reaper[:max(0, ser.reaper_len)],
                        cap=np.int64(cap), stats=np.frombuffer(stats, dtype=np.uint8),
                        levels=levels[:nres], grids=grids[:nres * ncells], ncells=np.int64(ncells),
                        version=np.int64(VERSION), state_size=np.int64(C.sizeof(capi.AvgpuCpuState)),
                        stats_size=np.int64(C.sizeof(capi.AvgpuUpdateStats)))


def _struct(cls, raw, what):
    """a raw structure of an older (shorter) layout, its missing tail zeroed"""
    size = C.sizeof(cls)
    if len(raw) > size:
        raise ValueError(f"checkpoint {what} record is {len(raw)} B, this build's is {size} B (newer file?)")
    return cls.from_buffer_copy(raw + b"\0" * (size - len(raw)))


def load(lib, prefix, handle, path):
    """Restore a checkpoint into a world created with the same configuration,
    instruction set and environment (resources loaded)."""
    z = np.load(path, allow_pickle=False)
    ncells, cap = int(z["ncells"]), int(z["cap"])
    if "version" in z.files and int(z["version"]) > VERSION:
        raise ValueError(f"checkpoint version {int(z['version'])} is newer than this reader ({VERSION})")
    raw = z["states"].tobytes()
    size = C.sizeof(capi.AvgpuCpuState)
    ssz = int(z["state_size"]) if "state_size" in z.files else len(raw) // max(1, ncells)
    if ssz == size - 8 and len(raw) == ssz * ncells:       # before `age` (version <= 2)
        raw = b"".join(raw[k * ssz:k * ssz + _AGE_OFF] + b"\0" * 8 + raw[k * ssz + _AGE_OFF:(k + 1) * ssz]
                       for k in range(ncells))
        ssz = size
    if ssz != size or len(raw) != ssz * ncells:
        raise ValueError(f"checkpoint state records are {ssz} B, this build's are {size} B")
    st = (capi.AvgpuCpuState * ncells).from_buffer_copy(raw)
    tape = z["tape"]
    ops = np.ascontiguousarray(tape & 0x3F)
    fl = np.ascontiguousarray(((tape >> 6) & 0x01) | (((tape >> 7) & 0x01) << 2))
    _call(lib, prefix, "set_states", handle, 0, ncells, st, ops.ctypes.data_as(C.POINTER(C.c_uint8)),
          fl.ctypes.data_as(C.POINTER(C.c_uint8)), cap)
    if "gkeys" in z.files:                     # genotype keys of the birth genomes
        gk = np.ascontiguousarray(z["gkeys"], dtype=np.uint64)
        _call(lib, prefix, "set_genotype_keys", handle, 0, ncells, gk.ctypes.data_as(C.c_void_p))
    if "serial" in z.files:                    # the serial world's own state (version >= 4)
        ser = _struct(capi.AvgpuSerialState, z["serial"].tobytes(), "serial state")
        arrs = [np.ascontiguousarray(z[k], dtype=t) for k, t in
                (("spec", np.int32), ("face", np.uint8), ("soup_perm", np.int32), ("reaper", np.int32))]
        _call(lib, prefix, "set_serial_state", handle, C.byref(ser), *[a.ctypes.data_as(C.c_void_p) for a in arrs])
    stats = _struct(capi.AvgpuUpdateStats, z["stats"].tobytes(), "stats")
    _call(lib, prefix, "set_clock", handle, C.byref(stats))
    levels = np.ascontiguousarray(z["levels"], dtype=np.float64)
    if len(levels):
        grids = np.ascontiguousarray(z["grids"], dtype=np.float64)
        _call(lib, prefix, "set_resources", handle, levels.ctypes.data_as(C.POINTER(C.c_double)),
              grids.ctypes.data_as(C.POINTER(C.c_double)))
    return stats
