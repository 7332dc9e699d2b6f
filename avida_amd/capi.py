"""ctypes mirror of include/avida_gpu.h (structures + the product library loader).

The product library is ``avida_amd/libavida_gpu.so`` (built in-tree by
``__graft_entry__.build()`` / ``avida_amd/build.py``).  There is no fallback:
if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

MAX_REACTIONS = 16
MAX_GENOME = 2048
STACK_SIZE = 10
MAX_LABEL = 10

MODE_WORLD, MODE_TEST, MODE_FROZEN = 0, 1, 2
# enum avgpu_counter
(CNT_INSTS, CNT_DEATHS, CNT_DIVIDES, CNT_BIRTHS, CNT_DROPPED, CNT_SPILLS, CNT_SLICES,
 CNT_LANESTEPS, CNT_C0_SLICES, CNT_C0_SITES, CNT_CLK_STAGE, CNT_CLK_LOOP, CNT_CLK_WB,
 CNT_ITERS, CNT_IT_FAST, CNT_IT_COPY, CNT_IT_SLOW, CNT_WAVES, CNT_HALO_SENT,
 CNT_HALO_LOST, CNT_REC_EXHAUSTED, CNT_OVERSIZE, CNT_SUB_OVERFLOW) = range(23)
RNG_COUNTER, RNG_RECORDED = 0, 1
NUM_COUNTERS = 48

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libavida_gpu.so")


class AvgpuCfg(C.Structure):
    _fields_ = [
        ("world_x", C.c_int32), ("world_y", C.c_int32), ("world_geometry", C.c_int32),
        ("ave_time_slice", C.c_int32), ("slicing_method", C.c_int32),
        ("base_merit_method", C.c_int32), ("base_const_merit", C.c_int32),
        ("default_bonus", C.c_double),
        ("copy_mut_prob", C.c_double), ("copy_ins_prob", C.c_double), ("copy_del_prob", C.c_double),
        ("divide_mut_prob", C.c_double), ("divide_ins_prob", C.c_double),
        ("divide_del_prob", C.c_double),
        ("offspring_size_range", C.c_double), ("min_copied_lines", C.c_double),
        ("min_exe_lines", C.c_double),
        ("require_allocate", C.c_int32), ("death_method", C.c_int32), ("age_limit", C.c_int32),
        ("alloc_method", C.c_int32), ("divide_method", C.c_int32),
        ("max_label_exe_size", C.c_int32), ("birth_method", C.c_int32),
        ("prefer_empty", C.c_int32), ("allow_parent", C.c_int32),
        ("test_cpu_time_mod", C.c_int32), ("min_genome_size", C.c_int32),
        ("max_genome_size", C.c_int32), ("inherit_merit", C.c_int32),
        ("merit_default_bonus", C.c_double), ("required_bonus", C.c_double),
        ("seed", C.c_uint64),
        ("divide_slip_prob", C.c_double), ("divide_uniform_prob", C.c_double),
        ("slip_fill_mode", C.c_int32), ("pad_cfg", C.c_int32),
        ("div_mut_prob", C.c_double), ("parent_mut_prob", C.c_double),
        ("divide_poisson_slip_mean", C.c_double), ("divide_poisson_mut_mean", C.c_double),
        ("divide_poisson_ins_mean", C.c_double), ("divide_poisson_del_mean", C.c_double),
        ("div_ins_prob", C.c_double), ("div_del_prob", C.c_double),
        ("div_uniform_prob", C.c_double), ("div_slip_prob", C.c_double),
        ("divide_trans_prob", C.c_double), ("divide_poisson_trans_mean", C.c_double),
        ("div_trans_prob", C.c_double),
    ]


class AvgpuReaction(C.Structure):
    _fields_ = [
        ("task", C.c_int32), ("type", C.c_int32), ("value", C.c_double),
        ("max_number", C.c_double), ("min_count", C.c_int32), ("max_count", C.c_int32),
        ("has_requisite", C.c_int32), ("resource", C.c_int32),
        ("min_number", C.c_double), ("max_fraction", C.c_double),
        ("depletable", C.c_int32), ("pad", C.c_int32),
    ]


class AvgpuResource(C.Structure):
    _fields_ = [
        ("geometry", C.c_int32), ("pad", C.c_int32),
        ("initial", C.c_double), ("inflow", C.c_double), ("outflow", C.c_double),
        ("inflow_x1", C.c_int32), ("inflow_x2", C.c_int32), ("inflow_y1", C.c_int32),
        ("inflow_y2", C.c_int32), ("outflow_x1", C.c_int32), ("outflow_x2", C.c_int32),
        ("outflow_y1", C.c_int32), ("outflow_y2", C.c_int32),
        ("xdiffuse", C.c_double), ("ydiffuse", C.c_double), ("xgravity", C.c_double),
        ("ygravity", C.c_double),
    ]


class AvgpuCellResource(C.Structure):
    _fields_ = [("resource", C.c_int32), ("cell", C.c_int32), ("initial", C.c_double),
                ("inflow", C.c_double), ("outflow", C.c_double)]


class AvgpuCpuState(C.Structure):
    _fields_ = [
        ("reg", C.c_int32 * 3), ("head", C.c_int32 * 4),
        ("stack", (C.c_int32 * STACK_SIZE) * 2), ("stack_ptr", C.c_int32 * 2),
        ("cur_stack", C.c_int32), ("read_label_len", C.c_int32),
        ("read_label", C.c_int8 * MAX_LABEL), ("pad0", C.c_int16),
        ("mal_active", C.c_int32), ("mem_size", C.c_int32),
        ("cpu_cycles_used", C.c_int32), ("time_used", C.c_int32),
        ("gestation_start", C.c_int32), ("gestation_time", C.c_int32),
        ("num_divides", C.c_int32), ("generation", C.c_int32), ("alive", C.c_int32),
        ("genome_length", C.c_int32), ("copied_size", C.c_int32),
        ("child_copied_size", C.c_int32), ("executed_size", C.c_int32),
        ("max_executed", C.c_int32), ("birth_length", C.c_int32), ("input_ptr", C.c_int32),
        ("input_buf", C.c_int32 * 3), ("input_total", C.c_int32),
        ("output_buf", C.c_int32), ("output_total", C.c_int32), ("inputs", C.c_int32 * 3),
        ("cur_task_count", C.c_int32 * MAX_REACTIONS),
        ("last_task_count", C.c_int32 * MAX_REACTIONS),
        ("cur_reaction_count", C.c_int32 * MAX_REACTIONS),
        ("rng_counter", C.c_uint32), ("rng_key_lo", C.c_uint32), ("rng_key_hi", C.c_uint32),
        ("errors", C.c_int32), ("pad1", C.c_int32),
        ("cur_bonus", C.c_double), ("merit", C.c_double), ("fitness", C.c_double),
        ("credit", C.c_double),
    ]


class AvgpuTestResult(C.Structure):
    _fields_ = [
        ("divided", C.c_int32), ("copy_true", C.c_int32), ("copied_size", C.c_int32),
        ("executed_size", C.c_int32), ("gestation_time", C.c_int32),
        ("offspring_len", C.c_int32), ("genome_length", C.c_int32), ("time_used", C.c_int32),
        ("merit", C.c_double), ("fitness", C.c_double),
        ("task_count", C.c_int32 * MAX_REACTIONS),
    ]


class AvgpuUpdateStats(C.Structure):
    _fields_ = [
        ("update", C.c_int64), ("num_organisms", C.c_int64), ("insts_executed", C.c_int64),
        ("births", C.c_int64), ("births_dropped", C.c_int64), ("deaths", C.c_int64),
        ("divides", C.c_int64), ("task_orgs", C.c_int64 * MAX_REACTIONS),
        ("sum_merit", C.c_double), ("sum_fitness", C.c_double), ("sum_gestation", C.c_double),
        ("sum_genome_length", C.c_double), ("max_fitness", C.c_double),
        ("ave_generation", C.c_double), ("sum_mem_size", C.c_double),
        ("cum_insts_executed", C.c_int64), ("cum_births", C.c_int64), ("slices", C.c_int64),
        ("lane_steps", C.c_int64),
    ]


# avgpu_census (include/avida_gpu.h), read straight into numpy
CENSUS_DTYPE = np.dtype([("genotype_key", "<u8"), ("merit", "<f8"), ("fitness", "<f8"),
                         ("genome_length", "<i4"), ("gestation_time", "<i4"), ("copied_size", "<i4"),
                         ("executed_size", "<i4"), ("generation", "<i4"), ("num_divides", "<i4")])
assert CENSUS_DTYPE.itemsize == 48


def get_census(lib, prefix, handle, first, count):
    """Census rows (CENSUS_DTYPE) of cells first .. first+count-1 through
    {prefix}get_census (avgpu_ = the product, orc_ = the oracle)."""
    out = np.zeros(count, dtype=CENSUS_DTYPE)
    rc = getattr(lib, prefix + "get_census")(handle, first, count, out.ctypes.data_as(C.c_void_p))
    if rc < 0:
        raise RuntimeError(f"{prefix}get_census: {getattr(lib, prefix + 'last_error')().decode()}")
    return out


# C-ABI symbols declared in include/avida_gpu.h (checked by tests/test_capi.py)
EXPORTED = [
    "avgpu_last_error", "avgpu_cfg_defaults", "avgpu_create", "avgpu_destroy", "avgpu_sync",
    "avgpu_load_instset", "avgpu_load_env", "avgpu_load_resources", "avgpu_get_resources",
    "avgpu_set_resources", "avgpu_set_org", "avgpu_set_orgs", "avgpu_kill", "avgpu_set_states", "avgpu_set_clock",
    "avgpu_step", "avgpu_run_update", "avgpu_run_updates", "avgpu_update_totals",
    "avgpu_update_run", "avgpu_set_stream", "avgpu_get_states", "avgpu_get_census", "avgpu_set_genotype_keys",
    "avgpu_test_genomes", "avgpu_get_stats", "avgpu_stats_vector", "avgpu_set_global_totals",
    "avgpu_set_tile", "avgpu_tile_buffer_bytes", "avgpu_set_tile_buffers", "avgpu_tile_partials",
    "avgpu_tile_begin", "avgpu_tile_place", "avgpu_tile_finish", "avgpu_tile_res_bytes",
    "avgpu_set_tile_res_buffers", "avgpu_tile_res_cons", "avgpu_tile_res_settle",
    "avgpu_last_step_insts", "avgpu_last_kernel_ms", "avgpu_kernel_times", "avgpu_counters",
    "avgpu_state_digests", "avgpu_set_rng_mode", "avgpu_run_serial_updates", "avgpu_set_timing",
]


# avida.cfg knobs that change the semantics of this path when non-zero and
# that it does not implement (main/cAvidaConfig.h:309-361, 372):
# lateral-transfer mutations (one-shot, Poisson and per-site), parent
# insertions / deletions, point, inject and meta mutations, copy uniform /
# slip, death on divide.  cfg_from_avida refuses a config that sets any of
# them rather than run it with different semantics.  (COPY_INS_PROB /
# COPY_DEL_PROB travel in avgpu_cfg; avgpu_create refuses them.)
UNSUPPORTED_NONZERO = [
    "COPY_UNIFORM_PROB", "COPY_SLIP_PROB",
    "POINT_MUT_PROB", "POINT_INS_PROB", "POINT_DEL_PROB", "INST_POINT_MUT_PROB",
    "DIV_LGT_PROB",
    "DIVIDE_LGT_PROB",
    "DIVIDE_POISSON_LGT_MEAN",
    "INJECT_MUT_PROB", "INJECT_INS_PROB", "INJECT_DEL_PROB",
    "PARENT_INS_PROB", "PARENT_DEL_PROB",
    "META_COPY_MUT", "META_STD_DEV", "DEATH_PROB",
]
# Knobs accepted without effect, with the reason.  SPECULATIVE only decides
# whether the reference's serial ProcessStep pre-executes up to 32 more
# instructions of the picked organism (main/cPopulation.cc:5740-5788); the
# batched update has no serial interleaving to speculate on.
IGNORED = {"SPECULATIVE": "batched update: no serial schedule to speculate on"}


def unsupported_knobs(cfg):
    """Names of the UNSUPPORTED_NONZERO keys a files.AvidaConfig sets non-zero."""
    bad = []
    for k in UNSUPPORTED_NONZERO:
        v = cfg.get(k, 0)
        try:
            nz = float(v) != 0.0
        except (TypeError, ValueError):
            nz = True
        if nz:
            bad.append(k)
    return bad


def cfg_from_avida(cfg, seed=None) -> AvgpuCfg:
    """Fill an AvgpuCfg from a files.AvidaConfig; raise ValueError for a knob
    of UNSUPPORTED_NONZERO set non-zero."""
    bad = unsupported_knobs(cfg)
    if bad:
        raise ValueError("avida.cfg sets mutation / death knobs this path does not implement: "
                         + ", ".join(bad))
    g = cfg.get
    c = AvgpuCfg()
    c.world_x, c.world_y = g("WORLD_X"), g("WORLD_Y")
    c.world_geometry = g("WORLD_GEOMETRY")
    c.ave_time_slice = g("AVE_TIME_SLICE")
    c.slicing_method = g("SLICING_METHOD")
    c.base_merit_method = g("BASE_MERIT_METHOD")
    c.base_const_merit = g("BASE_CONST_MERIT")
    c.default_bonus = g("DEFAULT_BONUS")
    c.copy_mut_prob = g("COPY_MUT_PROB")
    c.copy_ins_prob = g("COPY_INS_PROB")
    c.copy_del_prob = g("COPY_DEL_PROB")
    c.divide_mut_prob = g("DIVIDE_MUT_PROB")
    c.divide_ins_prob = g("DIVIDE_INS_PROB")
    c.divide_del_prob = g("DIVIDE_DEL_PROB")
    c.offspring_size_range = g("OFFSPRING_SIZE_RANGE")
    c.min_copied_lines = g("MIN_COPIED_LINES")
    c.min_exe_lines = g("MIN_EXE_LINES")
    c.require_allocate = g("REQUIRE_ALLOCATE")
    c.death_method = g("DEATH_METHOD")
    c.age_limit = g("AGE_LIMIT")
    c.alloc_method = g("ALLOC_METHOD")
    c.divide_method = g("DIVIDE_METHOD")
    c.max_label_exe_size = g("MAX_LABEL_EXE_SIZE")
    c.birth_method = g("BIRTH_METHOD")
    c.prefer_empty = g("PREFER_EMPTY")
    c.allow_parent = g("ALLOW_PARENT")
    c.test_cpu_time_mod = g("TEST_CPU_TIME_MOD")
    c.min_genome_size = g("MIN_GENOME_SIZE")
    c.max_genome_size = g("MAX_GENOME_SIZE")
    c.inherit_merit = g("INHERIT_MERIT")
    c.merit_default_bonus = g("MERIT_DEFAULT_BONUS")
    c.required_bonus = g("REQUIRED_BONUS")
    s = g("RANDOM_SEED") if seed is None else seed
    c.seed = int(s) & 0xFFFFFFFFFFFFFFFF if int(s) >= 0 else 0x1234ABCD
    c.divide_slip_prob = float(g("DIVIDE_SLIP_PROB", 0.0))
    c.divide_uniform_prob = float(g("DIVIDE_UNIFORM_PROB", 0.0))
    c.slip_fill_mode = int(float(g("SLIP_FILL_MODE", 0)))
    c.div_mut_prob = float(g("DIV_MUT_PROB", 0.0))
    c.parent_mut_prob = float(g("PARENT_MUT_PROB", 0.0))
    c.divide_poisson_slip_mean = float(g("DIVIDE_POISSON_SLIP_MEAN", 0.0))
    c.divide_poisson_mut_mean = float(g("DIVIDE_POISSON_MUT_MEAN", 0.0))
    c.divide_poisson_ins_mean = float(g("DIVIDE_POISSON_INS_MEAN", 0.0))
    c.divide_poisson_del_mean = float(g("DIVIDE_POISSON_DEL_MEAN", 0.0))
    c.div_ins_prob = float(g("DIV_INS_PROB", 0.0))
    c.div_del_prob = float(g("DIV_DEL_PROB", 0.0))
    c.div_uniform_prob = float(g("DIV_UNIFORM_PROB", 0.0))
    c.div_slip_prob = float(g("DIV_SLIP_PROB", 0.0))
    c.divide_trans_prob = float(g("DIVIDE_TRANS_PROB", 0.0))
    c.divide_poisson_trans_mean = float(g("DIVIDE_POISSON_TRANS_MEAN", 0.0))
    c.div_trans_prob = float(g("DIV_TRANS_PROB", 0.0))
    if (c.divide_trans_prob or c.divide_poisson_trans_mean or c.div_trans_prob) and \
            int(float(g("TRANS_FILL_MODE", 0))) != 0:
        raise ValueError("TRANS_FILL_MODE 1 (scrambled) is not on this path")
    return c


def reactions_array(reactions):
    arr = (AvgpuReaction * max(1, len(reactions)))()
    for i, r in enumerate(reactions):
        arr[i].task, arr[i].type, arr[i].value = r.task, r.proc_type, r.value
        arr[i].max_number, arr[i].min_count = r.max_number, r.min_count
        arr[i].max_count, arr[i].has_requisite = r.max_count, r.has_requisite
        arr[i].resource = getattr(r, "resource", 0)   # 1 + index, 0 = infinite
        arr[i].min_number = getattr(r, "min_number", 0.0)
        arr[i].max_fraction = getattr(r, "max_fraction", 1.0)
        arr[i].depletable = getattr(r, "depletable", 1)
    return arr


def resources_arrays(resources, cells):
    """files.Resource / files.CellResource lists -> ctypes arrays"""
    ra = (AvgpuResource * max(1, len(resources)))()
    for i, r in enumerate(resources):
        for f, _ in AvgpuResource._fields_:
            if f != "pad":
                setattr(ra[i], f, getattr(r, f))
    ca = (AvgpuCellResource * max(1, len(cells)))()
    for i, c in enumerate(cells):
        ca[i].resource, ca[i].cell = c.resource, c.cell
        ca[i].initial, ca[i].inflow, ca[i].outflow = c.initial, c.inflow, c.outflow
    return ra, ca


def bind_common(lib, prefix):
    """Declare argtypes for the functions shared by the product and the oracle."""
    p = prefix
    V, I64, I32 = C.c_void_p, C.c_int64, C.c_int32
    sig = {
        "load_instset": (C.c_int, [V, C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]),
        "load_env": (C.c_int, [V, C.c_int, C.POINTER(AvgpuReaction)]),
        "set_orgs": (C.c_int, [V, I64, I64, C.POINTER(C.c_uint8), C.POINTER(C.c_int32),
                               C.POINTER(C.c_double), C.POINTER(C.c_int32), C.c_int]),
        "kill": (C.c_int, [V, I64]),
        "step": (C.c_int, [V, I64, I64, C.POINTER(C.c_int32), I32, C.c_int]),
        "get_states": (C.c_int, [V, I64, I64, C.POINTER(AvgpuCpuState), C.POINTER(C.c_uint8),
                                 C.POINTER(C.c_uint8), C.c_int]),
        "test_genomes": (C.c_int, [V, C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_int32),
                                   C.POINTER(AvgpuTestResult), C.c_char_p, C.c_int,
                                   C.POINTER(C.c_uint8)]),
        "run_update": (C.c_int, [V, C.POINTER(AvgpuUpdateStats)]),
        "run_serial_updates": (C.c_int, [V, C.c_int, C.POINTER(AvgpuUpdateStats)]),
        "run_updates": (C.c_int, [V, C.c_int, C.POINTER(AvgpuUpdateStats)]),
        "last_step_insts": (C.c_int, [V, C.POINTER(C.c_int64)]),
        "set_global_totals": (C.c_int, [V, C.c_double, I64]),
        "destroy": (C.c_int, [V]),
        # strip tiles (include/avida_gpu.h "strip tiles")
        "set_tile": (C.c_int, [V, I64, I64]),
        "tile_buffer_bytes": (C.c_int, [V, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
        "set_tile_buffers": (C.c_int, [V] + [V] * 8),
        "tile_partials": (C.c_int, [V, V]),
        "tile_begin": (C.c_int, [V, V, C.c_int]),
        "tile_place": (C.c_int, [V, C.c_int, C.c_int]),
        "tile_finish": (C.c_int, [V, C.POINTER(AvgpuUpdateStats)]),
        "tile_res_bytes": (C.c_int, [V, C.POINTER(I64)]),
        "set_tile_res_buffers": (C.c_int, [V] * 5),
        "tile_res_cons": (C.c_int, [V, V]),
        "tile_res_settle": (C.c_int, [V, V]),
        "get_stats": (C.c_int, [V, C.POINTER(AvgpuUpdateStats)]),
        "load_resources": (C.c_int, [V, C.c_int, C.POINTER(AvgpuResource), C.c_int,
                                     C.POINTER(AvgpuCellResource)]),
        "get_resources": (C.c_int, [V, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "set_resources": (C.c_int, [V, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "set_states": (C.c_int, [V, I64, I64, C.POINTER(AvgpuCpuState), C.POINTER(C.c_uint8),
                                 C.POINTER(C.c_uint8), C.c_int]),
        "set_clock": (C.c_int, [V, C.POINTER(AvgpuUpdateStats)]),
        "get_census": (C.c_int, [V, I64, I64, V]),
        "set_genotype_keys": (C.c_int, [V, I64, I64, V]),
        "state_digests": (C.c_int, [V, I64, I64, V]),
        "set_rng_mode": (C.c_int, [V, C.c_int, V, I64, V]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, p + name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    getattr(lib, p + "last_error").restype = C.c_char_p
    return lib


_lib = None


def load_product(path=None):
    """Load the in-tree HIP library; raise if it is missing (no fallback).
    `path` selects a diagnostic build (tools/phase_clocks.py); it is not cached."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = path or os.environ.get("AVGPU_DIAG_LIB") or LIB_PATH   # diagnostic builds (tools/)
    if not os.path.exists(p):
        raise RuntimeError(f"{p} missing: run __graft_entry__.build() first")
    lib = C.CDLL(p)
    bind_common(lib, "avgpu_")
    lib.avgpu_create.restype = C.c_void_p
    lib.avgpu_create.argtypes = [C.POINTER(AvgpuCfg), C.c_int, C.c_int64]
    lib.avgpu_cfg_defaults.argtypes = [C.POINTER(AvgpuCfg)]
    lib.avgpu_sync.argtypes = [C.c_void_p]
    lib.avgpu_get_stats.argtypes = [C.c_void_p, C.POINTER(AvgpuUpdateStats)]
    lib.avgpu_stats_vector.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    lib.avgpu_last_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double),
                                         C.POINTER(C.c_int64)]
    lib.avgpu_kernel_times.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
    lib.avgpu_set_timing.argtypes = [C.c_void_p, C.c_int]
    lib.avgpu_counters.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int64), C.c_int]
    lib.avgpu_update_totals.argtypes = [C.c_void_p, C.c_void_p]
    lib.avgpu_update_run.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(AvgpuUpdateStats)]
    lib.avgpu_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    if path is None:
        _lib = lib
    return lib


def check(lib, rc, prefix="avgpu_"):
    if rc < 0:
        msg = getattr(lib, prefix + "last_error")()
        raise RuntimeError(f"{prefix}call failed ({rc}): {msg.decode() if msg else ''}")
    return rc
