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
 CNT_HALO_LOST, CNT_REC_EXHAUSTED, CNT_OVERSIZE, CNT_SUB_OVERFLOW, CNT_MEM_CAP,
 CNT_OVERWRITTEN, CNT_CANCELLED, CNT_BAD_RECORD, CNT_WASTED, CNT_STEPS) = range(29)
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
        ("slip_fill_mode", C.c_int32), ("sub_updates", C.c_int32),
        ("div_mut_prob", C.c_double), ("parent_mut_prob", C.c_double),
        ("divide_poisson_slip_mean", C.c_double), ("divide_poisson_mut_mean", C.c_double),
        ("divide_poisson_ins_mean", C.c_double), ("divide_poisson_del_mean", C.c_double),
        ("div_ins_prob", C.c_double), ("div_del_prob", C.c_double),
        ("div_uniform_prob", C.c_double), ("div_slip_prob", C.c_double),
        ("divide_trans_prob", C.c_double), ("divide_poisson_trans_mean", C.c_double),
        ("div_trans_prob", C.c_double),
        ("copy_uniform_prob", C.c_double), ("copy_slip_prob", C.c_double),
        ("slip_copy_mode", C.c_int32), ("trans_fill_mode", C.c_int32),
        ("parent_ins_prob", C.c_double), ("parent_del_prob", C.c_double),
        # knobs the library refuses away from their defaults (avgpu_create)
        ("point_mut_prob", C.c_double), ("point_ins_prob", C.c_double),
        ("point_del_prob", C.c_double), ("inst_point_mut_prob", C.c_double),
        ("div_lgt_prob", C.c_double), ("divide_lgt_prob", C.c_double),
        ("divide_poisson_lgt_mean", C.c_double),
        ("inject_mut_prob", C.c_double), ("inject_ins_prob", C.c_double),
        ("inject_del_prob", C.c_double),
        ("meta_copy_mut", C.c_double), ("meta_std_dev", C.c_double), ("death_prob", C.c_double),
        ("age_deviation", C.c_int32), ("divide_failure_resets", C.c_int32),
        ("special_mut_line", C.c_int32), ("population_cap", C.c_int32),
        ("generation_inc_method", C.c_int32), ("reset_inputs_on_divide", C.c_int32),
        ("epigenetic_method", C.c_int32), ("min_cycles", C.c_int32),
        ("required_task", C.c_int32), ("immunity_task", C.c_int32),
        ("required_reaction", C.c_int32), ("immunity_reaction", C.c_int32),
        ("require_single_reaction", C.c_int32), ("max_unique_task_count", C.c_int32),
        ("require_exact_copy", C.c_int32), ("fitness_method", C.c_int32),
        ("juv_period", C.c_int32), ("no_mut_insts_len", C.c_int32),
        ("test_fitness_measures", C.c_int32), ("pad_cfg2", C.c_int32),
        ("no_mut_insts", C.c_char * 64),
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
        ("errors", C.c_int32), ("head_start", C.c_uint32), ("age", C.c_int32), ("pad1", C.c_int32),
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


class AvgpuSerialState(C.Structure):
    """avgpu_serial_state (include/avida_gpu.h): the serial world's stream
    positions, reaper queue length and whether it has started"""
    _fields_ = [("sched_pos", C.c_int64), ("ctx_pos", C.c_int64), ("reaper_len", C.c_int64),
                ("started", C.c_int32), ("pad_", C.c_int32)]


class AvgpuUpdateStats(C.Structure):
    _fields_ = [
        ("update", C.c_int64), ("num_organisms", C.c_int64), ("insts_executed", C.c_int64),
        ("births", C.c_int64), ("births_dropped", C.c_int64), ("deaths", C.c_int64),
        ("divides", C.c_int64), ("task_orgs", C.c_int64 * MAX_REACTIONS),
        ("sum_merit", C.c_double), ("sum_fitness", C.c_double), ("sum_gestation", C.c_double),
        ("sum_genome_length", C.c_double), ("max_fitness", C.c_double),
        ("ave_generation", C.c_double), ("sum_mem_size", C.c_double),
        ("cum_insts_executed", C.c_int64), ("cum_births", C.c_int64), ("slices", C.c_int64),
        ("lane_steps", C.c_int64), ("births_overwritten", C.c_int64), ("births_cancelled", C.c_int64),
        ("seed", C.c_uint64), ("sched_pred", C.c_int64), ("sched_pred_n", C.c_int64), ("sub_steps", C.c_int64),
        ("sched_carry", C.c_int64), ("insts_wasted", C.c_int64), ("sched_pred_cnt", C.c_int64),
        ("sched_pred_bins", C.c_int64 * 4),
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
    "avgpu_last_error", "avgpu_cfg_defaults", "avgpu_check_cfg", "avgpu_create", "avgpu_destroy", "avgpu_sync",
    "avgpu_load_instset", "avgpu_load_env", "avgpu_load_resources", "avgpu_get_resources",
    "avgpu_set_resources", "avgpu_set_org", "avgpu_set_orgs", "avgpu_kill", "avgpu_set_states", "avgpu_set_clock",
    "avgpu_step", "avgpu_run_update", "avgpu_run_updates", "avgpu_update_totals",
    "avgpu_update_run", "avgpu_set_stream", "avgpu_get_states", "avgpu_get_census", "avgpu_set_genotype_keys",
    "avgpu_test_genomes", "avgpu_get_stats", "avgpu_stats_vector", "avgpu_set_global_totals",
    "avgpu_set_tile", "avgpu_tile_buffer_bytes", "avgpu_set_tile_buffers", "avgpu_tile_partials",
    "avgpu_tile_begin", "avgpu_tile_steps", "avgpu_tile_begin_step", "avgpu_tile_place", "avgpu_tile_finish", "avgpu_tile_res_bytes",
    "avgpu_set_tile_res_buffers", "avgpu_tile_res_cons", "avgpu_tile_res_settle",
    "avgpu_last_step_insts", "avgpu_last_kernel_ms", "avgpu_kernel_times", "avgpu_counters",
    "avgpu_state_digests", "avgpu_set_rng_mode", "avgpu_run_serial_updates", "avgpu_set_serial_streams",
    "avgpu_get_serial_state", "avgpu_set_serial_state", "avgpu_set_timing",
]


# avida.cfg knobs outside avgpu_cfg's implemented set travel in its refused
# block (include/avida_gpu.h): the library itself refuses any of them set away
# from the reference default (avgpu_create -> AVGPU_EUNSUPPORTED), so the
# Python driver and a C++ caller are refused alike.  (cfg key, field, default,
# kind) -- main/cAvidaConfig.h:309-420, :525-537, :546-559.
REFUSED_KNOBS = [
    ("POINT_MUT_PROB", "point_mut_prob", 0.0, float), ("POINT_INS_PROB", "point_ins_prob", 0.0, float),
    ("POINT_DEL_PROB", "point_del_prob", 0.0, float),
    ("INST_POINT_MUT_PROB", "inst_point_mut_prob", 0.0, float),
    ("DIV_LGT_PROB", "div_lgt_prob", 0.0, float), ("DIVIDE_LGT_PROB", "divide_lgt_prob", 0.0, float),
    ("DIVIDE_POISSON_LGT_MEAN", "divide_poisson_lgt_mean", 0.0, float),
    ("INJECT_MUT_PROB", "inject_mut_prob", 0.0, float), ("INJECT_INS_PROB", "inject_ins_prob", 0.0, float),
    ("INJECT_DEL_PROB", "inject_del_prob", 0.0, float),
    ("META_COPY_MUT", "meta_copy_mut", 0.0, float), ("META_STD_DEV", "meta_std_dev", 0.0, float),
    ("DEATH_PROB", "death_prob", 0.0, float),
    ("AGE_DEVIATION", "age_deviation", 0, int), ("DIVIDE_FAILURE_RESETS", "divide_failure_resets", 0, int),
    ("SPECIAL_MUT_LINE", "special_mut_line", -1, int), ("POPULATION_CAP", "population_cap", 0, int),
    ("GENERATION_INC_METHOD", "generation_inc_method", 1, int),
    ("RESET_INPUTS_ON_DIVIDE", "reset_inputs_on_divide", 0, int),
    ("EPIGENETIC_METHOD", "epigenetic_method", 0, int), ("MIN_CYCLES", "min_cycles", 0, int),
    ("REQUIRED_TASK", "required_task", -1, int), ("IMMUNITY_TASK", "immunity_task", -1, int),
    ("REQUIRED_REACTION", "required_reaction", -1, int), ("IMMUNITY_REACTION", "immunity_reaction", -1, int),
    ("REQUIRE_SINGLE_REACTION", "require_single_reaction", 0, int),
    ("MAX_UNIQUE_TASK_COUNT", "max_unique_task_count", -1, int),
    ("REQUIRE_EXACT_COPY", "require_exact_copy", 0, int), ("FITNESS_METHOD", "fitness_method", 0, int),
    ("JUV_PERIOD", "juv_period", 0, int),
]
# Divide_TestFitnessMeasures1 (cpu/cHardwareBase.cc:978-1085) runs a test CPU
# on every offspring when any of these is set: avgpu_cfg.test_fitness_measures
TEST_FITNESS_KNOBS = ["REVERT_FATAL", "REVERT_DETRIMENTAL", "REVERT_NEUTRAL", "REVERT_BENEFICIAL",
                      "REVERT_TASKLOSS", "REVERT_EQUALS", "STERILIZE_FATAL", "STERILIZE_DETRIMENTAL",
                      "STERILIZE_NEUTRAL", "STERILIZE_BENEFICIAL", "STERILIZE_TASKLOSS",
                      "STERILIZE_UNSTABLE", "FAIL_IMPLICIT"]
# Knobs accepted without effect, with the reason.  SPECULATIVE only decides
# whether the reference's serial ProcessStep pre-executes up to 32 more
# instructions of the picked organism (main/cPopulation.cc:5740-5788); the
# batched update has no serial interleaving to speculate on.
IGNORED = {"SPECULATIVE": "batched update: no serial schedule to speculate on"}


def _num(v, kind, default):
    try:
        return kind(float(v))
    except (TypeError, ValueError):
        return default


def cfg_from_avida(cfg, seed=None) -> AvgpuCfg:
    """Fill an AvgpuCfg from a files.AvidaConfig.  Every knob of the path is a
    field; the library refuses (avgpu_create) what it does not implement."""
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
    f = lambda k, d=0.0: _num(g(k, d), float, d)   # noqa: E731
    i = lambda k, d=0: _num(g(k, d), int, d)       # noqa: E731
    c.divide_slip_prob = f("DIVIDE_SLIP_PROB")
    c.divide_uniform_prob = f("DIVIDE_UNIFORM_PROB")
    c.slip_fill_mode = i("SLIP_FILL_MODE")
    c.div_mut_prob = f("DIV_MUT_PROB")
    c.parent_mut_prob = f("PARENT_MUT_PROB")
    c.divide_poisson_slip_mean = f("DIVIDE_POISSON_SLIP_MEAN")
    c.divide_poisson_mut_mean = f("DIVIDE_POISSON_MUT_MEAN")
    c.divide_poisson_ins_mean = f("DIVIDE_POISSON_INS_MEAN")
    c.divide_poisson_del_mean = f("DIVIDE_POISSON_DEL_MEAN")
    c.div_ins_prob = f("DIV_INS_PROB")
    c.div_del_prob = f("DIV_DEL_PROB")
    c.div_uniform_prob = f("DIV_UNIFORM_PROB")
    c.div_slip_prob = f("DIV_SLIP_PROB")
    c.divide_trans_prob = f("DIVIDE_TRANS_PROB")
    c.divide_poisson_trans_mean = f("DIVIDE_POISSON_TRANS_MEAN")
    c.div_trans_prob = f("DIV_TRANS_PROB")
    c.copy_uniform_prob = f("COPY_UNIFORM_PROB")
    c.copy_slip_prob = f("COPY_SLIP_PROB")
    c.slip_copy_mode = i("SLIP_COPY_MODE")
    c.trans_fill_mode = i("TRANS_FILL_MODE")
    c.parent_ins_prob = f("PARENT_INS_PROB")
    c.parent_del_prob = f("PARENT_DEL_PROB")
    for key, field, default, kind in REFUSED_KNOBS:
        setattr(c, field, _num(g(key, default), kind, default))
    nmi = g("NO_MUT_INSTS", "")
    nmi = str(nmi).strip() if nmi not in (None, 0) else ""
    c.no_mut_insts_len = len(nmi)
    c.no_mut_insts = nmi.encode()[:63]
    c.test_fitness_measures = int(any(_num(g(k, 0), float, 1.0) != 0.0 for k in TEST_FITNESS_KNOBS))
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
        "tile_steps": (C.c_int, [V, V, C.c_int, C.POINTER(C.c_int)]),
        "tile_begin_step": (C.c_int, [V, V, C.c_int, C.c_int, C.c_int]),
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
        "set_serial_streams": (C.c_int, [V, V, I64, V, I64]),
        "get_serial_state": (C.c_int, [V, C.POINTER(AvgpuSerialState), V, V, V, V, I64]),
        "set_serial_state": (C.c_int, [V, C.POINTER(AvgpuSerialState), V, V, V, V]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, p + name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    getattr(lib, p + "last_error").restype = C.c_char_p
    return lib


_lib = None


def lib_build_hash(path=None):
    """the first 16 hex digits of the SHA-256 of the library file: which
    build a measurement (profiles/pmc_k_interpret320.json) belongs to"""
    import hashlib
    with open(path or LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


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
    lib.avgpu_check_cfg.argtypes = [C.POINTER(AvgpuCfg)]
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
