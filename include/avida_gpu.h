/*
 * avida_gpu.h -- C-ABI of the MI355X batched Avida virtual-CPU interpreter.
 *
 * This is the drop-in boundary for ONE hot path of fortunalab/avida: the
 * per-organism heads-CPU execution loop (cHardwareCPU::SingleProcess) as driven
 * by cPopulation::ProcessStep, with its fused neighbours (Divide_DoMutations,
 * the IO-driven logic-9 task check, merit-weighted time slicing, birth
 * placement).  Every entry point below names the reference interface it
 * replaces (paths relative to avida-core/source/ of the reference).
 *
 * Conventions
 *   - plain C types only; no torch / HIP types cross this boundary;
 *   - every call returns >= 0 on success, a negative AVGPU_E* code on error,
 *     with a human readable message from avgpu_last_error();
 *   - one host thread per handle; work is enqueued on the handle's own HIP
 *     stream and avgpu_sync() waits for it;
 *   - genomes cross the boundary as instruction-set op codes (the byte values
 *     cInstSet assigns, i.e. INST line order), exactly like
 *     Avida::InstructionSequence (include/public/avida/core/InstructionSequence.h).
 */
#ifndef AVIDA_GPU_H
#define AVIDA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (include/public/avida/core/Definitions.h:28-29,
 *      cpu/nHardware.h:32-34, cpu/cCodeLabel.cc MAX_LENGTH) ---------------- */
#define AVGPU_MIN_GENOME 8
#define AVGPU_MAX_GENOME 2048
#define AVGPU_STACK_SIZE 10
#define AVGPU_MAX_LABEL 10
#define AVGPU_MAX_INST 64
#define AVGPU_MAX_REACTIONS 16
#define AVGPU_NUM_LOGIC_TASKS 9

/* error codes */
#define AVGPU_OK 0
#define AVGPU_EINVAL -1
#define AVGPU_EHIP -2
#define AVGPU_ESTATE -3
#define AVGPU_ENOMEM -4
#define AVGPU_EUNSUPPORTED -5

/* Canonical instruction handlers of the heads_default / classic instruction
 * sets: the 26 tInstLibEntry rows of cpu/cHardwareCPU.cc:85-375 that
 * support/config/instset-heads.cfg and tests/.../instset-classic.cfg name.
 * The value is the handler id, NOT the op code: the op code is the INST line
 * position, mapped to a handler by avgpu_load_instset (cInstSet::Load,
 * cpu/cInstSet.cc:152-312). */
enum avgpu_handler {
  AVGPU_H_NOP_A = 0,   /* cpu/cHardwareBase.cc:1179 (Inst_Nop), nop-mod 0 */
  AVGPU_H_NOP_B = 1,   /* nop-mod 1 */
  AVGPU_H_NOP_C = 2,   /* nop-mod 2 */
  AVGPU_H_IF_N_EQU = 3,  /* cpu/cHardwareCPU.cc:2190 */
  AVGPU_H_IF_LESS = 4,   /* :2235 */
  AVGPU_H_POP = 5,       /* :2698 */
  AVGPU_H_PUSH = 6,      /* :2705 */
  AVGPU_H_SWAP_STK = 7,  /* :2739 */
  AVGPU_H_SWAP = 8,      /* :2742 */
  AVGPU_H_SHIFT_R = 9,   /* :2806 */
  AVGPU_H_SHIFT_L = 10,  /* :2813 */
  AVGPU_H_INC = 11,      /* :2864 */
  AVGPU_H_DEC = 12,      /* :2871 */
  AVGPU_H_ADD = 13,      /* :2959 */
  AVGPU_H_SUB = 14,      /* :2968 */
  AVGPU_H_NAND = 15,     /* :3018 */
  AVGPU_H_IO = 16,       /* :4188 (Inst_TaskIO) */
  AVGPU_H_H_ALLOC = 17,  /* :3294 (Inst_MaxAlloc) */
  AVGPU_H_H_DIVIDE = 18, /* :6961 -> :6942 */
  AVGPU_H_H_COPY = 19,   /* :7130 */
  AVGPU_H_H_SEARCH = 20, /* :7245 */
  AVGPU_H_MOV_HEAD = 21, /* :6809 */
  AVGPU_H_JMP_HEAD = 22, /* :6859 */
  AVGPU_H_GET_HEAD = 23, /* :6907 */
  AVGPU_H_IF_LABEL = 24, /* :6914 */
  AVGPU_H_SET_FLOW = 25, /* :7270 */
  AVGPU_H_COUNT = 26
};

/* logic-9 task ids (main/cTaskLib.cc:511-575) */
enum avgpu_task {
  AVGPU_T_NOT = 0, AVGPU_T_NAND, AVGPU_T_AND, AVGPU_T_ORN, AVGPU_T_OR,
  AVGPU_T_ANDN, AVGPU_T_NOR, AVGPU_T_XOR, AVGPU_T_EQU
};

/* reaction process types (main/nReaction.h PROCTYPE_*) */
enum avgpu_proctype { AVGPU_PROC_ADD = 0, AVGPU_PROC_MULT = 1, AVGPU_PROC_POW = 2 };

/* Execution modes of avgpu_step.
 *  WORLD : cPopulation::ActivateOffspring semantics -- a successful divide runs
 *          Divide_DoMutations on the child and appends it to the birth queue;
 *  TEST  : cTestCPU::ProcessGestation semantics (cpu/cTestCPU.cc:144-188) --
 *          the organism stops at its first successful divide
 *          (cTestCPUInterface::Divide -> cPhenotype::TestDivideReset);
 *  FROZEN: divide resets the parent (DIVIDE_METHOD 1) and the offspring is
 *          discarded; used for frozen-population trace parity (BASELINE cfg 2). */
enum avgpu_mode { AVGPU_MODE_WORLD = 0, AVGPU_MODE_TEST = 1, AVGPU_MODE_FROZEN = 2 };

/* Scheduler (SLICING_METHOD, main/cPopulation.cc:7326-7358) */
enum avgpu_slicing { AVGPU_SLICE_CONSTANT = 0, AVGPU_SLICE_PROBABILISTIC = 1,
                     AVGPU_SLICE_INTEGRATED = 2 };

/* The avida.cfg subset on this path (main/cAvidaConfig.h; defaults are the
 * values of support/config/avida.cfg).  avgpu_cfg_defaults() fills them. */
typedef struct avgpu_cfg {
  int32_t world_x, world_y;        /* WORLD_X, WORLD_Y */
  int32_t world_geometry;          /* 1 grid, 2 torus */
  int32_t ave_time_slice;          /* AVE_TIME_SLICE */
  int32_t slicing_method;          /* SLICING_METHOD */
  int32_t base_merit_method;       /* BASE_MERIT_METHOD (0..5) */
  int32_t base_const_merit;        /* BASE_CONST_MERIT */
  double default_bonus;            /* DEFAULT_BONUS */
  double copy_mut_prob;            /* COPY_MUT_PROB */
  double copy_ins_prob;            /* COPY_INS_PROB */
  double copy_del_prob;            /* COPY_DEL_PROB */
  double divide_mut_prob;          /* DIVIDE_MUT_PROB */
  double divide_ins_prob;          /* DIVIDE_INS_PROB */
  double divide_del_prob;          /* DIVIDE_DEL_PROB */
  double offspring_size_range;     /* OFFSPRING_SIZE_RANGE */
  double min_copied_lines;         /* MIN_COPIED_LINES */
  double min_exe_lines;            /* MIN_EXE_LINES */
  int32_t require_allocate;        /* REQUIRE_ALLOCATE */
  int32_t death_method;            /* DEATH_METHOD 0/1/2 */
  int32_t age_limit;               /* AGE_LIMIT */
  int32_t alloc_method;            /* ALLOC_METHOD (0 default inst, 2 random) */
  int32_t divide_method;           /* DIVIDE_METHOD (1 split) */
  int32_t max_label_exe_size;      /* MAX_LABEL_EXE_SIZE */
  int32_t birth_method;            /* BIRTH_METHOD 0 random neighbour, 1 oldest, 2 age / merit, 3 empty only, 4 whole-world soup */
  int32_t prefer_empty;            /* PREFER_EMPTY */
  int32_t allow_parent;            /* ALLOW_PARENT */
  int32_t test_cpu_time_mod;       /* TEST_CPU_TIME_MOD */
  int32_t min_genome_size;         /* MIN_GENOME_SIZE (0 = none) */
  int32_t max_genome_size;         /* MAX_GENOME_SIZE (0 = none) */
  int32_t inherit_merit;           /* INHERIT_MERIT */
  double merit_default_bonus;      /* MERIT_DEFAULT_BONUS */
  double required_bonus;           /* REQUIRED_BONUS */
  uint64_t seed;                   /* RANDOM_SEED (counter-RNG key) */
  double divide_slip_prob;         /* DIVIDE_SLIP_PROB (TestDivideSlip always draws) */
  double divide_uniform_prob;      /* DIVIDE_UNIFORM_PROB */
  int32_t slip_fill_mode;          /* SLIP_FILL_MODE: 0 duplication, 2 random, 3 scrambled,
                                      4 nop-C (1, nop-X, refused) */
  int32_t sub_updates;             /* batch steps per update, no reference knob (DESIGN.md
                                      4.2): an update's AVE_TIME_SLICE x N picks are made in
                                      K batch steps, the scheduler weights re-read before
                                      each.  0 (default): adaptive -- from the previous
                                      step's predictor (avgpu_update_stats.sched_pred*),
                                      more steps the more the total weight is expected to
                                      move within the update or the more organisms are
                                      expected to divide in it (a cohort in lock step),
                                      else 1; K > 0: always K.  K > 1 needs SLICING_METHOD 1 and
                                      the world's own totals (strips take it through
                                      avgpu_tile_steps / avgpu_tile_begin_step) */
  double div_mut_prob;             /* DIV_MUT_PROB: per-site substitutions on divide,
                                      Binomial(offspring size, p) of them drawn after the
                                      uniform mutation (cpu/cHardwareBase.cc:447-460) */
  double parent_mut_prob;          /* PARENT_MUT_PROB: per-site substitutions in the parent's
                                      memory (cut to the divide point) after the offspring's
                                      mutations (cpu/cHardwareBase.cc:508-520) */
  /* DIVIDE_POISSON_{SLIP,MUT,INS,DEL}_MEAN: Poisson-distributed numbers of
   * slips / substitutions / insertions / deletions on divide, each right after
   * its one-shot test (cpu/cHardwareBase.cc:318-320, :383-391, :404-413,
   * :426-435; main/cMutationRates.h:137-144); means above 700 are refused */
  double divide_poisson_slip_mean, divide_poisson_mut_mean;
  double divide_poisson_ins_mean, divide_poisson_del_mean;
  /* DIV_INS_PROB, DIV_DEL_PROB, DIV_UNIFORM_PROB, DIV_SLIP_PROB: per-site
   * insertions / deletions / uniform mutations / slips on divide
   * (cpu/cHardwareBase.cc:323-327, :463-503) */
  double div_ins_prob, div_del_prob, div_uniform_prob, div_slip_prob;
  /* translocations (TRANS_FILL_MODE below): DIVIDE_TRANS_PROB,
   * DIVIDE_POISSON_TRANS_MEAN, DIV_TRANS_PROB (cpu/cHardwareBase.cc:331-343,
   * doTransMutation :700-760) */
  double divide_trans_prob, divide_poisson_trans_mean, div_trans_prob;
  /* copy mutations of Inst_HeadCopy beyond COPY_MUT/INS/DEL_PROB
   * (cpu/cHardwareCPU.cc:7153-7161): COPY_UNIFORM_PROB (doUniformCopyMutation,
   * cpu/cHardwareBase.cc:597-612) and COPY_SLIP_PROB under SLIP_COPY_MODE 0
   * (the read head jumps to GetInt(memory size)); SLIP_COPY_MODE 1 (a slip of
   * the whole memory at the write head) is refused */
  double copy_uniform_prob, copy_slip_prob;
  int32_t slip_copy_mode;          /* SLIP_COPY_MODE */
  int32_t trans_fill_mode;         /* TRANS_FILL_MODE: 0 duplication, 1 scrambled */
  /* PARENT_INS_PROB / PARENT_DEL_PROB: per-site insertions / deletions in the
   * parent's memory after its substitutions (cpu/cHardwareBase.cc:523-565) */
  double parent_ins_prob, parent_del_prob;
  /* ---- knobs this path does not implement: avgpu_create refuses any of them
   * set away from the reference default (main/cAvidaConfig.h) with
   * AVGPU_EUNSUPPORTED, so a C++ caller cannot run them with other semantics.
   * avgpu_cfg_defaults writes the defaults. ---- */
  double point_mut_prob, point_ins_prob, point_del_prob;   /* POINT_{MUT,INS,DEL}_PROB (0) */
  double inst_point_mut_prob;                              /* INST_POINT_MUT_PROB (0) */
  double div_lgt_prob, divide_lgt_prob, divide_poisson_lgt_mean;  /* lateral transfer (0) */
  double inject_mut_prob, inject_ins_prob, inject_del_prob;       /* INJECT_*_PROB (0) */
  double meta_copy_mut, meta_std_dev;                      /* META_COPY_MUT, META_STD_DEV (0) */
  double death_prob;                                       /* DEATH_PROB (0) */
  int32_t age_deviation;           /* AGE_DEVIATION (0) */
  int32_t divide_failure_resets;   /* DIVIDE_FAILURE_RESETS (0) */
  int32_t special_mut_line;        /* SPECIAL_MUT_LINE (-1) */
  int32_t population_cap;          /* POPULATION_CAP (0) */
  int32_t generation_inc_method;   /* GENERATION_INC_METHOD (1) */
  int32_t reset_inputs_on_divide;  /* RESET_INPUTS_ON_DIVIDE (0) */
  int32_t epigenetic_method;       /* EPIGENETIC_METHOD (0) */
  int32_t min_cycles;              /* MIN_CYCLES (0) */
  int32_t required_task, immunity_task;           /* REQUIRED_TASK, IMMUNITY_TASK (-1) */
  int32_t required_reaction, immunity_reaction;   /* REQUIRED_REACTION, IMMUNITY_REACTION (-1) */
  int32_t require_single_reaction; /* REQUIRE_SINGLE_REACTION (0) */
  int32_t max_unique_task_count;   /* MAX_UNIQUE_TASK_COUNT (-1) */
  int32_t require_exact_copy;      /* REQUIRE_EXACT_COPY (0) */
  int32_t fitness_method;          /* FITNESS_METHOD (0) */
  int32_t juv_period;              /* JUV_PERIOD (0) */
  int32_t no_mut_insts_len;        /* strlen(no_mut_insts) (0) */
  /* non-zero when any REVERT_* / STERILIZE_* probability or STERILIZE_UNSTABLE
   * is set (Divide_TestFitnessMeasures1, cpu/cHardwareBase.cc:978-1085) */
  int32_t test_fitness_measures;
  int32_t pad_cfg2;
  /* NO_MUT_INSTS (""): symbols of the instructions that copy mutations leave
   * alone (cHardwareCPU::checkNoMutList, cpu/cHardwareCPU.cc:797-810): an
   * h-copy whose read instruction's symbol (Instruction::GetSymbol's first
   * character, core/InstructionSequence.cc:69-106) is listed draws its copy
   * mutation but keeps the instruction (:7144), and a uniform copy mutation
   * leaves a listed write-head instruction (cpu/cHardwareBase.cc:597-612).
   * NUL-terminated, at most 63 symbols; no_mut_insts_len its length. */
  char no_mut_insts[64];
} avgpu_cfg;

/* One REACTION line of environment.cfg (main/cEnvironment.cc:1185-1211,
 * process settings :147-300) on a logic-9 task. */
typedef struct avgpu_reaction {
  int32_t task;          /* avgpu_task */
  int32_t type;          /* avgpu_proctype */
  double value;          /* process:value */
  double max_number;     /* process:max (consumed amount, default 1.0) */
  int32_t min_count;     /* requisite:min_count (default 0) */
  int32_t max_count;     /* requisite:max_count (INT32_MAX when absent) */
  int32_t has_requisite; /* 0: TestRequisites returns !on_divide */
  int32_t resource;      /* process:resource: 1 + index into avgpu_load_resources, 0 = infinite */
  double min_number;     /* process:min (default 0.0) */
  double max_fraction;   /* process:frac (default 1.0, capped at 1) */
  int32_t depletable;    /* process:depletable (default 1) */
  int32_t pad;
} avgpu_reaction;

/* One RESOURCE of environment.cfg (main/cEnvironment.cc:474-661; dynamics
 * main/cResourceCount.cc:207-358, :757-880, main/cSpatialResCount.cc:101-437). */
enum avgpu_res_geometry { AVGPU_RES_GLOBAL = 0, AVGPU_RES_GRID = 1, AVGPU_RES_TORUS = 2 };
#define AVGPU_RES_NONE (-99)   /* cResource::NONE */
#define AVGPU_MAX_RESOURCES 16
typedef struct avgpu_resource {
  int32_t geometry;      /* avgpu_res_geometry */
  int32_t pad;
  double initial, inflow, outflow;
  int32_t inflow_x1, inflow_x2, inflow_y1, inflow_y2;     /* AVGPU_RES_NONE when absent */
  int32_t outflow_x1, outflow_x2, outflow_y1, outflow_y2;
  double xdiffuse, ydiffuse, xgravity, ygravity;
} avgpu_resource;
/* One cell of a CELL line (main/cEnvironment.cc:663-755). */
typedef struct avgpu_cell_resource {
  int32_t resource, cell;
  double initial, inflow, outflow;
} avgpu_cell_resource;

/* Architectural + phenotype state of one organism: the tuple a
 * cHardwareStatusPrinter trace shows (cpu/cHardwareCPU.cc:1111-1169) plus the
 * phenotype counters the hot path mutates.  Used by avgpu_get_states /
 * avgpu_set_states and by the oracle, so traces compare field by field. */
typedef struct avgpu_cpu_state {
  int32_t reg[3];                      /* AX BX CX */
  int32_t head[4];                     /* IP READ WRITE FLOW */
  int32_t stack[2][AVGPU_STACK_SIZE];  /* [0] thread stack, [1] global stack (raw ring) */
  int32_t stack_ptr[2];
  int32_t cur_stack;
  int32_t read_label_len;
  int8_t read_label[AVGPU_MAX_LABEL];  /* nop-mods */
  int16_t pad0;
  int32_t mal_active;
  int32_t mem_size;
  int32_t cpu_cycles_used;             /* cPhenotype::cpu_cycles_used */
  int32_t time_used;                   /* cPhenotype::time_used */
  int32_t gestation_start;
  int32_t gestation_time;
  int32_t num_divides;
  int32_t generation;
  int32_t alive;
  int32_t genome_length;               /* cPhenotype::genome_length */
  int32_t copied_size;                 /* cPhenotype::copied_size (inherited) */
  int32_t child_copied_size;           /* cPhenotype::child_copied_size (SetLinesCopied) */
  int32_t executed_size;               /* cPhenotype::executed_size (SetLinesExecuted) */
  int32_t max_executed;                /* cOrganism::m_max_executed */
  int32_t birth_length;                /* length of the genome the organism was born with */
  int32_t input_ptr;                   /* cOrganism::m_input_pointer */
  int32_t input_buf[3];                /* tBuffer<int> ring, most recent first */
  int32_t input_total;
  int32_t output_buf;                  /* capacity-1 output buffer */
  int32_t output_total;
  int32_t inputs[3];                   /* cell inputs (cPopulationCell::m_inputs) */
  int32_t cur_task_count[AVGPU_MAX_REACTIONS];
  int32_t last_task_count[AVGPU_MAX_REACTIONS];
  int32_t cur_reaction_count[AVGPU_MAX_REACTIONS];
  uint32_t rng_counter;                /* draws consumed from this organism's stream */
  uint32_t rng_key_lo, rng_key_hi;
  int32_t errors;                      /* cPhenotype::cur_num_errors (faults) */
  uint32_t head_start;                 /* 2^16 - birth time of an offspring not yet allotted (its first
                                          allotment weights its merit by 1 + head_start / 2^16); 0 otherwise */
  int32_t age;                         /* cPhenotype::age: updates since birth or the last divide, as the
                                          reference's UpdateOrganismStats leaves it at the end of the last
                                          update (main/cPopulation.cc:6021, main/cPhenotype.cc:950) --
                                          BIRTH_METHOD 1 (PositionAge) and 2 (PositionMerit) compare it */
  int32_t pad1;
  double cur_bonus;
  double merit;
  double fitness;
  double credit;                       /* INTEGRATED slicing carry (cScheduler restated) */
} avgpu_cpu_state;

/* Result of one test-CPU gestation (cpu/cTestCPU.cc:144-326 +
 * main/cPlasticPhenotype.cc) */
typedef struct avgpu_test_result {
  int32_t divided;        /* 1 if a divide happened within TEST_CPU_TIME_MOD*len */
  int32_t copy_true;      /* offspring == genome */
  int32_t copied_size;
  int32_t executed_size;
  int32_t gestation_time;
  int32_t offspring_len;
  int32_t genome_length;
  int32_t time_used;
  double merit;
  double fitness;
  int32_t task_count[AVGPU_MAX_REACTIONS];  /* last_task_count after divide */
} avgpu_test_result;

/* Per-update statistics (the reduction inputs of cStats / count.dat:
 * main/cStats.cc:1081-1100). */
typedef struct avgpu_update_stats {
  int64_t update;
  int64_t num_organisms;
  int64_t insts_executed;      /* organism-instructions this update */
  int64_t births;              /* offspring placed this update */
  int64_t births_dropped;      /* never placed: birth-queue overflow, oversize, halo arena full */
  int64_t deaths;              /* old-age deaths this update */
  int64_t divides;             /* successful divides this update */
  int64_t task_orgs[AVGPU_MAX_REACTIONS]; /* organisms whose last gestation did task t */
  double sum_merit;
  double sum_fitness;
  double sum_gestation;
  double sum_genome_length;
  double max_fitness;
  double ave_generation;
  double sum_mem_size;         /* sum of memory-tape sizes after the update */
  int64_t cum_insts_executed;  /* since avgpu_create */
  int64_t cum_births;
  int64_t slices;              /* organism time slices interpreted this update */
  int64_t lane_steps;          /* 64 x longest lane per wave (SIMD lane-issue slots used) */
  int64_t births_overwritten;  /* placed, then killed by a later birth into the same cell this update */
  int64_t births_cancelled;    /* never placed: an earlier birth into the parent's cell killed the parent
                                  before this divide (every successful divide is births +
                                  births_overwritten + births_cancelled + births_dropped) */
  uint64_t seed;               /* the world's RANDOM_SEED, the key of the scheduler's draws: a checkpoint
                                  carries it and avgpu_set_clock restores it with the clock */
  int64_t sched_pred;          /* the adaptive sub-step predictor of the update's last batch step
                                  (2^-20 mean weights) and the living organisms it is relative to:
                                  the next update's step count follows from them (cfg.sub_updates
                                  0); avgpu_set_clock restores them */
  int64_t sched_pred_n;
  int64_t sub_steps;           /* batch steps this update ran */
  int64_t sched_carry;         /* picks the newborns ran beyond what the organisms they replaced had
                                  left, still to come out of the next allotment;
                                  avgpu_set_clock restores it */
  int64_t insts_wasted;        /* instructions the replaced organisms ran after their newborns' birth
                                  times (counted in insts_executed) */
  int64_t sched_pred_cnt;      /* organisms the predictor expects to divide within the densest
                                  quarter of the next update */
  int64_t sched_pred_bins[4];  /* ... in each quarter (avgpu_set_clock restores them) */
} avgpu_update_stats;

typedef struct avgpu_world avgpu_world;   /* opaque handle */

/* ---- lifecycle ---------------------------------------------------------- */
const char* avgpu_last_error(void);
void avgpu_cfg_defaults(avgpu_cfg* cfg);
/* cWorld::setup + cPopulation::SetupCellGrid (main/cWorld.cc:95-200,
 * main/cPopulation.cc:323-404): allocates SoA state for num_cells organisms
 * (world_x*world_y when num_cells <= 0) on HIP device `device`. */
avgpu_world* avgpu_create(const avgpu_cfg* cfg, int device, int64_t num_cells);
/* The configuration check avgpu_create runs first (no device needed): 0 when
 * every knob is on this path, AVGPU_EUNSUPPORTED naming the first knob that is
 * not (the refused block of avgpu_cfg, values outside the implemented ranges)
 * -- cAvidaConfig's knobs, main/cAvidaConfig.h:283-559. */
int avgpu_check_cfg(const avgpu_cfg* cfg);
int avgpu_destroy(avgpu_world* w);
int avgpu_sync(avgpu_world* w);

/* cInstSet::Load (cpu/cInstSet.cc:152-312): op code i runs handler
 * handler_id[i] and is drawn by GetRandomInst with weight redundancy[i]
 * (cpu/cInstSet.cc:83-88). The handler mapping must be injective. */
int avgpu_load_instset(avgpu_world* w, int n, const uint8_t* handler_id,
                       const int32_t* redundancy);
/* cEnvironment::Load REACTION lines (main/cEnvironment.cc:1185-1211). */
int avgpu_load_env(avgpu_world* w, int nreact, const avgpu_reaction* reactions);
/* RESOURCE / CELL lines: cPopulation's resource setup (main/cPopulation.cc:
 * 407-480 -> cResourceCount::Setup).  Call before avgpu_load_env when its
 * reactions name resources.  Update semantics (DESIGN.md "Resources"): at the
 * start of every update the spatial resources take one step of inflow /
 * outflow / diffusion (cSpatialResCount::Source, Sink, CellInflow,
 * CellOutflow, FlowAll, StateAll) and the global ones one update of decay +
 * inflow (DoNonSpatialUpdates over 1/UPDATE_STEP steps).  The first update
 * after this call is the reference's update 0: no spatial step, and 9999
 * global steps (its update_time sums to just under 1.0).  Organisms consume
 * from their own cell immediately and from global resources at the level the
 * update started with (the update's consumption is subtracted at its end). */
int avgpu_load_resources(avgpu_world* w, int nres, const avgpu_resource* res, int ncell,
                         const avgpu_cell_resource* cells);
/* checkpoint / resume: overwrite the levels (global[nres]; spatial[nres][cells]
 * rows of spatial resources) as read by avgpu_get_resources; the next update
 * then steps them like any later update (no update-0 rule) */
int avgpu_set_resources(avgpu_world* w, const double* levels, const double* spatial);
/* current levels: global[nres] (spatial resources: sum over cells, like
 * cStats::PrintResourceData main/cStats.cc:1551-1579); spatial (optional)
 * [nres][cells], zero rows for global resources */
int avgpu_get_resources(avgpu_world* w, double* levels, double* spatial);

/* ---- population --------------------------------------------------------- */
/* cPopulation::Inject / ActivateOrganism (main/cPopulation.cc:1320-1340) +
 * cPhenotype::SetupInject (main/cPhenotype.cc:599-640): put `genome` in
 * `cell`. inputs==NULL draws cell inputs from the cell's RNG stream
 * (cEnvironment::SetupInputs random, main/cEnvironment.cc:1252-1296);
 * deterministic_inputs!=0 uses the test-CPU constants instead. */
int avgpu_set_org(avgpu_world* w, int64_t cell, const uint8_t* genome, int len,
                  double merit, const int32_t* inputs);
/* bulk form: genomes packed back to back, lens[i] each. */
int avgpu_set_orgs(avgpu_world* w, int64_t first_cell, int64_t count,
                   const uint8_t* genomes, const int32_t* lens, const double* merits,
                   const int32_t* inputs /* count*3 or NULL */, int deterministic_inputs);
/* cPopulation::KillOrganism (main/cPopulation.cc:2219-2290) */
int avgpu_kill(avgpu_world* w, int64_t cell);

/* ---- the hot path ------------------------------------------------------- */
/* Batched cHardwareCPU::SingleProcess (cpu/cHardwareCPU.cc:908-1058): every
 * live organism in [first_cell, first_cell+count) executes budget[i]
 * instructions (budget==NULL: budget_uniform each) in the given avgpu_mode.
 * Asynchronous on the handle's stream. */
int avgpu_step(avgpu_world* w, int64_t first_cell, int64_t count,
               const int32_t* budget, int32_t budget_uniform, int mode);
/* One whole update of Avida2Driver::Run (targets/avida/Avida2Driver.cc:91-163):
 * merit-weighted allotment of AVE_TIME_SLICE*N instructions (cScheduler),
 * interpretation, birth placement (cPopulation::PositionOffspring,
 * main/cPopulation.cc:5185-5414), statistics. out may be NULL: no host sync,
 * and the update's statistics reduction is skipped until avgpu_get_stats /
 * avgpu_stats_vector asks for it (cumulative counters stay exact either way). */
int avgpu_run_update(avgpu_world* w, avgpu_update_stats* out);
int avgpu_run_updates(avgpu_world* w, int n_updates, avgpu_update_stats* last);
/* The serial world: n_updates updates under the reference's own schedule
 * (Avida2Driver::Run with cPopulation::ScheduleOrganism's merit-weighted pick
 * of one organism per step, main/cPopulation.cc:5698-5788, a cWeightedIndex
 * sum tree, tools/cWeightedIndex.cc:49-115; ProcessStepSpeculative's
 * run-ahead of up to 32 instructions, stopping before IO / h-divide,
 * :5740-5788; every offspring placed at once inside its h-divide,
 * ActivateOffspring / PositionOffspring :621-952, :5185-5414, on the
 * reference's rotated connection lists, tools/cTopology.h:40-55,
 * main/cPopulationCell.cc:122-141).  The picks draw from the scheduler's
 * stream, everything else from the world's context stream
 * (avgpu_set_serial_streams).  One wave steps the world, so this mode is for
 * reference-semantics runs of small worlds (statistical parity, replay), not
 * throughput.  Not with per-organism RECORDED streams (AVGPU_EUNSUPPORTED) or
 * strip tiles.  Statistics as
 * avgpu_run_update: insts_executed counts the update's picks of living
 * organisms, as cStats does. */
int avgpu_run_serial_updates(avgpu_world* w, int n_updates, avgpu_update_stats* last);
/* The serial world's two random streams, as the reference has them: the
 * scheduler's own generator (Apto::Scheduler::Probabilistic over an AvidaRNG
 * seeded from the world's, main/cPopulation.cc:7341-7346), drawn once per pick
 * (x = u * total merit), and the world's context stream (ctx.GetRandom()),
 * drawn by every organism instruction, PositionOffspring and the newborns'
 * SetupInputs in execution order.  sched / ctx: recorded doubles (k-th draw =
 * element k), or NULL for the counter stream keyed by the seed.  Both
 * positions restart at 0.  Draws past the end of an array return 0 and count
 * in AVGPU_CNT_REC_EXHAUSTED. */
int avgpu_set_serial_streams(avgpu_world* w, const double* sched, int64_t n_sched, const double* ctx,
                             int64_t n_ctx);
/* The serial world's own state beyond the organisms' (checkpoint / resume):
 * the two streams' positions (draws taken; recorded streams index their
 * arrays), every cell's speculative credit and m_spec_die
 * (ProcessStepSpeculative, main/cPopulation.cc:5740-5788; spec[c] = credit |
 * die << 16) and connection-list rotation (cPopulationCell::Rotate, face[c]),
 * and the persistent placement queues: soup_perm (n cells) -- BIRTH_METHOD 4's
 * empty_cell_id_array, whose swaps persist across placements (:338-340,
 * :5650-5668), the identity before its first use; reaper -- BIRTH_METHOD 5's
 * reaper_queue (Setup's cells, then every activated cell pushed at the front,
 * :343-347, :1358-1361), rear (eldest, the next PopRear) first, reaper_len -1
 * before it exists (it is built at the first serial update from the living
 * cells).  started = 0: no serial update has run (everything at its start).
 * get: any array may be NULL (reaper needs reaper_cap >= reaper_len, at most
 * 2n + 64).  set: after avgpu_set_states; started = 0 leaves the world alone;
 * NULL arrays keep theirs; reaper_len < 0 builds the queue again at the next
 * serial update.  Injection (avgpu_set_orgs / avgpu_set_org) into a serial
 * BIRTH_METHOD 5 world whose queue exists takes an occupied cell's entry out
 * (the first from the front, :6964-6968) and pushes the cell at the front, as
 * the reference's InjectGenome + ActivateOrganism do. */
typedef struct avgpu_serial_state {
  int64_t sched_pos;   /* draws taken from the scheduler's stream */
  int64_t ctx_pos;     /* draws taken from the context stream */
  int64_t reaper_len;  /* BIRTH_METHOD 5's queue length; -1: not built */
  int32_t started;     /* 1: the world has run a serial update (or had its state set) */
  int32_t pad_;
} avgpu_serial_state;
int avgpu_get_serial_state(avgpu_world* w, avgpu_serial_state* st, int32_t* spec, uint8_t* face,
                           int32_t* soup_perm, int32_t* reaper, int64_t reaper_cap);
int avgpu_set_serial_state(avgpu_world* w, const avgpu_serial_state* st, const int32_t* spec, const uint8_t* face,
                           const int32_t* soup_perm, const int32_t* reaper);
/* The same update split around an external all-reduce (multi-GPU tiles,
 * cMultiProcessWorld::CalculateUpdateSize main/cMultiProcessWorld.cc:375-405):
 * avgpu_update_totals writes the tile's {sum of scheduler weights, organisms}
 * into the 2-double device buffer dev_totals; after the caller sums it over
 * ranks (RCCL all-reduce, stream-ordered), avgpu_update_run allots
 * AVE_TIME_SLICE * N_global instructions in proportion to weight / global
 * weight.  The scheduler weight is the merit, times 1 + head start / 2^16 for
 * a newborn's first allotment, not the plain merit: a host that
 * hands in sum(merit) gives the world a different share of the picks. */
int avgpu_update_totals(avgpu_world* w, double* dev_totals);
int avgpu_update_run(avgpu_world* w, const double* dev_totals, avgpu_update_stats* out);
/* Run the handle's work on an external HIP stream (e.g. the framework's
 * current stream, so that collectives order against it).  NULL is the HIP
 * null stream (what PyTorch's default stream reports as 0); a new handle
 * starts on a private non-blocking stream of its own. */
int avgpu_set_stream(avgpu_world* w, void* hip_stream);

/* ---- systematics census ----
 * One row per cell for the host-side genotype classification that replaces
 * Systematics::GenotypeArbiter::ClassifyNewUnit (systematics/GenotypeArbiter.cc:
 * 280-380): the reference files every newborn under the genotype whose
 * InstructionSequence equals its birth genome (bucketed by hashGenome,
 * :470-480).  Here the device keys each birth genome once, when the
 * organism is activated (or set / restored), and the host groups cells by
 * key.  genotype_key is the 64-bit "genome key" of the birth genome over
 * canonical instruction codes (DESIGN.md section 10 gives the function;
 * oracle/oracle.cc and avida_amd/systematics.py restate it); 0 = empty cell.
 * The other fields are the phenotype values cStats / the Genotype data
 * providers average (systematics/Genotype.cc:493-540). */
typedef struct avgpu_census {
  uint64_t genotype_key;
  double merit;
  double fitness;
  int32_t genome_length;
  int32_t gestation_time;
  int32_t copied_size;
  int32_t executed_size;
  int32_t generation;
  int32_t num_divides;
} avgpu_census;

/* ---- random streams ------------------------------
 * Apto::RNG::AvidaRNG (main/cWorld.h:72) is absent, so every draw of the path
 * is a uniform u in [0,1) with the reference's interface on top (P(p) = u < p,
 * GetUInt(n) = floor(u n)), consumed in the reference's call order per
 * organism: copy mutation per h-copy (cpu/cHardwareCPU.cc:7144-7161), random
 * fill of ALLOC_METHOD 2, the divide-mutation sequence of Divide_DoMutations
 * (cpu/cHardwareBase.cc:296-569: TestDivideSlip, -Mut, -Ins, -Del always
 * draw; -Uniform only when non-zero).
 *   AVGPU_RNG_COUNTER (default): u from the organism's counter stream
 *     (key, counter; offspring keys derived from the parent's);
 *   AVGPU_RNG_RECORDED: organism c's k-th draw is stream[offsets[c] + k]
 *     (offsets NULL: every cell starts at 0), the reference's recorded
 *     ctx.GetRandom() doubles -- bit-exact traces with mutations on.  The call
 *     sets every cell's stream position (rng_counter) to 0; organisms set or
 *     born afterwards use counter streams; draws past the end of the array
 *     return 0 and count in AVGPU_CNT_REC_EXHAUSTED.
 * The allotment draw of SLICING_METHOD 1 is a stateless hash of the
 * organism's key and the update (the reference's scheduler has its own
 * generator, main/cPopulation.cc:7341-7346), in both modes. */
enum avgpu_rng_mode { AVGPU_RNG_COUNTER = 0, AVGPU_RNG_RECORDED = 1 };
int avgpu_set_rng_mode(avgpu_world* w, int mode, const double* stream, int64_t n,
                       const int64_t* offsets);

/* ---- inspection (cHardwareBase inspection API, cpu/cHardwareBase.h:145-200) */
int avgpu_get_states(avgpu_world* w, int64_t first_cell, int64_t count,
                     avgpu_cpu_state* states, uint8_t* mem_ops, uint8_t* mem_flags,
                     int mem_cap);
/* Census rows of cells first .. first+count-1 into host memory (48 B per
 * cell): the data PrintDominantData / PrintCountData's genotype columns and
 * the dominant genotype's averages are computed from on the host. */
int avgpu_get_census(avgpu_world* w, int64_t first_cell, int64_t count, avgpu_census* out);
/* Verification (no reference equivalent): one 64-bit digest per cell of
 * cells first .. first+count-1 into host memory -- a chained mix over the 32-bit
 * words of the cell's state record, as avgpu_get_states returns it, and its
 * memory tape in canonical bytes (handler id | copied << 6 | executed << 7).
 * oracle/oracle.cc computes the same digest, so worlds of any size (configs[2]
 * and [3]) compare cell for cell without copying 2 KiB tapes to the host. */
int avgpu_state_digests(avgpu_world* w, int64_t first_cell, int64_t count, uint64_t* out);
/* checkpoint / resume: genotype keys of cells first .. first+count-1 (as
 * avgpu_get_census reported them).  avgpu_set_states keys an organism from
 * its tape prefix, which differs from the birth genome once an organism has
 * copied into its own sites; a checkpoint carries the keys and sets them
 * after avgpu_set_states (avida_amd/checkpoint.py). */
int avgpu_set_genotype_keys(avgpu_world* w, int64_t first_cell, int64_t count, const uint64_t* keys);
/* checkpoint / resume: the inverse of avgpu_get_states -- cells first ..
 * first+count-1 take states[i] and their tapes from mem_ops / mem_flags
 * (instruction-set op codes; flags bit0 copied, bit2 executed), mem_cap bytes
 * per cell.  A world restored from avgpu_get_states + avgpu_get_stats +
 * avgpu_get_resources continues bit for bit (avida_amd/checkpoint.py). */
int avgpu_set_states(avgpu_world* w, int64_t first, int64_t count, const avgpu_cpu_state* states,
                     const uint8_t* mem_ops, const uint8_t* mem_flags, int mem_cap);
/* checkpoint / resume: the update counter and cumulative counters of
 * avgpu_get_stats (`last` = the stats of the checkpointed world's last update),
 * and its seed (the scheduler's key) unless last->seed is 0, which keeps the
 * world's configured seed */
int avgpu_set_clock(avgpu_world* w, const avgpu_update_stats* last);
/* Batched cTestCPU::TestGenome (cpu/cTestCPU.cc:190-326), one gestation
 * each, deterministic inputs, mutations off. executed_flags (n*flags_cap)
 * receives '+'/'-' for the parent part at the divide (or the whole memory
 * at timeout), offspring (n*AVGPU_MAX_GENOME) the offspring op codes. */
int avgpu_test_genomes(avgpu_world* w, int n, const uint8_t* genomes, const int32_t* lens,
                       avgpu_test_result* results, char* executed_flags, int flags_cap,
                       uint8_t* offspring);

/* ---- statistics / multi-GPU plumbing ------------------------------------ */
/* the last update's statistics (reduced here if that update ran with out == NULL) */
int avgpu_get_stats(avgpu_world* w, avgpu_update_stats* out);
/* device pointer of the 32-double reduction vector of the last update
 * (N, sum merit, executed, births, ...) for an external all-reduce
 * (RCCL, cMultiProcessWorld.cc:375-405); avgpu_set_global_merit feeds the
 * reduced totals back before the next allotment. */
int avgpu_stats_vector(avgpu_world* w, void** dev_ptr);
/* total_merit: the SUM OF SCHEDULER WEIGHTS over every world (as
 * avgpu_update_totals computes it, head starts included), total_orgs: the
 * living organisms of every world */
int avgpu_set_global_totals(avgpu_world* w, double total_merit, int64_t total_orgs);
/* ---- strip tiles: one global world over several GPUs --------------------
 * Replaces the reference's only multi-process world, cMultiProcessWorld
 * (main/cMultiProcessWorld.cc:142-190 migrant exchange, :375-405 update-size
 * all-reduce), with row strips of ONE torus / grid.  The world is created with
 * cfg.world_y = the GLOBAL row count and num_cells = rows*world_x of this tile;
 * avgpu_set_tile(row0) places it.  An update of a tiled world is identical,
 * cell for cell, to the same update of the untiled world (DESIGN.md
 * "Multi-GPU"), given this host schedule with exchange(halo) meaning: send
 * halo_send_up to the tile above (rank-1 mod T) and halo_send_down to the
 * tile below, receive into halo_recv_up from the tile above and into
 * halo_recv_down from the tile below (same for records):
 *
 *   avgpu_tile_partials(w, part)         all_gather(part) in tile order
 *   avgpu_tile_steps(w, gathered, T, &K) (the update's batch steps; the same K on
 *                                        every tile)
 *   for step s = 0 .. K-1:
 *    [s > 0: avgpu_tile_partials, all_gather(part)]
 *    [exchange(resource rows): spatial resources]
 *    avgpu_tile_begin_step(w, gathered, T, s, K)
 *                                        exchange(halo)
 *   avgpu_tile_place(w, 0, 0)            exchange(halo)
 *   avgpu_tile_place(w, 0, 3)            exchange(halo)
 *   for round 1..3:
 *     avgpu_tile_place(w, round, 0)      exchange(halo)
 *   avgpu_tile_place(w, 3, 1)            exchange(records) issued ...
 *   avgpu_tile_place(w, 3, 2)            ... and running beside this launch
 *                                        wait(records)
 *   avgpu_tile_finish(w, stats)          (the step's newborns; stats after the last step)
 *   [avgpu_tile_res_cons(w, cons)        all_reduce(cons, sum): global pools,
 *    avgpu_tile_res_settle(w, cons)      when avgpu_tile_res_cons returned > 0]
 *
 * Resources on tiles: call avgpu_set_tile before (or after: it re-seeds them)
 * avgpu_load_resources; CELL ids and inflow/outflow boxes stay global.
 * Every call is stream-ordered on the handle's stream (no host sync).
 * Requirements: rows >= 2, tile cells a multiple of 256 and of world_x.
 * arena_bytes (<= 0: default max(256 KiB, 256 B x world_x)) bounds the
 * offspring genome bytes shipped per direction per update; an offspring that
 * does not fit is dropped (AVGPU_CNT_HALO_LOST). */
int avgpu_set_tile(avgpu_world* w, int64_t row0, int64_t arena_bytes);
/* byte sizes of the partials vector (avgpu_tile_partials output, per tile),
 * of one halo buffer and of one record buffer */
int avgpu_tile_buffer_bytes(avgpu_world* w, int64_t* partial_bytes, int64_t* halo_bytes,
                            int64_t* record_bytes);
/* device buffers the host exchanges (8 distinct allocations) */
int avgpu_set_tile_buffers(avgpu_world* w, void* halo_send_up, void* halo_send_down,
                           void* halo_recv_up, void* halo_recv_down, void* rec_send_up,
                           void* rec_send_down, void* rec_recv_up, void* rec_recv_down);
/* per-256-cell merit partials, then alive counts (doubles), then the tile's
 * sub-step predictor (int64 bits), for the all-gather */
int avgpu_tile_partials(avgpu_world* w, double* dev_out);
/* the update's batch steps K from every tile's predictor in the gathered
 * partials (the single world's rule over the same integer sum; synchronises
 * with the handle's stream) */
int avgpu_tile_steps(avgpu_world* w, const double* dev_gathered, int ntiles, int* k_out);
/* batch step s of K: global totals from the gathered partials (T x partials,
 * tile order), then allotment + interpretation of this tile, occupancy of its
 * edge rows out.  avgpu_tile_begin = step 0 of 1. */
int avgpu_tile_begin_step(avgpu_world* w, const double* dev_gathered, int ntiles, int sub, int k);
int avgpu_tile_begin(avgpu_world* w, const double* dev_gathered, int ntiles);
/* placement round 0..3, phase 0: one launch that resolves round - 1 with the
 * claims both strips sent (a cell of an edge row is claimed only from the two
 * strips it touches, so both resolve it alike) and picks round `round`,
 * writing its claims on the ghost rows and on the own edge rows into the halo
 * send buffers.  Round 0, phase 0 picks and sends the kill times of its picks
 * on the ghost rows; round 0, phase 3 (after that exchange) cancels the
 * births whose parent's cell a pick of an earlier birth kills, here or from
 * the neighbour, and claims the others' round-0 targets (time-ordered
 * placement).  After round 3: phase 1 resolves round 3 and packs
 * the ghost-row winners into the record buffers, phase 2 activates this
 * tile's own winners (it reads no record buffer: it may run while the
 * records travel). */
int avgpu_tile_place(avgpu_world* w, int round, int phase);
/* activation of the received records; statistics (out may be NULL: see
 * avgpu_run_update) */
int avgpu_tile_finish(avgpu_world* w, avgpu_update_stats* out);
/* spatial resources on strips: bytes of one resource-row buffer (n_spatial x
 * world_x doubles, 0 without spatial resources) and the 4 device buffers
 * exchanged like the halo (avgpu_tile_partials fills the send rows: first and
 * last row of every spatial resource; the flow step of avgpu_tile_begin reads
 * the rows above and below from the receive buffers) */
int avgpu_tile_res_bytes(avgpu_world* w, int64_t* bytes);
int avgpu_set_tile_res_buffers(avgpu_world* w, void* send_up, void* send_down, void* recv_up,
                               void* recv_down);
/* global pools on strips: this tile's consumption of the update
 * (AVGPU_MAX_RESOURCES uint64, 2^-32 units, device memory); returns the number
 * of global resources (0: skip the all-reduce and the settle) */
int avgpu_tile_res_cons(avgpu_world* w, uint64_t* dev_out);
/* subtract the summed consumption of all tiles (same on every tile) */
int avgpu_tile_res_settle(avgpu_world* w, const uint64_t* dev_sum);

/* counters of the last avgpu_step: instructions executed (sum over lanes) */
int avgpu_last_step_insts(avgpu_world* w, int64_t* insts);
/* Interpreter-kernel time (HIP events recorded on the handle's stream around
 * every k_interpret launch sequence) accumulated since the previous call:
 * total milliseconds and number of interpret phases; resets the accumulator. */
int avgpu_last_kernel_ms(avgpu_world* w, double* ms, int64_t* launches);
/* The same accumulators split by interpreter size class (k_interpret<320>,
 * <768>, <1536>, <2048>): class_ms[4] milliseconds and the number of timed
 * interpret phases since the previous call; resets them (and
 * avgpu_last_kernel_ms's). */
int avgpu_kernel_times(avgpu_world* w, double* class_ms, int64_t* phases);
/* Bracket only every `every`-th interpret phase with the timing events (each
 * event record costs ~10 us of queue time); 0 = none, default 1. */
int avgpu_set_timing(avgpu_world* w, int every);

/* Device event counters (no reference equivalent: measurement only).
 * cumulative = 0: the last update (or avgpu_step); 1: summed over every
 * avgpu_run_update/update_run since creation.  Slots: */
enum avgpu_counter {
  AVGPU_CNT_INSTS = 0,      /* instructions executed (count.dat "insts executed") */
  AVGPU_CNT_DEATHS = 1,
  AVGPU_CNT_DIVIDES = 2,
  AVGPU_CNT_BIRTHS = 3,
  AVGPU_CNT_DROPPED = 4,    /* offspring never placed for capacity: birth-queue overflow, a slip past
                               AVGPU_MAX_GENOME, a full halo arena, BIRTH_METHOD 3 without a cell */
  AVGPU_CNT_SPILLS = 5,     /* slices handed to a larger LDS size class */
  AVGPU_CNT_SLICES = 6,     /* organisms with a non-zero allotment */
  AVGPU_CNT_LANESTEPS = 7,  /* 64 x longest lane per wave (lane efficiency = INSTS / this) */
  AVGPU_CNT_C0_SLICES = 8,  /* slices run by the class-0 launch (its windows, the list-class blocks inside it, its in-wave spill continuations) */
  AVGPU_CNT_C0_SITES = 9,   /* tape sites that launch staged in plus wrote back */
  /* 10..17: per-phase clocks of diagnostic (AVGPU_PHASE_CLOCKS) builds */
  AVGPU_CNT_HALO_SENT = 18, /* offspring shipped to a neighbouring tile */
  AVGPU_CNT_HALO_LOST = 19, /* offspring dropped because the halo arena was full */
  AVGPU_CNT_REC_EXHAUSTED = 20, /* RECORDED draws past the end of the stream */
  AVGPU_CNT_OVERSIZE = 21,  /* offspring longer than AVGPU_MAX_GENOME after a slip (dropped) */
  AVGPU_CNT_SUB_OVERFLOW = 22, /* DIV_MUT_PROB substitutions not kept: the per-update arena was full (must be 0) */
  AVGPU_CNT_OVERWRITTEN = 24, /* offspring placed, then replaced by a later birth into the same cell in
                                 the same update (the reference kills such a newborn too) */
  AVGPU_CNT_MEM_CAP = 23,   /* copy-time insertions skipped at AVGPU_MAX_GENOME memory sites (the
                               reference has no cap) and removals from a one-site memory */
  AVGPU_CNT_CANCELLED = 25, /* births whose parent's cell got an earlier offspring before the divide
                               (the reference's parent died first: never placed) */
  AVGPU_CNT_BAD_RECORD = 26, /* record or cell fields out of range where used as an index or length
                                (guarded, counted, never used; must be 0) */
  AVGPU_NUM_COUNTERS = 48   /* 32..47: AVGPU_PHASE_CLOCKS diagnostic builds */
};
int avgpu_counters(avgpu_world* w, int cumulative, int64_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* AVIDA_GPU_H */
