// device.h -- HBM layout of the organism SoA and device helpers shared by the
// HIP kernels of the batched heads-CPU interpreter (gfx950 / MI355X).
//
// Layout (DESIGN.md "Data layout in HBM"): one organism per cell, structure of
// arrays, every array indexed [field_row * N + cell] so that a wavefront of 64
// consecutive list entries touches 64 consecutive words when the list is in
// cell order.  The memory tape of cell c lives in tape[c * TAPE_SLOT ...] as one
// byte per site: bits 0-5 = canonical handler id (include/avida_gpu.h), bit 6 =
// copied flag, bit 7 = executed flag (cpu/cCPUMemory.h:31-37; the mutated /
// copy-mut flags are statistics only and are not kept on device).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/avida_gpu.h"

#define TAPE_SLOT 2048
// birth record row b_inh[r * BI_WORDS ..]: merit, fitness (doubles), generation,
// copied size, executed size, gestation time, the offspring's RNG key and
// counter, the parent's last task counts
// (BI_FINAL bit 0 = 1: the divide left the offspring's fitness and key and the
// parent's phenotype to finalize_key / finalize_phenotype, world.hip; bits
// 16..31 the offspring's birth time in the update, 1/2^16 -- DESIGN.md 5)
enum { BI_MERIT = 0, BI_FITNESS = 2, BI_GEN = 4, BI_CCOPIED = 5, BI_EXEC = 6, BI_GEST = 7,
       BI_RLO = 8, BI_RHI = 9, BI_RCTR = 10, BI_FINAL = 11, BI_LTASK = 12, BI_WORDS = 32 };
#define BI_TIME(w) ((uint32_t)(w) >> 16)
#define CODE_MASK 0x3F
#define TF_COPIED 0x40
#define TF_EXEC 0x80
#define CODE_ERROR 0x3F  /* cInstSet::GetInstError: never a nop */

// ctl word bits
#define CTL_SP0(c) ((c) & 0xF)
#define CTL_SP1(c) (((c) >> 4) & 0xF)
#define CTL_CURSTK 0x100u
#define CTL_MAL 0x200u
#define CTL_ALIVE 0x400u
// "fresh" offspring (k_activate): registers, heads, stacks, label, IO
// buffers, counters, task / reaction counts and bonus hold their birth values
// (zero, default bonus) implicitly -- the SoA rows are stale until the
// organism's first slice writes them back.  Every reader honours the bit.
#define CTL_FRESH 0x800u
// serial world: died in a speculative step (m_spec_die); removed at its next pick
#define CTL_SPECDIE 0x1000u
// head start of an offspring not yet allotted (17 bits: 2^16 - its birth
// time, 1..2^16; 0 = none): its first allotment weights its merit by
// 1 + hs / 2^16 (sched_weight), then clears it
#define CTL_HS_SHIFT 14
#define CTL_HS(c) (((c) >> CTL_HS_SHIFT) & 0x1FFFFu)
#define CTL_HS_MASK (0x1FFFFu << CTL_HS_SHIFT)

#define NUM_CLASSES 4
#define ACLASS_NONE 0xFF
// react_res row: resource slot+1 (0 infinite), spatial?, depletable, type, frac, min, max, value
#define RR_STRIDE 8
enum { RR_RES = 0, RR_SPATIAL = 1, RR_DEPL = 2, RR_TYPE = 3, RR_FRAC = 4, RR_MIN = 5, RR_MAX = 6, RR_VALUE = 7 };
#define RES_FIX 4294967296.0   /* global consumption accumulates in units of 2^-32 */

struct ResParam {
  int32_t geometry, slot;       // slot: row of res_amount (spatial) or -1
  int32_t in_x1, in_x2, in_y1, in_y2, out_x1, out_x2, out_y1, out_y2;
  double in_share;              // inflow / cells of the inflow box (cSpatialResCount::Source)
  double sink_frac;             // 1 - decay, decay = 1 - outflow (cPopulation.cc:440, Sink)
  double xdiffuse, ydiffuse, xgravity, ygravity;
  double decay100, inflow100;   // decay_precalc / inflow_precalc at PRECALC_DISTANCE (global)
  double decay99, inflow99;     // ... at 99 steps (the last block of update 0's 9999 steps)
  int32_t flows, has_sink;      // FlowAll does anything; the outflow box is set
  int32_t in_all, out_all;      // the inflow / outflow box covers every cell exactly once
};
#define NUM_LISTS 7
#define RT_STRIDE 12
enum { RT_TASK = 0, RT_TYPE = 1, RT_MIN = 2, RT_MAX = 3, RT_HASREQ = 4, RT_USED = 5, RT_MULT = 6, RT_ADD = 8 };
// budget bit carried by a slice handed to the next size class: its primary
// birth record is already in use (budgets are < 2^30: avgpu_step checks)
#define BUDGET_PRIM 0x40000000

// Per-cell execution record: the interpreter-private state of one organism
// (the fields only a slice and the state import / export touch), XS_WORDS
// int32 = 256 B per cell, 256-B aligned.  A slice reads and writes it with
// 13 16-byte accesses per lane (words 0..51) instead of ~50 scattered 4-byte
// SoA accesses -- in budget-sorted windows the lanes of a wave are scattered
// cells, and every SoA store was a partial-line HBM write.  A fresh offspring
// (CTL_FRESH) has none of it stored: its birth values are implied.
enum : int {
  XS_REG = 0,      // 3: registers AX BX CX
  XS_HEAD = 3,     // 4: IP, read, write, flow
  XS_RLABEL = 7,   // read_label: len (4b) | nop i at bits 4+2i
  XS_CYCLES = 8,   // cpu_cycles_used
  XS_TIME = 9,     // time_used
  XS_GEST = 10,    // gestation_start
  XS_ERRORS = 11,  // cur errors (faults)
  XS_INBUF = 12,   // 3: input buffer, most recent first
  XS_INTOT = 15,   // inputs received
  XS_INPTR = 16,   // next input index
  XS_OUTBUF = 17,  // last output
  XS_OUTTOT = 18,  // outputs made
  XS_BONUS = 20,   // 2: cur_bonus (double, 8-B aligned)
  XS_TASK = 22,    // 9: cur_task_count of the logic-9 tasks
  XS_STACK = 32,   // 20: stack k entry j at 32 + 10k + j
  XS_REACT = 52,   // 12: cur_reaction_count of reactions 0..11 (12..15 in cur_react rows)
  XS_NREACT = 12,
  XS_WORDS = 64
};

struct DevWorld {
  int64_t n;  // cells
  // --- hot state (registers in the interpreter) ---
  int32_t* xs;        // [n][XS_WORDS] execution records (above)
  uint32_t* ctl;      // [n]  sp0 | sp1<<4 | cur_stack | mal_active | alive
  int32_t* mem_size;  // [n]
  int32_t* max_exec;  // [n]
  int32_t* birth_len; // [n]  genome length at birth (cPhenotype::genome_length)
  uint64_t* gkey;     // [n]  genome key of the birth genome (systematics census)
  uint32_t* rng;      // [3][n] key_lo, key_hi, ctr
  int32_t* budget;    // [n]  instructions left in this update
  // [n] size class k_allot / k_classify_uniform gave the cell's slice this
  // update (0..3, ACLASS_NONE: no slice).  Only those kernels write it: the
  // class-0 launch and k_window_sort select their cells by this tag, never by
  // the live mem_size / budget that list classes running beside them on the
  // aux streams rewrite (a list-class slice that divides down to a class-0
  // size must not be picked up by class 0 in the same update).
  uint8_t* aclass;
  uint8_t* tape;      // [n][TAPE_SLOT]
  // --- cold state ---
  int32_t* inputs;    // [3][n] cell inputs
  int32_t* last_task; // [16][n]
  int32_t* cur_react; // [16][n]: rows XS_NREACT.. only (rows 0..11 live in the execution record)
  double* merit;      // [n]
  double* fitness;    // [n]
  double* credit;     // [n]
  int32_t* gest_time; // [n]
  int32_t* num_div;   // [n]
  int32_t* generation;// [n]
  int32_t* copied;    // [n]
  int32_t* child_copied; // [n]
  int32_t* executed;  // [n]
  // --- per-update work lists / queues ---
  // size-class lists: row k = 1..3 the organisms k_allot put in class k,
  // row 3 + k the organisms that spilled into class k during the update
  int32_t* class_list;   // [NUM_LISTS][n]
  int32_t* order;        // [n] class-0 order of a world update: cells of each SORT_WIN window by budget
  int32_t* class_count;  // [8] entries of each list row
  unsigned long long* counters; // [16] insts, deaths, divides, births, dropped, ...
  // birth records.  Record r < n holds the first offspring that cell r's
  // parent produced in its slice (no atomics in the interpreter loop); records
  // n .. n+ocap-1 hold further offspring of one slice, reserved atomically.
  // Queue entry i < b_count[0] is record b_list[i]; entry b_count[0] + j is
  // record n + j (rec_of below).
  int64_t rcap;       // n + ocap
  int32_t* b_count;   // [3] primary records listed, overflow records used, b_subs entries used
  int32_t* b_list;    // [n] primary record ids, appended per wave after the loop
  int32_t* b_parent;  // [rcap]
  uint32_t* b_seq;    // [rcap]
  int32_t* b_len;     // [rcap]  offspring length after the divide mutations
  int32_t* b_len0;    // [rcap]  the child's length before them (b_genome holds that child)
  int32_t* b_edit;    // [5][rcap] its divide-mutation edits (interp.hip edit_word; 0 = none)
  // variable-count divide-mutation edits of record r (only read when
  // seg_any): segment k holds b_pcnt[k][r] edit words from
  // b_subs[b_pofs[k][r]], applied at its place in Divide_DoMutations' order
  // (SEG_* below); b_count[2] is the arena's fill of this update, scap its size
  int32_t* b_subs;    // [scap]
  int64_t scap;
  int32_t* b_pofs;    // [NSEG][rcap]
  int32_t* b_pcnt;    // [NSEG][rcap]
  // what the offspring of record r inherits (cPhenotype::SetupOffspring,
  // main/cPhenotype.cc:349-447), one 128-B row per record (BI_* below):
  // written with 16-B stores at the divide, read with 16-B loads at
  // activation -- as [field][rcap] rows every field was a scattered 4-B
  // access whose line held no other field of the record
  int32_t* b_inh;     // [rcap][BI_WORDS]
  int32_t* b_target;  // [rcap]
  int8_t* b_state;    // [rcap]  BS_* (world.hip)
  unsigned long long* b_prio; // [rcap] claim key of the record's current round (world.hip claim_key)
  uint8_t* b_genome;  // [rcap][TAPE_SLOT]
  // placement scratch, n cells + 2 ghost rows (strip tiles, below)
  uint8_t* occ;       // [n + 2X]
  unsigned long long* claim; // [n + 2X]
  unsigned long long* claim2; // [n + 2X] (claim_r[1])
  // placement rounds 0..3 claim into their own arrays (k_place_round,
  // k_tile_round): claim_r[0] = claim, [1] = claim2, [2], [3], [n + 2X] each;
  // all zero between updates (records clear theirs at activation, k_allot
  // round 3's, k_tile_prep the ghost rows)
  unsigned long long* claim_r[4];
  int32_t* b_tgt;     // [4][rcap] the record's target in each placement round it claimed in
  int32_t* owner;     // [n + 2X]  record id, -1 none, REMOTE_OWNER(k, t) won by a halo birth in round k
  uint32_t* killt;    // [n] 2^16 - the earliest birth time of a round-0 pick that kills the cell's
                      // organism, 0 none (placement launch 0 -> the cancellations of launch 0b)
  // the scheduler's tree (k_block_counts -> k_allot): each 256-cell block's
  // share of the update's picks, then the tree's levels (scratch)
  int64_t* blk_count; // [nb]
  double* tree_scr;   // [2 * P] levels of the top tree over the block partials (P = pow2 >= blocks)
  int64_t* tree_cnt;  // [2 * P] their counts
  int64_t tree_cap;   // P of the allocation (strip tiles: >= every strip's blocks)
  int32_t* sdone;     // [n] instructions a spilled slice ran before it spilled (birth times)
  // test-CPU outputs
  uint8_t* t_flags;   // [n][TAPE_SLOT] executed flags snapshot ('+'/'-')
  int32_t* t_flags_len; // [n]
  uint8_t* t_child;   // [n][TAPE_SLOT]
  int32_t* t_child_len; // [n]
  // tables
  int32_t* rand_cum;  // [64] cumulative integer weights
  uint8_t* rand_code; // [64] canonical code of op i
  uint16_t* task_lut; // [256] logic id -> task bitmask
  int n_ops;
  int32_t rand_total;
  uint8_t* rand_lut;  // [256] draw -> canonical code when rand_total <= 256
  int32_t slow_batch;   // parked lanes that trigger the interpreter's slow phase (1..64)
  int32_t nb_slow_batch;  // the same in the newborn pass
  int n_react;
  // reactions, RT_STRIDE words each: task, process type, requisite min / max
  // count, has-requisite, in-use, bonus multiplier (f64), bonus addend (f64)
  int32_t* react_tab; // [AVGPU_MAX_REACTIONS][RT_STRIDE]
  // simple environment (reaction i rewards task i; requisites absent, or
  // min_count <= 0 with max_count 1 or unlimited): the IO check is bit logic
  int32_t env_simple;
  uint32_t env_react_mask;   // tasks with a reaction
  uint32_t env_once_mask;    // tasks whose reaction has max_count 1
  uint32_t env_res_mask;     // reactions drawing on a finite resource
  double* task_tab;          // [32]: bonus factor of task t's reaction, then its addend
  // ---- resources (resources.hip; DESIGN.md "Resources") ----
  int32_t n_res, n_cellres, env_resources;   // env_resources: some reaction consumes a resource
  struct ResParam* res_param;   // [AVGPU_MAX_RESOURCES]
  double* res_amount;           // [n_spatial][n] spatial amounts (row = ResParam::slot)
  double* res_delta;            // [n] rate scratch of the spatial step (+ 64: k_res_step's junk stores)
  double* res_global;           // [AVGPU_MAX_RESOURCES] global levels, fixed during an update
  unsigned long long* res_cons; // [AVGPU_MAX_RESOURCES] global consumption of the update, 2^-32 units
  avgpu_cell_resource* res_cells; // [n_cellres] CELL entries (cell ids are global)
  double* react_res;            // [AVGPU_MAX_REACTIONS][RR_STRIDE] resource-bound process settings
  int8_t res_spatial_host[AVGPU_MAX_RESOURCES];   // host-side launch flags
  int8_t res_flows_host[AVGPU_MAX_RESOURCES];
  int8_t res_cells_host[AVGPU_MAX_RESOURCES];     // resource has CELL entries
  int8_t res_grav_host[AVGPU_MAX_RESOURCES];      // resource has gravity on an axis
  double* res_amount_alt;       // [n_spatial][n] the other buffer of the spatial step
  int8_t res_first;             // host: the next update is the first since the load
  int32_t n_spatial;            // spatial resources (rows of res_amount)
  double* rs_send[2];           // strip tiles: [n_spatial][X] first / last row out
  double* rs_recv[2];           //   and the rows above / below in
  uint8_t fill_code;   // code of op 0 (new sites on allocate)
  // config scalars
  int32_t world_x, world_y, geometry;
  int32_t ave_time_slice, slicing;
  int32_t base_merit_method, base_const_merit;
  double default_bonus, size_range, min_copied_lines, min_exe_lines;
  double merit_default_bonus, required_bonus;
  int32_t inherit_merit, require_allocate, alloc_method, max_label_exe;
  int32_t min_genome, max_genome;  // resolved MIN/MAX (>= 8, <= 2048)
  int32_t cfg_min_genome, cfg_max_genome;  // raw MIN_GENOME_SIZE / MAX_GENOME_SIZE
  int32_t death_method, age_limit;
  int32_t prefer_empty, allow_parent, birth_method;
  // P(p) = u < p: counter threshold ceil(p 2^32), and p itself
  // for RECORDED draws
  uint64_t th_copy_mut, th_div_mut, th_div_ins, th_div_del, th_div_slip, th_div_uni;
  double p_copy_mut, p_div_mut, p_div_ins, p_div_del, p_div_slip, p_div_uni;
  // COPY_INS / COPY_DEL / COPY_UNIFORM / COPY_SLIP (SLIP_COPY_MODE 0) of
  // Inst_HeadCopy; copy_ext: any of them non-zero
  uint64_t th_copy_ins, th_copy_del, th_copy_uni, th_copy_slip;
  double p_copy_ins, p_copy_del, p_copy_uni, p_copy_slip;
  int32_t copy_ext;
  uint64_t no_mut_mask;   // NO_MUT_INSTS: handler codes copy mutations leave alone (bit per code)
  // Divide_CheckViable's task / reaction requirements (avgpu_load_env): the
  // required / immunity task (avgpu_task, -1 none), reaction (index, -1
  // none), REQUIRE_SINGLE_REACTION, MAX_UNIQUE_TASK_COUNT; div_req: any set
  int32_t req_task, imm_task, req_react, imm_react, single_react, max_task_cnt, div_req;
  uint64_t th_div_site;   // DIV_MUT_PROB (per-site substitutions on divide)
  double p_div_site;
  uint64_t th_par_site;   // PARENT_MUT_PROB (per-site substitutions in the parent)
  double p_par_site;
  uint64_t th_par_ins, th_par_del;   // PARENT_INS_PROB, PARENT_DEL_PROB (per site, in the parent)
  double p_par_ins, p_par_del;
  double pois_L[5];       // exp(-DIVIDE_POISSON_{SLIP,MUT,INS,DEL,TRANS}_MEAN), 0 = off
  int32_t pois_any;
  uint64_t th_dsite[5];   // DIV_INS_PROB, DIV_DEL_PROB, DIV_UNIFORM_PROB, DIV_SLIP_PROB, DIV_TRANS_PROB
  double p_dsite[5];
  uint64_t th_dtrans;     // DIVIDE_TRANS_PROB
  double p_dtrans;
  int32_t seg_any;        // some variable-count kind is on (b_subs / b_pofs / b_pcnt allocated)
  int32_t slip_fill_mode;
  int32_t trans_fill_mode;
  int32_t slip_copy_mode;   // SLIP_COPY_MODE: 0 the read head jumps, 1 a slip of the whole memory
  // RECORDED mode (avgpu_set_rng_mode): rec_n doubles; rec_off[c] = the start
  // of cell c's organism's segment, -1 = a counter stream.  rec == nullptr:
  // COUNTER mode everywhere (the REC-free interpreter instantiations run).
  const double* rec;
  int64_t rec_n;
  int64_t* rec_off;
  // the serial world (avgpu_run_serial_updates; allocated on its first use):
  // merit sum tree (stree[1] the root, leaves at stree_size + cell), each
  // organism's speculative-step credit, the world's scheduler stream
  double* stree;
  int64_t stree_size;
  int32_t* spec;     // [n]
  uint32_t* grng;    // [3] lo hi ctr: the scheduler's stream (picks)
  uint32_t* sctx;    // [3] lo hi ctr: the context stream (every other draw of the serial world)
  uint8_t* face;     // [n] connection-list rotation of each cell (cPopulationCell::Rotate)
  // recorded serial streams (avgpu_set_serial_streams): the k-th pick / context
  // draw is srec_sched[k] / srec_ctx[k] (the counters grng[2] / sctx[2])
  const double* srec_sched;
  int64_t srec_sched_n;
  const double* srec_ctx;
  int64_t srec_ctx_n;
  uint32_t seed_lo, seed_hi;
  // Strip tiles (multi-GPU, DESIGN.md "Multi-GPU"): this world holds rows
  // [row0, row0+rows) of a world_x x global_rows torus / grid.  When tiled,
  // occ / claim / owner carry two ghost rows after the n cells: [n, n+X) is
  // global row row0-1 (the tile above), [n+X, n+2X) global row row0+rows (the
  // tile below).  Single world: tiled = 0, row0 = 0, rows = global_rows = world_y.
  int32_t row0, global_rows, rows, tiled;
  int64_t cell0;          // row0 * world_x: global id of local cell 0 (RNG keys, priorities)
  // halo buffers per direction d (0: tile above, 1: tile below), registered by
  // the host: halo_bytes(X) = per round parity X u64 claims on the receiver's
  // edge row and X u64 the sender's own claims on its edge row, then X u8
  // edge-row occupancy (world.hip halo_cl / halo_occ)
  uint8_t* h_send[2];
  uint8_t* h_recv[2];
  // birth-record buffers per direction: HaloHdr, X HaloRec, arena of r_arena bytes
  uint8_t* r_send[2];
  uint8_t* r_recv[2];
  int64_t r_arena;
  // (appended, so that the hot fields keep their offsets in the scalar loads)
  int32_t* age;       // [n] cPhenotype::age during the update (k_allot ticks it; -1 injected, 0 born / divided),
                      // kept only when track_age (BIRTH_METHOD 1 / 2, its one consumer on this path)
  int32_t track_age;  // BIRTH_METHOD 1 / 2: the age row is maintained
  // the class-0 order's bucket histogram of each 4096-cell sub-window
  // (k_allot's workgroups write it, k_window_order scans it): [nsub][SORT_BUCKETS]
  int32_t* sub_hist;
  int32_t* e_list;    // BIRTH_METHOD 4 + PREFER_EMPTY: the cells empty at placement start, ascending
  int32_t* e_blk;     // its per-256-cell counts, then their exclusive offsets (e_blk[nb]: the total)
  int32_t* soup_perm; // serial world, BIRTH_METHOD 4: the reference's empty_cell_id_array (0..N-1 at creation)
  int32_t* reaper;    // serial world, BIRTH_METHOD 5: the reaper queue, a ring of reaper_cap cells
  int64_t* reaper_ix; // [0] its rear (oldest) position, [1] one past its front (newest)
  int64_t reaper_cap;
  // the batch step's newborns and sub-steps:
  int32_t* ran;       // [n] instructions each cell's organism ran in this step's main pass (k_allot zeroes)
  double* cons;       // [n_res][n] its depletable consumption in that pass (k_allot zeroes; env_resources)
  // [1] this step's pick carry (newborn picks beyond
  // their victims' leftovers, k_activate), [2] the carry not yet taken (taken
  // at an update's first step), [4] the update's UD (AVE_TIME_SLICE x the
  // organisms at its first step)
  long long* sched;
  // the sub-step predictor of this step's main pass, sharded by block like
  // the counters (k_block_counts zeroes it): shard s at pacc[s * PACC_STRIDE]
  // holds [0] its weight term (2^-20 mean weights), [1] its divide counts of
  // quarters 0 | 1 << 32, [2] of quarters 2 | 3 << 32 (pacc_sum)
  long long* pacc;
  const double* totals;   // the step's totals (k_block_counts): [1] organisms, [2] weight total, [3] UD
};

// a strip's partials vector (avgpu_tile_partials): nb block partials, nb alive
// counts, its sub-step predictor, its pick carry and its predictor's divide
// counts by quarter (int64 bits)
__host__ __device__ inline int64_t tile_part_stride(int64_t nb) { return 2 * nb + 6; }
// owner of a cell won by a neighbouring strip's offspring in round k at birth time t
#define REMOTE_OWNER(k, t) (-2 - ((k) + 4 * (int)(t)))
// halo buffer: per round parity X u64 claims on the receiver's edge row and X
// u64 the sender's own claims on its edge row, X u8 edge-row occupancy, then
// (round 0's picks) X u32 kill times of the sender's picks on the receiver's
// edge row (2^16 - t, max-reduced)
__host__ __device__ inline int64_t halo_kt_off(int x) { return ((int64_t)x * 33 + 3) / 4 * 4; }
__host__ __device__ inline int64_t halo_bytes(int x) { return (halo_kt_off(x) + 4 * (int64_t)x + 15) / 16 * 16; }
struct HaloHdr { int32_t count, arena_used, overflow, pad; };
// one offspring placed across a tile edge (the migrant record of
// cMultiProcessWorld.cc:142-190, restated for strip tiles)
struct HaloRec {
  int32_t col, round, len, gen, ccopied, exec, gest;
  uint32_t rng_lo, rng_hi, rng_ctr;
  int32_t off;
  uint32_t t;         // birth time (owner bookkeeping, head start)
  double merit, fitness;
  int32_t last_task[AVGPU_NUM_LOGIC_TASKS], pad2[3];   // the parent's (SetupOffspring)
};
__host__ __device__ inline int64_t record_bytes(int x, int64_t arena) {
  return (int64_t)sizeof(HaloHdr) + (int64_t)x * (int64_t)sizeof(HaloRec) + arena;
}

// counters[] slots
#define CNT_INSTS 0
#define CNT_DEATHS 1
#define CNT_DIVIDES 2
#define CNT_BIRTHS 3
#define CNT_DROPPED 4
#define CNT_SPILLS 5
#define CNT_SLICES 6
#define CNT_LANESTEPS 7   /* 64 x the longest lane of each wave: lane efficiency = insts / this */
#define CNT_C0_SLICES 8   /* slices run by the class-0 interpreter launch */
#define CNT_C0_SITES 9    /* tape sites it staged in + wrote back (sum of M at entry and exit) */
// slots 10..17: AVGPU_PHASE_CLOCKS diagnostic builds only (s_memtime per wave)
#define CNT_CLK_STAGE 10
#define CNT_CLK_LOOP 11
#define CNT_CLK_WB 12
#define CNT_ITERS 13      /* loop iterations of the wave */
#define CNT_IT_FAST 14    /* iterations in which some lane took the branch-free block */
#define CNT_IT_COPY 15    /* ... the h-copy block */
#define CNT_IT_SLOW 16    /* ... the switch */
#define CNT_WAVES 17
#define CNT_HALO_SENT 18  /* offspring shipped to a neighbouring tile */
#define CNT_HALO_LOST 19  /* offspring lost to a full halo arena (counted in DROPPED too) */
#define CNT_REC_OVER 20   /* RECORDED draws past the end of the stream */
// variable-count edit segments of a birth record, in the order applied:
// e0 (slip) or, with a data fill (SLIP_FILL_MODE 2 / 3), the one-shot slip as
// a segment, Poisson slips, per-site slips (two words each with a data fill:
// edit, fill offset), translocations (one-shot, Poisson, per site: two words
// each, three with TRANS_FILL_MODE 1; see births.h), e1 (mut), Poisson
// substitutions, e2 (ins), Poisson insertions, e3 (del), Poisson deletions,
// e4 (uniform), per-site substitutions, insertions, deletions, uniform
// mutations.  Data fills (a slip's or translocation's L codes / source
// sites) sit in the same arena, reserved per event.
enum { SEG_OSLIP = 0, SEG_PSLIP, SEG_SSLIP, SEG_TTRANS, SEG_PTRANS, SEG_STRANS, SEG_PMUT, SEG_PINS, SEG_PDEL, SEG_SMUT, SEG_SINS, SEG_SDEL, SEG_SUNI, NSEG };
#define CNT_SUB_OVERFLOW 22   /* DIV_MUT_PROB substitutions that found the b_subs arena full (must stay 0) */
#define CNT_OVERSIZE 21   /* offspring a slip grew past AVGPU_MAX_GENOME (counted in DROPPED too) */
#define CNT_MEM_CAP 23    /* copy insertions past AVGPU_MAX_GENOME sites / removals from one site (skipped) */
#define CNT_OVERWRITTEN 24  /* offspring placed, then killed by a later birth into the same cell this update */
#define CNT_CANCELLED 25  /* records whose parent's cell got an offspring before their divide (never placed) */
#define CNT_BAD_RECORD 26 /* record / cell fields out of range where used as an index (guarded; must be 0) */
#define CNT_WASTED 27     /* instructions replaced organisms ran after their newborns' birth times */
#define CNT_STEPS 28      /* batch steps (k_block_counts, one per step) */
// 32..37: AVGPU_PHASE_CLOCKS loop cycles by block (decode, fast, copy, switch,
// wave phase, advance); 38..43: slow-switch cycles in pop, push, IO, h-alloc,
// h-divide, h-search/if-label
#define CNT_CB0 32
#define CNT_CASE0 38
// Counters are sharded over NSHARD lines (CNT_STRIDE x u64 each) so that the
// per-wave adds of a 16K-wave launch do not serialise on one L2 address; they
// are cleared every update, and counters[CNT_CUM_BASE + k] accumulates slot k
// over all updates (k_stats_final).
#define NSHARD 64
#define CNT_STRIDE 64
#define CNT_CUM_BASE (NSHARD * CNT_STRIDE)
#define CNT_WORDS (NSHARD * CNT_STRIDE + CNT_STRIDE)
#define PACC_STRIDE 8
// the predictor's word k summed over the shards (a packed pair of 32-bit
// counts sums without carries for worlds below 2^32 organisms)
__device__ __forceinline__ long long pacc_sum(const DevWorld& W, int k) {
  long long s = 0;
  for (int sh = 0; sh < NSHARD; sh++) s += W.pacc[sh * PACC_STRIDE + k];
  return s;
}
// quarter k's divide count
__device__ __forceinline__ long long quarter_count(const DevWorld& W, int k) {
  return (long long)(((unsigned long long)pacc_sum(W, 1 + (k >> 1)) >> (32 * (k & 1))) & 0xFFFFFFFFull);
}
__device__ __forceinline__ long long densest_quarter(const DevWorld& W) {
  return max(max(quarter_count(W, 0), quarter_count(W, 1)), max(quarter_count(W, 2), quarter_count(W, 3)));
}
#define CNT_CUM_INSTS (CNT_CUM_BASE + CNT_INSTS)
#define CNT_CUM_BIRTHS (CNT_CUM_BASE + CNT_BIRTHS)
// 1 once this update's counts are in the running sums (k_stats_final); 0 after
// reset_counts_block, which folds them in itself when statistics were skipped
#define CNT_CUM_FLAG (CNT_CUM_BASE + CNT_STRIDE - 1)

__device__ __forceinline__ int queue_len(const DevWorld& W) {
  const int64_t n = (int64_t)W.b_count[0] + (int64_t)min(W.b_count[1], (int)(W.rcap - W.n));
  return (int)n;
}
__device__ __forceinline__ int64_t rec_of(const DevWorld& W, int64_t i) {
  const int p = W.b_count[0];
  return i < p ? (int64_t)W.b_list[i] : W.n + (i - p);
}

// Stores issued from inside the interpreter loop for write-only data (birth
// records, test-CPU snapshots) that no later instruction of the kernel reads.
// As inline asm they are outside the compiler's s_waitcnt bookkeeping, so no
// loop iteration waits on vmcnt for them: with compiler-visible stores there,
// every following iteration drained all of the wave's outstanding memory
// operations (~3000 cycles under load) before its first LDS read.  expcnt(0)
// lets the data VGPRs be reused immediately.
__device__ __forceinline__ void st_async_u32(void* p, uint32_t v) {
  asm volatile("global_store_dword %0, %1, off\n\ts_waitcnt expcnt(0)" ::"v"(p), "v"(v));
}
__device__ __forceinline__ void st_async_u64(void* p, uint64_t v) {
  asm volatile("global_store_dwordx2 %0, %1, off\n\ts_waitcnt expcnt(0)" ::"v"(p), "v"(v));
}
// global loads on rarely taken paths that wait for their own data, so that
// the compiler's wait bookkeeping sees no load outstanding after them
__device__ __forceinline__ uint32_t ld_sync_u32(const void* p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t ld_sync_u8(const void* p) {
  uint32_t v;
  asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// the same without the memory clobber: a read-only table load that orders
// nothing else (it still waits for itself)
__device__ __forceinline__ uint32_t ld_sync_ro_u32(const void* p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p));
  return v;
}
__device__ __forceinline__ uint32_t ld_sync_ro_u8(const void* p) {
  uint32_t v;
  asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p));
  return v;
}
// Read-only tables read through the scalar cache (s_load, counted by lgkmcnt):
// a vector load in the interpreter's loop waits on vmcnt, which also counts
// every store the wave still has in flight (the divide's record stores).
typedef const __attribute__((address_space(4))) double const_f64_t;
// p[0] at a wave-uniform address
__device__ __forceinline__ double ld_uniform_f64(const double* p) {
  return *(const_f64_t*)p;
}
// tab[idx] for a per-lane idx: one scalar load per distinct index among the
// active lanes (waterfall)
__device__ __forceinline__ uint32_t sgather_u8(const uint8_t* tab, uint32_t idx) {
  uint32_t out = 0;
  bool todo = true;
  while (todo) {
    const uint32_t u = __builtin_amdgcn_readfirstlane(idx);
    if (idx == u) {
      // the address made explicitly scalar (an "s" operand computed by VALU
      // was otherwise handed over in a VGPR)
      const uint64_t a = (uint64_t)(tab + (u & ~3u));
      // (readfirstlane returns int: each half through uint32_t, no sign extension)
      const uint64_t sa = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
      uint32_t w;
      asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w) : "s"(sa));
      out = (w >> ((u & 3u) * 8u)) & 0xFFu;
      todo = false;
    }
  }
  return out;
}
// one 16-B store of four words (p 16-byte aligned).  A store of more than 8
// bytes leaves a hazard on its data VGPRs: a VALU write to them right after
// the store can change what is stored.  The compiler pads its own stores; an
// asm store must carry the wait states itself (without them the rows came out
// corrupted, nondeterministically).
__device__ __forceinline__ void st_async_b128(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {a, b, c, d};
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_waitcnt expcnt(0)\n\ts_nop 2" ::"v"(p), "v"(v));
}
__device__ __forceinline__ void st_async_u8(void* p, uint32_t v) {
  asm volatile("global_store_byte %0, %1, off\n\ts_waitcnt expcnt(0)" ::"v"(p), "v"(v));
}

// ---------------------------------------------------------------------------
// RNG spec: identical arithmetic to the oracle's Stream.
__host__ __device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t rng_next(uint32_t lo, uint32_t hi, uint32_t& ctr) {
  uint32_t a = lowbias32(ctr * 0x9E3779B9U + hi);
  uint32_t b = lowbias32(a ^ lo);
  ++ctr;
  return b;
}
__device__ __forceinline__ uint32_t rng_below(uint32_t lo, uint32_t hi, uint32_t& ctr, uint32_t n) {
  return (uint32_t)(((uint64_t)rng_next(lo, hi, ctr) * n) >> 32);
}
__device__ __forceinline__ bool rng_p(uint32_t lo, uint32_t hi, uint32_t& ctr, uint64_t th) {
  return (uint64_t)rng_next(lo, hi, ctr) < th;
}
__host__ __device__ __forceinline__ void derive_key(uint32_t a_lo, uint32_t a_hi, uint32_t x, uint32_t y,
                                                    uint32_t& lo, uint32_t& hi) {
  lo = lowbias32(lowbias32(x ^ a_lo) + y);
  hi = lowbias32(lowbias32(y ^ a_hi) + x + 0x632BE5ABU);
}

// cHeadCPU::Adjust (cpu/cHeadCPU.cc:27-50)
// Genome key (restated in oracle/oracle.cc and
// avida_amd/systematics.py): words w = 0 .. ceil(len/4)-1 of the birth genome
// in canonical codes (4 sites little-endian, sites >= len zero) each mixed with
// their index, summed mod 2^64, then mixed with the length.  The sum makes it
// wave-parallel: each lane folds the words it copies, one wave_sum finishes.
__device__ __forceinline__ uint64_t gk_mix(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t gk_word(uint32_t word, int w, int len) {
  word &= 0x3F3F3F3Fu;
  const int keep = len - 4 * w;                 // sites of this word inside the genome
  if (keep < 4) word &= (1u << (8 * keep)) - 1u;
  return gk_mix(((uint64_t)(w + 1) << 32) | word);
}
__device__ __forceinline__ uint64_t gk_final(uint64_t sum, int len) {
  const uint64_t k = gk_mix(sum ^ ((uint64_t)len * 0x9E3779B97F4A7C15ull));
  return k ? k : 1ull;
}
// serial form over a tape (one lane)
__device__ __forceinline__ uint64_t gk_tape(const uint8_t* t, int len) {
  uint64_t s = 0;
  for (int w = 0; w < (len + 3) / 4; w++) {
    uint32_t v = 0;
    for (int j = 0; j < 4 && 4 * w + j < len; j++) v |= (uint32_t)t[4 * w + j] << (8 * j);
    s += gk_word(v, w, len);
  }
  return gk_final(s, len);
}

__device__ __forceinline__ int head_adjust(int pos, int size) {
  // wave-uniform test first: the common case (every active lane in range)
  // falls through without entering the divergent adjustment
  const bool out = (unsigned)pos >= (unsigned)size;
  if (__builtin_expect(__ballot(out) != 0ull, 0)) {
    if (out) pos = pos < 0 ? 0 : (pos < 2 * size ? pos - size : pos % size);
  }
  return pos;
}
// head_adjust of a position known to lie in [0, size] (one past a valid site)
__device__ __forceinline__ int head_wrap(int pos, int size) {
  return (unsigned)pos < (unsigned)size ? pos : pos - size;
}

// cInstSet::GetRandomInst (cpu/cInstSet.cc:83-88) -> canonical code
__device__ __forceinline__ uint8_t random_code(const DevWorld& W, uint32_t lo, uint32_t hi,
                                               uint32_t& ctr) {
  uint32_t r = rng_below(lo, hi, ctr, (uint32_t)W.rand_total);
  int i = 0;
  while (i < W.n_ops - 1 && W.rand_cum[i] <= (int32_t)r) i++;
  return W.rand_code[i];
}

// 2^x from IEEE adds / multiplies only (Horner on the Taylor series of
// e^(f ln2), f in [0,1), then an exact scale by 2^n): the same bits on the
// device and in the oracle (oracle/oracle.cc det_exp2); within 1 ulp of
// pow(2, x) (cEnvironment::DoProcesses PROCTYPE_POW, main/cEnvironment.cc:1752)
__device__ __forceinline__ double det_exp2(double x) {
  const double n = floor(x);
  const double t = __dmul_rn(__dsub_rn(x, n), 0.6931471805599453094);
  double y = 1.0;
  for (int k = 22; k >= 1; k--) y = __dadd_rn(1.0, __dmul_rn(y, __ddiv_rn(t, (double)k)));
  return ldexp(y, (int)n);
}

__device__ __forceinline__ double pow_int(double q, int64_t n) {
  double r = 1.0, b = q;
  while (n) { if (n & 1) r = __dmul_rn(r, b); b = __dmul_rn(b, b); n >>= 1; }
  return r;
}
// 1/k for k = 1..64 (oracle INV_K)
__constant__ const double INV_K[65] = {0.0,
  1.0 / 1, 1.0 / 2, 1.0 / 3, 1.0 / 4, 1.0 / 5, 1.0 / 6, 1.0 / 7, 1.0 / 8, 1.0 / 9, 1.0 / 10, 1.0 / 11, 1.0 / 12,
  1.0 / 13, 1.0 / 14, 1.0 / 15, 1.0 / 16, 1.0 / 17, 1.0 / 18, 1.0 / 19, 1.0 / 20, 1.0 / 21, 1.0 / 22, 1.0 / 23,
  1.0 / 24, 1.0 / 25, 1.0 / 26, 1.0 / 27, 1.0 / 28, 1.0 / 29, 1.0 / 30, 1.0 / 31, 1.0 / 32, 1.0 / 33, 1.0 / 34,
  1.0 / 35, 1.0 / 36, 1.0 / 37, 1.0 / 38, 1.0 / 39, 1.0 / 40, 1.0 / 41, 1.0 / 42, 1.0 / 43, 1.0 / 44, 1.0 / 45,
  1.0 / 46, 1.0 / 47, 1.0 / 48, 1.0 / 49, 1.0 / 50, 1.0 / 51, 1.0 / 52, 1.0 / 53, 1.0 / 54, 1.0 / 55, 1.0 / 56,
  1.0 / 57, 1.0 / 58, 1.0 / 59, 1.0 / 60, 1.0 / 61, 1.0 / 62, 1.0 / 63, 1.0 / 64};
// Binomial(n, p) from one 32-bit word h (oracle binom_draw: inversion below a
// mean of 6 on the smaller side, else normal with the binomial's skew, z the
// centred, scaled sum of 4 16-bit uniforms)
__device__ __forceinline__ int64_t binom_draw(int64_t n, double p, uint32_t h) {
  if (n <= 0 || !(p > 0.0)) return 0;
  if (p >= 1.0) return n;
  const bool flip = p > 0.5;
  const double pp = flip ? __dsub_rn(1.0, p) : p, q = __dsub_rn(1.0, pp);
  const double mean = __dmul_rn((double)n, pp);
  int64_t k;
  if (mean < 6.0) {
    const double u = __dmul_rn(__dadd_rn((double)h, 0.5), 2.3283064365386962890625e-10);
    const double r = __ddiv_rn(pp, q);
    double f = pow_int(q, n);
    double F = f;
    k = 0;
    while (F < u && k < n && k < 64) {
      f = __dmul_rn(__dmul_rn(f, __dmul_rn((double)(n - k), r)), INV_K[k + 1]);
      k++;
      F = __dadd_rn(F, f);
    }
  } else {
    uint32_t x = lowbias32(h + 0x9E3779B9U);
    uint32_t sum = (x & 0xFFFFu) + (x >> 16);
    x = lowbias32(x + 0x9E3779B9U);
    sum += (x & 0xFFFFu) + (x >> 16);
    const double z = __dmul_rn(__dsub_rn(__dmul_rn(__dadd_rn((double)sum, 2.0), 1.52587890625e-05), 2.0),
                               1.7320508075688772);
    const double sd = __dsqrt_rn(__dmul_rn(mean, q));   // IEEE, correctly rounded (oracle std::sqrt)
    const double skew = __dmul_rn(__dmul_rn(__dsub_rn(q, pp), __dsub_rn(__dmul_rn(z, z), 1.0)), 0.16666666666666666);
    const double v = __dadd_rn(__dadd_rn(__dadd_rn(mean, __dmul_rn(sd, z)), skew), 0.5);
    k = v < 1.0 ? 0 : (int64_t)floor(v);
    if (k > n) k = n;
  }
  return flip ? n - k : k;
}
// the word of scheduler-tree node `node` in update u (oracle node_draw)
#define SALT_TOP 0x7A11C0DEu
#define SALT_BLOCK 0x51CEB10Cu
#define SALT_NEWBORN 0x4E3B0A17u
__device__ __forceinline__ uint32_t node_draw(uint32_t slo, uint32_t shi, uint32_t update, uint32_t salt,
                                              uint64_t node) {
  return lowbias32(lowbias32(lowbias32(update * 0x85EBCA6BU + shi) ^ (uint32_t)node ^ salt) +
                   (uint32_t)(node >> 32) + slo);
}
// a merit the scheduler can weigh: finite and not negative (NaN, -x and inf
// are never scheduled; large finite merits of multiplicative environments are)
__device__ __forceinline__ bool merit_ok(double m) { return m >= 0.0 && m <= 1.7976931348623157e308; }
// the scheduler weight of a living organism (oracle sched_weight): the same
// in k_merit_partial's partials and k_allot's leaves; at most 2^990, so that
// the scheduler's sums over up to 2^33 organisms stay finite
#define WEIGHT_CAP 0x1p990
__device__ __forceinline__ double sched_weight(double merit, uint32_t ctl) {
  if (!merit_ok(merit)) return 0.0;
  const uint32_t hs = CTL_HS(ctl);
  const double w = hs ? __dmul_rn(merit, __dadd_rn(1.0, __dmul_rn((double)hs, 1.0 / 65536.0))) : merit;
  return merit_ok(w) ? fmin(w, WEIGHT_CAP) : 0.0;
}

// CalcSizeMerit (main/cPhenotype.cc:1760-1816)
__device__ __forceinline__ int size_merit(int method, int base_const, int glen, int copied, int exe) {
  int s;
  switch (method) {
    case 1: return copied;
    case 2: return exe;
    case 3: return glen;
    case 4: s = glen; if (s > copied) s = copied; if (s > exe) s = exe; return s;
    case 5: s = glen; if (s > copied) s = copied; if (s > exe) s = exe;
            return (int)sqrt((double)s);
    default: return base_const;
  }
}
__device__ __forceinline__ int calc_size_merit(const DevWorld& W, int glen, int copied, int exe) {
  return size_merit(W.base_merit_method, W.base_const_merit, glen, copied, exe);
}
// a value the compiler must keep (in an SGPR, or spilled) rather than
// re-load from its invariant source at each use
#define OPQ(x) asm("" : "+s"(x))

__device__ __forceinline__ void count_add(const DevWorld& W, int slot, unsigned long long v) {
  atomicAdd(&W.counters[(blockIdx.x & (NSHARD - 1)) * CNT_STRIDE + slot], v);
}

// LDS size classes of k_interpret (bytes of tape per lane)
// (a block of class S uses 64 x tape_stride(S) B of LDS for tapes; class 0
// holds nothing else: 64 x 320 B = 20 KiB, so 8 one-wave blocks fill a CU's
// 160 KiB -- as many as its ~216 VGPRs admit.  A 316-B stride (79 dwords:
// equal offsets of the 64 lanes in 64 banks) cut the bank conflicts from 47
// to 22 % of LDS cycles but needs dword LDS-DMA staging: class 0 1.12 ->
// 1.50 ms per launch, A/B on one box, profiles/r04c_*).  A split
// slot -- 208 sites in LDS, the rest in the HBM tape, 13 KiB per wave -- for 3
// waves per SIMD was bit-exact but slower, 1.36 against 1.02 ms: 3 waves cap
// the kernel at 168 VGPRs and the spills land in the loop (profiles/r04k_*)
#define CLASS0_SIZE 320
#define CLASS1_SIZE 768
#define CLASS2_SIZE 1536
#define CLASS3_SIZE 2048
__device__ __forceinline__ int class_of(int need) {
  return need <= CLASS0_SIZE ? 0 : (need <= CLASS1_SIZE ? 1 : (need <= CLASS2_SIZE ? 2 : 3));
}
// tape capacity an organism may need this slice: its memory, or the size
// h-alloc would grow it to when it has not allocated yet
__device__ __forceinline__ int need_of(int m, uint32_t ctl, double size_range) {
  if (ctl & CTL_MAL) return m;
  const int grown = m + min((int)(size_range * m), AVGPU_MAX_GENOME - m);
  return grown > m ? grown : m;
}

// ---------------------------------------------------------------------------
// host-side launchers (defined next to their kernels)
struct LaunchInfo {
  hipStream_t stream;
  hipEvent_t ev0, ev1;
  bool timed;
};

// class 0 runs densely over cells [first, first+count); classes 1..3 over their lists
// after_class[k] (optional): event recorded after the class-k launch
// dW: device copy of W (avgpu_world::push_world)
// aux (optional): three streams on which the classes 1..3 of k_allot's
// lists run concurrently with class 0 (ev_fork / ev_join[3] order them)
void launch_serial_update(const DevWorld& W, const DevWorld* dW, hipStream_t s);
void launch_serial_post(const DevWorld& W, hipStream_t s, double* stats);
void launch_reset_counts(const DevWorld& W, hipStream_t s);
void launch_interpret_classes(const DevWorld& W, const DevWorld* dW, int mode, hipStream_t s,
                              int64_t first, int64_t count, int* launches,
                              hipEvent_t* after_class = nullptr, bool sorted = false,
                              hipStream_t* aux = nullptr, hipEvent_t ev_fork = nullptr,
                              hipEvent_t* ev_join = nullptr);
// class-0 windows: k_allot's budgets sorted (descending) inside windows of
// SORT_WIN cells, so that a wave's 64 organisms get similar time slices
#define SORT_WIN 32768
// k_allot_sort's buckets: budgets 0 .. SORT_BUCKETS-3 (larger ones share the
// last of them), then one bucket for the window's cells that are not class 0
#define SORT_BUCKETS 258
bool class_timing_all();   // AVGPU_CLASS_TIMING (interp.hip)
bool mix_lists();          // list classes inside class 0's launch (interp.hip; AVGPU_NO_MIX=1 off)
void launch_age_tick(const DevWorld& W, hipStream_t s);
// sub-update `sub` of `nsub` (avgpu_cfg.sub_updates): the
// resources step and the update's counters are reset at sub 0 only; the key
// of the scheduler's node draws is update x nsub + sub (the caller's `update`)
void launch_world_begin(const DevWorld& W, hipStream_t s, double* d_totals, double* d_scratch,
                        hipEvent_t lists_ready, uint32_t update, int sub = 0, int nsub = 1);
// a sub-update's share of the update's picks n (oracle sub_share)
__host__ __device__ __forceinline__ long long sub_share(long long n, int s, int K) {
  return K == 1 ? n : (n * (s + 1)) / K - (n * s) / K;
}
void launch_world_pre(const DevWorld& W, hipStream_t s, double* d_totals, double* d_scratch, hipEvent_t lists_ready,
                      uint32_t update, bool reset = true);
void launch_tile_pre(const DevWorld& W, hipStream_t s, const double* d_gathered, int ntiles, double* d_totals,
                     hipEvent_t lists_ready, uint32_t update, int sub = 0, int nsub = 1);
// allotment draw of organism (lo, hi) in update u (oracle allot_draw)
__device__ __forceinline__ uint32_t allot_draw(uint32_t lo, uint32_t hi, uint32_t update) {
  return lowbias32(lowbias32(update * 0x85EBCA6BU + hi) ^ lo ^ 0x27D4EB2FU);
}
void launch_resources_begin(const DevWorld& W, hipStream_t s);
void launch_resources_end(const DevWorld& W, hipStream_t s);
void launch_resources_pack(const DevWorld& W, hipStream_t s);
bool res_stepped(const DevWorld& W);   // launch_resources_begin wrote res_amount_alt
void launch_resources_settle(const DevWorld& W, hipStream_t s, const unsigned long long* sum);
// placement and activation of batch step `sub` of `nsub` (key: its scheduler
// key), the newborns listed for the newborn pass; then launch_world_end
// pred_out (coherent mapped host memory, the update's last step): the
// predictor, its organisms and divide count, then pred_seq at system scope
void launch_world_post(const DevWorld& W, hipStream_t s, uint32_t key, int sub, int nsub,
                       long long* pred_out = nullptr, long long pred_seq = 0);
void launch_world_end(const DevWorld& W, hipStream_t s, double* d_stats, bool eager);
// the newborn pass of a batch step (interp.hip): the organisms k_activate listed
void launch_newborns(const DevWorld& W, const DevWorld* dW, hipStream_t s);
// the update's statistics into d_stats (k_stats_partial + k_stats_final)
void launch_stats(const DevWorld& W, hipStream_t s, double* d_stats);
void launch_classify_uniform(const DevWorld& W, hipStream_t s, int64_t first, int64_t count,
                             const int32_t* d_budget, int32_t uniform);
void launch_set_orgs(const DevWorld& W, hipStream_t s, int64_t first, int64_t count,
                     const uint8_t* d_codes, const int32_t* d_offsets, const int32_t* d_lens,
                     const double* d_merits, const int32_t* d_inputs, int deterministic);
void launch_get_states(const DevWorld& W, hipStream_t s, int64_t first, int64_t count,
                       avgpu_cpu_state* d_states, uint8_t* d_codes, int cap);
void launch_set_states(const DevWorld& W, hipStream_t s, int64_t first, int64_t count, const avgpu_cpu_state* in,
                       const uint8_t* codes, int cap);
void launch_state_digest(const DevWorld& W, hipStream_t s, int64_t first, int64_t count, uint64_t* d_out);
void launch_get_census(const DevWorld& W, hipStream_t s, int64_t first, int64_t count, avgpu_census* d_out);
void launch_merit_total(const DevWorld& W, hipStream_t s, double* d_totals, double* d_scratch);
// strip tiles
void launch_tile_partials(const DevWorld& W, hipStream_t s, double* d_out, int reset);
void launch_tile_after_interpret(const DevWorld& W, hipStream_t s);
void launch_tile_place(const DevWorld& W, hipStream_t s, int round, int phase, uint32_t key, int sub, int nsub);
void launch_tile_finish(const DevWorld& W, hipStream_t s, uint32_t key, int sub, int nsub);
