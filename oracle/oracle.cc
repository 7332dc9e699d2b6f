// oracle/oracle.cc -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the fortunalab/avida hot path (heads-CPU execution,
// test CPU, divide/mutation, logic-9 tasks, batch world update, and the
// reference-style serial world loop used as the CPU baseline).  It is the
// parity checker for the HIP path in avida_amd/csrc and is never linked into,
// called by, or shipped with the product.  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load liboracle.so.
//
// The reference itself cannot be built here (libs/apto is an empty submodule;
// see DESIGN.md "Oracle"), so this file restates its algorithms line by line.
// Citations are avida-core/source/<path>:<line> of /root/reference.
// Pinning: tests/test_oracle_golden.py checks it against the reference's own
// RNG-free golden vectors (tests/_analyze_detail_all/expected/data/
// detail-recalc.dat, 1794 genomes; the default-heads ancestor 389/97/100).
//
// RNG: Apto::RNG::AvidaRNG is absent, so (like the product) the oracle uses the
// project's counter-based stream spec (DESIGN.md "RNG spec"); RNG-dependent
// trajectories are therefore compared statistically to the reference, and
// bit-exactly only between this oracle and the GPU path.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off).

#include "../include/avida_gpu.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <deque>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// RNG spec.  Every draw is a uniform u in [0, 1) with the
// reference's RNG interface on top of it (Apto::RNG: P(p) = u < p, GetUInt(n) =
// GetInt(n) = floor(u n), GetDouble(x) = u x).  u comes from the organism's
// COUNTER stream (32-bit draws x, u = x 2^-32, so P(p) = x < ceil(p 2^32) and
// GetUInt(n) = (x n) >> 32 exactly) or, in RECORDED mode
// (avgpu_set_rng_mode), from its segment of a host-supplied array of doubles.
static inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// a probability and its COUNTER-mode threshold ceil(p 2^32) (P(p) = u < p)
struct Prob {
  double p = 0.0;
  uint64_t th = 0;
};
static inline Prob make_prob(double p) {
  Prob r;
  r.p = p;
  if (!(p > 0.0)) r.th = 0;
  else if (p >= 1.0) r.th = 1ULL << 32;
  else r.th = (uint64_t)std::ceil(p * 4294967296.0);
  return r;
}
static int64_t g_rec_over = 0;   // RECORDED draws past the end of a segment
struct Stream {
  uint32_t lo = 0, hi = 0, ctr = 0;
  const double* rec = nullptr;   // RECORDED: this organism's segment
  int64_t rec_len = 0;
  uint32_t next() {
    uint32_t a = lowbias32(ctr * 0x9E3779B9U + hi);
    uint32_t b = lowbias32(a ^ lo);
    ++ctr;
    return b;
  }
  double rd() {
    const uint32_t k = ctr++;
    if ((int64_t)k < rec_len) return rec[k];
    g_rec_over++;
    return 0.0;
  }
  // Apto::RNG::GetUInt(n) / GetInt(n): floor(u n)
  uint32_t uint_below(uint32_t n) {
    if (rec) { const uint32_t v = (uint32_t)(rd() * (double)n); return v < n ? v : n - 1; }
    return (uint32_t)(((uint64_t)next() * n) >> 32);
  }
  // a uniform double: the recorded value, or the counter draw times 2^-32
  double u() {
    if (rec) return rd();
    return (double)next() * 2.3283064365386963e-10;
  }
  // Apto::RNG::GetRandPoisson(mean) (Apto is absent; restated as the classic
  // product-of-uniforms method of Avida's own cRandom: multiply uniforms until
  // the product falls below exp(-mean), capped at 4096 events); L = exp(-mean)
  // is computed once by the host (the device gets the same double)
  uint32_t poisson(double L) {
    double x = u();
    uint32_t k = 0;
    while (x >= L && k < 4096) { x = x * u(); k++; }
    return k;
  }
  // Apto::RNG::P(p): u < p
  bool p(const Prob& q) {
    if (rec) return rd() < q.p;
    return (uint64_t)next() < q.th;
  }
};
// Allotment draw of organism (lo, hi) in update u: a stateless hash, so the
// organism's own stream carries exactly the reference's ctx.GetRandom() calls
// (the reference's scheduler draws from its own generator,
// main/cPopulation.cc:7341-7346)
static inline uint32_t allot_draw(uint32_t lo, uint32_t hi, uint32_t update) {
  return lowbias32(lowbias32(update * 0x85EBCA6BU + hi) ^ lo ^ 0x27D4EB2FU);
}
static inline void derive_key(uint32_t a_lo, uint32_t a_hi, uint32_t x, uint32_t y,
                              uint32_t* lo, uint32_t* hi) {
  *lo = lowbias32(lowbias32(x ^ a_lo) + y);
  *hi = lowbias32(lowbias32(y ^ a_hi) + x + 0x632BE5ABU);
}

// ---------------------------------------------------------------------------
// heads_default handler ids (include/avida_gpu.h enum avgpu_handler)
enum { H_NOP_A = 0, H_NOP_B, H_NOP_C, H_IF_N_EQU, H_IF_LESS, H_POP, H_PUSH, H_SWAP_STK,
       H_SWAP, H_SHIFT_R, H_SHIFT_L, H_INC, H_DEC, H_ADD, H_SUB, H_NAND, H_IO, H_H_ALLOC,
       H_H_DIVIDE, H_H_COPY, H_H_SEARCH, H_MOV_HEAD, H_JMP_HEAD, H_GET_HEAD, H_IF_LABEL,
       H_SET_FLOW };

const int INST_ERROR = 255;  // cInstSet::GetInstError (cpu/cHeadCPU.h:167-170)
const int REG_AX = 0, REG_BX = 1, REG_CX = 2;
const int HEAD_IP = 0, HEAD_READ = 1, HEAD_WRITE = 2, HEAD_FLOW = 3;  // cpu/nHardware.h:32
const int NUM_NOPS = 3;      // cpu/cHardwareCPU.h:64

// cCPUMemory flag masks (cpu/cCPUMemory.h:31-37)
const uint8_t F_COPIED = 0x01, F_MUTATED = 0x02, F_EXECUTED = 0x04, F_COPYMUT = 0x10;

struct InstSet {
  int n = 0;
  int handler[256];
  int nopmod[256];   // -1 if not a nop (cInstSet::IsNop / GetNopMod, cpu/cInstSet.h:127-131)
  int64_t cum[256];  // cOrderedWeightedIndex cumulative weights (tools/cOrderedWeightedIndex.cc:43-50)
  int64_t total = 0;
  bool is_nop(int op) const { return op >= 0 && op < n && nopmod[op] >= 0; }
  uint64_t nomut = 0;   // NO_MUT_INSTS: the ops (bit per op) copy mutations leave alone
  bool no_mut(int op) const { return op >= 0 && op < 64 && ((nomut >> op) & 1ull); }
  // cInstSet::GetRandomInst (cpu/cInstSet.cc:83-88) on the project RNG
  int random_inst(Stream& s) const {
    uint32_t r = s.uint_below((uint32_t)total);
    for (int i = 0; i < n; i++) if (cum[i] > (int64_t)r) return i;
    return n - 1;
  }
};

struct Reaction {
  avgpu_reaction r;
  double mult;  // pow: 2^(max_number*value) ; mult: max_number*value
  double add;
};

// cCodeLabel (cpu/cCodeLabel.h:76-100): nop sequence, AddNop ignores overflow.
struct Label {
  int8_t nops[AVGPU_MAX_LABEL];
  int size = 0;
  void clear() { size = 0; }
  void add(int n) { if (size < AVGPU_MAX_LABEL) nops[size++] = (int8_t)n; }
  void rotate(int rot, int base) {
    for (int i = 0; i < size; i++) { nops[i] += rot; if (nops[i] >= base) nops[i] -= base; }
  }
  bool eq(const Label& o) const {
    if (size != o.size) return false;
    for (int i = 0; i < size; i++) if (nops[i] != o.nops[i]) return false;
    return true;
  }
};

// cCPUStack (cpu/cCPUStack.h:60-90)
struct CPUStack {
  int s[AVGPU_STACK_SIZE];
  int sp = 0;
  void clear() { for (int i = 0; i < AVGPU_STACK_SIZE; i++) s[i] = 0; sp = 0; }
  void push(int v) { sp = (sp == 0) ? AVGPU_STACK_SIZE - 1 : sp - 1; s[sp] = v; }
  int pop() { int v = s[sp]; s[sp] = 0; sp++; if (sp == AVGPU_STACK_SIZE) sp = 0; return v; }
};

// tBuffer<int> (tools/tBuffer.h:32-84)
struct Buffer {
  int data[3] = {0, 0, 0};
  int cap = 1, offset = 0, total = 0;
  void clear() { offset = 0; total = 0; }
  void add(int v) { data[offset] = v; total++; offset++; offset %= cap; }
  int operator[](int i) const { int idx = offset - i - 1; if (idx < 0) idx += cap; return data[idx]; }
  int num_stored() const { return total <= cap ? total : cap; }
};

struct Org {
  bool alive = false;
  // hardware (cpu/cHardwareCPU.h:61-129)
  std::vector<uint8_t> mem, flg;
  int reg[3];
  int head[4];
  CPUStack stk[2];       // [0] thread-local stack, [1] m_global_stack
  int cur_stack = 0;
  Label read_label, next_label;
  bool mal_active = false;
  bool advance_ip = true;
  // organism (main/cOrganism.h)
  std::vector<uint8_t> genome;  // m_initial_genome (birth genome)
  uint64_t gkey_restored = 0;    // genotype key carried by a checkpoint (orc_set_genotype_keys)
  Buffer input_buf, output_buf;
  int input_ptr = 0;
  int max_executed = 0;
  int inputs[3];
  // phenotype (main/cPhenotype.h)
  int cpu_cycles_used = 0, time_used = 0, gestation_start = 0, gestation_time = 0;
  int num_divides = 0, generation = 0;
  int genome_length = 0, copied_size = 0, child_copied_size = 0, executed_size = 0;
  int errors = 0;
  double cur_bonus = 1.0, merit = 0.0, fitness = 0.0;
  int cur_task[AVGPU_MAX_REACTIONS], last_task[AVGPU_MAX_REACTIONS];
  int cur_react[AVGPU_MAX_REACTIONS];
  bool to_die = false;
  bool spec_die = false;   // serial world: died in a speculative step (m_spec_die), removed when next picked
  // batch-world bookkeeping
  Stream rng;
  double credit = 0.0;
  int age = 0;           // cPhenotype::age during the update (BIRTH_METHOD 1 / 2; age_tick)
  uint32_t hstart = 0;   // head start: 2^16 - birth time, for the first allotment after birth (sched_weight)
  int spec_count = 0;
  // test-CPU outputs
  std::vector<uint8_t> offspring;
  std::string exec_flags_at_divide;
};

struct Birth {
  int64_t parent;
  uint32_t seq;
  std::vector<uint8_t> genome;
  double merit;
  int generation;
  int child_copied, executed, gestation_time;
  double fitness;
  int last_task[AVGPU_NUM_LOGIC_TASKS];   // SetupOffspring copies the parent's (main/cPhenotype.cc:447)
  Stream rng;     // the child's stream
  int64_t target = -1;
  bool placed = false;
  uint32_t t = 0;   // birth time in the update, 1/2^16 (birth_time)
};

struct World {
  avgpu_cfg cfg;
  int64_t ncells = 0;
  InstSet is;
  std::vector<Reaction> react;
  int num_tasks_in_env = 0;
  std::vector<Org> orgs;
  Prob p_copy_mut, p_copy_ins, p_copy_del, p_copy_uni, p_copy_slip;
  Prob p_div_mut, p_div_ins, p_div_del, p_div_slip, p_div_uni;
  Prob p_div_site;           // DIV_MUT_PROB (per-site substitutions on divide)
  Prob p_par_site;           // PARENT_MUT_PROB (per-site substitutions in the parent)
  Prob p_par_ins, p_par_del; // PARENT_INS_PROB, PARENT_DEL_PROB
  Prob p_dsite[5];           // DIV_INS_PROB, DIV_DEL_PROB, DIV_UNIFORM_PROB, DIV_SLIP_PROB, DIV_TRANS_PROB (per site)
  Prob p_div_trans;          // DIVIDE_TRANS_PROB
  double pois_L[5] = {0, 0, 0, 0, 0};   // + DIVIDE_POISSON_TRANS_MEAN   // exp(-DIVIDE_POISSON_{SLIP,MUT,INS,DEL}_MEAN); 0 = off
  std::vector<double> rec;   // RECORDED mode: the host's stream (organisms point into it)
  // batch world
  std::vector<Birth> births;
  int64_t update = 0;
  int64_t cum_insts = 0, cum_births = 0;
  avgpu_update_stats stats;
  int64_t step_insts = 0;
  // multi-GPU style overrides (unused by the oracle tests unless set)
  bool have_global = false;
  double global_merit = 0.0;
  int64_t global_orgs = 0;
  Stream global_rng;   // serial world: the scheduler's own stream (main/cPopulation.cc:7341-7346)
  Stream ctx_rng;      // serial world: the context stream every ctx.GetRandom() draw comes from
  std::vector<double> srec_sched, srec_ctx;   // their recorded values (avgpu_set_serial_streams)
  std::vector<uint8_t> face;   // serial world: each cell's connection-list rotation (cPopulationCell::Rotate)
  std::vector<int64_t> soup_cells;   // serial world, BIRTH_METHOD 4: cPopulation::empty_cell_id_array
  std::deque<int64_t> reaper;        // serial world, BIRTH_METHOD 5: cPopulation::reaper_queue (front: newest)
  bool reaper_init = false;
  // strip tiles (avgpu_set_tile): rows [row0, row0+rows) of a world_x x
  // global_rows world; occ / claim / owner carry two ghost rows after n
  int64_t row0 = 0, rows = 0, global_rows = 0, cell0 = 0;
  bool tiled = false;
  int64_t r_arena = 0;
  uint8_t* h_send[2] = {nullptr, nullptr};
  uint8_t* h_recv[2] = {nullptr, nullptr};
  uint8_t* r_send[2] = {nullptr, nullptr};
  uint8_t* r_recv[2] = {nullptr, nullptr};
  // per-update placement state of the tiled path
  std::vector<uint8_t> occ;
  std::vector<uint64_t> claim_r[4];   // each placement round's claims
  std::vector<int64_t> tgt_r[4];      // each record's target in each round it picked in
  std::vector<int64_t> owner;     // birth index, -1 none, remote_owner(m, t) won by a halo birth
  std::vector<uint32_t> killt;    // per cell: 2^16 - the earliest kill pick's birth time, 0 none
  std::vector<uint64_t> prio;     // each record's claim key in its current round
  std::vector<int8_t> bstate;     // BS_* (place_pick)
  std::vector<int64_t> empty_cells;   // BIRTH_METHOD 4: the cells empty at placement start, ascending
  int64_t t_insts = 0, t_deaths = 0, t_divides = 0, t_slices = 0, t_born = 0, t_dropped = 0;
  uint32_t sched_key = 0;  // the scheduler's node-draw key: update x K + sub-update (sub_share)
  int64_t t_oversize = 0;   // offspring longer than AVGPU_MAX_GENOME after a slip (dropped at the divide)
  int64_t t_memcap = 0;     // copy insertions past AVGPU_MAX_GENOME sites / removals from one site (skipped)
  int64_t t_overwritten = 0;   // offspring placed, then killed by a later birth into the same cell
  int64_t t_cancelled = 0;     // records whose parent's cell got an offspring before their divide
  std::vector<int32_t> last_budget;   // the last allotment's budgets (orc_last_budgets, diagnostics)
  int64_t t_placed = 0;        // strip tiles: this tile's own winners activated (avgpu_tile_place(3, 2))
  // resources (avgpu_load_resources): literal restatement of cResourceCount /
  // cSpatialResCount, stepped once per update
  std::vector<avgpu_resource> res;
  std::vector<avgpu_cell_resource> res_cells;
  std::vector<std::vector<double>> res_amount, res_delta;   // spatial grids (empty for global)
  std::vector<double> res_global, res_decay100, res_inflow100, res_decay99, res_inflow99;
  bool res_first = false;   // the first update after the load: no spatial step, 9999 global steps
  std::vector<uint64_t> res_cons;
  // strip tiles: edge rows of the spatial amounts, [slot][X] (0 = above, 1 = below)
  std::vector<int> res_slot;   // resource -> spatial slot or -1
  int n_spatial = 0;
  double* rs_send[2] = {nullptr, nullptr};
  double* rs_recv[2] = {nullptr, nullptr};
  // the birth-step model: each cell's depletable consumption
  // in this batch step's main pass, [resource][cell] (credited back when an
  // offspring replaces the organism); the step's newborns (cell, birth time)
  std::vector<std::vector<double>> cons_cell;
  std::vector<std::pair<int64_t, uint32_t>> newborns;
  // the adaptive sub-step predictor: the last batch step's sum
  // (2^-20 units) and the living organisms it was relative to; the batch
  // steps the last update ran
  int64_t pred_acc = 0, pred_n = 0;
  int64_t pred_bin[4] = {0, 0, 0, 0};   // the divide count by quarter of the update (pred_term)
  int64_t last_k = 1;
  // the picks the last batch step's newborns took beyond what the organisms
  // they replaced left (newborn_pass), taken from the next step's allotment;
  // each cell's instructions in this step's main pass
  int64_t carry_rem = 0, carry_new = 0;   // the carry not yet taken (all strips alike); this step's own
  int64_t t_wasted = 0;                    // the replaced organisms' instructions after their newborns' times
  std::vector<int32_t> ran;
  // strip tiles: the current batch step (avgpu_tile_begin_step) and the
  // update's counts summed over its steps
  int step_sub = 0, step_k = 1;
  int64_t step_uds = 0;
  int64_t upd_ud = 0;      // the update's picks UD, fixed at its first batch step
  int req_task = -1, imm_task = -1;   // REQUIRED_TASK / IMMUNITY_TASK as avgpu_task ids (orc_load_env)
  double step_total = 0.0;
  int64_t acc_placed = 0, acc_dropped = 0, acc_insts = 0, acc_deaths = 0, acc_divides = 0, acc_slices = 0;
  int64_t acc_overwritten = 0, acc_cancelled = 0;
};

thread_local std::string g_err;
static int g_trace = getenv("ORACLE_TRACE") ? 1 : 0;
static int64_t g_op_hist[64];   // executed instructions per handler (instruction-mix statistics)
static inline bool tracks_age(const World& w) { return w.cfg.birth_method == 1 || w.cfg.birth_method == 2; }
int fail(int code, const std::string& msg) { g_err = msg; return code; }

// cHeadCPU::Adjust / fullAdjust (cpu/cHeadCPU.h:63, cpu/cHeadCPU.cc:27-50)
static inline int adjust(int pos, int size) {
  if (pos >= 0 && pos < size) return pos;
  if (size == 0 || pos < 0) return 0;
  if (pos < 2 * size) return pos - size;
  return pos % size;
}
static inline int wrap_add(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }

// 2^x from IEEE adds / multiplies only (the device's det_exp2, device.h):
// cEnvironment::DoProcesses PROCTYPE_POW (main/cEnvironment.cc:1752) uses
// pow(2, bonus); this restatement is within 1 ulp of it and identical on both sides.
static double det_exp2(double x) {
  const double n = std::floor(x);
  const double t = (x - n) * 0.6931471805599453094;
  double y = 1.0;
  for (int k = 22; k >= 1; k--) y = 1.0 + y * (t / (double)k);
  return std::ldexp(y, (int)n);
}

struct Exec {
  World& w;
  Org& o;
  int mode;
  bool stop = false;   // TEST mode: gestation finished
  // the newborn pass (newborn_pass): a viable h-divide is not run -- the
  // instruction's cycle is taken back and the slice ends before it
  bool nb_stop = false, nb_halted = false;
  int64_t cur_cell = -1;  // the organism's cell (spatial resources)
  // where the organism's ctx.GetRandom() draws come from: its own stream, or
  // (serial world) the world's single context stream
  Stream* ctx = nullptr;
  Stream& rng() { return ctx ? *ctx : o.rng; }

  int size() const { return (int)o.mem.size(); }
  // cHeadCPU::GetNextInst (cpu/cHeadCPU.h:167-170)
  int next_inst(int pos) const { return (pos + 1 == size()) ? INST_ERROR : o.mem[pos + 1]; }
  void advance_ip() { o.head[HEAD_IP] = adjust(o.head[HEAD_IP] + 1, size()); }

  // FindModifiedRegister / FindModifiedHead (cpu/cHardwareCPU.cc:1622-1672)
  int find_modified(int def) {
    int nx = next_inst(o.head[HEAD_IP]);
    if (w.is.is_nop(nx)) {
      advance_ip();
      def = w.is.nopmod[o.mem[o.head[HEAD_IP]]];
      o.flg[o.head[HEAD_IP]] |= F_EXECUTED;
    }
    return def;
  }
  static int next_reg(int r) { return (r + 1) % 3; }  // FindNextRegister :1676-1679

  // cHardwareCPU::ReadLabel (cpu/cHardwareCPU.cc:1484-1502)
  void read_label() {
    int count = 0;
    o.next_label.clear();
    while (w.is.is_nop(next_inst(o.head[HEAD_IP])) && count < AVGPU_MAX_LABEL) {
      count++;
      advance_ip();
      o.next_label.add(w.is.nopmod[o.mem[o.head[HEAD_IP]]]);
      if (o.next_label.size <= w.cfg.max_label_exe_size) o.flg[o.head[HEAD_IP]] |= F_EXECUTED;
    }
  }

  // FindLabel_Forward (cpu/cHardwareCPU.cc:1219-1295)
  int find_label_forward(const Label& lab, int pos) {
    const int gsize = size();
    int search_start = pos;
    int label_size = lab.size;
    bool found = false;
    pos += label_size;
    while (pos < gsize) {
      if (w.is.is_nop(o.mem[pos])) {
        int start_pos = pos, end_pos = pos + 1;
        while (start_pos > search_start && w.is.is_nop(o.mem[start_pos - 1])) start_pos--;
        while (end_pos < gsize && w.is.is_nop(o.mem[end_pos])) end_pos++;
        int test_size = end_pos - start_pos;
        int max_offset = test_size - label_size + 1;
        int offset;
        for (offset = start_pos; offset < start_pos + max_offset; offset++) {
          int m;
          for (m = 0; m < label_size; m++)
            if (lab.nops[m] != w.is.nopmod[o.mem[offset + m]]) break;
          if (m == label_size) { found = true; break; }
        }
        if (found) { pos = label_size + offset; break; }
        pos = end_pos;
      }
      pos += label_size;
    }
    if (!found) pos = -1;
    return pos;
  }

  // FindLabel(0) (cpu/cHardwareCPU.cc:1177-1212): returns the position of the
  // search head (IP copy when label empty / not found)
  int find_label_from_start() {
    int ip = o.head[HEAD_IP];
    if (o.next_label.size == 0) return ip;
    int found = find_label_forward(o.next_label, 0);
    if (found >= 0) return adjust(found - 1, size());  // search_head.Set(found_pos - 1)
    return ip;
  }

  // cHardwareCPU::Allocate_Main (cpu/cHardwareCPU.cc:1707-1763)
  bool allocate_main(int allocated_size) {
    if (w.cfg.require_allocate && o.mal_active) { o.errors++; return false; }
    if (allocated_size < 1) { o.errors++; return false; }
    const int old_size = size();
    const int new_size = old_size + allocated_size;
    if (new_size > AVGPU_MAX_GENOME || new_size < AVGPU_MIN_GENOME) { o.errors++; return false; }
    const int max_alloc = (int)(old_size * w.cfg.offspring_size_range);
    if (allocated_size > max_alloc) { o.errors++; return false; }
    const int max_old = (int)(allocated_size * w.cfg.offspring_size_range);
    if (old_size > max_old) { o.errors++; return false; }
    o.mem.resize(new_size, 0);   // ALLOC_METHOD 0: new sites are op 0 (Allocate_Default :1698-1705)
    o.flg.resize(new_size, 0);
    if (w.cfg.alloc_method == 2) {  // ALLOC_METHOD_RANDOM (Allocate_Random :1688-1696)
      for (int i = old_size; i < new_size; i++) o.mem[i] = (uint8_t)w.is.random_inst(rng());
    }
    o.mal_active = true;
    return true;
  }

  // CalcSizeMerit (main/cPhenotype.cc:1760-1816)
  int calc_size_merit() const {
    switch (w.cfg.base_merit_method) {
      case 1: return o.copied_size;
      case 2: return o.executed_size;
      case 3: return o.genome_length;
      case 4: { int s = o.genome_length; if (s > o.copied_size) s = o.copied_size;
                if (s > o.executed_size) s = o.executed_size; return s; }
      case 5: { int s = o.genome_length; if (s > o.copied_size) s = o.copied_size;
                if (s > o.executed_size) s = o.executed_size; return (int)std::sqrt((double)s); }
      default: return w.cfg.base_const_merit;
    }
  }

  // cHardwareCPU::Reset -> internalReset + cLocalThread::Reset (cpu/cHardwareCPU.cc:813-900)
  void hw_reset() {
    for (int i = 0; i < 3; i++) o.reg[i] = 0;
    for (int i = 0; i < 4; i++) o.head[i] = 0;
    o.stk[0].clear(); o.stk[1].clear();
    o.cur_stack = 0;
    o.read_label.clear(); o.next_label.clear();
    o.mal_active = false;
  }

  // cPhenotype::DivideReset / TestDivideReset (main/cPhenotype.cc:824-1000, :1064-1180)
  void divide_reset() {
    double base = (double)calc_size_merit();
    if (w.cfg.merit_default_bonus != 0.0) o.cur_bonus = w.cfg.merit_default_bonus;
    o.merit = base * o.cur_bonus;
    if (w.cfg.inherit_merit == 0) o.merit = base;
    o.genome_length = (int)o.genome.size();
    o.gestation_time = o.time_used - o.gestation_start;
    o.gestation_start = o.time_used;
    o.fitness = base * o.cur_bonus / o.gestation_time;   // CalcFitness :1827 (FITNESS_METHOD 0)
    for (int i = 0; i < AVGPU_MAX_REACTIONS; i++) {
      o.last_task[i] = o.cur_task[i];
      o.cur_task[i] = 0;
      o.cur_react[i] = 0;
    }
    o.cur_bonus = w.cfg.default_bonus;
    o.cpu_cycles_used = 0;
    o.errors = 0;
    o.age = 0;   // DivideReset (main/cPhenotype.cc:950)
    o.num_divides++;
    if (mode == AVGPU_MODE_TEST) o.generation++;  // TestDivideReset :1160; world: GENERATION_INC_METHOD 1
    else o.generation++;
  }

  // the op code of nop-C in this instruction set (cInstSet::GetInst("nop-C"))
  uint8_t nop_c_op() const {
    for (int i = 0; i < w.is.n; i++) if (w.is.nopmod[i] == 2) return (uint8_t)i;
    return 2;
  }
  // The scrambled fills' index pick (cpu/cHardwareBase.cc:652-664, :727-739):
  // GetInt(L - i), then the walk over copied_so_far that skips the indices
  // already taken -- the draw-th index not yet copied.
  static int scrambled_index(std::vector<bool>& taken, int draw) {
    int copy_index = draw, test = 0, passed = draw;
    while (passed >= 0) {
      if (taken[test]) copy_index++;
      else passed--;
      test++;
    }
    taken[copy_index] = true;
    return copy_index;
  }

  // cHardwareBase::doSlipMutation (cpu/cHardwareBase.cc:621-694), SLIP_FILL_MODE
  // 0 duplication, 2 random instructions, 3 scrambled duplication, 4 nop-C
  // (1, nop-X, is refused).  The scrambled fill reads genome[to + k] of the
  // sequence being filled: [to, from) is never written by the fill, so that is
  // the copy's.
  void slip_mutation(std::vector<uint8_t>& g, Stream& r) {
    const std::vector<uint8_t> copy = g;
    const int size = (int)copy.size();
    const int from = (int)r.uint_below((uint32_t)size + 1);
    const int to = (from == 0) ? (int)r.uint_below((uint32_t)size) : (int)r.uint_below((uint32_t)size + 1);
    int ins = from - to;
    g.resize(size + ins);
    lmax = std::max(lmax, (int)g.size());
    const int mode = w.cfg.slip_fill_mode;
    std::vector<bool> taken(ins > 0 ? ins : 0, false);
    for (int i = 0; i < ins; i++) {
      if (mode == 2) g[from + i] = (uint8_t)w.is.random_inst(r);
      else if (mode == 3) g[from + i] = g[to + scrambled_index(taken, (int)r.uint_below((uint32_t)(ins - i)))];
      else if (mode == 4) g[from + i] = nop_c_op();
      else g[from + i] = copy[to + i];
    }
    if (ins < 0) ins = 0;
    for (int i = ins; i < size - to; i++) g[from + i] = copy[to + i];
  }

  // cHardwareBase::doTransMutation (cpu/cHardwareBase.cc:700-760), TRANS_FILL_MODE
  // 0 duplication, 1 scrambled: copy[to, from) is inserted at ins_loc when
  // from > to, copy[ins_loc, ins_loc + to - from) is cut when from < to.  The
  // scrambled fill reads genome[to + k] of the sequence being filled, which may
  // be a site this fill already wrote (ins_loc inside [to, from)).
  void trans_mutation(std::vector<uint8_t>& g, Stream& r) {
    const std::vector<uint8_t> copy = g;
    const int size = (int)copy.size();
    const int from = (int)r.uint_below((uint32_t)size + 1);
    const int to = (from == 0) ? (int)r.uint_below((uint32_t)size) : (int)r.uint_below((uint32_t)size + 1);
    const int ins = from - to;
    g.resize(size + ins);
    lmax = std::max(lmax, (int)g.size());
    const int ins_loc = (int)r.uint_below((uint32_t)size + 1);
    if (ins > 0) {
      if (w.cfg.trans_fill_mode == 1) {
        std::vector<bool> taken(ins, false);
        for (int i = 0; i < ins; i++)
          g[ins_loc + i] = g[to + scrambled_index(taken, (int)r.uint_below((uint32_t)(ins - i)))];
      } else {
        for (int i = 0; i < ins; i++) g[ins_loc + i] = copy[to + i];
      }
      for (int i = ins_loc; i < size; i++) g[i + ins] = copy[i];
    } else if (ins < 0) {
      for (int i = ins_loc; i < (int)g.size(); i++) g[i] = copy[i - ins];
    }
  }

  // Divide_DoMutations (cpu/cHardwareBase.cc:296-569) in the reference's order
  // of draws: TestDivideSlip always draws (main/cMutationRates.h:128);
  // TestDivideMut / Ins / Del always draw (:121-123; the size limits are
  // tested after the draw); TestDivideUniform and every variable-count kind --
  // Poisson (:318-435), per site (:323-327, :447-503), translocations
  // (:331-343) -- draw only at a non-zero rate or mean; the parent's own
  // substitutions, insertions and deletions (:509-563) come last, in
  // divide() on the parent's memory.  LGT (:345-357) is refused by the
  // library (avgpu_check_cfg) and never reaches this code.
  int lmax = 0;   // the longest the offspring got during its divide mutations
  void divide_mutations(std::vector<uint8_t>& child) {
    Stream& r = rng();
    lmax = (int)child.size();
    int max_g = w.cfg.max_genome_size; if (!max_g || max_g > AVGPU_MAX_GENOME) max_g = AVGPU_MAX_GENOME;
    int min_g = w.cfg.min_genome_size; if (!min_g || min_g < AVGPU_MIN_GENOME) min_g = AVGPU_MIN_GENOME;
    // NumDividePoisson* draws only at a non-zero mean (main/cMutationRates.h:137-144)
    auto npois = [&](int k) -> uint32_t { return w.pois_L[k] > 0.0 ? r.poisson(w.pois_L[k]) : 0u; };
    // doUniformMutation (cpu/cHardwareBase.cc:572-595): op codes, not weighted
    auto uniform_mutation = [&]() {
      const int n_ops = w.is.n;
      const int mut = (int)r.uint_below((uint32_t)(2 * n_ops + 1));
      if (mut < n_ops) {
        child[r.uint_below((uint32_t)child.size())] = (uint8_t)mut;
      } else if (mut == n_ops) {
        if ((int)child.size() != min_g) child.erase(child.begin() + r.uint_below((uint32_t)child.size()));
      } else if ((int)child.size() != max_g) {
        const uint32_t site = r.uint_below((uint32_t)child.size() + 1);
        child.insert(child.begin() + site, (uint8_t)(mut - n_ops - 1));
        lmax = std::max(lmax, (int)child.size());
      }
    };
    // GetRandBinomial(size, p) restated as one P(p) per site (see DIV_MUT_PROB below)
    auto binom = [&](const Prob& q, int size) -> int {
      int n = 0;
      for (int i = 0; i < size; i++) n += r.p(q) ? 1 : 0;
      return n;
    };
    if (r.p(w.p_div_slip)) slip_mutation(child, r);
    for (uint32_t i = 0, n = npois(0); i < n; i++) slip_mutation(child, r);   // :318-320
    if (w.p_dsite[3].p > 0.0) {                                               // per site :323-327
      const int n = binom(w.p_dsite[3], (int)child.size());
      for (int i = 0; i < n; i++) slip_mutation(child, r);
    }
    // translocations (:331-343): one-shot (drawn only at a non-zero rate),
    // Poisson, per site
    if (w.p_div_trans.p != 0.0 && r.p(w.p_div_trans)) trans_mutation(child, r);
    for (uint32_t i = 0, n = w.pois_L[4] > 0.0 ? r.poisson(w.pois_L[4]) : 0u; i < n; i++) trans_mutation(child, r);
    if (w.p_dsite[4].p > 0.0) {
      const int n = binom(w.p_dsite[4], (int)child.size());
      for (int i = 0; i < n; i++) trans_mutation(child, r);
    }
    if (r.p(w.p_div_mut)) {
      uint32_t line = r.uint_below((uint32_t)child.size());
      child[line] = (uint8_t)w.is.random_inst(r);
    }
    for (uint32_t i = 0, n = npois(1); i < n; i++) {                         // :383-391
      uint32_t line = r.uint_below((uint32_t)child.size());
      child[line] = (uint8_t)w.is.random_inst(r);
    }
    if (r.p(w.p_div_ins) && (int)child.size() < max_g) {
      uint32_t line = r.uint_below((uint32_t)child.size() + 1);
      child.insert(child.begin() + line, (uint8_t)w.is.random_inst(r));
      lmax = std::max(lmax, (int)child.size());
    }
    for (uint32_t i = 0, n = npois(2); i < n; i++) {                         // :404-413
      if ((int)child.size() >= max_g) break;
      uint32_t line = r.uint_below((uint32_t)child.size() + 1);
      child.insert(child.begin() + line, (uint8_t)w.is.random_inst(r));
      lmax = std::max(lmax, (int)child.size());
    }
    if (r.p(w.p_div_del) && (int)child.size() > min_g) {
      uint32_t line = r.uint_below((uint32_t)child.size());
      child.erase(child.begin() + line);
    }
    for (uint32_t i = 0, n = npois(3); i < n; i++) {                         // :426-435
      if ((int)child.size() <= min_g) break;
      uint32_t line = r.uint_below((uint32_t)child.size());
      child.erase(child.begin() + line);
    }
    if (w.p_div_uni.p != 0.0 && r.p(w.p_div_uni)) uniform_mutation();
    // Divide Mutations (per site) (cpu/cHardwareBase.cc:447-460): only at a
    // non-zero DIV_MUT_PROB; mut_multiplier 1 and maxmut INT_MAX on this path
    // (Divide_Main :1806).  GetRandBinomial lives in Apto (absent here): it is
    // restated as its exact form, one P(p) per offspring site, so the count is
    // Binomial(size, p) and every draw comes from the organism's own stream.
    // Then one GetUInt(size) site and one GetRandomInst per substitution.
    if (w.p_div_site.p > 0.0) {
      const int size = (int)child.size();
      int num_mut = 0;
      for (int i = 0; i < size; i++) num_mut += r.p(w.p_div_site) ? 1 : 0;
      for (int i = 0; i < num_mut; i++) {
        const uint32_t site = r.uint_below((uint32_t)size);
        child[site] = (uint8_t)w.is.random_inst(r);
      }
    }
    // Insert Mutations (per site) (:463-485): all sites first, sorted, then
    // inserted from the highest down, one GetRandomInst each
    if (w.p_dsite[0].p > 0.0) {
      int n = binom(w.p_dsite[0], (int)child.size());
      if (n + (int)child.size() > max_g) n = max_g - (int)child.size();
      if (n > 0) {
        std::vector<int> sites(n);
        for (int i = 0; i < n; i++) sites[i] = (int)r.uint_below((uint32_t)child.size() + 1);
        std::sort(sites.begin(), sites.end());
        for (int i = n - 1; i >= 0; i--) child.insert(child.begin() + sites[i], (uint8_t)w.is.random_inst(r));
        lmax = std::max(lmax, (int)child.size());
      }
    }
    // Delete Mutations (per site) (:473-488)
    if (w.p_dsite[1].p > 0.0) {
      int n = binom(w.p_dsite[1], (int)child.size());
      if ((int)child.size() - n < min_g) n = (int)child.size() - min_g;
      for (int i = 0; i < n; i++) child.erase(child.begin() + r.uint_below((uint32_t)child.size()));
    }
    // Uniform Mutations (per site) (:492-503)
    if (w.p_dsite[2].p > 0.0) {
      const int n = binom(w.p_dsite[2], (int)child.size());
      for (int i = 0; i < n; i++) uniform_mutation();
    }
    // Parent Substitution Mutations (per site) (cpu/cHardwareBase.cc:508-520):
    // the parent's memory, already cut to the divide point (Divide_Main
    // :1803-1806); the same Binomial restatement; flags are untouched
    if (w.p_par_site.p > 0.0) {
      const int size = (int)o.mem.size();
      int num_mut = 0;
      for (int i = 0; i < size; i++) num_mut += r.p(w.p_par_site) ? 1 : 0;
      for (int i = 0; i < num_mut; i++) {
        const uint32_t site = r.uint_below((uint32_t)size);
        o.mem[site] = (uint8_t)w.is.random_inst(r);
      }
    }
    // Parent Insert Mutations (per site) (:523-547): the count capped at the
    // largest genome, every site drawn (GetUInt(size + 1)), sorted (Apto::QSort),
    // inserted from the highest down, one GetRandomInst each; new sites flags 0
    if (w.p_par_ins.p > 0.0) {
      int n = binom(w.p_par_ins, (int)o.mem.size());
      if (n + (int)o.mem.size() > max_g) n = max_g - (int)o.mem.size();
      if (n > 0) {
        std::vector<int> sites(n);
        for (int i = 0; i < n; i++) sites[i] = (int)r.uint_below((uint32_t)o.mem.size() + 1);
        std::sort(sites.begin(), sites.end());
        for (int i = n - 1; i >= 0; i--) {
          o.mem.insert(o.mem.begin() + sites[i], (uint8_t)w.is.random_inst(r));
          o.flg.insert(o.flg.begin() + sites[i], 0);
        }
      }
    }
    // Parent Deletion Mutations (per site) (:550-565): capped at the smallest genome
    if (w.p_par_del.p > 0.0) {
      int n = binom(w.p_par_del, (int)o.mem.size());
      if ((int)o.mem.size() - n < min_g) n = (int)o.mem.size() - min_g;
      for (int i = 0; i < n; i++) {
        const uint32_t site = r.uint_below((uint32_t)o.mem.size());
        o.mem.erase(o.mem.begin() + site);
        o.flg.erase(o.flg.begin() + site);
      }
    }
  }

  // Divide_CheckViable (cpu/cHardwareBase.cc:140-289 + main/cOrganism.cc:788-919);
  // ORG_FAULT is gated by ctx.OrgFaultReporting(), off by default
  // (main/cAvidaContext.h:45), so these failures do not count errors.
  bool check_viable(int parent_size, int child_size, int* exe_out, int* copied_out) {
    const int genome_size = (int)o.genome.size();
    const double range = w.cfg.offspring_size_range;
    const int min_size = std::max(AVGPU_MIN_GENOME, (int)(genome_size / range));
    const int max_size = std::min(AVGPU_MAX_GENOME, (int)(genome_size * range));
    if (child_size < min_size || child_size > max_size) { return false; }
    if (parent_size < min_size || parent_size > max_size) { return false; }
    const int ming = w.cfg.min_genome_size, maxg = w.cfg.max_genome_size;
    if ((ming && child_size < ming) || (maxg && child_size > maxg)) { return false; }
    if ((ming && parent_size < ming) || (maxg && parent_size > maxg)) { return false; }
    int executed = 0;
    for (int i = 0; i < parent_size; i++) if (o.flg[i] & F_EXECUTED) executed++;
    const int min_exe = (int)(parent_size * w.cfg.min_exe_lines);
    if (executed < min_exe) { return false; }
    int copied = 0;
    for (int i = parent_size; i < parent_size + child_size; i++) if (o.flg[i] & F_COPIED) copied++;
    const int min_copied = (int)(child_size * w.cfg.min_copied_lines);
    if (copied < min_copied) { return false; }
    // cOrganism::Divide_CheckViable (main/cOrganism.cc:788-919)
    if (o.cur_bonus < w.cfg.required_bonus) return false;
    // the required task unless the immunity task was done (:826-832)
    if (w.req_task >= 0 && o.cur_task[w.req_task] == 0 && (w.imm_task < 0 || o.cur_task[w.imm_task] == 0))
      return false;
    // the required reaction likewise (:839-847; nothing is stolen on this path)
    const int rr = w.cfg.required_reaction, ir = w.cfg.immunity_reaction;
    if (w.cfg.require_single_reaction == 0 && rr >= 0 && o.cur_react[rr] == 0 && (ir < 0 || o.cur_react[ir] == 0))
      return false;
    // at most MAX_UNIQUE_TASK_COUNT distinct tasks (:849-862)
    if (w.cfg.max_unique_task_count > 0) {
      int nt = 0;
      for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) nt += o.cur_task[t] > 0;
      if (nt > w.cfg.max_unique_task_count) return false;
    }
    // REQUIRE_SINGLE_REACTION: some reaction (:864-880)
    if (w.cfg.require_single_reaction != 0) {
      bool any = false;
      for (int i = 0; i < (int)w.react.size(); i++) any = any || o.cur_react[i] > 0;
      if (!any) return false;
    }
    double base = (double)calc_size_merit();
    double bonus = o.cur_bonus;
    if (w.cfg.merit_default_bonus != 0.0) bonus = w.cfg.merit_default_bonus;
    double off_merit = base * bonus;
    if (w.cfg.inherit_merit == 0) off_merit = base;
    if (off_merit == 0) return false;
    *exe_out = executed; *copied_out = copied;
    return true;
  }

  // Inst_HeadDivideMut -> Divide_Main (cpu/cHardwareCPU.cc:6942-6959, :1775-1843)
  bool h_divide(int64_t cell) {
    const int sz0 = size();
    for (int i = 0; i < 4; i++) o.head[i] = adjust(o.head[i], sz0);  // AdjustHeads
    const int div_point = o.head[HEAD_READ];
    int child_end = o.head[HEAD_WRITE];
    if (child_end == 0) child_end = sz0;
    const int extra = sz0 - child_end;
    const int child_size = sz0 - div_point - extra;
    int exe = 0, cop = 0;
    if (!check_viable(div_point, child_size, &exe, &cop)) {
      for (int i = 0; i < 4; i++) o.head[i] = adjust(o.head[i], size());
      return false;
    }
    if (nb_stop) { nb_halted = true; return false; }
    o.executed_size = exe;       // SetLinesExecuted
    o.child_copied_size = cop;   // SetLinesCopied
    std::vector<uint8_t> child(o.mem.begin() + div_point, o.mem.begin() + div_point + child_size);
    if (mode == AVGPU_MODE_TEST) {
      o.exec_flags_at_divide.assign(div_point, '-');
      for (int i = 0; i < div_point; i++) if (o.flg[i] & F_EXECUTED) o.exec_flags_at_divide[i] = '+';
    }
    o.mem.resize(div_point);
    o.flg.resize(div_point);
    // the reference draws the divide mutations in every mode with a world
    // (Divide_Main :1806); FROZEN discards the offspring afterwards, the test
    // CPU runs without mutations and stops at its divide
    if (mode != AVGPU_MODE_TEST) divide_mutations(child);
    o.mal_active = false;
    o.advance_ip = false;   // DIVIDE_METHOD_SPLIT
    // ActivateDivide: the on-divide DoOutput runs no reaction for logic-9
    // environments (every requisite has divide_only 0; TestRequisites :1408).
    divide_reset();
    // a slip outgrew the largest genome (or passed 4095 sites on the way: the
    // device's edit words hold 12-bit positions): the offspring is dropped
    if (mode == AVGPU_MODE_WORLD && ((int)child.size() > AVGPU_MAX_GENOME || lmax > 4095)) {
      w.t_oversize++;
    } else if (mode == AVGPU_MODE_WORLD) {
      Birth b;
      b.parent = cell;
      b.seq = (uint32_t)o.num_divides;
      b.genome = child;
      b.merit = o.merit;
      b.generation = o.generation;
      b.child_copied = o.child_copied_size;
      b.executed = o.executed_size;
      b.gestation_time = o.gestation_time;
      b.fitness = o.fitness;
      for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) b.last_task[t] = o.last_task[t];
      derive_key(o.rng.lo, o.rng.hi, (uint32_t)o.num_divides, 0x1B873593U, &b.rng.lo, &b.rng.hi);
      b.rng.ctr = 0;
      w.births.push_back(std::move(b));
    } else if (mode == AVGPU_MODE_TEST) {
      o.offspring = child;
      stop = true;
    }
    // parent alive: Reset + ClearFlags (:1836-1839)
    hw_reset();
    std::fill(o.flg.begin(), o.flg.end(), 0);
    return true;
  }

  // cTaskLib::SetupTests logic id (main/cTaskLib.cc:369-448)
  static int logic_id(const Buffer& in, int out_val) {
    const int num_inputs = in.num_stored();
    int ti[3];
    for (int i = 0; i < 3; i++) ti[i] = (num_inputs > i) ? in[i] : 0;
    int to = out_val;
    int lo[8];
    for (int i = 0; i < 8; i++) lo[i] = -1;
    for (int tp = 0; tp < 32; tp++) {
      int lp = 0;
      for (int i = 0; i < 3; i++) lp += (ti[i] & 1) << i;
      if (lo[lp] != -1 && lo[lp] != (to & 1)) return -1;
      lo[lp] = to & 1;
      to >>= 1;
      for (int i = 0; i < 3; i++) ti[i] >>= 1;
    }
    if (num_inputs < 1) lo[1] = lo[0];
    if (num_inputs < 2) { lo[2] = lo[0]; lo[3] = lo[1]; }
    if (num_inputs < 3) { lo[4] = lo[0]; lo[5] = lo[1]; lo[6] = lo[2]; lo[7] = lo[3]; }
    int id = 0;
    for (int i = 0; i < 8; i++) id += lo[i] * (1 << i);  // -1 entries contribute -2^i
    return id;
  }
  // Task_Not ... Task_Equ (main/cTaskLib.cc:511-575)
  static bool task_done(int task, int id) {
    switch (task) {
      case 0: return id == 15 || id == 51 || id == 85;
      case 1: return id == 63 || id == 95 || id == 119;
      case 2: return id == 136 || id == 160 || id == 192;
      case 3: return id == 175 || id == 187 || id == 207 || id == 221 || id == 243 || id == 245;
      case 4: return id == 238 || id == 250 || id == 252;
      case 5: return id == 10 || id == 12 || id == 34 || id == 48 || id == 68 || id == 80;
      case 6: return id == 3 || id == 5 || id == 17;
      case 7: return id == 60 || id == 90 || id == 102;
      case 8: return id == 153 || id == 165 || id == 195;
    }
    return false;
  }

  // cOrganism::DoOutput -> cPhenotype::TestOutput -> cEnvironment::TestOutput
  // (main/cOrganism.cc:385-521, main/cPhenotype.cc:1493-1700,
  //  main/cEnvironment.cc:1314-1406, :1408-1503, :1610-1760)
  void do_output(int value) {
    o.output_buf.add(value);
    const int id = logic_id(o.input_buf, o.output_buf[0]);
    bool done[AVGPU_MAX_REACTIONS] = {false};
    double mult = 1.0, add = 0.0;
    bool any = false;
    for (size_t i = 0; i < w.react.size(); i++) {
      const avgpu_reaction& r = w.react[i].r;
      const int task_cnt = o.cur_task[r.task];    // eff_task_count
      if (r.has_requisite) {
        if (task_cnt < r.min_count) continue;
        if (task_cnt >= r.max_count) continue;
      }
      if (id < 0 || !task_done(r.task, id)) continue;
      done[r.task] = true;                          // MarkTask precedes DoProcesses
      any = true;
      if (r.resource == 0 || mode == AVGPU_MODE_TEST) {   // infinite (the test CPU: no resource grid)
        if (r.type == AVGPU_PROC_POW) mult *= w.react[i].mult;
        else if (r.type == AVGPU_PROC_MULT) mult *= w.react[i].mult;
        else add += w.react[i].add;
        o.cur_react[i]++;
        continue;
      }
      // cEnvironment::DoProcesses, finite resource (main/cEnvironment.cc:1660-1724)
      const int res = r.resource - 1;
      const bool spatial = w.res[res].geometry != AVGPU_RES_GLOBAL;
      const double level = spatial ? w.res_amount[res][cur_cell] : w.res_global[res];
      double consumed;
      if (level == 0) consumed = 0;
      else consumed = level * std::min(r.max_fraction, 1.0);
      if (consumed > r.max_number) consumed = r.max_number;
      consumed = consumed * 1.0 * 1.0;              // task quality, plasticity modifier
      if (consumed < r.min_number) consumed = 0.0;
      if (consumed == 0.0) continue;
      consumed = std::min(consumed, level);
      if (r.depletable) {
        if (spatial) w.res_amount[res][cur_cell] = level + (-consumed);   // ModifyCell: Rate + State
        else w.res_cons[res] += (uint64_t)(consumed * 4294967296.0);
        if (mode == AVGPU_MODE_WORLD) w.cons_cell[res][cur_cell] += consumed;   // (newborn credit)
      }
      const double bonus = consumed * r.value;
      if (r.type == AVGPU_PROC_ADD) add += bonus;
      else if (r.type == AVGPU_PROC_MULT) mult *= bonus;
      else mult *= det_exp2(bonus);
      o.cur_react[i]++;
    }
    if (!any) return;
    for (int t = 0; t < AVGPU_MAX_REACTIONS; t++) if (done[t]) o.cur_task[t]++;
    o.cur_bonus *= mult;
    o.cur_bonus += add;
  }

  // cOrganism::GetNextInput (main/cOrganism.h:249 -> main/cPopulationCell.h:214-218,
  // cpu/cTestCPU.h:132-136)
  int next_input() {
    if (o.input_ptr >= 3) o.input_ptr = 0;
    return o.inputs[o.input_ptr++];
  }

  // doSlipMutation(ctx, m_memory, write head) (cpu/cHardwareBase.cc:621-694)
  // on the organism's whole memory -- SLIP_COPY_MODE 1's copy slip
  // (cpu/cHardwareCPU.cc:7157-7161): `to` = GetInt(size) when from is 0, else
  // GetInt(size + 1); the memory is resized by from - to (cCPUMemory::Resize,
  // cpu/cCPUMemory.cc:66-77: new sites op 0 / flags 0, a shrink keeps the
  // leading flags) and the sites from `from` on are rewritten -- the
  // insertion [from, from + (from - to)) filled per SLIP_FILL_MODE (0: the
  // duplicated sites [to, from); 2: GetRandomInst each; 4: nop-C), then the
  // old sites from `to` on.  Only the instructions move: every site keeps the
  // flags of its position (the slip writes InstructionSequence elements, not
  // the cCPUMemory flag array).  A slip that would take the memory past
  // AVGPU_MAX_GENOME sites is skipped after its draw and counted
  // (AVGPU_CNT_MEM_CAP).  SLIP_FILL_MODE 1 (nop-X) and 3 are refused with
  // SLIP_COPY_MODE 1 (avgpu_check_cfg).
  void slip_memory(Stream& r, int from) {
    const int M = size();
    const int to = (int)(from == 0 ? r.uint_below((uint32_t)M) : r.uint_below((uint32_t)M + 1u));
    const int ins = from - to, Mn = M + ins;
    if (Mn > AVGPU_MAX_GENOME) { w.t_memcap++; return; }
    const std::vector<uint8_t> copy = o.mem;
    o.mem.resize(Mn, 0);
    o.flg.resize(Mn, 0);
    for (int i = 0; i < ins; i++) {
      const int sfm = w.cfg.slip_fill_mode;
      o.mem[from + i] = sfm == 0 ? copy[to + i] : sfm == 2 ? (uint8_t)w.is.random_inst(r) : (uint8_t)2;   // nop-C
    }
    for (int i = std::max(ins, 0); i < M - to; i++) o.mem[from + i] = copy[to + i];
  }

  // Inst_HeadCopy (cpu/cHardwareCPU.cc:7130-7167)
  void h_copy() {
    const int sz = size();
    int& rh = o.head[HEAD_READ];
    int& wh = o.head[HEAD_WRITE];
    rh = adjust(rh, sz);
    wh = adjust(wh, sz);
    int read_inst = o.mem[rh];
    // ReadInst (:1459-1466)
    if (w.is.is_nop(read_inst)) o.read_label.add(read_inst); else o.read_label.clear();
    // the test CPU runs with cleared mutation rates (cpu/cTestCPU.cc:270,
    // main/cMutationRates.cc:78-120)
    const bool muts = mode != AVGPU_MODE_TEST;
    // TestCopy*: no draw when the rate is 0 (main/cMutationRates.h:111-120)
    Stream& r = rng();
    // checkNoMutList (cpu/cHardwareCPU.cc:797-810, :7144): the draw always,
    // the mutation (and its GetRandomInst draw) only for an unlisted instruction
    if (muts && w.p_copy_mut.th && r.p(w.p_copy_mut) && !w.is.no_mut(read_inst)) {
      read_inst = w.is.random_inst(r);
      o.flg[wh] |= F_MUTATED | F_COPYMUT;
    }
    o.mem[wh] = (uint8_t)read_inst;
    o.flg[wh] |= F_COPIED;
    // cHeadCPU::InsertInst / RemoveInst at the write head (cpu/cHeadCPU.h:87-88
    // -> cCPUMemory::Insert / Remove, cpu/cCPUMemory.cc:103-138: the new site
    // has flags 0, later sites shift with their flags; no head moves).  The
    // memory is capped at AVGPU_MAX_GENOME sites here (the reference has no
    // cap): an insertion past it is skipped, its draws consumed, and counted
    // (AVGPU_CNT_MEM_CAP); a removal from a one-site memory is skipped.
    auto insert_at = [&](int pos, int op) {
      if (size() >= AVGPU_MAX_GENOME) { w.t_memcap++; return; }
      o.mem.insert(o.mem.begin() + pos, (uint8_t)op);
      o.flg.insert(o.flg.begin() + pos, 0);
    };
    // After a deletion at the last site the write head sits one past the end:
    // cCPUMemory::Remove(size) then drops the last site (its shift loop is
    // empty, adjustCapacity shrinks) and SetInst writes outside the sequence
    // (no visible effect).
    auto remove_at = [&](int pos) {
      if (size() <= 1) { w.t_memcap++; return; }
      if (pos > size() - 1) pos = size() - 1;
      o.mem.erase(o.mem.begin() + pos);
      o.flg.erase(o.flg.begin() + pos);
    };
    // TestCopyIns, TestCopyDel, TestCopyUniform, TestCopySlip in that order
    // (cpu/cHardwareCPU.cc:7153-7161), each drawing only at a non-zero rate
    if (muts && w.p_copy_ins.th && r.p(w.p_copy_ins)) insert_at(wh, w.is.random_inst(r));
    if (muts && w.p_copy_del.th && r.p(w.p_copy_del)) remove_at(wh);
    if (muts && w.p_copy_uni.th && r.p(w.p_copy_uni)) {
      // doUniformCopyMutation (cpu/cHardwareBase.cc:597-612): op codes, not
      // weighted; nothing for a write-head instruction NO_MUT_INSTS lists
      const int n_ops = w.is.n;
      const int mut = (int)r.uint_below((uint32_t)(2 * n_ops + 1));
      if (!(wh < size() && w.is.no_mut(o.mem[wh]))) {
        if (mut < n_ops) { if (wh < size()) o.mem[wh] = (uint8_t)mut; }   // SetInst: flags kept
        else if (mut == n_ops) remove_at(wh);
        else insert_at(wh, mut - n_ops - 1);
      }
    }
    // SLIP_COPY_MODE 0 (m_slip_read_head, cpu/cHardwareCPU.cc:785): the read
    // head jumps to GetInt(memory size) (:7157-7158); SLIP_COPY_MODE 1: a slip
    // of the whole memory at the write head (:7160, slip_memory)
    if (muts && w.p_copy_slip.th && r.p(w.p_copy_slip)) {
      if (w.cfg.slip_copy_mode == 0) rh = adjust((int)r.uint_below((uint32_t)size()), size());
      else slip_memory(r, wh);
    }
    rh = adjust(rh + 1, size());
    wh = adjust(wh + 1, size());
  }

  // One SingleProcess cycle (cpu/cHardwareCPU.cc:908-1058), single thread,
  // no costs / promoters / speculation.  Returns true if the instruction ran.
  void single_process(int64_t cell) {
    cur_cell = cell;
    o.cpu_cycles_used++;
    o.time_used++;
    o.advance_ip = true;
    o.head[HEAD_IP] = adjust(o.head[HEAD_IP], size());
    const int op = o.mem[o.head[HEAD_IP]];
    if (g_trace) {
      fprintf(stderr, "%d IP:%d op:%d AX:%d BX:%d CX:%d R:%d W:%d F:%d RL:", o.cpu_cycles_used,
              o.head[HEAD_IP], op, o.reg[0], o.reg[1], o.reg[2], o.head[1], o.head[2], o.head[3]);
      for (int i = 0; i < o.read_label.size; i++) fputc('A' + o.read_label.nops[i], stderr);
      fprintf(stderr, " mem:%d\n", (int)o.mem.size());
    }
    o.flg[o.head[HEAD_IP]] |= F_EXECUTED;
    g_op_hist[w.is.handler[op]]++;
    switch (w.is.handler[op]) {
      case H_NOP_A: case H_NOP_B: case H_NOP_C: break;
      case H_IF_N_EQU: { int a = find_modified(REG_BX), b = next_reg(a);
        if (o.reg[a] == o.reg[b]) advance_ip(); break; }
      case H_IF_LESS: { int a = find_modified(REG_BX), b = next_reg(a);
        if (o.reg[a] >= o.reg[b]) advance_ip(); break; }
      case H_POP: { int r = find_modified(REG_BX); o.reg[r] = o.stk[o.cur_stack].pop(); break; }
      case H_PUSH: { int r = find_modified(REG_BX); o.stk[o.cur_stack].push(o.reg[r]); break; }
      case H_SWAP_STK: o.cur_stack = o.cur_stack ? 0 : 1; break;
      case H_SWAP: { int a = find_modified(REG_BX), b = next_reg(a);
        std::swap(o.reg[a], o.reg[b]); break; }
      case H_SHIFT_R: { int r = find_modified(REG_BX); o.reg[r] >>= 1; break; }
      case H_SHIFT_L: { int r = find_modified(REG_BX); o.reg[r] = (int)((uint32_t)o.reg[r] << 1); break; }
      case H_INC: { int r = find_modified(REG_BX); o.reg[r] = wrap_add(o.reg[r], 1); break; }
      case H_DEC: { int r = find_modified(REG_BX); o.reg[r] = wrap_add(o.reg[r], -1); break; }
      case H_ADD: { int r = find_modified(REG_BX); o.reg[r] = wrap_add(o.reg[REG_BX], o.reg[REG_CX]); break; }
      case H_SUB: { int r = find_modified(REG_BX);
        o.reg[r] = (int)((uint32_t)o.reg[REG_BX] - (uint32_t)o.reg[REG_CX]); break; }
      case H_NAND: { int r = find_modified(REG_BX); o.reg[r] = ~(o.reg[REG_BX] & o.reg[REG_CX]); break; }
      case H_IO: { int r = find_modified(REG_BX);
        do_output(o.reg[r]);
        int in = next_input();
        o.reg[r] = in;
        o.input_buf.add(in);
        break; }
      case H_H_ALLOC: {  // Inst_MaxAlloc (:3294-3303)
        const int cur = size();
        const int alloc = std::min((int)(w.cfg.offspring_size_range * cur), AVGPU_MAX_GENOME - cur);
        if (allocate_main(alloc)) o.reg[REG_AX] = cur;
        break; }
      case H_H_DIVIDE: h_divide(cell); break;
      case H_H_COPY: h_copy(); break;
      case H_H_SEARCH: {  // :7245-7256
        read_label();
        o.next_label.rotate(1, NUM_NOPS);
        int found = find_label_from_start();
        o.reg[REG_BX] = found - o.head[HEAD_IP];
        o.reg[REG_CX] = o.next_label.size;
        o.head[HEAD_FLOW] = found;                               // Set(found_pos): copy, no adjust
        o.head[HEAD_FLOW] = adjust(o.head[HEAD_FLOW] + 1, size()); // Advance
        break; }
      case H_MOV_HEAD: { int h = find_modified(HEAD_IP);
        o.head[h] = o.head[HEAD_FLOW];
        if (h == HEAD_IP) o.advance_ip = false;
        break; }
      case H_JMP_HEAD: { int h = find_modified(HEAD_IP);
        o.head[h] = adjust(wrap_add(o.head[h], o.reg[REG_CX]), size()); break; }
      case H_GET_HEAD: { int h = find_modified(HEAD_IP); o.reg[REG_CX] = o.head[h]; break; }
      case H_IF_LABEL: {
        read_label();
        o.next_label.rotate(1, NUM_NOPS);
        if (!o.next_label.eq(o.read_label)) advance_ip();
        break; }
      case H_SET_FLOW: { int r = find_modified(REG_CX);
        o.head[HEAD_FLOW] = adjust(o.reg[r], size()); break; }
      default: break;
    }
    if (stop) return;
    if (nb_halted) { o.cpu_cycles_used--; o.time_used--; return; }   // (its executed flag stays: set again when it runs)
    if (o.advance_ip) advance_ip();
    // death (:1045-1049)
    if ((o.max_executed > 0 && o.time_used >= o.max_executed) || o.to_die) o.alive = false;
  }
};

// cPhenotype::SetupInject + cOrganism::initialize (main/cPhenotype.cc:599-640,
// main/cOrganism.cc:216-236)
void setup_inject(World& w, Org& o, const uint8_t* genome, int len, double merit) {
  o = Org();
  o.alive = true;
  o.age = -1;   // injected between updates: age 0 during the next one (age_tick)
  o.genome.assign(genome, genome + len);
  o.mem = o.genome;
  o.flg.assign(len, 0);
  for (int i = 0; i < 3; i++) o.reg[i] = 0;
  for (int i = 0; i < 4; i++) o.head[i] = 0;
  o.stk[0].clear(); o.stk[1].clear();
  o.input_buf.cap = 3; o.output_buf.cap = 1;
  o.genome_length = len; o.copied_size = len; o.executed_size = len; o.child_copied_size = 0;
  o.merit = merit > 0 ? merit : (double)len;
  o.cur_bonus = w.cfg.default_bonus;
  for (int i = 0; i < AVGPU_MAX_REACTIONS; i++) { o.cur_task[i] = o.last_task[i] = o.cur_react[i] = 0; }
  o.max_executed = 0;
  if (w.cfg.death_method > 0) {
    o.max_executed = w.cfg.age_limit;
    if (w.cfg.death_method == 2) o.max_executed *= len;
    if (o.max_executed < 1) o.max_executed = 1;
  }
}

void dump_state(const World& w, const Org& o, avgpu_cpu_state* s, uint8_t* ops, uint8_t* flags, int cap) {
  memset(s, 0, sizeof(*s));
  for (int i = 0; i < 3; i++) s->reg[i] = o.reg[i];
  for (int i = 0; i < 4; i++) s->head[i] = o.head[i];
  for (int k = 0; k < 2; k++) {
    for (int i = 0; i < AVGPU_STACK_SIZE; i++) s->stack[k][i] = o.stk[k].s[i];
    s->stack_ptr[k] = o.stk[k].sp;
  }
  s->cur_stack = o.cur_stack;
  s->read_label_len = o.read_label.size;
  for (int i = 0; i < o.read_label.size; i++) s->read_label[i] = o.read_label.nops[i];
  s->mal_active = o.mal_active;
  s->mem_size = (int)o.mem.size();
  s->cpu_cycles_used = o.cpu_cycles_used;
  s->time_used = o.time_used;
  s->gestation_start = o.gestation_start;
  s->gestation_time = o.gestation_time;
  s->num_divides = o.num_divides;
  s->generation = o.generation;
  s->alive = o.alive;
  s->genome_length = o.genome_length;
  s->copied_size = o.copied_size;
  s->child_copied_size = o.child_copied_size;
  s->executed_size = o.executed_size;
  s->max_executed = o.max_executed;
  s->birth_length = (int)o.genome.size();
  s->input_ptr = o.input_ptr;
  for (int i = 0; i < 3; i++) s->input_buf[i] = (i < o.input_buf.num_stored()) ? o.input_buf[i] : 0;
  s->input_total = o.input_buf.total;
  s->output_buf = o.output_buf.total ? o.output_buf[0] : 0;
  s->output_total = o.output_buf.total;
  for (int i = 0; i < 3; i++) s->inputs[i] = o.inputs[i];
  for (int i = 0; i < AVGPU_MAX_REACTIONS; i++) {
    s->cur_task_count[i] = o.cur_task[i];
    s->last_task_count[i] = o.last_task[i];
    s->cur_reaction_count[i] = o.cur_react[i];
  }
  s->rng_counter = o.rng.ctr;
  s->rng_key_lo = o.rng.lo;
  s->rng_key_hi = o.rng.hi;
  s->errors = o.errors;
  s->cur_bonus = o.cur_bonus;
  s->merit = o.merit;
  s->fitness = o.fitness;
  s->credit = o.credit;
  s->head_start = o.hstart;
  // as the reference's UpdateOrganismStats leaves it (age_tick); kept only
  // for BIRTH_METHOD 1 / 2, its one consumer on this path (the device's
  // track_age), 0 otherwise
  s->age = tracks_age(w) ? o.age + 1 : 0;
  (void)w;
  if (ops && flags) {
    for (int i = 0; i < cap; i++) {
      ops[i] = i < (int)o.mem.size() ? o.mem[i] : 0;
      // exported flags: bit0 copied, bit2 executed (the execution-relevant bits)
      flags[i] = i < (int)o.flg.size() ? (o.flg[i] & (F_COPIED | F_EXECUTED)) : 0;
    }
  }
}

// The scheduler weight of a living organism: its merit, raised for its first
// allotment after birth by the share of the birth update it did not run
// (hstart / 2^16, DESIGN.md 5 "head start"): the reference places an
// offspring inside its parent's divide and schedules it for the rest of that
// update; the batch update places it at the update's end and gives it that
// share in the next.  hstart 0 -> the merit itself.
// A merit that is NaN, negative or infinite is never scheduled (weight 0),
// nor is a weight that overflows; a weight is at most 2^990, so that the
// scheduler's sums over up to 2^33 organisms stay finite (a few merits near
// DBL_MAX would sum to inf and zero every draw); the device's merit_ok /
// sched_weight.
static constexpr double WEIGHT_CAP = 0x1p990;
static inline bool merit_ok(double m) { return m >= 0.0 && m <= 1.7976931348623157e308; }
static inline double sched_weight(const Org& o) {
  if (!merit_ok(o.merit)) return 0.0;
  const double w = o.hstart ? o.merit * (1.0 + (double)o.hstart * (1.0 / 65536.0)) : o.merit;
  return merit_ok(w) ? std::min(w, WEIGHT_CAP) : 0.0;
}

// ---------------------------------------------------------------------------
// The scheduler (SLICING_METHOD 1, the default: Apto::Scheduler::Probabilistic,
// main/cPopulation.cc:7341-7346): each update the reference makes
// UD = AVE_TIME_SLICE x N picks (cWorld::CalculateUpdateSize,
// main/cWorld.cc:247-250), each one instruction of an organism drawn with
// probability weight / total weight -- so the update's instruction counts are
// Multinomial(UD, weights).  The batch update draws exactly that, in parallel,
// by splitting UD down a fixed binary tree of the cells with a Binomial at
// every node:
//   * 256-cell blocks; a block's partial is the pairwise tree of strides 128,
//     64, ..., 1 over its cells' weights (s[t] += s[t + stride]): node (k, t)
//     of level k covers the block's cells = t (mod 2^k);
//   * the top tree over the blocks (global order, padded to a power of two
//     with zeros): node i of level l = left + right, children 2i, 2i + 1;
//   * top down: the root holds UD; a node holding n gives its left child
//     Binomial(n, S_left / S_node) (binom_draw) and its right child the rest,
//     down to the blocks and inside each block down to the cells.
// The sums are the same additions in the same order on both sides, and every
// node draws from its own stateless word (node_draw), so the budgets do not
// depend on execution order or on how the world is cut into strips.
static double pow_int(double q, int64_t n) {
  double r = 1.0, b = q;
  while (n) { if (n & 1) r = r * b; b = b * b; n >>= 1; }
  return r;
}

// 1/k for k = 1..64, correctly rounded (the same doubles on both sides)
static const double INV_K[65] = {0.0,
  1.0 / 1, 1.0 / 2, 1.0 / 3, 1.0 / 4, 1.0 / 5, 1.0 / 6, 1.0 / 7, 1.0 / 8, 1.0 / 9, 1.0 / 10, 1.0 / 11, 1.0 / 12,
  1.0 / 13, 1.0 / 14, 1.0 / 15, 1.0 / 16, 1.0 / 17, 1.0 / 18, 1.0 / 19, 1.0 / 20, 1.0 / 21, 1.0 / 22, 1.0 / 23,
  1.0 / 24, 1.0 / 25, 1.0 / 26, 1.0 / 27, 1.0 / 28, 1.0 / 29, 1.0 / 30, 1.0 / 31, 1.0 / 32, 1.0 / 33, 1.0 / 34,
  1.0 / 35, 1.0 / 36, 1.0 / 37, 1.0 / 38, 1.0 / 39, 1.0 / 40, 1.0 / 41, 1.0 / 42, 1.0 / 43, 1.0 / 44, 1.0 / 45,
  1.0 / 46, 1.0 / 47, 1.0 / 48, 1.0 / 49, 1.0 / 50, 1.0 / 51, 1.0 / 52, 1.0 / 53, 1.0 / 54, 1.0 / 55, 1.0 / 56,
  1.0 / 57, 1.0 / 58, 1.0 / 59, 1.0 / 60, 1.0 / 61, 1.0 / 62, 1.0 / 63, 1.0 / 64};

// Binomial(n, p) from one 32-bit word h (the device's binom_draw, device.h):
// on the smaller side pp = min(p, 1 - p), mean n pp < 6 by inversion
// (f_0 = (1 - pp)^n by squaring, f_{k+1} = f_k (n - k) (pp / (1 - pp)) / (k + 1),
// at most 64 steps); otherwise normal with the binomial's skew
// (Cornish-Fisher: mean + sd z + (1 - 2 pp)(z^2 - 1) / 6, rounded), z the
// centred, scaled sum of 4 16-bit uniforms from h (Irwin-Hall), clamped to
// [0, n].  IEEE adds, multiplies, divisions and square roots only (correctly
// rounded on both sides, no fused multiply-add).
static int64_t binom_draw(int64_t n, double p, uint32_t h) {
  if (n <= 0 || !(p > 0.0)) return 0;
  if (p >= 1.0) return n;
  const bool flip = p > 0.5;
  const double pp = flip ? 1.0 - p : p, q = 1.0 - pp;
  const double mean = (double)n * pp;
  int64_t k;
  if (mean < 6.0) {
    const double u = ((double)h + 0.5) * 2.3283064365386962890625e-10;
    const double r = pp / q;
    double f = pow_int(q, n);
    double F = f;
    k = 0;
    while (F < u && k < n && k < 64) { f = (f * ((double)(n - k) * r)) * INV_K[k + 1]; k++; F = F + f; }
  } else {
    uint32_t x = lowbias32(h + 0x9E3779B9U);
    uint32_t sum = (x & 0xFFFFu) + (x >> 16);
    x = lowbias32(x + 0x9E3779B9U);
    sum += (x & 0xFFFFu) + (x >> 16);
    const double z = (((double)sum + 2.0) * 1.52587890625e-05 - 2.0) * 1.7320508075688772;
    const double sd = std::sqrt(mean * q);   // IEEE, correctly rounded (the device's __dsqrt_rn)
    const double v = mean + sd * z + ((q - pp) * (z * z - 1.0)) * 0.16666666666666666 + 0.5;
    k = v < 1.0 ? 0 : (int64_t)std::floor(v);
    if (k > n) k = n;
  }
  return flip ? n - k : k;
}

// the word of tree node `node` in update u (salt: top tree / block trees)
static inline uint32_t node_draw(const World& w, uint32_t update, uint32_t salt, uint64_t node) {
  const uint32_t slo = (uint32_t)w.cfg.seed, shi = (uint32_t)(w.cfg.seed >> 32);
  return lowbias32(lowbias32(lowbias32(update * 0x85EBCA6BU + shi) ^ (uint32_t)node ^ salt) +
                   (uint32_t)(node >> 32) + slo);
}
enum : uint32_t { SALT_TOP = 0x7A11C0DEu, SALT_BLOCK = 0x51CEB10Cu };

// a block's partial: the stride tree over its cells' weights (levels kept)
static double block_levels(const World& w, int64_t b, double lv[9][256]) {
  for (int t = 0; t < 256; t++) {
    const int64_t c = b * 256 + t;
    lv[8][t] = (c < w.ncells && w.orgs[c].alive) ? sched_weight(w.orgs[c]) : 0.0;
  }
  for (int k = 7; k >= 0; k--)
    for (int t = 0; t < (1 << k); t++) lv[k][t] = lv[k + 1][t] + lv[k + 1][t + (1 << k)];
  return lv[0][0];
}

// the top tree over block partials `leaf` (global block order): returns the
// root (the total weight) and, when n_root >= 0, splits n_root down to the
// blocks [b0, b0 + nloc) into cnt
static double top_tree(const World& w, const std::vector<double>& leaf, int64_t n_root, int64_t b0, int64_t nloc,
                       std::vector<int64_t>* cnt) {
  int L = 0;
  while (((int64_t)1 << L) < (int64_t)leaf.size()) L++;
  std::vector<std::vector<double>> lv(L + 1);
  lv[L].assign((size_t)1 << L, 0.0);
  for (size_t i = 0; i < leaf.size(); i++) lv[L][i] = leaf[i];
  for (int l = L - 1; l >= 0; l--) {
    lv[l].resize((size_t)1 << l);
    for (size_t i = 0; i < lv[l].size(); i++) lv[l][i] = lv[l + 1][2 * i] + lv[l + 1][2 * i + 1];
  }
  if (cnt) {
    std::vector<int64_t> c(1, n_root);
    for (int l = 0; l < L; l++) {
      std::vector<int64_t> nc((size_t)2 << l, 0);
      for (size_t i = 0; i < c.size(); i++) {
        const int64_t left = binom_draw(c[i], lv[l + 1][2 * i] / lv[l][i],
                                        node_draw(w, w.sched_key, SALT_TOP, ((uint64_t)1 << l) + i));
        nc[2 * i] = left;
        nc[2 * i + 1] = c[i] - left;
      }
      c.swap(nc);
    }
    cnt->assign(nloc, 0);
    for (int64_t j = 0; j < nloc; j++) (*cnt)[j] = c[b0 + j];
  }
  return lv[0][0];
}

// a block's count split down its stride tree into its cells' budgets
static void block_split(const World& w, int64_t b, int64_t n, int32_t* budget) {
  double lv[9][256];
  block_levels(w, b, lv);
  int64_t cnt[256];
  cnt[0] = n;
  const uint64_t gb = (uint64_t)(w.cell0 / 256 + b);
  for (int k = 0; k < 8; k++)
    for (int t = 0; t < (1 << k); t++) {
      const int64_t c0 = cnt[t];
      const int64_t left = binom_draw(c0, lv[k + 1][t] / lv[k][t],
                                      node_draw(w, w.sched_key, SALT_BLOCK, (gb << 9) | ((1u << k) + t)));
      cnt[t] = left;
      cnt[t + (1 << k)] = c0 - left;
    }
  for (int t = 0; t < 256; t++) {
    const int64_t c = b * 256 + t;
    if (c < w.ncells) budget[c] = (int32_t)std::min<int64_t>(cnt[t], (1 << 30) - 1);   // the device's budget range
  }
}

// this world's block partials and living organisms (the strip tiles' partials)
static void world_partials(const World& w, std::vector<double>& part, int64_t* n_alive) {
  const int64_t nb = (w.ncells + 255) / 256;
  part.resize(nb);
  double lv[9][256];
  for (int64_t b = 0; b < nb; b++) part[b] = block_levels(w, b, lv);
  int64_t cnt = 0;
  for (int64_t c = 0; c < w.ncells; c++) cnt += w.orgs[c].alive ? 1 : 0;
  *n_alive = cnt;
}

// torus / grid neighbourhood (tools/cTopology.h:40-55 build_torus/build_grid),
// fixed order: NW N NE W E SW S SE.  A strip tile maps the rows above / below
// it to the ghost rows [n, n+X) / [n+X, n+2X).
int neighbours(const World& w, int64_t cell, int64_t* out) {
  const int X = w.cfg.world_x;
  const int64_t R = w.rows;
  const int x = (int)(cell % X);
  const int64_t y = cell / X;
  int n = 0;
  for (int dy = -1; dy <= 1; dy++)
    for (int dx = -1; dx <= 1; dx++) {
      if (dx == 0 && dy == 0) continue;
      int nx = x + dx;
      int64_t ny = y + dy;
      if (w.cfg.world_geometry == 1) {
        if (nx < 0 || nx >= X) continue;
      } else {
        nx = (nx + X) % X;
      }
      if (ny >= 0 && ny < R) {
        out[n++] = ny * X + nx;
      } else if (!w.tiled) {
        if (w.cfg.world_geometry == 1) continue;
        ny = (ny + R) % R;
        out[n++] = ny * X + nx;
      } else {
        const int64_t gy = w.row0 + ny;
        if (w.cfg.world_geometry == 1 && (gy < 0 || gy >= w.global_rows)) continue;
        out[n++] = w.ncells + (ny < 0 ? 0 : X) + nx;
      }
    }
  return n;
}

// cPopulation::ActivateOrganism for a child (main/cPopulation.cc:1320-1340)
// + cPhenotype::SetupOffspring (main/cPhenotype.cc:349-420)
// ctx: the serial world's context stream (the three input draws of
// SetupInputs come from it); nullptr: the offspring's own stream
void activate_child(World& w, Birth& b, int64_t cell, Stream* ctx = nullptr) {
  Org& o = w.orgs[cell];
  setup_inject(w, o, b.genome.data(), (int)b.genome.size(), b.merit);
  o.merit = b.merit;
  o.copied_size = b.child_copied;
  o.executed_size = b.executed;
  o.gestation_time = b.gestation_time;
  o.fitness = b.fitness;
  o.generation = b.generation;
  for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) o.last_task[t] = b.last_task[t];
  o.rng = b.rng;
  o.age = 0;   // cPhenotype::SetupOffspring (main/cPhenotype.cc:705): 0 for the rest of its birth update
  // cEnvironment::SetupInputs random (main/cEnvironment.cc:1268-1271)
  Stream& r = ctx ? *ctx : o.rng;
  o.inputs[0] = (15 << 24) + (int)r.uint_below(1u << 24);
  o.inputs[1] = (51 << 24) + (int)r.uint_below(1u << 24);
  o.inputs[2] = (85 << 24) + (int)r.uint_below(1u << 24);
}

}  // namespace

// ===========================================================================
extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }

void* orc_create(const avgpu_cfg* cfg, int64_t ncells) {
  World* w = new World();
  w->cfg = *cfg;
  w->ncells = ncells > 0 ? ncells : (int64_t)cfg->world_x * cfg->world_y;
  w->orgs.resize(w->ncells);
  w->rows = cfg->world_y;
  w->global_rows = cfg->world_y;
  w->p_copy_mut = make_prob(cfg->copy_mut_prob);
  w->p_copy_ins = make_prob(cfg->copy_ins_prob);
  w->p_copy_del = make_prob(cfg->copy_del_prob);
  w->p_copy_uni = make_prob(cfg->copy_uniform_prob);
  w->p_copy_slip = make_prob(cfg->copy_slip_prob);
  w->p_div_mut = make_prob(cfg->divide_mut_prob);
  w->p_div_ins = make_prob(cfg->divide_ins_prob);
  w->p_div_del = make_prob(cfg->divide_del_prob);
  w->p_div_slip = make_prob(cfg->divide_slip_prob);
  w->p_div_uni = make_prob(cfg->divide_uniform_prob);
  w->p_div_site = make_prob(cfg->div_mut_prob);
  w->p_par_site = make_prob(cfg->parent_mut_prob);
  w->p_par_ins = make_prob(cfg->parent_ins_prob);
  w->p_par_del = make_prob(cfg->parent_del_prob);
  w->p_dsite[0] = make_prob(cfg->div_ins_prob);
  w->p_dsite[1] = make_prob(cfg->div_del_prob);
  w->p_dsite[2] = make_prob(cfg->div_uniform_prob);
  w->p_dsite[3] = make_prob(cfg->div_slip_prob);
  w->p_dsite[4] = make_prob(cfg->div_trans_prob);
  w->p_div_trans = make_prob(cfg->divide_trans_prob);
  w->pois_L[4] = cfg->divide_poisson_trans_mean > 0.0 ? std::exp(-cfg->divide_poisson_trans_mean) : 0.0;
  {
    const double means[4] = {cfg->divide_poisson_slip_mean, cfg->divide_poisson_mut_mean,
                             cfg->divide_poisson_ins_mean, cfg->divide_poisson_del_mean};
    for (int k = 0; k < 4; k++) w->pois_L[k] = means[k] > 0.0 ? std::exp(-means[k]) : 0.0;
  }
  memset(&w->stats, 0, sizeof(w->stats));
  derive_key((uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32), 0x5CEDu, 0xC0FFEEu,
             &w->global_rng.lo, &w->global_rng.hi);
  derive_key((uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32), 0xC7C7u, 0x5EED5u,
             &w->ctx_rng.lo, &w->ctx_rng.hi);
  return w;
}

void orc_destroy(void* h) { delete (World*)h; }

// avgpu_set_rng_mode restated (include/avida_gpu.h "random streams")
int orc_set_rng_mode(void* h, int mode, const double* stream, int64_t n, const int64_t* offsets) {
  World& w = *(World*)h;
  if (mode == AVGPU_RNG_COUNTER) {
    for (Org& o : w.orgs) { o.rng.rec = nullptr; o.rng.rec_len = 0; }
    w.rec.clear();
    return 0;
  }
  if (mode != AVGPU_RNG_RECORDED || !stream || n <= 0) return fail(AVGPU_EINVAL, "rng mode / stream");
  w.rec.assign(stream, stream + n);
  for (int64_t c = 0; c < w.ncells; c++) {
    const int64_t off = offsets ? offsets[c] : 0;
    if (off < 0 || off > n) return fail(AVGPU_EINVAL, "stream offset outside the stream");
    Org& o = w.orgs[c];
    o.rng.rec = w.rec.data() + off;
    o.rng.rec_len = n - off;
    o.rng.ctr = 0;
  }
  return 0;
}

int64_t orc_rec_exhausted(void) { return g_rec_over; }

int orc_load_instset(void* h, int n, const uint8_t* handler_id, const int32_t* redundancy) {
  World& w = *(World*)h;
  if (n <= 0 || n > AVGPU_MAX_INST) return fail(AVGPU_EINVAL, "bad instset size");
  w.is.n = n;
  int64_t cum = 0;
  for (int i = 0; i < n; i++) {
    w.is.handler[i] = handler_id[i];
    w.is.nopmod[i] = handler_id[i] <= 2 ? handler_id[i] : -1;
    cum += redundancy[i];
    w.is.cum[i] = cum;
  }
  w.is.total = cum;
  // NO_MUT_INSTS: op i's symbol (Instruction::GetSymbol, core/InstructionSequence.cc:
  // 69-106), its first character
  w.is.nomut = 0;
  for (int i = 0; i < n; i++) {
    const int k = i % 62;
    const char sym = i >= 62 ? "+-~?"[std::min(i / 62, 4) - 1]
                             : (char)(k < 26 ? 'a' + k : (k < 52 ? 'A' + k - 26 : '0' + k - 52));
    if (memchr(w.cfg.no_mut_insts, sym, (size_t)w.cfg.no_mut_insts_len)) w.is.nomut |= 1ull << i;
  }
  return 0;
}

// initial amounts (cResourceCount::Setup: RateAll(initial / size) + StateAll,
// main/cResourceCount.cc:323-328; SetCellList: Rate + State,
// main/cSpatialResCount.cc:216-231) of this world's cells (a strip tile holds
// rows [row0, row0 + rows) of the global grid)
static void res_init(World& w) {
  const int64_t n = w.ncells, nglobal = (int64_t)w.cfg.world_x * w.global_rows;
  const int nres = (int)w.res.size();
  w.res_amount.assign(nres, {});
  w.res_delta.assign(nres, {});
  w.res_global.assign(nres, 0.0);
  w.res_cons.assign(nres, 0);
  w.cons_cell.assign(nres, std::vector<double>(n, 0.0));
  w.res_first = true;
  for (int r = 0; r < nres; r++) {
    const avgpu_resource& q = w.res[r];
    if (q.geometry == AVGPU_RES_GLOBAL) { w.res_global[r] = q.initial; continue; }
    w.res_amount[r].assign(n, 0.0 + q.initial / (double)nglobal);
    w.res_delta[r].assign(n, 0.0);
  }
  for (const auto& c : w.res_cells) {
    const int64_t l = c.cell - w.cell0;
    if (c.cell >= 0 && c.cell < nglobal && l >= 0 && l < n) w.res_amount[c.resource][l] += (0.0 + c.initial);
  }
}

int orc_load_resources(void* h, int nres, const avgpu_resource* res, int ncell,
                       const avgpu_cell_resource* cells) {
  World& w = *(World*)h;
  if (nres < 0 || nres > AVGPU_MAX_RESOURCES) return fail(AVGPU_EINVAL, "resource count");
  w.res.assign(res, res + nres);
  w.res_cells.assign(cells, cells + ncell);
  w.res_decay100.assign(nres, 1.0);
  w.res_inflow100.assign(nres, 0.0);
  w.res_decay99.assign(nres, 1.0);
  w.res_inflow99.assign(nres, 0.0);
  w.res_slot.assign(nres, -1);
  w.n_spatial = 0;
  for (int r = 0; r < nres; r++) {
    const avgpu_resource& q = res[r];
    if (q.geometry != AVGPU_RES_GLOBAL) w.res_slot[r] = w.n_spatial++;
    // decay_precalc / inflow_precalc (main/cResourceCount.cc:336-345)
    const double decay = 1.0 - q.outflow;
    const double step_decay = std::pow(decay, 1.0 / 10000.0), step_inflow = q.inflow * (1.0 / 10000.0);
    double dp = 1.0, ip = 0.0;
    for (int i = 1; i <= 100; i++) {
      dp = dp * step_decay;
      ip = ip * step_decay + step_inflow;
      if (i == 99) { w.res_decay99[r] = dp; w.res_inflow99[r] = ip; }
    }
    w.res_decay100[r] = dp;
    w.res_inflow100[r] = ip;
  }
  res_init(w);
  return 0;
}

int orc_set_resources(void* h, const double* levels, const double* spatial) {
  World& w = *(World*)h;
  const int64_t n = w.ncells;
  for (size_t r = 0; r < w.res.size(); r++) {
    if (w.res[r].geometry == AVGPU_RES_GLOBAL) { w.res_global[r] = levels[r]; continue; }
    if (!spatial) return fail(AVGPU_EINVAL, "spatial resources need their grids");
    std::copy(spatial + r * n, spatial + (r + 1) * n, w.res_amount[r].begin());
  }
  std::fill(w.res_cons.begin(), w.res_cons.end(), 0);
  w.res_first = false;
  return 0;
}

int orc_get_resources(void* h, double* levels, double* spatial) {
  World& w = *(World*)h;
  const int64_t n = w.ncells;
  for (size_t r = 0; r < w.res.size(); r++) {
    if (w.res[r].geometry == AVGPU_RES_GLOBAL) {
      levels[r] = w.res_global[r];
      if (spatial) std::fill(spatial + r * n, spatial + (r + 1) * n, 0.0);
      continue;
    }
    double sum = 0.0;
    for (int64_t c = 0; c < n; c++) sum += w.res_amount[r][c];
    levels[r] = sum;
    if (spatial) std::copy(w.res_amount[r].begin(), w.res_amount[r].end(), spatial + r * n);
  }
  return 0;
}

int orc_load_env(void* h, int n, const avgpu_reaction* r) {
  World& w = *(World*)h;
  w.react.clear();
  for (int i = 0; i < n; i++) {
    Reaction x;
    x.r = r[i];
    double bonus = r[i].max_number * r[i].value;
    x.mult = (r[i].type == AVGPU_PROC_POW) ? std::pow(2.0, bonus) : bonus;
    x.add = bonus;
    w.react.push_back(x);
  }
  // REQUIRED_TASK / IMMUNITY_TASK index the task library: the distinct tasks
  // in the order of their first REACTION line (cTaskLib::AddTask)
  std::vector<int> lib;
  for (int i = 0; i < n; i++)
    if (std::find(lib.begin(), lib.end(), r[i].task) == lib.end()) lib.push_back(r[i].task);
  auto task_of = [&](int t) { return t >= 0 && t < (int)lib.size() ? lib[t] : -1; };
  w.req_task = task_of(w.cfg.required_task);
  w.imm_task = task_of(w.cfg.immunity_task);
  return 0;
}

static void reaper_inject(World& w, int64_t c, bool was_alive);
int orc_set_orgs(void* h, int64_t first, int64_t count, const uint8_t* genomes, const int32_t* lens,
                 const double* merits, const int32_t* inputs, int deterministic) {
  World& w = *(World*)h;
  size_t off = 0;
  for (int64_t i = 0; i < count; i++) {
    int64_t c = first + i;
    Org& o = w.orgs[c];
    reaper_inject(w, c, o.alive);
    setup_inject(w, o, genomes + off, lens[i], merits ? merits[i] : 0.0);
    off += lens[i];
    derive_key((uint32_t)w.cfg.seed, (uint32_t)(w.cfg.seed >> 32), (uint32_t)(w.cell0 + c), 0xA5A5A5A5U,
               &o.rng.lo, &o.rng.hi);
    o.rng.ctr = 0;
    if (inputs) { for (int k = 0; k < 3; k++) o.inputs[k] = inputs[i * 3 + k]; }
    else if (deterministic) {  // cEnvironment::SetupInputs(random=false) :1286-1289
      o.inputs[0] = 0x0f13149f; o.inputs[1] = 0x3308e53e; o.inputs[2] = 0x556241eb;
    } else {
      o.inputs[0] = (15 << 24) + (int)o.rng.uint_below(1u << 24);
      o.inputs[1] = (51 << 24) + (int)o.rng.uint_below(1u << 24);
      o.inputs[2] = (85 << 24) + (int)o.rng.uint_below(1u << 24);
    }
  }
  return 0;
}

int orc_kill(void* h, int64_t cell) { ((World*)h)->orgs[cell].alive = false; return 0; }

// instruction-mix histogram over everything executed since the last call
int orc_op_hist(int64_t* out, int n) {
  for (int i = 0; i < n && i < 64; i++) { out[i] = g_op_hist[i]; g_op_hist[i] = 0; }
  return 0;
}

// Batched SingleProcess for a range (FROZEN / TEST / WORLD semantics).
int orc_step(void* h, int64_t first, int64_t count, const int32_t* budget, int32_t uniform, int mode) {
  World& w = *(World*)h;
  int64_t insts = 0;
  for (int64_t i = 0; i < count; i++) {
    int64_t c = first + i;
    Org& o = w.orgs[c];
    int b = budget ? budget[i] : uniform;
    Exec ex{w, o, mode};
    for (int k = 0; k < b && o.alive && !ex.stop; k++) { ex.single_process(c); insts++; }
  }
  w.step_insts = insts;
  return 0;
}

int orc_last_step_insts(void* h, int64_t* out) { *out = ((World*)h)->step_insts; return 0; }

int orc_get_states(void* h, int64_t first, int64_t count, avgpu_cpu_state* st, uint8_t* ops,
                   uint8_t* flags, int cap) {
  World& w = *(World*)h;
  for (int64_t i = 0; i < count; i++)
    dump_state(w, w.orgs[first + i], &st[i], ops ? ops + i * cap : nullptr,
               flags ? flags + i * cap : nullptr, cap);
  return 0;
}

// Genome key of a birth genome (the device's
// gk_* in avida_amd/csrc/device.h): canonical codes handler[op] in 4-site
// little-endian words, each mixed with its index, summed mod 2^64, mixed with
// the length.  Stands in for the genome equality that files a newborn under
// its genotype (Systematics::GenotypeArbiter::ClassifyNewUnit,
// systematics/GenotypeArbiter.cc:280-380; hashGenome :470-480).
static uint64_t gk_mix(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t genome_key(const World& w, const std::vector<uint8_t>& g) {
  const int len = (int)g.size();
  uint64_t sum = 0;
  for (int wd = 0; wd < (len + 3) / 4; wd++) {
    uint32_t v = 0;
    for (int j = 0; j < 4 && 4 * wd + j < len; j++)
      v |= (uint32_t)(w.is.handler[g[4 * wd + j]] & 0x3F) << (8 * j);
    sum += gk_mix(((uint64_t)(wd + 1) << 32) | v);
  }
  const uint64_t k = gk_mix(sum ^ ((uint64_t)len * 0x9E3779B97F4A7C15ull));
  return k ? k : 1ull;
}

// Per-cell state digest, restating the device's k_state_digest (avida_amd/
// csrc/world.hip): chained mix over the words of the dump_state tuple, then the
// tape in canonical bytes (handler | copied << 6 | executed << 7).  0 for a
// cell that never held an organism.
int orc_state_digests(void* h, int64_t first, int64_t count, uint64_t* out) {
  World& w = *(World*)h;
  if (first < 0 || count < 0 || first + count > w.ncells) return fail(AVGPU_EINVAL, "cell range");
  for (int64_t i = 0; i < count; i++) {
    const Org& o = w.orgs[first + i];
    if (o.genome.empty()) { out[i] = 0; continue; }
    avgpu_cpu_state s;
    dump_state(w, o, &s, nullptr, nullptr, 0);
    uint32_t wd[sizeof(s) / 4];
    memcpy(wd, &s, sizeof(wd));
    uint64_t hsh = 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < (int)(sizeof(s) / 4); k++) hsh = gk_mix(hsh ^ ((uint64_t)k << 32 | wd[k]));
    const int m = (int)o.mem.size();
    for (int k = 0; k < (m + 3) / 4; k++) {
      uint32_t v = 0;
      for (int j = 0; j < 4 && 4 * k + j < m; j++) {
        const int q = 4 * k + j;
        const uint32_t b = (uint32_t)(w.is.handler[o.mem[q]] & 0x3F) | ((o.flg[q] & F_COPIED) ? 0x40u : 0u) |
                           ((o.flg[q] & F_EXECUTED) ? 0x80u : 0u);
        v |= b << (8 * j);
      }
      hsh = gk_mix(hsh ^ ((uint64_t)(0x10000 + k) << 32 | v));
    }
    out[i] = hsh;
  }
  return 0;
}

int orc_get_census(void* h, int64_t first, int64_t count, avgpu_census* out) {
  World& w = *(World*)h;
  if (first < 0 || count < 0 || first + count > w.ncells) return fail(AVGPU_EINVAL, "cell range");
  for (int64_t i = 0; i < count; i++) {
    const Org& o = w.orgs[first + i];
    avgpu_census& r = out[i];
    memset(&r, 0, sizeof(r));
    if (!o.alive) continue;
    r.genotype_key = o.gkey_restored ? o.gkey_restored : genome_key(w, o.genome);
    r.merit = o.merit;
    r.fitness = o.fitness;
    r.genome_length = (int)o.genome.size();
    r.gestation_time = o.gestation_time;
    r.copied_size = o.copied_size;
    r.executed_size = o.executed_size;
    r.generation = o.generation;
    r.num_divides = o.num_divides;
  }
  return 0;
}

int orc_set_genotype_keys(void* h, int64_t first, int64_t count, const uint64_t* keys) {
  World& w = *(World*)h;
  if (first < 0 || count < 0 || first + count > w.ncells) return fail(AVGPU_EINVAL, "cell range");
  for (int64_t i = 0; i < count; i++) w.orgs[first + i].gkey_restored = keys[i];
  return 0;
}

// checkpoint restore: the inverse of dump_state (ops are instruction-set op
// codes; flags bit0 copied, bit2 executed)
int orc_set_states(void* h, int64_t first, int64_t count, const avgpu_cpu_state* st, const uint8_t* ops,
                   const uint8_t* flags, int cap) {
  World& w = *(World*)h;
  if (first < 0 || count < 0 || first + count > w.ncells) return fail(AVGPU_EINVAL, "cell range");
  for (int64_t i = 0; i < count; i++) {
    const avgpu_cpu_state& s = st[i];
    if (s.mem_size < 0 || s.mem_size > cap) return fail(AVGPU_EINVAL, "memory size outside mem_cap");
    Org& o = w.orgs[first + i];
    o = Org();
    o.alive = s.alive != 0;
    o.mem.assign(ops + i * cap, ops + i * cap + s.mem_size);
    o.flg.assign(flags + i * cap, flags + i * cap + s.mem_size);
    for (auto& f : o.flg) f &= (F_COPIED | F_EXECUTED);
    for (int k = 0; k < 3; k++) o.reg[k] = s.reg[k];
    for (int k = 0; k < 4; k++) o.head[k] = s.head[k];
    for (int k = 0; k < 2; k++) {
      for (int j = 0; j < AVGPU_STACK_SIZE; j++) o.stk[k].s[j] = s.stack[k][j];
      o.stk[k].sp = s.stack_ptr[k];
    }
    o.cur_stack = s.cur_stack;
    o.read_label.size = s.read_label_len;
    for (int k = 0; k < s.read_label_len && k < AVGPU_MAX_LABEL; k++) o.read_label.nops[k] = s.read_label[k];
    o.mal_active = s.mal_active != 0;
    // the birth genome: only its length is state (birth_length); its sites are
    // the memory's leading sites at the checkpoint
    o.genome.assign(o.mem.begin(), o.mem.begin() + std::min<int>(s.birth_length, (int)o.mem.size()));
    o.genome.resize(s.birth_length, 0);
    o.cpu_cycles_used = s.cpu_cycles_used; o.time_used = s.time_used;
    o.gestation_start = s.gestation_start; o.gestation_time = s.gestation_time;
    o.num_divides = s.num_divides; o.generation = s.generation;
    o.genome_length = s.genome_length; o.copied_size = s.copied_size;
    o.child_copied_size = s.child_copied_size; o.executed_size = s.executed_size;
    o.max_executed = s.max_executed;
    o.input_ptr = s.input_ptr;
    o.input_buf.cap = 3; o.input_buf.offset = 0; o.input_buf.total = s.input_total;
    for (int k = 0; k < 3; k++) o.input_buf.data[2 - k] = s.input_buf[k];   // [i] = data[cap-1-i]
    o.output_buf.cap = 1; o.output_buf.offset = 0; o.output_buf.total = s.output_total;
    o.output_buf.data[0] = s.output_buf;
    for (int k = 0; k < 3; k++) o.inputs[k] = s.inputs[k];
    for (int k = 0; k < AVGPU_MAX_REACTIONS; k++) {
      o.cur_task[k] = s.cur_task_count[k];
      o.last_task[k] = s.last_task_count[k];
      o.cur_react[k] = s.cur_reaction_count[k];
    }
    o.rng.lo = s.rng_key_lo; o.rng.hi = s.rng_key_hi; o.rng.ctr = s.rng_counter;
    o.rng.rec = nullptr; o.rng.rec_len = 0;   // restored organisms draw from counter streams
    o.errors = s.errors;
    o.cur_bonus = s.cur_bonus; o.merit = s.merit; o.fitness = s.fitness; o.credit = s.credit;
    o.hstart = s.head_start;
    if (tracks_age(w)) o.age = s.age - 1;
  }
  return 0;
}

int orc_set_clock(void* h, const avgpu_update_stats* last) {
  World& w = *(World*)h;
  w.update = last->update + 1;
  w.cum_insts = last->cum_insts_executed;
  w.cum_births = last->cum_births;
  if (last->seed != 0) {   // zero: stats of an older checkpoint -- the configured seed stays
    w.cfg.seed = last->seed;
    w.stats.seed = last->seed;
    // the serial world's two streams are keyed by the seed too (positions stay)
    derive_key((uint32_t)w.cfg.seed, (uint32_t)(w.cfg.seed >> 32), 0x5CEDu, 0xC0FFEEu,
               &w.global_rng.lo, &w.global_rng.hi);
    derive_key((uint32_t)w.cfg.seed, (uint32_t)(w.cfg.seed >> 32), 0xC7C7u, 0x5EED5u,
               &w.ctx_rng.lo, &w.ctx_rng.hi);
  }
  // the adaptive sub-step predictor the next update decides by (0: one step)
  w.pred_acc = last->sched_pred;
  w.pred_n = last->sched_pred_n;
  w.carry_rem = last->sched_carry;
  w.carry_new = 0;
  for (int k = 0; k < 4; k++) w.pred_bin[k] = last->sched_pred_bins[k];
  return 0;
}

// cTestCPU::TestGenome_Body for one gestation (cpu/cTestCPU.cc:144-188, :233-326)
int orc_test_genomes(void* h, int n, const uint8_t* genomes, const int32_t* lens,
                     avgpu_test_result* res, char* exec_flags, int flags_cap, uint8_t* offspring) {
  World& w = *(World*)h;
  size_t off = 0;
  for (int i = 0; i < n; i++) {
    Org o;
    const int len = lens[i];
    setup_inject(w, o, genomes + off, len, 0.0);
    off += len;
    o.inputs[0] = 0x0f13149f; o.inputs[1] = 0x3308e53e; o.inputs[2] = 0x556241eb;
    Exec ex{w, o, AVGPU_MODE_TEST};
    const int time_allocated = w.cfg.test_cpu_time_mod * len;
    int t = 0;
    while (t < time_allocated && o.num_divides == 0 && o.alive) { t++; ex.single_process(-1); }
    avgpu_test_result& r = res[i];
    memset(&r, 0, sizeof(r));
    r.divided = o.num_divides > 0;
    r.copied_size = o.copied_size;
    r.executed_size = o.executed_size;
    r.gestation_time = o.gestation_time;
    r.genome_length = o.genome_length;
    r.time_used = o.time_used;
    r.merit = o.merit;
    r.fitness = o.fitness;
    for (int k = 0; k < AVGPU_MAX_REACTIONS; k++) r.task_count[k] = o.last_task[k];
    r.offspring_len = (int)o.offspring.size();
    r.copy_true = r.divided && o.offspring == o.genome;
    if (exec_flags) {
      std::string f = o.exec_flags_at_divide;
      if (!r.divided) {
        f.assign(o.mem.size(), '-');
        for (size_t k = 0; k < o.mem.size(); k++) if (o.flg[k] & F_EXECUTED) f[k] = '+';
      }
      char* dst = exec_flags + (size_t)i * flags_cap;
      memset(dst, 0, flags_cap);
      memcpy(dst, f.data(), std::min((int)f.size(), flags_cap - 1));
    }
    if (offspring) {
      uint8_t* dst = offspring + (size_t)i * AVGPU_MAX_GENOME;
      memset(dst, 0, AVGPU_MAX_GENOME);
      memcpy(dst, o.offspring.data(), o.offspring.size());
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Batch-synchronous world update: the exact semantics the device implements
// (DESIGN.md "Update semantics"): allot -> interpret -> place births -> stats.
static int amod(int x, int y) { x %= y; return x < 0 ? x + y : x; }   // AvidaTools::Mod

// FlowMatter (main/cResourceCount.cc:40-110)
static void flow_matter(double a1, double a2, double& d1, double& d2, const avgpu_resource& r,
                        int xdist, int ydist, double dist) {
  double diff, flowamt, xgravity, xdiffuse, ygravity, ydiffuse;
  diff = (a1 - a2);
  if (xdist != 0) {
    if (((xdist > 0) && (r.xgravity > 0.0)) || ((xdist < 0) && (r.xgravity < 0.0)))
      xgravity = a1 * std::fabs(r.xgravity) / 3.0;
    else
      xgravity = -a2 * std::fabs(r.xgravity) / 3.0;
    xdiffuse = r.xdiffuse * diff / 16.0;
  } else {
    xdiffuse = 0.0;
    xgravity = 0.0;
  }
  if (ydist != 0) {
    if (((ydist > 0) && (r.ygravity > 0.0)) || ((ydist < 0) && (r.ygravity < 0.0)))
      ygravity = a1 * std::fabs(r.ygravity) / 3.0;
    else
      ygravity = -a2 * std::fabs(r.ygravity) / 3.0;
    ydiffuse = r.ydiffuse * diff / 16.0;
  } else {
    ydiffuse = 0.0;
    ygravity = 0.0;
  }
  flowamt = ((xdiffuse + ydiffuse + xgravity + ygravity) /
             (std::fabs(xdist * 1.0) + std::fabs(ydist * 1.0))) / dist;
  d1 -= flowamt;
  d2 += flowamt;
}

// one update of resources at its start (cPopulation::ProcessPreUpdate + the
// first DoUpdates: DoSpatialUpdates main/cResourceCount.cc:830-846 with
// Source / Sink / CellInflow / CellOutflow / FlowAll / StateAll of
// main/cSpatialResCount.cc, and DoNonSpatialUpdates :814-827).
// Update 0 has no spatial step (m_spatial_update == m_last_updated == 0,
// :797) and 9999 global steps: the update_time the steps of update 0 add up
// to falls just short of 1.0, so (int)(update_time / UPDATE_STEP) is 9999
// (:780) and the remainder carries, making every later update 10000 steps.
// Pinned by tests/golden/spatial_res_100u (test_resources.py).
static void res_begin(World& w) {
  const int X = w.cfg.world_x, Yg = (int)w.global_rows;
  const int64_t n = w.ncells;
  const bool first = w.res_first;
  w.res_first = false;
  // this world's rows of the global grid; a strip tile reads the rows above
  // and below from the edge rows its neighbours sent (rs_recv)
  auto local = [&](int64_t g) -> int64_t {
    const int64_t l = g - w.cell0;
    return (l >= 0 && l < n) ? l : -1;
  };
  for (size_t r = 0; r < w.res.size(); r++) {
    const avgpu_resource& q = w.res[r];
    if (q.geometry == AVGPU_RES_GLOBAL) {
      double R = w.res_global[r];
      int steps = first ? 9999 : 10000;
      while (steps > 100) { R *= w.res_decay100[r]; R += w.res_inflow100[r]; steps -= 100; }
      if (steps == 100) { R *= w.res_decay100[r]; R += w.res_inflow100[r]; }
      else { R *= w.res_decay99[r]; R += w.res_inflow99[r]; }
      w.res_global[r] = R;
      continue;
    }
    if (first) continue;
    std::vector<double>& amt = w.res_amount[r];
    std::vector<double>& d = w.res_delta[r];
    const int slot = w.res_slot[r];
    auto amount = [&](int gy, int x) -> double {
      const int ly = gy - (int)w.row0;
      if (ly >= 0 && ly < w.rows) return amt[(int64_t)ly * X + x];
      if (gy == amod((int)w.row0 - 1, Yg)) return w.rs_recv[0][(int64_t)slot * X + x];
      return w.rs_recv[1][(int64_t)slot * X + x];
    };
    // Source
    double amount_in = q.inflow;
    const double totalcells = (q.inflow_y2 - q.inflow_y1 + 1) * (q.inflow_x2 - q.inflow_x1 + 1) * 1.0;
    amount_in /= totalcells;
    for (int i = q.inflow_y1; i <= q.inflow_y2; i++)
      for (int j = q.inflow_x1; j <= q.inflow_x2; j++) {
        const int64_t l = local((int64_t)amod(i, Yg) * X + amod(j, X));
        if (l >= 0) d[l] += amount_in;
      }
    // Sink
    const double decay = 1.0 - q.outflow;
    if (!(q.outflow_x1 == AVGPU_RES_NONE || q.outflow_y1 == AVGPU_RES_NONE ||
          q.outflow_x2 == AVGPU_RES_NONE || q.outflow_y2 == AVGPU_RES_NONE))
      for (int i = q.outflow_y1; i <= q.outflow_y2; i++)
        for (int j = q.outflow_x1; j <= q.outflow_x2; j++) {
          const int64_t l = local((int64_t)amod(i, Yg) * X + amod(j, X));
          if (l >= 0) d[l] += -std::max(amt[l] * (1.0 - decay), 0.0);
        }
    // CellInflow / CellOutflow (cell ids are global)
    bool any_cells = false;
    for (const auto& c : w.res_cells) if (c.resource == (int)r) any_cells = true;
    if (any_cells) {
      for (const auto& c : w.res_cells) {
        const int64_t l = local(c.cell);
        if (c.resource == (int)r && l >= 0) d[l] += c.inflow;
      }
      for (const auto& c : w.res_cells) {
        const int64_t l = local(c.cell);
        if (c.resource == (int)r && l >= 0) d[l] += -std::max(amt[l] * c.outflow, 0.0);
      }
    }
    // FlowAll: pointers 3..6 of every cell in global cell order; the cells
    // that reach this world's rows are its own and those of the row above
    if (q.xdiffuse != 0.0 || q.ydiffuse != 0.0 || q.xgravity != 0.0 || q.ygravity != 0.0) {
      const double SQRT2 = std::sqrt(2.0);
      const int dxk[7] = {0, 0, 0, 1, 1, 0, -1}, dyk[7] = {0, 0, 0, 0, 1, 1, 1};
      std::vector<int> rows_g;
      for (int ly = 0; ly < w.rows; ly++) rows_g.push_back((int)w.row0 + ly);
      if (w.tiled && (w.row0 > 0 || q.geometry != AVGPU_RES_GRID)) rows_g.push_back(amod((int)w.row0 - 1, Yg));
      std::sort(rows_g.begin(), rows_g.end());
      for (int gy : rows_g)
        for (int x = 0; x < X; x++) {
          const int64_t li = local((int64_t)gy * X + x);
          for (int k = 3; k <= 6; k++) {
            if (q.geometry == AVGPU_RES_GRID) {
              if ((k == 3 || k == 4) && x == X - 1) continue;
              if (k == 6 && x == 0) continue;
              if (k != 3 && gy == Yg - 1) continue;
            }
            const int ny = amod(gy + dyk[k], Yg), nx = amod(x + dxk[k], X);
            const int64_t lii = local((int64_t)ny * X + nx);
            if (li < 0 && lii < 0) continue;
            double sink1 = 0.0, sink2 = 0.0;
            flow_matter(amount(gy, x), amount(ny, nx), li >= 0 ? d[li] : sink1, lii >= 0 ? d[lii] : sink2,
                        q, dxk[k], dyk[k], (k == 4 || k == 6) ? SQRT2 : 1.0);
          }
        }
    }
    // StateAll
    for (int64_t i = 0; i < n; i++) { amt[i] += d[i]; d[i] = 0.0; }
  }
}

// the update's consumption of global resources (fixed point, DESIGN.md "Resources")
static void res_end(World& w) {
  for (size_t r = 0; r < w.res.size(); r++) {
    if (w.res[r].geometry != AVGPU_RES_GLOBAL) continue;
    w.res_global[r] = std::max(w.res_global[r] - (double)w.res_cons[r] / 4294967296.0, 0.0);
    w.res_cons[r] = 0;
  }
}

// 1. allotment (cScheduler restated; DESIGN.md "Scheduler") + 2. interpretation
// PROBABILISTIC: the update's picks split down the cell tree (block_split);
// INTEGRATED: lambda = UD * weight / total with a credit carry;
// CONSTANT: AVE_TIME_SLICE.  A divide stamps its birth record
// with its time in the update, t = k / (b + 1) in 1/2^16 (k: the slice's
// instructions up to and including the h-divide, b: the slice's budget) --
// the expected position of the k-th of b instructions spread uniformly over
// the update, which is how the reference's one-instruction picks interleave
// organisms (main/cPopulation.cc:5698-5701).
static inline uint32_t birth_time(int k, int budget) {
  return (uint32_t)(((double)k * 65536.0) / (double)((int64_t)budget + 1));
}

// the densest quarter's divide count (choose_k)
static int64_t densest(const int64_t* bins) {
  int64_t m = 0;
  for (int k = 0; k < 4; k++) m = std::max(m, bins[k]);
  return m;
}

// The adaptive sub-step predictor, one organism's term at the
// end of its slice: an organism expected to reach its divide within the next
// update's share of picks (its gestation time, or for one that never divided
// its genome length, against the cycles of its current gestation) is counted
// in the quarter of the update its divide is expected in (the divide
// density: a cohort in lock step fills one quarter, a steady state spreads
// over all four), and it changes the scheduler's total weight by its
// merit's change at the divide (its size times its bonus so far, for one
// that never divided; else its merit stays) and by as much again through its
// offspring, which takes the merit to a neighbour's cell (a relative's, of
// about its old merit) -- from that point of the update on: the
// within-update weight change the batch step reads only once
// (main/cPopulation.cc:610-615 AdjustSchedule at every divide).  In units of
// the mean weight, 2^-20 fixed point (an order-free sum).  Organisms that
// divided in this slice are left out (their next divide is a gestation away).
// The device's pred_term (interp.hip) is the same arithmetic.
static int64_t pred_term(const World& w, const Org& o, double total, int64_t nalive, int64_t* bins) {
  const double wbar = total / (double)nalive;
  const double wi = o.merit;
  if (!(wi > 0.0) || !(wi <= 1.7976931348623157e308) || !(wbar > 0.0)) return 0;
  const double e = ((double)w.cfg.ave_time_slice * wi) / wbar;
  const int G = o.gestation_time > 0 ? o.gestation_time : o.genome_length;
  const double r = (double)(G - (o.time_used - o.gestation_start));
  if (!(r <= e * 1.25)) return 0;
  const double t = r <= 0.0 ? 0.0 : std::fmin(r / e, 1.0);
  bins[std::min(3, (int)(t * 4.0))]++;
  int sz = o.genome_length;
  if (sz > o.copied_size) sz = o.copied_size;
  if (sz > o.executed_size) sz = o.executed_size;
  const double m = o.gestation_time > 0 ? wi : (double)sz * o.cur_bonus;
  double term = (((m - wi) + (m - wi)) * (1.0 - t)) / wbar;
  if (!(term <= 1.0e6)) term = 1.0e6;
  if (!(term >= -1.0e6)) term = -1.0e6;
  return (int64_t)(term * 1048576.0);
}

// blk: each of this world's blocks' share of the update's picks (top_tree),
// total: the total weight, ud: the update size (INTEGRATED's lambda =
// ud * weight / total), nalive: the living organisms the weights are over
// (the predictor's mean weight)
static void allot_interpret(World& w, const std::vector<int64_t>& blk, double total, double ud, int64_t nalive) {
  std::vector<int32_t> budget(w.ncells, 0);
  const bool consts = w.cfg.slicing_method == AVGPU_SLICE_CONSTANT || !(total > 0.0);
  if (!consts && w.cfg.slicing_method != AVGPU_SLICE_INTEGRATED)
    for (int64_t b = 0; b < (int64_t)blk.size(); b++) block_split(w, b, blk[b], budget.data());
  for (int64_t c = 0; c < w.ncells; c++) {
    Org& o = w.orgs[c];
    if (!o.alive) { budget[c] = 0; continue; }
    const double wt = sched_weight(o);
    o.hstart = 0;                               // consumed by this allotment
    if (consts) {
      budget[c] = w.cfg.ave_time_slice;
    } else if (w.cfg.slicing_method == AVGPU_SLICE_INTEGRATED) {
      double lam = (ud * wt) / total;
      if (lam > 1.0e8) lam = 1.0e8;
      o.credit = o.credit + lam;
      double fl = std::floor(o.credit);
      budget[c] = (int32_t)fl;
      o.credit = o.credit - fl;
    }
  }
  w.t_slices = 0;
  for (int64_t c = 0; c < w.ncells; c++) w.t_slices += budget[c] > 0;
  w.last_budget = budget;
  w.births.clear();
  for (auto& v : w.cons_cell) std::fill(v.begin(), v.end(), 0.0);
  w.pred_acc = 0;
  for (int k = 0; k < 4; k++) w.pred_bin[k] = 0;
  w.pred_n = nalive;
  w.ran.assign(w.ncells, 0);
  int64_t insts = 0, deaths = 0, divides = 0;
  for (int64_t c = 0; c < w.ncells; c++) {
    Org& o = w.orgs[c];
    if (!o.alive) continue;
    Exec ex{w, o, AVGPU_MODE_WORLD};
    int d0 = o.num_divides;
    const int tu0 = o.time_used;
    for (int k = 0; k < budget[c] && o.alive; k++) {
      const size_t nb0 = w.births.size();
      ex.single_process(c); insts++;
      w.ran[c]++;
      if (w.births.size() != nb0) w.births.back().t = birth_time(k + 1, budget[c]);
    }
    divides += o.num_divides - d0;
    if (!o.alive) deaths++;
    else if (budget[c] > 0 && o.gestation_start <= tu0 && total > 0.0 && nalive > 0)
      w.pred_acc += pred_term(w, o, total, nalive, w.pred_bin);
  }
  w.t_insts = insts; w.t_deaths = deaths; w.t_divides = divides;
}

// The newborns of a batch step (the reference places an
// offspring inside its parent's divide and schedules it for the rest of that
// update, main/cPopulation.cc:621-952): each activated offspring first gives
// back what the organism it replaced consumed in this step's main pass after
// the birth -- (1 - t) of the cell's depletable consumption -- and then runs
// its own share of the step's remaining picks, Binomial(round(UD_s (1 - t)),
// weight / total) from a stateless node draw of its global cell, stopping
// before an h-divide (its offspring would need a placement this step has
// already done).  The device's k_activate / newborn pass (world.hip,
// interp.hip NB) run the same.
enum : uint32_t { SALT_NEWBORN = 0x4E3B0A17u };
static int64_t newborn_budget(const World& w, int64_t cell, uint32_t t, int64_t uds, double total) {
  const Org& o = w.orgs[cell];
  if (!(total > 0.0) || uds <= 0) return 0;
  const double f = (double)(0x10000u - t) * (1.0 / 65536.0);
  const int64_t n = (int64_t)std::floor((double)uds * f + 0.5);
  const double p = sched_weight(o) / total;
  int64_t b = binom_draw(n, p, node_draw(w, w.sched_key, SALT_NEWBORN, (uint64_t)(w.cell0 + cell)));
  return std::min<int64_t>(b, (1 << 30) - 1);
}
static void newborn_credit(World& w, int64_t cell, uint32_t t) {
  const double f = (double)(0x10000u - t) * (1.0 / 65536.0);
  for (size_t r = 0; r < w.res.size(); r++) {
    const double v = w.cons_cell[r][cell];
    if (v == 0.0) continue;
    const double back = v * f;
    if (w.res[r].geometry != AVGPU_RES_GLOBAL) w.res_amount[r][cell] = w.res_amount[r][cell] + back;
    else w.res_cons[r] -= (uint64_t)(back * 4294967296.0);
  }
}
static void newborn_pass(World& w, int64_t uds, double total) {
  int64_t insts = 0, deaths = 0;
  for (const auto& nb : w.newborns) {
    const int64_t c = nb.first;
    if (!w.res.empty()) newborn_credit(w, c, nb.second);
    Org& o = w.orgs[c];
    const int64_t bud = newborn_budget(w, c, nb.second, uds, total);
    const int64_t left = (int64_t)((double)w.ran[c] * ((double)(0x10000u - nb.second) * (1.0 / 65536.0)));
    w.carry_new += bud - left;
    w.t_wasted += left;
    if (bud <= 0) continue;
    w.t_slices++;
    Exec ex{w, o, AVGPU_MODE_WORLD};
    ex.nb_stop = true;
    for (int64_t k = 0; k < bud && o.alive; k++) {
      ex.single_process(c);
      if (ex.nb_halted) break;
      insts++;
    }
    if (!o.alive) deaths++;
  }
  w.newborns.clear();
  w.t_insts += insts;
  w.t_deaths += deaths;
}

// 5. statistics (main/cStats.cc:1081-1100 inputs)
static void finish_stats(World& w, int64_t placed, int64_t dropped) {
  avgpu_update_stats& st = w.stats;
  memset(&st, 0, sizeof(st));
  st.update = w.update;
  st.insts_executed = w.t_insts;
  st.births = placed;
  st.births_dropped = dropped + w.t_oversize;
  w.t_oversize = 0;
  st.deaths = w.t_deaths;
  st.divides = w.t_divides;
  double gen = 0.0;
  for (int64_t c = 0; c < w.ncells; c++) {
    const Org& o = w.orgs[c];
    if (!o.alive) continue;
    st.num_organisms++;
    st.sum_merit += o.merit;
    st.sum_fitness += o.fitness;
    st.sum_gestation += o.gestation_time;
    st.sum_genome_length += (double)o.genome.size();
    if (o.fitness > st.max_fitness) st.max_fitness = o.fitness;
    gen += o.generation;
    for (int t = 0; t < AVGPU_MAX_REACTIONS; t++) if (o.last_task[t] > 0) st.task_orgs[t]++;
  }
  st.ave_generation = st.num_organisms ? gen / st.num_organisms : 0.0;
  for (int64_t c = 0; c < w.ncells; c++) if (w.orgs[c].alive) st.sum_mem_size += (double)w.orgs[c].mem.size();
  w.cum_insts += w.t_insts;
  w.cum_births += placed;
  st.cum_insts_executed = w.cum_insts;
  st.cum_births = w.cum_births;
  st.slices = w.t_slices;
  st.births_overwritten = w.t_overwritten;
  st.births_cancelled = w.t_cancelled;
  st.seed = w.cfg.seed;
  st.sched_pred = w.pred_acc;
  st.sched_pred_n = w.pred_n;
  st.sub_steps = w.last_k;
  st.sched_carry = w.carry_rem + w.carry_new;
  st.sched_pred_cnt = densest(w.pred_bin);
  for (int k = 0; k < 4; k++) st.sched_pred_bins[k] = w.pred_bin[k];
  st.insts_wasted = w.t_wasted;
  w.t_wasted = 0;
  w.t_overwritten = 0;
  w.t_cancelled = 0;
  w.update++;
}

extern "C++" {
// ---------------------------------------------------------------------------
// 3. Time-ordered placement.  The reference places each
// offspring inside its parent's h-divide (ActivateOffspring,
// main/cPopulation.cc:621-952 -> PositionOffspring :5185-5414), so an
// organism whose cell receives an offspring before its own divide never
// divides, an earlier birth takes an empty cell before a later one, and a
// later birth into an occupied cell kills whatever is there.  The batch update
// restates that order from the records' birth times t:
//   launch 0  every record picks a target (PositionOffspring: an empty
//             neighbour, else any neighbour or the parent); a pick whose
//             target is taken is a kill, and the cell's kill time is the
//             earliest such t (killt = 2^16 - t, max-reduced);
//   launch 0b a record whose parent's cell was killed before its own time
//             (killt[parent] > 2^16 - t) is cancelled -- its parent died
//             before dividing; the rest claim their targets;
//   launch m  (1..3) round m-1 resolved: the maximum claim wins.  Claim keys
//             order empty-cell claims earliest first and kill claims latest
//             first, so an empty cell goes to its earliest claimer and a kill
//             target to its latest -- the earlier kills were placed and
//             overwritten, as in the reference.  A winner owns its cell
//             unless the cell's owner from an earlier round is later in time
//             (that owner overwrote it).  A lost empty claim picks again
//             (cells claimed in round m-1 count as taken); a lost kill claim
//             is placed and overwritten;
//   activation round 3 resolved the same way; every owner is activated.
// claim key: [63:48] time key (kill: t, empty: 0xFFFF - t), [47] kill,
// [46:32] the pick's draw >> 17, [31:8] the parent's GLOBAL cell id (tiles
// agree), [7:0] its divide number -- unique per record.
static inline uint64_t claim_key(uint32_t t, bool kill, uint32_t draw, int64_t gparent, uint32_t seq) {
  const uint64_t tk = kill ? (uint64_t)(t & 0xFFFFu) : (uint64_t)(0xFFFFu - (t & 0xFFFFu));
  return (tk << 48) | ((uint64_t)(kill ? 1 : 0) << 47) | ((uint64_t)(draw >> 17) << 32) |
         ((uint64_t)(gparent & 0xFFFFFF) << 8) | (uint64_t)(seq & 0xFF);
}
static inline bool key_kill(uint64_t k) { return ((k >> 47) & 1ull) != 0; }
static inline uint32_t key_time(uint64_t k) {
  const uint32_t tk = (uint32_t)(k >> 48);
  return key_kill(k) ? tk : 0xFFFFu - tk;
}
// record states (Birth index i -> bstate[i])
enum : int8_t { BS_PENDING = 0, BS_WON = 1 /* 1 + round */, BS_KILL_LOST = 8 /* 8 + round */,
                BS_CANCELLED = -1, BS_NO_CELL = -2 /* - round */ };
// owner: >= 0 a record of this world, -1 none, <= -2 a neighbouring strip's
// offspring that won round m at time t (strip tiles)
static inline int64_t remote_owner(int m, uint32_t t) { return -2 - ((int64_t)m + 4 * (int64_t)t); }
static inline uint32_t owner_time(const World& w, int64_t o) {
  return o >= 0 ? w.births[o].t : (uint32_t)((-2 - o) >> 2);
}
// a cell's owner after a round-m winner with time t: it replaces the owner
// unless the owner is later in time
static inline bool takes_cell(const World& w, int64_t owner, uint32_t t) {
  return owner == -1 || owner_time(w, owner) <= t;
}

// PositionOffspring for record i in round m (main/cPopulation.cc:5353-5413):
// an empty neighbour (not taken) when PREFER_EMPTY, else any of the eight
// neighbours or the parent (ALLOW_PARENT).  BIRTH_METHOD 3 with no empty
// neighbour: PositionOffspring returns the parent's cell without a draw
// (:5407) and ActivateOffspring places the offspring there only if
// ALLOW_PARENT (:706-713); otherwise it is never placed (BS_NO_CELL).
// Writes the record's target and key (and w.tgt_r[m][i]); returns false for
// no cell.
// A cell's value for BIRTH_METHOD 1 (its organism's age) or 2
// (cOrganism::CalcMeritRatio, main/cOrganism.cc:703-708: age / merit, or the
// age without a positive merit) at the batch step's end; an empty cell (a
// newborn's to be) is worth 0.
static double position_value(const World& w, int64_t c) {
  if (c >= w.ncells || !w.orgs[c].alive) return 0.0;
  const Org& o = w.orgs[c];
  const double age = (double)o.age;
  if (w.cfg.birth_method == 1) return age;
  return o.merit > 0.0 ? age / o.merit : age;
}

// BIRTH_METHOD 4 (POSITION_OFFSPRING_FULL_SOUP_RANDOM, main/cPopulation.cc:
// 5297-5310): with PREFER_EMPTY, FindRandEmptyCell (:5650-5668) -- a cell drawn
// uniformly among the empty ones (the reference swap-removes the occupied
// entries it draws and draws again); here one draw among the cells empty at
// the batch step's end that this round has not taken (empty_cells, ascending,
// recompacted before every round: soup_round_cells); none (a full world, or
// every empty cell claimed by earlier births): GetUInt(size) over the whole
// world.  Without PREFER_EMPTY: GetUInt(size), redrawn while it is the parent
// and ALLOW_PARENT is 0.  The parent's cell without ALLOW_PARENT:
// ActivateOffspring drops the offspring (:706-713).
static int64_t soup_target(World& w, Birth& b) {
  const uint32_t n = (uint32_t)w.ncells;
  if (w.cfg.prefer_empty) {
    const uint32_t ne = (uint32_t)w.empty_cells.size();
    if (ne > 0) return w.empty_cells[b.rng.uint_below(ne)];
    return b.rng.uint_below(n);
  }
  int64_t c = b.rng.uint_below(n);
  while (!w.cfg.allow_parent && n > 1 && c == b.parent) c = b.rng.uint_below(n);
  return c;
}

template <class Taken>
static bool place_pick(World& w, int64_t i, int m, Taken taken) {
  Birth& b = w.births[i];
  if (w.cfg.birth_method == 4) {
    const int64_t t = soup_target(w, b);
    if (t == b.parent && !w.cfg.allow_parent) { b.target = -1; w.bstate[i] = (int8_t)(BS_NO_CELL - m); return false; }
    b.target = t;
    w.prio[i] = claim_key(b.t, taken(t), b.rng.next(), w.cell0 + b.parent, b.seq);
    w.tgt_r[m][i] = t;
    return true;
  }
  int64_t nb[8];
  const int nn = neighbours(w, b.parent, nb);
  int64_t cand[9];
  int nc = 0;
  if (w.cfg.prefer_empty)
    for (int k = 0; k < nn; k++) if (!taken(nb[k])) cand[nc++] = nb[k];
  if (nc == 0 && (w.cfg.birth_method == 1 || w.cfg.birth_method == 2)) {
    // PositionAge / PositionMerit (main/cPopulation.cc:5416-5470): the parent
    // first, valued -1 without ALLOW_PARENT; each neighbour of a larger value
    // replaces the list, one of an equal value joins it
    double best = w.cfg.allow_parent ? position_value(w, b.parent) : -1.0;
    cand[nc++] = b.parent;
    for (int k = 0; k < nn; k++) {
      const double v = position_value(w, nb[k]);
      if (v > best) { best = v; nc = 0; cand[nc++] = nb[k]; }
      else if (v == best) cand[nc++] = nb[k];
    }
  } else if (nc == 0 && w.cfg.birth_method != 3) {
    for (int k = 0; k < nn; k++) cand[nc++] = nb[k];
    if (w.cfg.allow_parent) cand[nc++] = b.parent;
  }
  if (nc == 0 && !w.cfg.allow_parent) { b.target = -1; w.bstate[i] = (int8_t)(BS_NO_CELL - m); return false; }
  b.target = nc > 0 ? cand[b.rng.uint_below((uint32_t)nc)] : b.parent;
  w.prio[i] = claim_key(b.t, taken(b.target), b.rng.next(), w.cell0 + b.parent, b.seq);
  w.tgt_r[m][i] = b.target;
  return true;
}

// round m > 0's soup candidates: the cells still empty and not claimed in
// round m - 1 (the device's k_empty_* with m)
static void soup_round_cells(World& w, int m) {
  if (w.cfg.birth_method != 4 || !w.cfg.prefer_empty) return;
  const std::vector<uint64_t>& prev = w.claim_r[m - 1];
  w.empty_cells.clear();
  for (int64_t c = 0; c < w.ncells; c++) if (!w.occ[c] && !prev[c]) w.empty_cells.push_back(c);
}

static void place_reset(World& w, int64_t ext) {
  const int64_t nbirth = (int64_t)w.births.size();
  w.occ.assign(ext, 0);
  for (int64_t c = 0; c < w.ncells; c++) w.occ[c] = w.orgs[c].alive ? 1 : 0;
  w.empty_cells.clear();
  if (w.cfg.birth_method == 4 && w.cfg.prefer_empty)
    for (int64_t c = 0; c < w.ncells; c++) if (!w.occ[c]) w.empty_cells.push_back(c);
  for (int k = 0; k < 4; k++) { w.claim_r[k].assign(ext, 0); w.tgt_r[k].assign(nbirth, -1); }
  w.owner.assign(ext, -1);
  w.killt.assign(w.ncells, 0);
  w.prio.assign(nbirth, 0);
  w.bstate.assign(nbirth, BS_PENDING);
}

// launch 0b, one record: cancelled if its parent's cell was killed earlier
// (kt: the cell's merged kill time), else it claims its round-0 target
static inline bool place_cancelled(const World& w, int64_t i, uint32_t kt) {
  return kt > 0x10000u - w.births[i].t;
}

// the single world's activation: round 3 resolved, owners activated, the
// rest counted (main/cPopulation.cc:5382-5413: PositionOffspring always
// returns a cell, so a record that is neither cancelled nor without a cell
// was placed -- it owns its cell, or a later birth overwrote it)
static void place_finish_single(World& w, int64_t& placed_out, int64_t& dropped_out) {
  const int64_t nbirth = (int64_t)w.births.size();
  int64_t placed = 0, overwritten = 0, cancelled = 0, dropped = 0;
  for (int64_t i = 0; i < nbirth; i++) {
    Birth& b = w.births[i];
    const int8_t st = w.bstate[i];
    bool own = false;
    if (st == BS_PENDING) {
      own = w.claim_r[3][b.target] == w.prio[i] && takes_cell(w, w.owner[b.target], b.t);
    } else if (st >= BS_WON && st < BS_WON + 4) {
      const uint64_t c3 = w.claim_r[3][b.target];
      own = w.owner[b.target] == i && !(c3 != 0 && key_time(c3) >= b.t);
    }
    if (own) { activate_child(w, b, b.target); w.newborns.push_back({b.target, b.t}); placed++; }
    else if (st == BS_CANCELLED) cancelled++;
    else if (st <= BS_NO_CELL) dropped++;
    else overwritten++;
  }
  w.t_overwritten += overwritten;
  w.t_cancelled += cancelled;
  placed_out += placed;
  dropped_out += dropped;
}

}  // extern "C++"

// Sub-steps: an update's UD picks are made in K consecutive
// batch steps of floor(UD (s + 1) / K) - floor(UD s / K) picks each, the
// weights re-read before each one -- the reference re-weights its scheduler
// at every divide (cPopulation::ActivateOffspring -> AdjustSchedule,
// main/cPopulation.cc:621-952).  avgpu_cfg.sub_updates = K > 0 fixes K;
// 0 (the default) chooses it per update from the previous step's predictor
// (pred_term): more steps the more the total weight is expected to move
// within the update (a cohort reaching its divides together: the lock-step
// start of injected or loaded organisms), one step below a tenth.  Resources
// step once per update (at sub-step 0); global consumption settles after each
// step.
// cPhenotype::IncAge for every living organism (UpdateOrganismStats,
// main/cPopulation.cc:6021, at the end of each update): here at the start of
// the next, so that Org::age is the reference's age DURING the update --
// injected organisms start at -1, newborns and dividers are set to 0.
static void age_tick(World& w) {
  if (!tracks_age(w)) return;
  for (int64_t c = 0; c < w.ncells; c++) if (w.orgs[c].alive) w.orgs[c].age++;
}

static inline int64_t sub_share(int64_t n, int s, int K) {
  return K == 1 ? n : (n * (s + 1)) / K - (n * s) / K;
}
// The picks the last batch step's newborns ran beyond what the organisms they
// replaced had left after their births (newborn_pass) come out of the next
// update's first step's allotment (taken within the update, from steps whose
// weights are older than the births, it starved the organisms that had not
// divided yet), so that the updates' picks stay the reference's UD
// (newborns into empty cells take picks from the living there, as the
// reference's scheduler gives a newborn its share of the remaining picks);
// a negative carry (victims left more) adds picks.  `fresh`: the summed new
// carry of every strip (the single world's own); returns the picks to take
// from the step's n_root (at most n_root either way; the rest waits).
static int64_t take_carry(World& w, int64_t fresh, int64_t n_root, bool first) {
  w.carry_rem += fresh;
  w.carry_new = 0;
  if (!first) return 0;
  const int64_t take = std::min(std::max<int64_t>(w.carry_rem, -n_root), n_root);
  w.carry_rem -= take;
  return take;
}
// the update's batch steps (the device's choose_k, capi.hip): sub_updates
// when set; else the more of two rules, each one step up to its threshold:
// with E = |predictor| in mean weights per organism (the total weight's
// expected move within the update), ceil(E / 0.05) steps above E = 0.1; with
// D the fraction of organisms expected to divide within its densest quarter
// (a cohort in lock step), ceil(D / 0.15) steps above D = 0.3; at most
// ADAPT_KMAX
static constexpr int ADAPT_KMAX = 16;
static int choose_k(const avgpu_cfg& c, int64_t pred, int64_t n, bool handed_in, int64_t cnt) {
  if (c.sub_updates > 0) return c.sub_updates;
  if (handed_in || c.slicing_method != AVGPU_SLICE_PROBABILISTIC || n <= 0) return 1;
  const double a = (double)(pred < 0 ? -pred : pred), dn = (double)n;
  int k = 1;
  if (a > 104857.6 * dn) k = std::max(k, (int)std::ceil(a / (52428.8 * dn)));
  if ((double)cnt > 0.3 * dn) k = std::max(k, (int)std::ceil((double)cnt / (0.15 * dn)));
  return std::min(k, ADAPT_KMAX);
}

// Batch-synchronous world update: the exact semantics the device implements
// (DESIGN.md "Update semantics"): allot -> interpret -> place births ->
// newborns -> stats.
static int run_update_impl(World& w) {
  if (w.cfg.birth_method == 5)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 5 (the reaper queue) runs on the serial world only");
  const int K = choose_k(w.cfg, w.pred_acc, w.pred_n, w.have_global, densest(w.pred_bin));
  if (K > 1 && w.have_global)
    return fail(AVGPU_EUNSUPPORTED, "sub_updates > 1 needs the world's own totals (no handed-in totals)");
  int64_t placed = 0, dropped = 0, insts = 0, deaths = 0, divides = 0, slices = 0;
  w.t_overwritten = 0;
  w.t_cancelled = 0;
  for (int sub = 0; sub < K; sub++) {
    w.sched_key = (uint32_t)w.update * (uint32_t)K + (uint32_t)sub;
    int64_t n_alive = 0;
    std::vector<double> part;
    world_partials(w, part, &n_alive);
    const double local = top_tree(w, part, -1, 0, 0, nullptr);
    const double ave = (double)w.cfg.ave_time_slice;
    // the update's UD = AVE_TIME_SLICE x the organisms at its start
    // (cAvidaDriver's update loop), its later steps' shares of that
    if (sub == 0) w.upd_ud = (int64_t)w.cfg.ave_time_slice * n_alive;
    double total = local, ud = (double)w.upd_ud;
    int64_t n_all = n_alive;
    int64_t n_root = w.upd_ud;
    if (w.have_global) {   // cMultiProcessWorld::CalculateUpdateSize (main/cMultiProcessWorld.cc:396-405)
      total = w.global_merit;
      ud = ave * (double)w.global_orgs;
      n_all = w.global_orgs;
      n_root = total > 0.0 ? (int64_t)((local / total) * ave * (double)w.global_orgs) : 0;
    }
    n_root = sub_share(n_root, sub, K);
    n_root -= take_carry(w, w.carry_new, n_root, sub == 0);
    std::vector<int64_t> blk;
    top_tree(w, part, n_root, 0, (int64_t)part.size(), &blk);
    if (sub == 0) res_begin(w);   // resources step once per update, at its start
    if (sub == 0) age_tick(w);
    allot_interpret(w, blk, total, ud, n_all);
    insts += w.t_insts; deaths += w.t_deaths; divides += w.t_divides; slices += w.t_slices;
    const int64_t nbirth = (int64_t)w.births.size();
    place_reset(w, w.ncells);
    // launch 0: picks, kill times
    for (int64_t i = 0; i < nbirth; i++) {
      if (!place_pick(w, i, 0, [&](int64_t c) { return w.occ[c] != 0; })) continue;
      const Birth& b = w.births[i];
      if (key_kill(w.prio[i])) w.killt[b.target] = std::max(w.killt[b.target], 0x10000u - b.t);
    }
    // launch 0b: cancellations, round-0 claims
    for (int64_t i = 0; i < nbirth; i++) {
      if (w.bstate[i] != BS_PENDING) continue;
      const Birth& b = w.births[i];
      if (place_cancelled(w, i, w.killt[b.parent])) { w.bstate[i] = BS_CANCELLED; continue; }
      w.claim_r[0][b.target] = std::max(w.claim_r[0][b.target], w.prio[i]);
    }
    // launches 1..3: resolve round m-1, pick round m
    for (int m = 1; m < 4; m++) {
      const std::vector<uint64_t>& prev = w.claim_r[m - 1];
      soup_round_cells(w, m);
      for (int64_t i = 0; i < nbirth; i++) {
        if (w.bstate[i] != BS_PENDING) continue;
        Birth& b = w.births[i];
        if (prev[b.target] == w.prio[i]) {
          w.bstate[i] = (int8_t)(BS_WON + m - 1);
          w.occ[b.target] = 1;
          if (takes_cell(w, w.owner[b.target], b.t)) w.owner[b.target] = i;
          continue;
        }
        if (key_kill(w.prio[i])) { w.bstate[i] = (int8_t)(BS_KILL_LOST + m - 1); continue; }
        if (!place_pick(w, i, m, [&](int64_t c) { return w.occ[c] != 0 || prev[c] != 0; })) continue;
        w.claim_r[m][b.target] = std::max(w.claim_r[m][b.target], w.prio[i]);
      }
    }
    place_finish_single(w, placed, dropped);
    // the newborns' credit and their share of the step (newborn_pass)
    w.t_insts = 0; w.t_deaths = 0; w.t_slices = 0;
    newborn_pass(w, sub_share((int64_t)ud, sub, K), total);
    insts += w.t_insts; deaths += w.t_deaths; slices += w.t_slices;
    res_end(w);
  }
  w.t_insts = insts; w.t_deaths = deaths; w.t_divides = divides; w.t_slices = slices;
  w.last_k = K;
  finish_stats(w, placed, dropped);
  return 0;
}

int orc_run_update(void* h, avgpu_update_stats* out) {
  World& w = *(World*)h;
  int rc = run_update_impl(w);
  if (out) *out = w.stats;
  return rc;
}

int orc_run_updates(void* h, int n, avgpu_update_stats* out) {
  World& w = *(World*)h;
  for (int i = 0; i < n; i++) run_update_impl(w);
  if (out) *out = w.stats;
  return 0;
}

int orc_set_global_totals(void* h, double merit, int64_t orgs) {
  World& w = *(World*)h;
  w.have_global = true; w.global_merit = merit; w.global_orgs = orgs;
  return 0;
}

// ---------------------------------------------------------------------------
// Strip tiles (include/avida_gpu.h "strip tiles"; DESIGN.md "Multi-GPU"): the
// same update as run_update_impl, split around the halo exchanges the host
// performs.  Buffer layouts are the device's: halo = per round parity X u64
// claims on the receiver's edge row and X u64 the sender's own claims on its
// edge row, then X u8 edge-row occupancy; records = HaloHdr, X HaloRec,
// genome arena.  A cell of an edge row is claimed only from the two strips it
// touches, so one exchange per placement round gives both strips every claim
// on it: each resolves the cell alike (the neighbour's own claims merged into
// the ghost row), at the start of the next round's call.
namespace {
struct HaloHdr { int32_t count, arena_used, overflow, pad; };
struct HaloRec {
  int32_t col, round, len, gen, ccopied, exec, gest;
  uint32_t rng_lo, rng_hi, rng_ctr;
  int32_t off;
  uint32_t t;         // the offspring's birth time (owner bookkeeping, head start)
  double merit, fitness;
  int32_t last_task[AVGPU_NUM_LOGIC_TASKS], pad2[3];
};
static_assert(sizeof(HaloRec) == 112, "HaloRec layout");
// per round parity p: k = 0 the sender's claims on the receiver's edge row
// (its ghost row), k = 1 its own claims on its edge row; then the occupancy;
// then (round 0's picks) the kill times of the sender's picks on the
// receiver's edge row (u32, 2^16 - t, max-reduced)
int64_t halo_kt_off(int x) { return ((int64_t)x * 33 + 3) / 4 * 4; }
int64_t halo_bytes_of(int x) { return (halo_kt_off(x) + 4 * (int64_t)x + 15) / 16 * 16; }
uint64_t* hcl(uint8_t* b, int x, int p, int k) { return reinterpret_cast<uint64_t*>(b) + (int64_t)(2 * p + k) * x; }
uint8_t* hocc(uint8_t* b, int x) { return b + (int64_t)x * 32; }
uint32_t* hkt(uint8_t* b, int x) { return reinterpret_cast<uint32_t*>(b + halo_kt_off(x)); }
int64_t edge_cell(const World& w, int d, int x) { return d == 0 ? x : (w.rows - 1) * w.cfg.world_x + x; }
int64_t ghost_cell(const World& w, int d, int x) { return w.ncells + (int64_t)d * w.cfg.world_x + x; }
bool tile_ok(World& w) { return w.tiled && w.h_send[0] && w.r_recv[1]; }
}  // namespace

int orc_set_tile(void* h, int64_t row0, int64_t arena) {
  World& w = *(World*)h;
  if (w.cfg.birth_method == 1 || w.cfg.birth_method == 2)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 1 / 2 on strip tiles (the ghost rows carry no age or merit)");
  if (w.cfg.birth_method == 4 || w.cfg.birth_method == 5)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 4 / 5 on strip tiles (a soup birth may land in any strip)");
  const int64_t X = w.cfg.world_x;
  if (X <= 0 || w.ncells % X) return fail(AVGPU_EINVAL, "tile cells must be whole rows of WORLD_X");
  const int64_t rows = w.ncells / X;
  if (rows < 2) return fail(AVGPU_EINVAL, "a tile needs at least 2 rows");
  if (w.ncells % 256) return fail(AVGPU_EINVAL, "tile cells must be a multiple of 256 (merit blocks)");
  if (row0 < 0 || row0 + rows > w.global_rows) return fail(AVGPU_EINVAL, "tile rows outside WORLD_Y");
  if (arena <= 0) arena = std::max<int64_t>(256 * 1024, X * 256);
  w.row0 = row0; w.rows = rows; w.tiled = rows < w.global_rows; w.cell0 = row0 * X;
  w.r_arena = (arena + 15) / 16 * 16;
  if (!w.res.empty()) res_init(w);   // this strip's share of the initial amounts
  return 0;
}

int orc_tile_res_bytes(void* h, int64_t* bytes) {
  World& w = *(World*)h;
  if (bytes) *bytes = (int64_t)w.n_spatial * w.cfg.world_x * 8;
  return 0;
}

int orc_set_tile_res_buffers(void* h, void* send_up, void* send_down, void* recv_up, void* recv_down) {
  World& w = *(World*)h;
  if (!w.tiled) return fail(AVGPU_ESTATE, "not a strip tile");
  w.rs_send[0] = (double*)send_up; w.rs_send[1] = (double*)send_down;
  w.rs_recv[0] = (double*)recv_up; w.rs_recv[1] = (double*)recv_down;
  return 0;
}

// the update's consumption of the global pools by this strip (2^-32 units)
int orc_tile_res_cons(void* h, uint64_t* out) {
  World& w = *(World*)h;
  int g = 0;
  for (int r = 0; r < AVGPU_MAX_RESOURCES; r++) out[r] = 0;
  for (size_t r = 0; r < w.res.size(); r++) {
    out[r] = w.res_cons[r];
    g += w.res[r].geometry == AVGPU_RES_GLOBAL;
  }
  return g;
}

// subtract every strip's consumption (summed over the strips): res_end
int orc_tile_res_settle(void* h, const uint64_t* sum) {
  World& w = *(World*)h;
  for (size_t r = 0; r < w.res.size(); r++) w.res_cons[r] = sum[r];
  res_end(w);
  return 0;
}

int orc_tile_buffer_bytes(void* h, int64_t* part, int64_t* halo, int64_t* rec) {
  World& w = *(World*)h;
  const int X = w.cfg.world_x;
  if (part) *part = (2 * ((w.ncells + 255) / 256) + 6) * 8;
  if (halo) *halo = halo_bytes_of(X);
  if (rec) *rec = (int64_t)sizeof(HaloHdr) + (int64_t)X * (int64_t)sizeof(HaloRec) + w.r_arena;
  return 0;
}

int orc_set_tile_buffers(void* h, void* hs0, void* hs1, void* hr0, void* hr1, void* rs0, void* rs1,
                         void* rr0, void* rr1) {
  World& w = *(World*)h;
  if (!w.tiled) return fail(AVGPU_ESTATE, "not a strip tile");
  w.h_send[0] = (uint8_t*)hs0; w.h_send[1] = (uint8_t*)hs1;
  w.h_recv[0] = (uint8_t*)hr0; w.h_recv[1] = (uint8_t*)hr1;
  w.r_send[0] = (uint8_t*)rs0; w.r_send[1] = (uint8_t*)rs1;
  w.r_recv[0] = (uint8_t*)rr0; w.r_recv[1] = (uint8_t*)rr1;
  return 0;
}

// the 256-cell block partials of the scheduler tree (block_levels), then alive counts
int orc_tile_partials(void* h, double* out) {
  World& w = *(World*)h;
  const int64_t nb = (w.ncells + 255) / 256;
  double lv[9][256];
  for (int64_t b = 0; b < nb; b++) {
    out[b] = block_levels(w, b, lv);
    int64_t cnt = 0;
    for (int i = 0; i < 256; i++) cnt += (b * 256 + i < w.ncells && w.orgs[b * 256 + i].alive) ? 1 : 0;
    out[nb + b] = (double)cnt;
  }
  // the predictor of the strip's last batch step (its bits), summed by
  // avgpu_tile_steps on every strip
  memcpy(out + 2 * nb, &w.pred_acc, 8);
  memcpy(out + 2 * nb + 1, &w.carry_new, 8);
  for (int k = 0; k < 4; k++) memcpy(out + 2 * nb + 2 + k, &w.pred_bin[k], 8);
  // edge rows of the spatial amounts for the neighbours' flow step
  const int X = w.cfg.world_x;
  if (w.tiled && w.rs_send[0])
    for (size_t r = 0; r < w.res.size(); r++) {
      const int slot = w.res_slot[r];
      if (slot < 0) continue;
      for (int x = 0; x < X; x++) {
        w.rs_send[0][(int64_t)slot * X + x] = w.res_amount[r][x];
        w.rs_send[1][(int64_t)slot * X + x] = w.res_amount[r][(w.rows - 1) * X + x];
      }
    }
  return 0;
}

// the update's batch steps from every strip's predictor in the gathered
// partials (the single world's choose_k over the same integer sum)
int orc_tile_steps(void* h, const double* gathered, int ntiles, int* k_out) {
  World& w = *(World*)h;
  const int64_t nb = (w.ncells + 255) / 256, stride = 2 * nb + 6;
  int64_t sum = 0, bins[4] = {0, 0, 0, 0};
  for (int k = 0; k < ntiles; k++) {
    int64_t v;
    memcpy(&v, gathered + k * stride + 2 * nb, 8);
    sum += v;
    for (int q = 0; q < 4; q++) {
      int64_t c;
      memcpy(&c, gathered + k * stride + 2 * nb + 2 + q, 8);
      bins[q] += c;
    }
  }
  if (k_out) *k_out = choose_k(w.cfg, sum, w.pred_n, false, densest(bins));
  return 0;
}

int orc_tile_begin_step(void* h, const double* gathered, int ntiles, int sub, int K) {
  World& w = *(World*)h;
  if (!tile_ok(w)) return fail(AVGPU_ESTATE, "not a strip tile with buffers");
  if (K < 1 || sub < 0 || sub >= K) return fail(AVGPU_EINVAL, "batch step sub of K");
  w.sched_key = (uint32_t)w.update * (uint32_t)K + (uint32_t)sub;
  if (sub == 0) {
    age_tick(w);
    w.acc_placed = w.acc_dropped = w.acc_insts = w.acc_deaths = w.acc_divides = w.acc_slices = 0;
    w.acc_overwritten = w.acc_cancelled = 0;
  }
  // the top tree over every strip's block partials (tile order = block order)
  const int64_t nb = (w.ncells + 255) / 256, stride = 2 * nb + 6;
  std::vector<double> leaf((size_t)(nb * ntiles));
  int64_t cnt = 0, fresh = 0;
  for (int k = 0; k < ntiles; k++) {
    for (int64_t j = 0; j < nb; j++) {
      leaf[k * nb + j] = gathered[k * stride + j];
      cnt += (int64_t)gathered[k * stride + nb + j];
    }
    int64_t v;
    memcpy(&v, gathered + k * stride + 2 * nb + 1, 8);
    fresh += v;
  }
  std::vector<int64_t> blk;
  if (sub == 0) w.upd_ud = (int64_t)w.cfg.ave_time_slice * cnt;
  const int64_t ud = w.upd_ud;
  int64_t n_root = sub_share(ud, sub, K);
  n_root -= take_carry(w, fresh, n_root, sub == 0);
  const double total = top_tree(w, leaf, n_root, w.cell0 / 256, nb, &blk);
  if (w.n_spatial && !w.rs_recv[0]) return fail(AVGPU_ESTATE, "spatial resources need the tile resource buffers");
  if (sub == 0) res_begin(w);
  allot_interpret(w, blk, total, (double)ud, cnt);
  w.step_sub = sub; w.step_k = K;
  w.step_uds = sub_share(ud, sub, K);
  w.step_total = total;
  const int X = w.cfg.world_x;
  place_reset(w, w.ncells + 2 * X);
  for (int d = 0; d < 2; d++)
    for (int x = 0; x < X; x++) {
      hocc(w.h_send[d], X)[x] = w.occ[edge_cell(w, d, x)];
      for (int k = 0; k < 4; k++) hcl(w.h_send[d], X, k >> 1, k & 1)[x] = 0;
      hkt(w.h_send[d], X)[x] = 0;
    }
  w.t_placed = 0; w.t_overwritten = 0; w.t_dropped = 0;
  return 0;
}

int orc_tile_begin(void* h, const double* gathered, int ntiles) { return orc_tile_begin_step(h, gathered, ntiles, 0, 1); }

namespace {
// the halo slot of a cell: direction, column, ghost row (else edge row)
bool tile_slot(const World& w, int64_t c, int& d, int& x, bool& ghost) {
  const int X = w.cfg.world_x;
  if (c >= w.ncells) { d = (int)((c - w.ncells) / X); x = (int)((c - w.ncells) % X); ghost = true; return true; }
  ghost = false;
  if (c < X) { d = 0; x = (int)c; return true; }
  if (c >= w.ncells - X) { d = 1; x = (int)(c - (w.ncells - X)); return true; }
  return false;
}
// a tile's cell taken for round m's pick (the device's tile_taken): round 0
// the occupancy (ghost rows: the neighbour's edge occupancy, imported); later
// rounds also every cell claimed in round m - 1, here or by the neighbour
bool tile_taken(const World& w, int64_t c, int m) {
  if (w.occ[c]) return true;
  if (m == 0) return false;
  if (w.claim_r[m - 1][c] != 0) return true;
  int d, x;
  bool ghost;
  return tile_slot(w, c, d, x, ghost) && hcl(w.h_recv[d], w.cfg.world_x, (m - 1) & 1, ghost ? 1 : 0)[x] != 0;
}
// round m's merged claim on cell t: mine, the neighbour's
uint64_t tile_merged(const World& w, int64_t t, int m) {
  uint64_t v = w.claim_r[m][t];
  int d, x;
  bool ghost;
  if (tile_slot(w, t, d, x, ghost)) v = std::max(v, hcl(w.h_recv[d], w.cfg.world_x, m & 1, ghost ? 1 : 0)[x]);
  return v;
}
// launch m = 1..4 of a tile (the device's k_tile_round): round m - 1
// resolved with the merged claims -- the halo cells' remote winners (an edge
// or ghost cell whose maximum came from the neighbour: owner
// remote_owner(m - 1, t) by the time rule, occupied), this tile's winners
// (takes_cell), lost kill claims placed and overwritten -- then (m < 4) the
// pending records pick round m
void tile_launch(World& w, int m) {
  const int X = w.cfg.world_x, p = (m - 1) & 1;
  const std::vector<uint64_t>& cl = w.claim_r[m - 1];
  for (int d = 0; d < 2; d++)
    for (int x = 0; x < X; x++) {
      const int64_t c = edge_cell(w, d, x), g = ghost_cell(w, d, x);
      const uint64_t rc = hcl(w.h_recv[d], X, p, 0)[x], rg = hcl(w.h_recv[d], X, p, 1)[x];
      if (rc != 0 && rc > cl[c]) {
        if (takes_cell(w, w.owner[c], key_time(rc))) w.owner[c] = remote_owner(m - 1, key_time(rc));
        w.occ[c] = 1;
      }
      if (rg != 0 && rg > cl[g] && takes_cell(w, w.owner[g], key_time(rg)))
        w.owner[g] = remote_owner(m - 1, key_time(rg));
      if (cl[g] != 0 || rg != 0) w.occ[g] = 1;
    }
  const int64_t nbirth = (int64_t)w.births.size();
  for (int64_t i = 0; i < nbirth; i++) {
    if (w.bstate[i] != BS_PENDING) continue;
    Birth& b = w.births[i];
    if (tile_merged(w, b.target, m - 1) == w.prio[i]) {
      w.bstate[i] = (int8_t)(BS_WON + m - 1);
      w.occ[b.target] = 1;
      if (takes_cell(w, w.owner[b.target], b.t)) w.owner[b.target] = i;
      continue;
    }
    if (key_kill(w.prio[i])) { w.bstate[i] = (int8_t)(BS_KILL_LOST + m - 1); continue; }
    if (m == 4) continue;
    if (!place_pick(w, i, m, [&](int64_t c) { return tile_taken(w, c, m); })) continue;
    w.claim_r[m][b.target] = std::max(w.claim_r[m][b.target], w.prio[i]);
    int d, x;
    bool ghost;
    if (tile_slot(w, b.target, d, x, ghost)) {
      uint64_t& slot = hcl(w.h_send[d], X, m & 1, ghost ? 0 : 1)[x];
      slot = std::max(slot, w.prio[i]);
    }
  }
}
}  // namespace

// phase 0, round 0: picks and kill times (own cells; picks on a ghost row go
// to the neighbour in the halo's kill-time slots); phase 3 (after that
// exchange): cancellations with the merged kill times, round 0's claims;
// phase 0, rounds 1..3: tile_launch; phase 1: round 3 resolved, the ghost
// cells' owners packed; phase 2: this tile's owners activated
int orc_tile_place(void* h, int round, int phase) {
  World& w = *(World*)h;
  if (!tile_ok(w)) return fail(AVGPU_ESTATE, "not a strip tile with buffers");
  if (round < 0 || round > 3 || phase < 0 || phase > 3 || (phase >= 1 && phase <= 2 && round != 3) ||
      (phase == 3 && round != 0))
    return fail(AVGPU_EINVAL, "round 0..3 with phase 0, round 0 with phase 3; phases 1, 2 after round 3");
  const int X = w.cfg.world_x;
  const int64_t nbirth = (int64_t)w.births.size();
  if (phase == 0 && round == 0) {
    for (int d = 0; d < 2; d++)
      for (int x = 0; x < X; x++) w.occ[ghost_cell(w, d, x)] = hocc(w.h_recv[d], X)[x];
    for (int64_t i = 0; i < nbirth; i++) {
      if (!place_pick(w, i, 0, [&](int64_t c) { return tile_taken(w, c, 0); })) continue;
      const Birth& b = w.births[i];
      if (!key_kill(w.prio[i])) continue;
      int d, x;
      bool ghost;
      if (b.target >= w.ncells && tile_slot(w, b.target, d, x, ghost)) {
        uint32_t& k = hkt(w.h_send[d], X)[x];
        k = std::max(k, 0x10000u - b.t);
      } else {
        w.killt[b.target] = std::max(w.killt[b.target], 0x10000u - b.t);
      }
    }
  } else if (phase == 3) {
    for (int64_t i = 0; i < nbirth; i++) {
      if (w.bstate[i] != BS_PENDING) continue;
      const Birth& b = w.births[i];
      uint32_t kt = w.killt[b.parent];
      int d, x;
      bool ghost;
      if (tile_slot(w, b.parent, d, x, ghost)) kt = std::max(kt, hkt(w.h_recv[d], X)[x]);
      if (place_cancelled(w, i, kt)) { w.bstate[i] = BS_CANCELLED; continue; }
      w.claim_r[0][b.target] = std::max(w.claim_r[0][b.target], w.prio[i]);
      if (tile_slot(w, b.target, d, x, ghost)) {
        uint64_t& slot = hcl(w.h_send[d], X, 0, ghost ? 0 : 1)[x];
        slot = std::max(slot, w.prio[i]);
      }
    }
  } else if (phase == 0) {
    // this round's send slots (their last contents, round - 2's, went out)
    const int p = round & 1;
    for (int d = 0; d < 2; d++)
      for (int x = 0; x < X; x++) { hcl(w.h_send[d], X, p, 0)[x] = 0; hcl(w.h_send[d], X, p, 1)[x] = 0; }
    tile_launch(w, round);
  } else if (phase == 2) {
    // this tile's own winners (the records travel meanwhile)
    int64_t placed = 0, overwritten = 0, cancelled = 0, nocell = 0;
    for (int64_t i = 0; i < nbirth; i++) {
      Birth& b = w.births[i];
      const int8_t st = w.bstate[i];
      const bool won = st >= BS_WON && st < BS_WON + 4 && w.owner[b.target] == i;
      if (won && b.target >= w.ncells) continue;   // shipped to the neighbour
      if (won) { activate_child(w, b, b.target); w.newborns.push_back({b.target, b.t}); placed++; }
      else if (st == BS_CANCELLED) cancelled++;
      else if (st <= BS_NO_CELL) nocell++;
      else overwritten++;                          // placed, then overwritten (run_update_impl)
    }
    w.t_placed = placed;
    w.t_overwritten = overwritten;
    w.t_cancelled = cancelled;
    w.t_dropped += nocell;
  } else {
    tile_launch(w, 4);
    // then pack the owner of every ghost cell (births in queue order)
    w.t_born = 0; w.t_dropped = 0;
    for (int d = 0; d < 2; d++) memset(w.r_send[d], 0, sizeof(HaloHdr));
    for (int64_t i = 0; i < nbirth; i++) {
      const Birth& b = w.births[i];
      const int8_t st = w.bstate[i];
      if (st < BS_WON || st >= BS_WON + 4 || b.target < w.ncells || w.owner[b.target] != i) continue;
      const int d = (int)((b.target - w.ncells) / X), col = (int)((b.target - w.ncells) % X);
      HaloHdr* hdr = reinterpret_cast<HaloHdr*>(w.r_send[d]);
      HaloRec* recs = reinterpret_cast<HaloRec*>(w.r_send[d] + sizeof(HaloHdr));
      uint8_t* arena = w.r_send[d] + sizeof(HaloHdr) + (int64_t)X * sizeof(HaloRec);
      const int len = (int)b.genome.size();
      const int slot = hdr->count++;
      const int off = hdr->arena_used;
      hdr->arena_used += (len + 3) & ~3;
      const bool fits = (int64_t)off + len <= w.r_arena;
      HaloRec r;
      r.col = col; r.round = st - BS_WON; r.len = fits ? len : -1;
      r.gen = b.generation; r.ccopied = b.child_copied; r.exec = b.executed; r.gest = b.gestation_time;
      r.rng_lo = b.rng.lo; r.rng_hi = b.rng.hi; r.rng_ctr = b.rng.ctr;
      r.off = off; r.t = b.t; r.merit = b.merit; r.fitness = b.fitness;
      for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) r.last_task[t] = b.last_task[t];
      r.pad2[0] = r.pad2[1] = r.pad2[2] = 0;
      recs[slot] = r;
      if (fits) memcpy(arena + off, b.genome.data(), len);
      else { hdr->overflow++; w.t_dropped++; }
    }
  }
  return 0;
}

int orc_tile_finish(void* h, avgpu_update_stats* out) {
  World& w = *(World*)h;
  if (!tile_ok(w)) return fail(AVGPU_ESTATE, "not a strip tile with buffers");
  const int X = w.cfg.world_x;
  int64_t placed = w.t_placed, dropped = w.t_dropped, overwritten = w.t_overwritten;
  for (int d = 0; d < 2; d++) {
    const HaloHdr* hdr = reinterpret_cast<const HaloHdr*>(w.r_recv[d]);
    const HaloRec* recs = reinterpret_cast<const HaloRec*>(w.r_recv[d] + sizeof(HaloHdr));
    const uint8_t* arena = w.r_recv[d] + sizeof(HaloHdr) + (int64_t)X * sizeof(HaloRec);
    const int nrec = std::min(hdr->count, X);
    for (int q = 0; q < nrec; q++) {
      const HaloRec& r = recs[q];
      if (r.len < 0) continue;
      const int64_t c = edge_cell(w, d, r.col);
      if (w.owner[c] != remote_owner(r.round, r.t)) { overwritten++; continue; }
      Birth b;
      b.parent = -1; b.seq = 0;
      b.genome.assign(arena + r.off, arena + r.off + r.len);
      b.merit = r.merit; b.generation = r.gen; b.child_copied = r.ccopied; b.executed = r.exec;
      b.gestation_time = r.gest; b.fitness = r.fitness;
      for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) b.last_task[t] = r.last_task[t];
      b.rng.lo = r.rng_lo; b.rng.hi = r.rng_hi; b.rng.ctr = r.rng_ctr;
      activate_child(w, b, c);
      w.newborns.push_back({c, r.t});
      placed++;
    }
  }
  // the step's newborns, the update's counts over its steps
  const int64_t mi = w.t_insts, md = w.t_deaths, ms = w.t_slices;
  w.t_insts = 0; w.t_deaths = 0; w.t_slices = 0;
  newborn_pass(w, w.step_uds, w.step_total);
  w.acc_insts += mi + w.t_insts; w.acc_deaths += md + w.t_deaths; w.acc_slices += ms + w.t_slices;
  w.acc_divides += w.t_divides;
  w.acc_placed += placed; w.acc_dropped += dropped;
  w.acc_overwritten += overwritten; w.acc_cancelled += w.t_cancelled;
  if (w.step_sub == w.step_k - 1) {
    w.t_insts = w.acc_insts; w.t_deaths = w.acc_deaths; w.t_slices = w.acc_slices; w.t_divides = w.acc_divides;
    w.t_overwritten = w.acc_overwritten; w.t_cancelled = w.acc_cancelled;
    w.last_k = w.step_k;
    finish_stats(w, w.acc_placed, w.acc_dropped);
  }
  if (out) *out = w.stats;
  return 0;
}

int orc_get_stats(void* h, avgpu_update_stats* out) { *out = ((World*)h)->stats; return 0; }

// the last allotment's budgets (diagnostics: tools/budget_spread.py)
int orc_last_budgets(void* h, int32_t* out) {
  const World& w = *(World*)h;
  for (size_t c = 0; c < w.last_budget.size(); c++) out[c] = w.last_budget[c];
  return (int)w.last_budget.size();
}

// ---------------------------------------------------------------------------
// Reference-style serial world (the CPU baseline): Avida2Driver::Run's update
// loop (targets/avida/Avida2Driver.cc:91-163) with cPopulation::ScheduleOrganism
// (probabilistic pick proportional to merit; a cWeightedIndex-style sum tree,
// tools/cWeightedIndex.cc:49-115) and ProcessStepSpeculative
// (main/cPopulation.cc:5740-5788), births placed immediately
// (ActivateOffspring main/cPopulation.cc:621-952).
struct SerialSched {
  int64_t n = 0, size = 1;
  std::vector<double> tree;
  void init(int64_t cells) {
    n = cells; size = 1; while (size < n) size <<= 1;
    tree.assign(2 * size, 0.0);
  }
  void set(int64_t i, double v) {
    int64_t p = size + i; tree[p] = v;
    for (p >>= 1; p >= 1; p >>= 1) tree[p] = tree[2 * p] + tree[2 * p + 1];
  }
  int64_t find(double x) const {
    int64_t p = 1;
    while (p < size) {
      if (x < tree[2 * p]) p = 2 * p; else { x -= tree[2 * p]; p = 2 * p + 1; }
    }
    return p - size;
  }
};

// The reference's connection list of a cell (tools/cTopology.h:40-55
// build_torus: eight Push()es, and tList::Push prepends, tools/tList.h:140-147,
// so the list runs W, SW, S, SE, E, NE, N, NW -- (dx, dy) below; build_grid
// :62-95 removes the wrapped entries, keeping the order), rotated by the cell's
// facing (cPopulationCell::Rotate, main/cPopulationCell.cc:122-141: CircNext
// until the given cell is first).
static const int CONN_DX[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, CONN_DY[8] = {0, 1, 1, 1, 0, -1, -1, -1};
static int conn_base(const World& w, int64_t cell, int64_t* out) {
  const int X = w.cfg.world_x, Y = w.cfg.world_y;
  const int x = (int)(cell % X), y = (int)(cell / X);
  int n = 0;
  for (int k = 0; k < 8; k++) {
    const int nx = x + CONN_DX[k], ny = y + CONN_DY[k];
    if (w.cfg.world_geometry == 1 && (nx < 0 || nx >= X || ny < 0 || ny >= Y)) continue;
    out[n++] = (int64_t)((ny + Y) % Y) * X + (nx + X) % X;
  }
  return n;
}

// PositionOffspring (main/cPopulation.cc:5353-5413) on the rotated list:
// FindEmptyCell walks the list from its first cell and Push()es (prepends)
// every empty one (:7361-7370), so the found list is the empty cells in
// reverse list order; with none, BIRTH_METHOD 0 takes the whole list in order
// (Append) with the parent pushed in front (ALLOW_PARENT); one GetUInt(size)
// from the context stream picks.  No candidate: the parent's cell (no draw).
// BIRTH_METHOD 4 in the serial world: PositionOffspring's FULL_SOUP_RANDOM
// (main/cPopulation.cc:5297-5310) with FindRandEmptyCell (:5650-5668) on the
// reference's persistent empty_cell_id_array (0..N-1 at setup, :338-340):
// a full world (num_organisms >= size) or a walk that runs out of cells ->
// GetUInt(size); each occupied draw is swapped behind the shrinking range,
// and the swaps persist.  Without PREFER_EMPTY GetUInt(size), redrawn while
// it is the parent and ALLOW_PARENT is 0.  Every draw from the context stream.
static int64_t serial_soup(World& w, int64_t parent) {
  const uint32_t n = (uint32_t)w.ncells;
  if ((int64_t)w.soup_cells.size() != w.ncells) {
    w.soup_cells.resize(w.ncells);
    for (int64_t c = 0; c < w.ncells; c++) w.soup_cells[c] = c;
  }
  if (w.cfg.prefer_empty) {
    int64_t alive = 0;
    for (int64_t c = 0; c < w.ncells; c++) alive += w.orgs[c].alive ? 1 : 0;
    if (alive < (int64_t)n) {
      uint32_t ws = n;
      uint32_t idx = w.ctx_rng.uint_below(ws);
      int64_t c = w.soup_cells[idx];
      bool found = true;
      while (w.orgs[c].alive) {
        std::swap(w.soup_cells[idx], w.soup_cells[--ws]);
        if (ws == 1) { found = false; break; }
        idx = w.ctx_rng.uint_below(ws);
        c = w.soup_cells[idx];
      }
      if (found) return c;
    }
    return w.ctx_rng.uint_below(n);
  }
  int64_t c = w.ctx_rng.uint_below(n);
  while (!w.cfg.allow_parent && n > 1 && c == parent) c = w.ctx_rng.uint_below(n);
  return c;
}

// BIRTH_METHOD 5 in the serial world: FULL_SOUP_ELDEST (main/cPopulation.cc:
// 5312-5319) -- the cell of the reaper queue's rear entry (PopRear; the
// parent's, without ALLOW_PARENT, is pushed back to the rear and the next one
// taken); ActivateOrganism pushes every newborn's cell at the front (:1358-
// 1361).  Deaths leave the queue alone, so a cell may be in it more than once.
// The queue is the reference's Setup order (cells 0..N-1 pushed, :343-347)
// followed by the living cells in ascending order (their injections, each
// an ActivateOrganism), built at the first serial update.
static void reaper_setup(World& w) {
  if (w.reaper_init) return;
  w.reaper_init = true;
  w.reaper.clear();
  for (int64_t c = 0; c < w.ncells; c++) w.reaper.push_front(c);
  for (int64_t c = 0; c < w.ncells; c++) if (w.orgs[c].alive) w.reaper.push_front(c);
}
// an injection into cell c once the queue exists: an occupied cell's entry
// out (the first from the front, InjectGenome main/cPopulation.cc:6964-6968),
// the cell pushed at the front (ActivateOrganism :1358-1361)
static void reaper_inject(World& w, int64_t c, bool was_alive) {
  if (w.cfg.birth_method != 5 || !w.reaper_init) return;
  if (was_alive) {
    auto it = std::find(w.reaper.begin(), w.reaper.end(), c);
    if (it != w.reaper.end()) w.reaper.erase(it);
  }
  w.reaper.push_front(c);
}
static int64_t serial_eldest(World& w, int64_t parent) {
  int64_t c = w.reaper.back();
  w.reaper.pop_back();
  if (!w.cfg.allow_parent && c == parent && !w.reaper.empty()) {
    c = w.reaper.back();
    w.reaper.pop_back();
    w.reaper.push_back(parent);
  }
  return c;
}

static int64_t serial_target(World& w, int64_t parent) {
  if (w.cfg.birth_method == 4) return serial_soup(w, parent);
  if (w.cfg.birth_method == 5) return serial_eldest(w, parent);
  int64_t base[8], conn[8], found[9];
  const int nb = conn_base(w, parent, base);
  const int f = nb ? w.face[parent] % nb : 0;
  for (int k = 0; k < nb; k++) conn[k] = base[(f + k) % nb];
  int nf = 0;
  if (w.cfg.prefer_empty)
    for (int k = 0; k < nb; k++)
      if (!w.orgs[conn[k]].alive) { for (int q = nf; q > 0; q--) found[q] = found[q - 1]; found[0] = conn[k]; nf++; }
  if (nf == 0 && w.cfg.birth_method == 0) {
    if (w.cfg.allow_parent) found[nf++] = parent;
    for (int k = 0; k < nb; k++) found[nf++] = conn[k];
  }
  if (nf == 0) return parent;
  return found[w.ctx_rng.uint_below((uint32_t)nf)];
}

// ActivateOffspring after the divide (main/cPopulation.cc:621-960): the
// target cell, the kill of its occupant, ActivateOrganism with SetupInputs
// from the context stream, the parent's and the child's scheduler weights,
// and -- the parent still alive -- the child's cell rotated to face the
// parent (:935-944).  Returns 0 dropped (BIRTH_METHOD 3, no empty cell, no
// ALLOW_PARENT), 1 placed, 2 placed over a living organism, 3 over the parent.
static int serial_place(World& w, SerialSched& sch, Birth& b) {
  const int64_t t = serial_target(w, b.parent);
  if (t == b.parent && !w.cfg.allow_parent) return 0;     // target_cells[i] = -1 (:706-712)
  const bool parent_alive = t != b.parent;
  if (parent_alive) sch.set(b.parent, w.orgs[b.parent].merit);   // AdjustSchedule(parent) :933
  const int killed = w.orgs[t].alive ? 1 : 0;
  activate_child(w, b, t, &w.ctx_rng);
  if (w.cfg.birth_method == 5) w.reaper.push_front(t);   // ActivateOrganism (:1358-1361)
  w.orgs[t].spec_count = 0;                               // InsertOrganism (main/cPopulationCell.cc:270-271)
  w.orgs[t].spec_die = false;
  sch.set(t, w.orgs[t].merit);
  if (parent_alive && w.cfg.birth_method < 4) {          // Rotate(parent_cell) :935-944 (local methods, :938)
    int64_t base[8];
    const int nb = conn_base(w, t, base);
    for (int k = 0; k < nb; k++) if (base[k] == b.parent) { w.face[t] = (uint8_t)k; break; }
  }
  return parent_alive ? 1 + killed : 3;
}

// avgpu_set_serial_streams restated: the scheduler's and the context's
// recorded doubles (NULL / 0: counter streams)
int orc_set_serial_streams(void* h, const double* sched, int64_t n_sched, const double* ctx, int64_t n_ctx) {
  World& w = *(World*)h;
  w.srec_sched.assign(sched ? sched : (const double*)nullptr, sched ? sched + n_sched : nullptr);
  w.srec_ctx.assign(ctx ? ctx : (const double*)nullptr, ctx ? ctx + n_ctx : nullptr);
  w.global_rng.rec = w.srec_sched.empty() ? nullptr : w.srec_sched.data();
  w.global_rng.rec_len = (int64_t)w.srec_sched.size();
  w.global_rng.ctr = 0;
  w.ctx_rng.rec = w.srec_ctx.empty() ? nullptr : w.srec_ctx.data();
  w.ctx_rng.rec_len = (int64_t)w.srec_ctx.size();
  w.ctx_rng.ctr = 0;
  return 0;
}

// The serial world: Avida2Driver::Run's update loop (targets/avida/
// Avida2Driver.cc:91-163) with the reference's own schedule.
//  * Two streams, as in the reference: the scheduler's own generator for the
//    picks (Apto::Scheduler::Probabilistic over an AvidaRNG seeded from the
//    world's, main/cPopulation.cc:7341-7346; restated as x = u * total merit
//    and a cWeightedIndex-style sum-tree descent, tools/cWeightedIndex.cc:49-115)
//    and ONE context stream for every other draw -- every organism's
//    mutations, placement, the newborns' inputs -- in execution order.
//  * ProcessStepSpeculative (main/cPopulation.cc:5740-5788): a cell with
//    speculative credit spends one; otherwise one SingleProcess, then while it
//    returns true up to 32 speculative ones, each rejected before a STALL
//    instruction (IO, h-divide: cpu/cHardwareCPU.cc:961-968).  A speculative
//    instruction that reaches the age limit sets m_spec_die (:1045-1049) and is
//    not counted; the organism dies when next picked with no credit left
//    (:917-921).  An organism replaced by its own offspring gets no speculation.
//  * Offspring are placed inside the h-divide (ActivateOffspring), i.e.
//    before the speculative run: rotated connection lists (serial_target).
int orc_run_serial_updates(void* h, int n_updates, avgpu_update_stats* out) {
  World& w = *(World*)h;
  if (w.cfg.birth_method == 1 || w.cfg.birth_method == 2)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 1 / 2 run on the batch world, not the serial world");
  if ((int64_t)w.face.size() != w.ncells) w.face.assign(w.ncells, 0);
  if (w.cfg.birth_method == 5) reaper_setup(w);
  SerialSched sch;
  sch.init(w.ncells);
  for (int64_t c = 0; c < w.ncells; c++) sch.set(c, w.orgs[c].alive ? w.orgs[c].merit : 0.0);
  for (int u = 0; u < n_updates; u++) {
    int64_t n_alive = 0;
    for (int64_t c = 0; c < w.ncells; c++) n_alive += w.orgs[c].alive;
    const int64_t ud = (int64_t)w.cfg.ave_time_slice * n_alive;   // cWorld::CalculateUpdateSize
    int64_t insts = 0, births = 0, deaths = 0, divides = 0, dropped = 0;
    age_tick(w);
    res_begin(w);   // ProcessPreUpdate + the update's first DoUpdates
    for (int64_t i = 0; i < ud; i++) {
      const double tot = sch.tree[1];
      if (!(tot > 0.0)) break;
      const double x = w.global_rng.rec ? w.global_rng.u() * tot
                                        : (double)w.global_rng.next() * (1.0 / 4294967296.0) * tot;
      int64_t c = sch.find(x);
      Org& o = w.orgs[c];
      if (!o.alive) continue;
      insts++;
      if (o.spec_count > 0) { o.spec_count--; continue; }
      if (o.spec_die) {                        // SingleProcess: m_spec_die -> Die (:917-921)
        o.alive = false; o.spec_die = false;
        sch.set(c, 0.0);
        deaths++;
        continue;
      }
      Exec ex{w, o, AVGPU_MODE_WORLD};
      ex.ctx = &w.ctx_rng;
      w.births.clear();
      const int d0 = o.num_divides;
      ex.single_process(c);
      divides += o.num_divides - d0;
      bool replaced = false;
      for (auto& b : w.births) {               // placed inside the h-divide
        const int r = serial_place(w, sch, b);
        births += r > 0;
        deaths += r == 2 || r == 3;            // KillOrganism of the replaced occupant
        dropped += r == 0;
        replaced = replaced || r == 3;
      }
      w.births.clear();
      if (replaced) continue;                  // the parent was killed in its own step
      if (!o.alive) { sch.set(c, 0.0); deaths++; continue; }
      // speculative run (SingleProcess(ctx, true) while it returns true)
      int spec = 0;
      while (spec < 32) {
        const int hid = w.is.handler[o.mem[adjust(o.head[HEAD_IP], (int)o.mem.size())]];
        if (hid == H_IO || hid == H_H_DIVIDE) break;   // STALL: rejected, nothing counted
        const int tu_max = o.max_executed;
        ex.single_process(c);
        if (!o.alive) {                        // reached the age limit speculatively: m_spec_die
          if (tu_max > 0) { o.alive = true; o.spec_die = true; }
          break;
        }
        spec++;
      }
      o.spec_count = spec;
    }
    res_end(w);
    // cStats for the update (finish_stats advances the update counter)
    w.t_insts = insts; w.t_deaths = deaths; w.t_divides = divides; w.t_slices = 0;
    finish_stats(w, births, dropped);
  }
  if (out) *out = w.stats;
  return 0;
}

}  // extern "C"

extern "C" {
// the serial world's own state (avgpu_get_serial_state / avgpu_set_serial_state):
// stream positions, speculative credit and death, faces, soup_perm (identity
// before its first use), the reaper queue rear first (-1: not built yet)
int orc_get_serial_state(void* h, avgpu_serial_state* st, int32_t* spec, uint8_t* face, int32_t* soup_perm,
                         int32_t* reaper, int64_t cap) {
  World& w = *(World*)h;
  const bool started = (int64_t)w.face.size() == w.ncells;
  const int64_t n = w.reaper_init ? (int64_t)w.reaper.size() : -1;
  if (st) {
    memset(st, 0, sizeof(*st));
    st->sched_pos = w.global_rng.ctr;
    st->ctx_pos = w.ctx_rng.ctr;
    st->reaper_len = n;
    st->started = started ? 1 : 0;
  }
  for (int64_t c = 0; c < w.ncells; c++) {
    if (spec) spec[c] = (w.orgs[c].spec_count & 0xFFFF) | (w.orgs[c].spec_die ? 1 << 16 : 0);
    if (face) face[c] = started ? w.face[c] : 0;
    if (soup_perm) soup_perm[c] = (int32_t)((int64_t)w.soup_cells.size() == w.ncells ? w.soup_cells[c] : c);
  }
  if (reaper && n > 0) {
    if (cap < n) return fail(AVGPU_EINVAL, "reaper buffer too small");
    int64_t k = 0;
    for (auto it = w.reaper.rbegin(); it != w.reaper.rend(); ++it) reaper[k++] = (int32_t)*it;
  }
  return 0;
}

int orc_set_serial_state(void* h, const avgpu_serial_state* st, const int32_t* spec, const uint8_t* face,
                         const int32_t* soup_perm, const int32_t* reaper) {
  World& w = *(World*)h;
  if (!st) return fail(AVGPU_EINVAL, "serial state");
  if (!st->started) return 0;
  if (soup_perm) {
    std::vector<char> seen((size_t)w.ncells, 0);
    for (int64_t c = 0; c < w.ncells; c++) {
      if (soup_perm[c] < 0 || soup_perm[c] >= w.ncells || seen[(size_t)soup_perm[c]])
        return fail(AVGPU_EINVAL, "soup_perm is not a permutation of the cells");
      seen[(size_t)soup_perm[c]] = 1;
    }
  }
  const int64_t len = st->reaper_len;
  if (len > 2 * w.ncells + 64) return fail(AVGPU_EINVAL, "reaper queue longer than 2n + 64");
  if (len > 0 && !reaper) return fail(AVGPU_EINVAL, "reaper queue");
  for (int64_t k = 0; k < len; k++)
    if (reaper[k] < 0 || reaper[k] >= w.ncells) return fail(AVGPU_EINVAL, "reaper queue cell out of range");
  w.global_rng.ctr = (uint32_t)st->sched_pos;
  w.ctx_rng.ctr = (uint32_t)st->ctx_pos;
  if ((int64_t)w.face.size() != w.ncells) w.face.assign(w.ncells, 0);
  for (int64_t c = 0; c < w.ncells; c++) {
    if (spec) { w.orgs[c].spec_count = spec[c] & 0xFFFF; w.orgs[c].spec_die = (spec[c] >> 16) & 1; }
    if (face) w.face[c] = face[c];
  }
  if (soup_perm) w.soup_cells.assign(soup_perm, soup_perm + w.ncells);
  if (w.cfg.birth_method == 5) {
    w.reaper.clear();
    w.reaper_init = len >= 0;
    for (int64_t k = 0; k < len; k++) w.reaper.push_front(reaper[k]);
  }
  return 0;
}
}  // extern "C"
