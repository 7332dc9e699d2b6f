// world.hip -- the per-update kernels around k_interpret:
//   k_set_orgs       cPopulation::Inject / ActivateOrganism + cPhenotype::SetupInject
//   k_get_states     cHardwareBase inspection API (trace tuple gather)
//   k_classify_*     budget + LDS size-class lists for k_interpret
//   k_merit_*        deterministic total merit (scheduler input)
//   k_block_counts, k_allot  the scheduler (cScheduler restated): the update's picks
//                    split down a binary tree of the cells
//   k_place_*, k_tile_*  cPopulation::PositionOffspring in conflict-resolving rounds
//   k_activate       cPopulation::ActivateOrganism + cPhenotype::SetupOffspring
//   k_stats          cStats reduction inputs
// Paths are relative to avida-core/source/ of the reference.
#include "device.h"
#include "births.h"

#pragma clang fp contract(off)

namespace {

// Append `cell` to its size-class list (rows 1..3).  Class 0 is not listed:
// k_interpret<CLASS0_SIZE> sweeps the cells densely.  Block-aggregated: one
// global atomic per class and block (a per-wave atomic on three addresses
// serialised ~16K waves in L2), lanes then write at block base + wave offset
// + rank.  blockDim.x must be 64 * WAVES.
template <int WAVES = 4>
__device__ __forceinline__ void enqueue_class(const DevWorld& W, int cell, bool want, int cls) {
  __shared__ int s_pc[NUM_CLASSES][WAVES], s_base[NUM_CLASSES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long masks[NUM_CLASSES];
  __syncthreads();                             // s_pc / s_base free (repeat calls)
#pragma unroll
  for (int k = 1; k < NUM_CLASSES; k++) {
    masks[k] = __ballot(want && cls == k);
    if (lane == 0) s_pc[k][wv] = __popcll(masks[k]);
  }
  __syncthreads();
  // waves take their offsets in wave order (deterministic list order)
  if (threadIdx.x > 0 && threadIdx.x < NUM_CLASSES) {
    const int k = threadIdx.x;
    int tot = 0;
    for (int w = 0; w < WAVES; w++) tot += s_pc[k][w];
    s_base[k] = tot ? atomicAdd(&W.class_count[k], tot) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 1; k < NUM_CLASSES; k++) {
    if (want && cls == k) {
      int woff = 0;
      for (int w = 0; w < wv; w++) woff += s_pc[k][w];
      const int rank = __popcll(masks[k] & ((1ull << lane) - 1ull));
      W.class_list[(int64_t)k * W.n + s_base[k] + woff + rank] = cell;
    }
  }
}

// The same for CPT cells per thread (cells[j], j-major order inside the
// block): one global atomic per class and block for all of them.
template <int WAVES, int CPT>
__device__ __forceinline__ void enqueue_class_multi(const DevWorld& W, const int* cell, const bool* want,
                                                    const int* cls) {
  __shared__ int s_pc[NUM_CLASSES][WAVES], s_base[NUM_CLASSES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long masks[NUM_CLASSES][CPT];
  __syncthreads();                             // s_pc / s_base free (repeat calls)
#pragma unroll
  for (int k = 1; k < NUM_CLASSES; k++) {
    int n = 0;
#pragma unroll
    for (int j = 0; j < CPT; j++) {
      masks[k][j] = __ballot(want[j] && cls[j] == k);
      n += __popcll(masks[k][j]);
    }
    if (lane == 0) s_pc[k][wv] = n;
  }
  __syncthreads();
  if (threadIdx.x > 0 && threadIdx.x < NUM_CLASSES) {
    const int k = threadIdx.x;
    int tot = 0;
    for (int w = 0; w < WAVES; w++) tot += s_pc[k][w];
    s_base[k] = tot ? atomicAdd(&W.class_count[k], tot) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 1; k < NUM_CLASSES; k++) {
    int woff = 0;
    for (int w = 0; w < wv; w++) woff += s_pc[k][w];
    int jbase = 0;
#pragma unroll
    for (int j = 0; j < CPT; j++) {
      if (want[j] && cls[j] == k) {
        const int rank = __popcll(masks[k][j] & ((1ull << lane) - 1ull));
        W.class_list[(int64_t)k * W.n + s_base[k] + woff + jbase + rank] = cell[j];
      }
      jbase += __popcll(masks[k][j]);
    }
  }
}

__device__ __forceinline__ int need_of_cell(const DevWorld& W, int cell) {
  return ::need_of(W.mem_size[cell], W.ctl[cell], W.size_range);
}

// ---------------------------------------------------------------------------
__global__ void k_set_orgs(DevWorld W, int64_t first, int64_t count, const uint8_t* codes,
                           const int32_t* offsets, const int32_t* lens, const double* merits,
                           const int32_t* inputs, int deterministic) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t N = W.n;
  const int64_t c = first + i;
  const int len = lens[i];
  const uint8_t* g = codes + offsets[i];
  uint8_t* t = W.tape + c * TAPE_SLOT;
  for (int k = 0; k < len; k++) t[k] = g[k] & CODE_MASK;
  // registers, heads, label, counters, buffers, task counts, stacks: zero
  int32_t* x = W.xs + c * XS_WORDS;
  for (int k = 0; k < XS_WORDS; k++) x[k] = 0;
  W.ctl[c] = CTL_ALIVE;
  W.mem_size[c] = len;
  int mx = 0;
  if (W.death_method > 0) {                 // cOrganism::initialize (main/cOrganism.cc:216-236)
    mx = W.age_limit;
    if (W.death_method == 2) mx *= len;
    if (mx < 1) mx = 1;
  }
  W.max_exec[c] = mx;
  W.birth_len[c] = len;
  if (W.track_age) W.age[c] = -1;          // injected between updates: age 0 during the next one
  W.gkey[c] = gk_tape(t, len);
  // stream key (DESIGN.md RNG spec)
  uint32_t lo, hi, ctr = 0;
  derive_key(W.seed_lo, W.seed_hi, (uint32_t)(W.cell0 + c), 0xA5A5A5A5U, lo, hi);
  int in0, in1, in2;
  if (inputs) { in0 = inputs[3 * i]; in1 = inputs[3 * i + 1]; in2 = inputs[3 * i + 2]; }
  else if (deterministic) { in0 = 0x0f13149f; in1 = 0x3308e53e; in2 = 0x556241eb; }
  else {                                      // cEnvironment::SetupInputs random
    in0 = (15 << 24) + (int)rng_below(lo, hi, ctr, 1u << 24);
    in1 = (51 << 24) + (int)rng_below(lo, hi, ctr, 1u << 24);
    in2 = (85 << 24) + (int)rng_below(lo, hi, ctr, 1u << 24);
  }
  W.rng[c] = lo; W.rng[N + c] = hi; W.rng[2 * N + c] = ctr;
  if (W.rec_off) W.rec_off[c] = -1;   // a new organism draws from its counter stream
  if (W.spec) W.spec[c] = 0;           // serial world: no speculative credit yet
  W.inputs[c] = in0; W.inputs[N + c] = in1; W.inputs[2 * N + c] = in2;
  W.budget[c] = 0;
  for (int k = 0; k < AVGPU_MAX_REACTIONS; k++) {
    W.last_task[k * N + c] = 0; W.cur_react[k * N + c] = 0;   // record words: zeroed above
  }
  // cPhenotype::SetupInject (main/cPhenotype.cc:599-640)
  *reinterpret_cast<double*>(x + XS_BONUS) = W.default_bonus;
  W.merit[c] = (merits && merits[i] > 0.0) ? merits[i] : (double)len;
  W.fitness[c] = 0.0;
  W.credit[c] = 0.0;
  W.gest_time[c] = 0; W.num_div[c] = 0; W.generation[c] = 0;
  W.copied[c] = len; W.child_copied[c] = 0; W.executed[c] = len;
}

// the cHardwareBase inspection tuple of cell c (zero padding: the digest below
// hashes its bytes)
__device__ void build_state(const DevWorld& W, int64_t c, avgpu_cpu_state& s) {
  const int64_t N = W.n;
  memset(&s, 0, sizeof(s));
  const bool fresh = (W.ctl[c] & CTL_FRESH) != 0;   // birth values implied (setup_child)
  const int32_t* x = W.xs + c * XS_WORDS;
  if (!fresh) {
  for (int k = 0; k < 3; k++) s.reg[k] = x[XS_REG + k];
  for (int k = 0; k < 4; k++) s.head[k] = x[XS_HEAD + k];
  for (int k = 0; k < 2; k++)
    for (int j = 0; j < AVGPU_STACK_SIZE; j++) s.stack[k][j] = x[XS_STACK + k * AVGPU_STACK_SIZE + j];
  }
  const uint32_t ctl = W.ctl[c];
  s.stack_ptr[0] = CTL_SP0(ctl); s.stack_ptr[1] = CTL_SP1(ctl);
  s.cur_stack = (ctl & CTL_CURSTK) ? 1 : 0;
  s.mal_active = (ctl & CTL_MAL) ? 1 : 0;
  s.alive = (ctl & CTL_ALIVE) ? 1 : 0;
  const uint32_t rl = fresh ? 0u : (uint32_t)x[XS_RLABEL];
  s.read_label_len = rl & 15;
  for (int k = 0; k < (int)(rl & 15); k++) s.read_label[k] = (int8_t)((rl >> (4 + 2 * k)) & 3);
  s.mem_size = W.mem_size[c];
  s.cpu_cycles_used = fresh ? 0 : x[XS_CYCLES];
  s.time_used = fresh ? 0 : x[XS_TIME];
  s.gestation_start = fresh ? 0 : x[XS_GEST];
  s.gestation_time = W.gest_time[c];
  s.num_divides = fresh ? 0 : W.num_div[c];
  s.generation = W.generation[c];
  s.genome_length = W.birth_len[c];
  s.copied_size = W.copied[c];
  s.child_copied_size = fresh ? 0 : W.child_copied[c];
  s.executed_size = W.executed[c];
  s.max_executed = W.max_exec[c];
  s.birth_length = W.birth_len[c];
  s.input_ptr = fresh ? 0 : x[XS_INPTR];
  const int tot = fresh ? 0 : x[XS_INTOT];
  for (int k = 0; k < 3; k++) s.input_buf[k] = (k < tot) ? x[XS_INBUF + k] : 0;
  s.input_total = tot;
  s.output_total = fresh ? 0 : x[XS_OUTTOT];
  s.output_buf = s.output_total ? x[XS_OUTBUF] : 0;
  for (int k = 0; k < 3; k++) s.inputs[k] = W.inputs[k * N + c];
  // task counts past the logic-9 tasks stay 0 (no reaction can count them)
  for (int k = 0; k < AVGPU_MAX_REACTIONS && !fresh; k++) {
    s.cur_task_count[k] = k < AVGPU_NUM_LOGIC_TASKS ? x[XS_TASK + k] : 0;
    s.cur_reaction_count[k] = k < XS_NREACT ? x[XS_REACT + k] : W.cur_react[k * N + c];
  }
  for (int k = 0; k < AVGPU_MAX_REACTIONS; k++)   // a fresh offspring's were set at activation
    s.last_task_count[k] = (fresh && k >= AVGPU_NUM_LOGIC_TASKS) ? 0 : W.last_task[k * N + c];
  s.rng_key_lo = W.rng[c]; s.rng_key_hi = W.rng[N + c]; s.rng_counter = W.rng[2 * N + c];
  s.errors = fresh ? 0 : x[XS_ERRORS];
  s.cur_bonus = fresh ? W.default_bonus : *reinterpret_cast<const double*>(x + XS_BONUS);
  s.merit = W.merit[c];
  s.fitness = W.fitness[c];
  s.credit = W.credit[c];
  s.head_start = CTL_HS(ctl);
  s.age = W.track_age ? W.age[c] + 1 : 0;   // as UpdateOrganismStats leaves it at the update's end
}

__global__ void k_get_states(DevWorld W, int64_t first, int64_t count, avgpu_cpu_state* out,
                             uint8_t* codes, int cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t c = first + i;
  avgpu_cpu_state s;
  build_state(W, c, s);
  out[i] = s;
  if (codes) {
    const uint8_t* t = W.tape + c * TAPE_SLOT;
    uint8_t* d = codes + i * cap;
    const int m = s.mem_size < cap ? s.mem_size : cap;
    for (int k = 0; k < m; k++) d[k] = t[k];
  }
}

// Per-cell state digest (include/avida_gpu.h avgpu_state_digests): a chained
// 64-bit mix over the 32-bit words of the inspection tuple, then over the
// memory tape in canonical bytes (handler id | copied << 6 | executed << 7, 4
// sites per word, sites >= mem_size zero).  oracle/oracle.cc restates it on its
// own state, so GPU and oracle worlds of any size compare digest for digest.
__global__ void k_state_digest(DevWorld W, int64_t first, int64_t count, uint64_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t c = first + i;
  avgpu_cpu_state s;
  build_state(W, c, s);
  if (s.birth_length == 0) { out[i] = 0; return; }   // never occupied
  uint32_t w[sizeof(s) / 4];
  memcpy(w, &s, sizeof(s));              // the record's bytes (no type-punned loads)
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int k = 0; k < (int)(sizeof(s) / 4); k++) h = gk_mix(h ^ ((uint64_t)k << 32 | w[k]));
  const uint32_t* t = reinterpret_cast<const uint32_t*>(W.tape + c * TAPE_SLOT);
  const int m = min(max(s.mem_size, 0), TAPE_SLOT);
  for (int k = 0; k < (m + 3) / 4; k++) {
    uint32_t v = t[k];
    const int keep = m - 4 * k;
    if (keep < 4) v &= (1u << (8 * keep)) - 1u;
    h = gk_mix(h ^ ((uint64_t)(0x10000 + k) << 32 | v));
  }
  out[i] = h;
}

// checkpoint restore: the inverse of k_get_states; `codes` holds device codes
// with the TF_* flag bits, cap bytes per cell
__global__ void k_set_states(DevWorld W, int64_t first, int64_t count, const avgpu_cpu_state* in,
                             const uint8_t* codes, int cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t N = W.n;
  const int64_t c = first + i;
  const avgpu_cpu_state s = in[i];
  if (W.track_age) W.age[c] = s.age - 1;
  int32_t* x = W.xs + c * XS_WORDS;
  for (int k = 0; k < XS_WORDS; k++) x[k] = 0;
  for (int k = 0; k < 3; k++) x[XS_REG + k] = s.reg[k];
  for (int k = 0; k < 4; k++) x[XS_HEAD + k] = s.head[k];
  for (int k = 0; k < 2; k++)
    for (int j = 0; j < AVGPU_STACK_SIZE; j++) x[XS_STACK + k * AVGPU_STACK_SIZE + j] = s.stack[k][j];
  W.ctl[c] = (uint32_t)(s.stack_ptr[0] & 0xF) | ((uint32_t)(s.stack_ptr[1] & 0xF) << 4) |
             (s.cur_stack ? CTL_CURSTK : 0u) | (s.mal_active ? CTL_MAL : 0u) | (s.alive ? CTL_ALIVE : 0u) |
             ((s.head_start & 0x1FFFFu) << CTL_HS_SHIFT);
  uint32_t rl = (uint32_t)(s.read_label_len & 15);
  for (int k = 0; k < (s.read_label_len & 15) && k < AVGPU_MAX_LABEL; k++)
    rl |= (uint32_t)(s.read_label[k] & 3) << (4 + 2 * k);
  x[XS_RLABEL] = (int32_t)rl;
  W.mem_size[c] = s.mem_size;
  x[XS_CYCLES] = s.cpu_cycles_used; x[XS_TIME] = s.time_used; x[XS_GEST] = s.gestation_start;
  W.gest_time[c] = s.gestation_time; W.num_div[c] = s.num_divides; W.generation[c] = s.generation;
  W.birth_len[c] = s.birth_length;
  W.copied[c] = s.copied_size; W.child_copied[c] = s.child_copied_size; W.executed[c] = s.executed_size;
  W.max_exec[c] = s.max_executed;
  x[XS_INPTR] = s.input_ptr;
  for (int k = 0; k < 3; k++) x[XS_INBUF + k] = s.input_buf[k];
  x[XS_INTOT] = s.input_total;
  x[XS_OUTBUF] = s.output_buf; x[XS_OUTTOT] = s.output_total;
  for (int k = 0; k < 3; k++) W.inputs[k * N + c] = s.inputs[k];
  for (int k = 0; k < AVGPU_MAX_REACTIONS; k++) {
    if (k < AVGPU_NUM_LOGIC_TASKS) x[XS_TASK + k] = s.cur_task_count[k];
    W.last_task[k * N + c] = s.last_task_count[k];
    if (k < XS_NREACT) x[XS_REACT + k] = s.cur_reaction_count[k];
    else W.cur_react[k * N + c] = s.cur_reaction_count[k];
  }
  W.rng[c] = s.rng_key_lo; W.rng[N + c] = s.rng_key_hi; W.rng[2 * N + c] = s.rng_counter;
  if (W.rec_off) W.rec_off[c] = -1;   // restored organisms draw from counter streams
  x[XS_ERRORS] = s.errors;
  *reinterpret_cast<double*>(x + XS_BONUS) = s.cur_bonus;
  W.merit[c] = s.merit; W.fitness[c] = s.fitness; W.credit[c] = s.credit;
  W.budget[c] = 0;
  uint8_t* t = W.tape + c * TAPE_SLOT;
  const uint8_t* src = codes + i * cap;
  const int m = s.mem_size < cap ? s.mem_size : cap;
  for (int k = 0; k < m; k++) t[k] = src[k];
  // the birth genome is the tape prefix (as the oracle restores it)
  uint64_t gs = 0;
  const int bl = s.birth_length < m ? s.birth_length : m;
  for (int w = 0; w < (bl + 3) / 4; w++) {
    uint32_t v = 0;
    for (int j = 0; j < 4 && 4 * w + j < bl; j++) v |= (uint32_t)(t[4 * w + j] & CODE_MASK) << (8 * j);
    gs += gk_word(v, w, s.birth_length);
  }
  W.gkey[c] = gk_final(gs, s.birth_length);
}

// systematics census (include/avida_gpu.h avgpu_census): one row per cell,
// written as one coalesced 48-B struct per lane
__global__ void k_census(DevWorld W, int64_t first, int64_t count, avgpu_census* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t c = first + i;
  const uint32_t ctl = W.ctl[c];
  avgpu_census r;
  memset(&r, 0, sizeof(r));
  if (ctl & CTL_ALIVE) {
    r.genotype_key = W.gkey[c];
    r.merit = W.merit[c];
    r.fitness = W.fitness[c];
    r.genome_length = W.birth_len[c];
    r.gestation_time = W.gest_time[c];
    r.copied_size = W.copied[c];
    r.executed_size = W.executed[c];
    r.generation = W.generation[c];
    r.num_divides = (ctl & CTL_FRESH) ? 0 : W.num_div[c];
  }
  out[i] = r;
}

// budget = uniform or per-cell array, all live cells of [first, first+count)
__global__ void k_classify_uniform(DevWorld W, int64_t first, int64_t count, const int32_t* budget,
                                   int32_t uniform) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < count;
  const int cell = in ? (int)(first + i) : 0;
  int b = 0;
  bool want = false;
  int cls = 0;
  if (in) {
    b = budget ? budget[i] : uniform;
    W.budget[cell] = b;
    want = (W.ctl[cell] & CTL_ALIVE) && b > 0;
    if (want) cls = class_of(need_of_cell(W, cell));
    W.aclass[cell] = want ? (uint8_t)cls : (uint8_t)ACLASS_NONE;
  }
  enqueue_class(W, cell, want, cls);
}

// ---- deterministic total merit: 256-cell blocks, fixed pairwise tree ----
// (strip tiles hold whole 256-cell blocks, so the block partials of a tiled
// world are the single world's partials; alive_d: alive counts as doubles
// after the merits, the layout tiles exchange)
// Before the shards are cleared, an update whose statistics were never asked
// for (lazy: run with out == NULL, CNT_CUM_FLAG still 0) has its counts added
// to the running sums here instead of in k_stats_final.  One block, >= 256
// threads; the caller's condition is block-uniform.
__device__ __forceinline__ void reset_queues_block(const DevWorld& W) {
  if (threadIdx.x < 3) W.b_count[threadIdx.x] = 0;
  if (threadIdx.x < 8) W.class_count[threadIdx.x] = 0;
}
__device__ __forceinline__ void reset_counts_block(const DevWorld& W) {
  constexpr int NG = 256 / CNT_STRIDE;
  __shared__ unsigned long long cs[NG][CNT_STRIDE];
  const bool fold = W.counters[CNT_CUM_FLAG] == 0ull;
  if (threadIdx.x < 256) {
    const int slot = threadIdx.x & (CNT_STRIDE - 1), g = threadIdx.x / CNT_STRIDE;
    unsigned long long a = 0;
    if (fold && slot != CNT_STRIDE - 1) {
      unsigned long long v[NSHARD / NG];         // all loads in flight together (this block is
#pragma unroll                                   // the launch's long pole: ~16 L2 round trips)
      for (int k = 0; k < NSHARD / NG; k++) v[k] = W.counters[(g + k * NG) * CNT_STRIDE + slot];
#pragma unroll
      for (int k = 0; k < NSHARD / NG; k++) a += v[k];
    }
    cs[g][slot] = a;
  }
  __syncthreads();
  if (threadIdx.x < CNT_STRIDE) {
    unsigned long long t = 0;
    for (int g = 0; g < NG; g++) t += cs[g][threadIdx.x];
    if (threadIdx.x == CNT_STRIDE - 1) W.counters[CNT_CUM_FLAG] = 0ull;
    else if (t) W.counters[CNT_CUM_BASE + threadIdx.x] += t;
  }
  for (int i = threadIdx.x; i < NSHARD * CNT_STRIDE; i += blockDim.x) W.counters[i] = 0ull;
  if (threadIdx.x < 3) W.b_count[threadIdx.x] = 0;
  if (threadIdx.x < 8) W.class_count[threadIdx.x] = 0;
}

// reset 1: block 0 also zeroes the update's counters, birth-queue and class-list
// lengths (k_reset_counts' work; the previous update's statistics have read them);
// reset 2 (a later sub-update): the queue and list lengths only, the counters
// go on adding up the update
// One wave per 256-cell block b (partial[b]): the pairwise tree of strides
// 128, 64, ..., 1 (s[t] += s[t + stride]), the oracle's tree_merit_sum order.
// Lane l loads cells l, l+64, l+128, l+192 and forms the stride-128 and -64
// sums itself; strides 32 .. 1 are lane shuffles -- the same additions in the
// same order, without the LDS tree's 8 barriers.  Four blocks per workgroup.
__global__ __launch_bounds__(256) void k_merit_partial(DevWorld W, double* partial, int32_t* alive_partial,
                                                       double* alive_d, int reset) {
  if (reset == 1 && blockIdx.x == 0) reset_counts_block(W);
  if (reset == 2 && blockIdx.x == 0) reset_queues_block(W);
  // a strip's partials end with its last step's predictor, pick carry and
  // divide counts by quarter (the oracle's orc_tile_partials; summed on every
  // strip after the gather)
  if (alive_d && blockIdx.x == 0 && threadIdx.x < 6) {
    const int64_t nbl = (W.n + 255) / 256;
    const long long v = threadIdx.x == 0 ? pacc_sum(W, 0)
                        : (threadIdx.x == 1 ? W.sched[1] : quarter_count(W, (int)threadIdx.x - 2));
    partial[2 * nbl + threadIdx.x] = __longlong_as_double(v);
  }
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nb = (W.n + 255) / 256;
  if (b >= nb) return;
  double m[4];
  int a = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int64_t c = b * 256 + lane + 64 * k;
    const uint32_t ctl = c < W.n ? W.ctl[c] : 0u;
    const bool live = (ctl & CTL_ALIVE) != 0;
    m[k] = live ? sched_weight(W.merit[c], ctl) : 0.0;   // the scheduler weight (oracle block_levels)
    a += live ? 1 : 0;
  }
  double z = __dadd_rn(__dadd_rn(m[0], m[2]), __dadd_rn(m[1], m[3]));
  for (int off = 32; off >= 1; off >>= 1) {
    const double o = __shfl_down(z, off);
    z = __dadd_rn(z, o);                       // lanes < off hold the tree's s[t]
    a += __shfl_down(a, off);
  }
  if (lane == 0) {
    partial[b] = z;
    if (alive_partial) alive_partial[b] = a;
    if (alive_d) alive_d[b] = (double)a;
  }
}

// ---- the scheduler: PROBABILISTIC slicing as the reference's picks ----
// (oracle/oracle.cc block_levels / top_tree / block_split) The
// update's UD = AVE_TIME_SLICE x N picks are split down a fixed binary tree
// with a Binomial at every node: the top tree over the 256-cell blocks'
// partials (k_block_counts, one workgroup), then each block's stride tree
// down to its cells (k_allot).
//
// k_block_counts: heap-ordered top tree in tree_scr (node h = (1 << l) + i,
// children 2h, 2h + 1; leaves at P + block, zero-padded to P = 2^L), built
// bottom up, split top down in tree_cnt.  mode 0: this world's partials
// (part doubles, alive int32); mode 1: a strip's gathered vector (tile k's
// block j at gathered[k * 2 nb + j], its alive count nb after); mode 2: this
// world's partials with the totals of every world handed in (totals[0..1]:
// cMultiProcessWorld::CalculateUpdateSize, main/cMultiProcessWorld.cc:
// 396-405 -- this world's picks = (int)((local / total) * AVE_TIME_SLICE *
// N_total)); mode 3: the totals only (totals[0..1] = root, N).
// totals[2] = the weight total INTEGRATED divides by, totals[3] = UD.
// LDS: the whole tree in the workgroup's LDS (P <= TREE_LDS_P: 2 x 4096 doubles
// + counts = 128 KiB of gfx950's 160).  A larger tree (strips of a world of
// more than 4096 blocks: the weak-scaling bench at N >= 2, configs[3]) is
// cut at the level of its 4096-block subtrees ("chunks"): k_tree_up builds
// every chunk's sums (a workgroup each), k_block_counts runs the tree above
// the chunk roots (chunked = 1: its leaves are the chunk roots, its output
// the chunk roots' counts), k_tree_down splits each chunk over this world's
// blocks (a workgroup each).  The same pairwise sums, the same draws at the
// same heap nodes: the same counts as one tree (oracle top_tree).  (One
// workgroup over a 65536-block tree in global memory took 124 us.)
#define TREE_LDS_P 4096
#define TREE_C_LOG 12

// leaf g of the block level (0 past the blocks); alive count into a
__device__ __forceinline__ double tree_leaf(const double* part, const int32_t* alive_part, int64_t nb, int64_t nbt,
                                            int mode, int64_t g, long long& a) {
  if (g >= nbt) return 0.0;
  if (mode == 1) {
    const int64_t k = g / nb, j = g - k * nb;
    a += (long long)part[k * tile_part_stride(nb) + nb + j];
    return part[k * tile_part_stride(nb) + j];
  }
  a += alive_part[g];
  return part[g];
}
template <bool LDS>
__global__ __launch_bounds__(1024) void k_block_counts(DevWorld W, const double* part, const int32_t* alive_part,
                                                       int64_t nb, int ntiles, int L, double* totals,
                                                       uint32_t update, int mode, int chunked, int sub,
                                                       int nsub) {
  __shared__ long long s_cnt[1024];
  __shared__ double l_scr[LDS ? 2 * TREE_LDS_P : 1];
  __shared__ long long l_cnt[LDS ? 2 * TREE_LDS_P : 1];
  const int tid = threadIdx.x;
  const int64_t P = (int64_t)1 << L, nbt = mode == 1 ? nb * ntiles : nb;
  double* scr = LDS ? l_scr : W.tree_scr;
  long long* cnt = LDS ? l_cnt : reinterpret_cast<long long*>(W.tree_cnt);
  long long a = 0;
  for (int64_t g = tid; g < P; g += 1024) {
    double v;
    if (chunked) {                              // the chunk roots of k_tree_up
      v = W.tree_scr[g];
      a += W.tree_cnt[g];
    } else {
      v = tree_leaf(part, alive_part, nb, nbt, mode, g, a);
    }
    scr[P + g] = v;
  }
  s_cnt[tid] = a;
  __syncthreads();
  for (int st = 512; st >= 1; st >>= 1) {      // living organisms (integer: any order)
    if (tid < st) s_cnt[tid] += s_cnt[tid + st];
    __syncthreads();
  }
  for (int l = L - 1; l >= 0; l--) {
    const int64_t w0 = (int64_t)1 << l;
    for (int64_t i = tid; i < w0; i += 1024) scr[w0 + i] = __dadd_rn(scr[2 * (w0 + i)], scr[2 * (w0 + i) + 1]);
    __syncthreads();
  }
  if (tid == 0) {
    const long long n = s_cnt[0];
    const double root = scr[1];
    const double ave = (double)W.ave_time_slice;
    // the update's UD = AVE_TIME_SLICE x the organisms at its start
    // (cAvidaDriver's update loop; W.sched[4]), a step's share of that
    if (sub == 0 && mode != 2) W.sched[4] = (long long)W.ave_time_slice * n;
    long long nroot = sub_share(W.sched[4], sub, nsub);
    if (mode == 2) {
      const double tot = totals[0];
      nroot = tot > 0.0 ? (long long)__dmul_rn(__dmul_rn(__ddiv_rn(root, tot), ave), totals[1]) : 0;
      totals[2] = tot;
      totals[3] = __dmul_rn(ave, totals[1]);
    } else {
      totals[0] = root;
      totals[1] = (double)n;
      totals[2] = root;
      totals[3] = (double)W.sched[4];
    }
    if (mode != 3) {
      // the picks the last steps' newborns ran beyond their victims'
      // leftovers come out of an update's first step (oracle take_carry): a
      // strip sums every strip's carry from the gathered partials
      long long fresh = W.sched[1];
      if (mode == 1) {
        fresh = 0;
        for (int k = 0; k < ntiles; k++) fresh += __double_as_longlong(part[k * tile_part_stride(nb) + 2 * nb + 1]);
      }
      long long rem = W.sched[2] + fresh;
      if (sub == 0) {
        const long long take = min(max(rem, -nroot), nroot);
        rem -= take;
        nroot -= take;
      }
      W.sched[1] = 0;
      W.sched[2] = rem;
      count_add(W, CNT_STEPS, 1ull);
    }
    cnt[1] = nroot;
  }
  __syncthreads();
  if (mode == 3) return;
  for (int i = tid; i < NSHARD * PACC_STRIDE; i += 1024) W.pacc[i] = 0;   // this step's predictor (interp.hip pred_term)
  // top down, only the nodes over this world's blocks [b0, b0 + nloc) (a
  // node's count depends on its ancestors' alone): a strip of T splits its
  // own subtree and the path to it, not the whole gathered world's tree
  // (chunked: the leaves are chunks, the range in chunks)
  const int sh = chunked ? TREE_C_LOG : 0;
  const int64_t b0 = mode == 1 ? W.cell0 / 256 : 0;
  const int64_t nloc = (W.n + 255) / 256;
  const int64_t lo = b0 >> sh, hi = (b0 + nloc - 1) >> sh;
  for (int l = 0; l < L; l++) {
    const int64_t w0 = (int64_t)1 << l;
    const int64_t ilo = lo >> (L - l), ihi = hi >> (L - l);
    for (int64_t i = ilo + tid; i <= ihi; i += 1024) {
      const int64_t h = w0 + i;
      const long long n = cnt[h];
      const long long left = binom_draw(n, __ddiv_rn(scr[2 * h], scr[h]),
                                        node_draw(W.seed_lo, W.seed_hi, update, SALT_TOP, (uint64_t)h));
      cnt[2 * h] = left;
      cnt[2 * h + 1] = n - left;
    }
    __syncthreads();
  }
  if (chunked) {
    for (int64_t j = lo + tid; j <= hi; j += 1024) W.tree_cnt[P + j] = cnt[P + j];
  } else {
    for (int64_t j = tid; j < nloc; j += 1024) W.blk_count[j] = cnt[P + b0 + j];
  }
}

// a chunk's subtree sums in LDS (t[1 .. 2 C), leaves at C + i), its alive count
__device__ __forceinline__ long long chunk_sums(double* t, long long* s_cnt, const double* part,
                                                const int32_t* alive_part, int64_t nb, int64_t nbt, int mode,
                                                int64_t k) {
  constexpr int C = 1 << TREE_C_LOG;
  const int tid = threadIdx.x;
  long long a = 0;
  for (int i = tid; i < C; i += 1024) t[C + i] = tree_leaf(part, alive_part, nb, nbt, mode, k * C + i, a);
  s_cnt[tid] = a;
  __syncthreads();
  for (int st = 512; st >= 1; st >>= 1) {
    if (tid < st) s_cnt[tid] += s_cnt[tid + st];
    __syncthreads();
  }
  for (int l = TREE_C_LOG - 1; l >= 0; l--) {
    const int w0 = 1 << l;
    for (int i = tid; i < w0; i += 1024) t[w0 + i] = __dadd_rn(t[2 * (w0 + i)], t[2 * (w0 + i) + 1]);
    __syncthreads();
  }
  return s_cnt[0];
}
// chunk k = blockIdx.x: its root's sum -> tree_scr[k], its organisms -> tree_cnt[k]
__global__ __launch_bounds__(1024) void k_tree_up(DevWorld W, const double* part, const int32_t* alive_part,
                                                  int64_t nb, int ntiles, int mode) {
  __shared__ double t[2 << TREE_C_LOG];
  __shared__ long long s_cnt[1024];
  const int64_t nbt = mode == 1 ? nb * ntiles : nb;
  const long long a = chunk_sums(t, s_cnt, part, alive_part, nb, nbt, mode, blockIdx.x);
  if (threadIdx.x == 0) {
    W.tree_scr[blockIdx.x] = t[1];
    W.tree_cnt[blockIdx.x] = a;
  }
}
// chunk k = k0 + blockIdx.x of this world's range: its count (tree_cnt[K + k],
// k_block_counts chunked) split down its subtree over this world's blocks;
// node i of local level l is heap node (K + k) 2^l + i
__global__ __launch_bounds__(1024) void k_tree_down(DevWorld W, const double* part, const int32_t* alive_part,
                                                    int64_t nb, int ntiles, int mode, int64_t K, uint32_t update) {
  constexpr int C = 1 << TREE_C_LOG;
  __shared__ double t[2 * C];
  __shared__ long long c[2 * C];
  __shared__ long long s_cnt[1024];
  const int tid = threadIdx.x;
  const int64_t nbt = mode == 1 ? nb * ntiles : nb;
  const int64_t b0 = mode == 1 ? W.cell0 / 256 : 0;
  const int64_t nloc = (W.n + 255) / 256;
  const int64_t k = (b0 >> TREE_C_LOG) + blockIdx.x;
  chunk_sums(t, s_cnt, part, alive_part, nb, nbt, mode, k);
  if (tid == 0) c[1] = W.tree_cnt[K + k];
  __syncthreads();
  // this world's blocks inside the chunk: local leaves [lo, hi]
  const int64_t g0 = k * C;
  const int lo = (int)(max(b0, g0) - g0), hi = (int)(min(b0 + nloc, g0 + C) - 1 - g0);
  for (int l = 0; l < TREE_C_LOG; l++) {
    const int w0 = 1 << l;
    const int ilo = lo >> (TREE_C_LOG - l), ihi = hi >> (TREE_C_LOG - l);
    for (int i = ilo + tid; i <= ihi; i += 1024) {
      const int h = w0 + i;
      const long long n = c[h];
      const uint64_t H = (uint64_t)(K + k) * (uint64_t)w0 + (uint64_t)i;
      const long long left = binom_draw(n, __ddiv_rn(t[2 * h], t[h]),
                                        node_draw(W.seed_lo, W.seed_hi, update, SALT_TOP, H));
      c[2 * h] = left;
      c[2 * h + 1] = n - left;
    }
    __syncthreads();
  }
  for (int i = lo + tid; i <= hi; i += 1024) W.blk_count[g0 + i - b0] = c[C + i];
}

__device__ __forceinline__ void occ_init_cell(const DevWorld& W, int64_t c) {
  W.occ[c] = (c < W.n && (W.ctl[c] & CTL_ALIVE)) ? 1 : 0;
  W.owner[c] = -1;
}

// k_allot: one wave per 256-cell block, 16 blocks per workgroup.  Lane l
// holds cells l, l + 64, l + 128, l + 192.  The block's stride tree over its
// cells' weights (node (k, t) = the cells = t mod 2^k, the additions of
// k_merit_partial): levels 7 and 6 in the lane, levels 5..0 by shuffles; then
// its count blk_count[b] split top down (PROBABILISTIC): levels 0..5 across
// the lanes (lane t holds node (k, t), the right child's count goes to lane
// t + 2^k by shuffle), levels 6 and 7 in the lane -- no barrier, no LDS.
// INTEGRATED: lambda = UD * weight / total with a credit carry; CONSTANT (or
// no weight at all): AVE_TIME_SLICE.  Each cell's head start is consumed here.
// Also the cell's budget and class tag, the placement occupancy of this
// update (living cells occupied; an organism that dies in its slice clears
// its cell at write-back), its kill time, the previous update's round-3
// claim, and the class lists.
// a cell's bucket of the class-0 order: class-0 slices by budget, descending
// (clamped both ways: a bucket outside the histogram would place the cell
// outside its window of W.order), every other cell in the last bucket
__device__ __forceinline__ int window_bucket(bool c0, int budget) {
  return c0 ? SORT_BUCKETS - 2 - min(max(budget, 0), SORT_BUCKETS - 2) : SORT_BUCKETS - 1;
}
__global__ __launch_bounds__(1024) void k_allot(DevWorld W, const double* totals, uint32_t update, int tick) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const int64_t nb = (W.n + 255) / 256;
  const double total = totals[2];
  const bool consts = W.slicing == AVGPU_SLICE_CONSTANT || !(total > 0.0);
  const bool prob = !consts && W.slicing != AVGPU_SLICE_INTEGRATED;
  uint32_t ctl[4];
  double wt[4];
  bool alive[4];
  int msz[4];                                  // loaded ahead of the tree (the class needs it)
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int64_t c = b * 256 + lane + 64 * j;
    ctl[j] = (b < nb && c < W.n) ? W.ctl[c] : 0u;
    alive[j] = (ctl[j] & CTL_ALIVE) != 0;
    msz[j] = alive[j] ? W.mem_size[c] : 0;
    const double m = alive[j] ? W.merit[c] : 0.0;
    if (alive[j] && !merit_ok(m)) count_add(W, CNT_BAD_RECORD, 1ull);   // counted; sched_weight gives it 0
    wt[j] = alive[j] ? sched_weight(m, ctl[j]) : 0.0;
  }
  long long cnt[4] = {0, 0, 0, 0};
  if (prob && b < nb) {                        // wave-uniform
    const uint64_t gb = (uint64_t)(W.cell0 / 256 + b);
    const uint32_t slo = W.seed_lo, shi = W.seed_hi;
    // bottom up: L7[l] = x[l] + x[l+128], L7[l+64] = x[l+64] + x[l+192], L6[l] = L7[l] + L7[l+64]
    const double l7a = __dadd_rn(wt[0], wt[2]), l7b = __dadd_rn(wt[1], wt[3]);
    const double l6 = __dadd_rn(l7a, l7b);
    double lv[7];                                // lv[k] = L_k[lane] (k = 0..6; lanes >= 2^k: unused)
    lv[6] = l6;
#pragma unroll
    for (int k = 5; k >= 0; k--) {
      const double o = __shfl_down(lv[k + 1], 1 << k);
      lv[k] = __dadd_rn(lv[k + 1], o);
    }
    // top down: lane t < 2^k holds count(k, t)
    long long c = lane == 0 ? (long long)W.blk_count[b] : 0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      long long left = 0;
      const bool act = lane < (1 << k);
      if (act)
        left = binom_draw(c, __ddiv_rn(lv[k + 1], lv[k]),
                          node_draw(slo, shi, update, SALT_BLOCK, (gb << 9) | (uint64_t)((1 << k) + lane)));
      const long long right = c - left;
      const long long got = __shfl_up(right, 1 << k);   // lane t + 2^k takes node (k, t)'s right child
      if (act) c = left;
      else if (lane < (2 << k)) c = got;
    }
    // level 6 (node (6, l) -> (7, l), (7, l + 64)) and level 7 (-> the cells)
    const long long l6l = binom_draw(c, __ddiv_rn(l7a, l6),
                                     node_draw(slo, shi, update, SALT_BLOCK, (gb << 9) | (uint64_t)(64 + lane)));
    const long long c7a = l6l, c7b = c - l6l;
    const long long x0 = binom_draw(c7a, __ddiv_rn(wt[0], l7a),
                                    node_draw(slo, shi, update, SALT_BLOCK, (gb << 9) | (uint64_t)(128 + lane)));
    const long long x1 = binom_draw(c7b, __ddiv_rn(wt[1], l7b),
                                    node_draw(slo, shi, update, SALT_BLOCK, (gb << 9) | (uint64_t)(192 + lane)));
    cnt[0] = x0; cnt[2] = c7a - x0; cnt[1] = x1; cnt[3] = c7b - x1;
  }
  bool want[4] = {false, false, false, false};
  int cls[4] = {0, 0, 0, 0}, buds[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int64_t c = b * 256 + lane + 64 * j;
    if (b >= nb || c >= W.n) continue;
    int bud = 0;
    if (alive[j]) {
      if (consts) {
        bud = W.ave_time_slice;
      } else if (prob) {
        bud = (int)min(cnt[j], (long long)(BUDGET_PRIM - 1));   // budgets are < 2^30 (device.h)
      } else {
        double lam = __ddiv_rn(__dmul_rn(totals[3], wt[j]), total);
        if (lam > 1.0e8) lam = 1.0e8;
        const double cr = __dadd_rn(W.credit[c], lam);
        const double fl = floor(cr);
        bud = (int)fl;
        W.credit[c] = __dsub_rn(cr, fl);
      }
      if (ctl[j] & CTL_HS_MASK) W.ctl[c] = ctl[j] & ~CTL_HS_MASK;   // the head start is used up
      if (tick && W.track_age) W.age[c] += 1;   // cPhenotype::IncAge at the previous update's end (oracle age_tick)
      want[j] = bud > 0;
      if (want[j]) cls[j] = class_of(need_of(msz[j], ctl[j], W.size_range));   // need_of_cell
    }
    buds[j] = bud;
    W.budget[c] = bud;
    W.aclass[c] = want[j] ? (uint8_t)cls[j] : (uint8_t)ACLASS_NONE;
    W.ran[c] = 0;
    if (W.env_resources)
      for (int r = 0; r < W.n_res; r++) W.cons[(int64_t)r * W.n + c] = 0.0;
    occ_init_cell(W, c);
    W.killt[c] = 0u;
    W.claim_r[3][c] = 0ull;   // the previous update's round-3 claims (k_activate read them last)
  }
  unsigned long long ns = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) ns += (unsigned long long)__popcll(__ballot(want[j]));
  if (lane == 0 && ns) count_add(W, CNT_SLICES, ns);
  int cells[4];
#pragma unroll
  for (int j = 0; j < 4; j++) cells[j] = (int)(b * 256 + lane + 64 * j);
  enqueue_class_multi<16, 4>(W, cells, want, cls);
  // this 4096-cell sub-window's histogram of the class-0 order's buckets
  // (k_window_order; the bucket rule of window_bucket)
  __shared__ int sh[SORT_BUCKETS];
  for (int i = threadIdx.x; i < SORT_BUCKETS; i += 1024) sh[i] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int64_t c = b * 256 + lane + 64 * j;
    if (b < nb && c < W.n) atomicAdd(&sh[window_bucket(want[j] && cls[j] == 0, buds[j])], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SORT_BUCKETS; i += 1024) W.sub_hist[(int64_t)blockIdx.x * SORT_BUCKETS + i] = sh[i];
}

// exclusive scan of the SORT_BUCKETS counts in h, in place, by one wave
__device__ __forceinline__ void bucket_scan(int* h) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    constexpr int PER = (SORT_BUCKETS + 63) / 64;
    int loc[PER], t = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int i = tid * PER + k;
      loc[k] = i < SORT_BUCKETS ? h[i] : 0;
      t += loc[k];
    }
    int incl = t;
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off);
      if (tid >= off) incl += o;
    }
    int run = incl - t;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int i = tid * PER + k;
      if (i < SORT_BUCKETS) h[i] = run;
      run += loc[k];
    }
  }
}

// The class-0 order: each SORT_WIN window's class-0 cells by budget
// (descending), a counting sort.  Which cell runs in which wave changes no
// organism's result (per-organism streams, placement by birth time and key),
// it only groups similar slices, so the order inside a budget is free (LDS
// atomics).  A wave loses about (window's budget range) / (2 x its waves) per
// lane to the spread of its budgets: 8192-cell windows (128 waves) took the
// lane efficiency of the multinomial budgets from 0.94 to 0.98
// (tools/budget_spread.py), 32768 cells measured fastest (HISTORY.md,
// profiles/r04w_ab.txt).
// One 1024-thread block per 4096-cell sub-window (the blocks of k_allot,
// which left each sub-window's bucket histogram in sub_hist): the window's
// bucket starts plus the counts of its earlier sub-windows, then this
// sub-window's cells by LDS atomics.  (One block per 32768-cell window, all
// of its 32768 LDS atomics on ~25 busy buckets, took 33 us: the list classes
// used that as their head start before they ran inside class 0's launch.)
__global__ __launch_bounds__(1024) void k_window_order(DevWorld W) {
  constexpr int SUBS = SORT_WIN / 4096;
  __shared__ int start[SORT_BUCKETS];
  const int tid = threadIdx.x;
  const int64_t sub = blockIdx.x;
  const int64_t s0 = (sub / SUBS) * SUBS, nsub = (W.n + 4095) / 4096;
  int before = 0;
  if (tid < SORT_BUCKETS) {
    int tot = 0;
    for (int64_t k = s0; k < s0 + SUBS && k < nsub; k++) {
      const int v = W.sub_hist[k * SORT_BUCKETS + tid];
      tot += v;
      if (k < sub) before += v;
    }
    start[tid] = tot;
  }
  __syncthreads();
  bucket_scan(start);
  __syncthreads();
  if (tid < SORT_BUCKETS) start[tid] += before;
  __syncthreads();
  const int64_t wbase = (sub / SUBS) * SORT_WIN;
#pragma unroll
  for (int h = 0; h < 4; h++) {
    const int64_t c = sub * 4096 + h * 1024 + tid;
    if (c < W.n) {
      const int pos = atomicAdd(&start[window_bucket(W.aclass[c] == 0, W.budget[c])], 1);
      W.order[wbase + pos] = (int32_t)c;
    }
  }
}


// ---- budget-sorted class-0 windows ----
// A wave runs until its longest slice ends, so the class-0 interpreter takes
// its 64 organisms from a window of SORT_WIN cells sorted by budget
// (k_window_order above).

// ---- strip-tile halo (DESIGN.md "Multi-GPU") ----
// Edge rows: top = local row 0, bottom = local row rows-1; ghost rows after n.
__device__ __forceinline__ int64_t edge_cell(const DevWorld& W, int d, int x) {
  return d == 0 ? (int64_t)x : (int64_t)(W.rows - 1) * W.world_x + x;
}
__device__ __forceinline__ int64_t ghost_cell(const DevWorld& W, int d, int x) {
  return W.n + (int64_t)d * W.world_x + x;
}
// Halo buffer (one per direction): per round parity p = round & 1, [X u64]
// the sender's claims on the receiver's edge row (its ghost row, k = 0) and
// [X u64] the sender's own claims on its edge row (the receiver's ghost row,
// k = 1); then [X u8] the sender's edge-row occupancy after interpretation.
// A cell of an edge row is claimed only from the two strips it touches, so
// after ONE exchange per placement round both strips know every claim on
// both rows and resolve them alike; the parities let round m + 1's claims
// go out while round m's are still being read (DESIGN.md "Multi-GPU").
__device__ __forceinline__ unsigned long long* halo_cl(uint8_t* b, int X, int p, int k) {
  return reinterpret_cast<unsigned long long*>(b) + (int64_t)(2 * p + k) * X;
}
__device__ __forceinline__ uint8_t* halo_occ(uint8_t* b, int X) { return b + (int64_t)X * 32; }
// round 0's kill times of the sender's picks on the receiver's edge row
__device__ __forceinline__ uint32_t* halo_kt(uint8_t* b, int X) { return reinterpret_cast<uint32_t*>(b + halo_kt_off(X)); }
// which halo slot a cell maps to: d = direction, x = column, k = 0 for a
// ghost cell (my claims on the neighbour's edge), 1 for an edge cell
__device__ __forceinline__ bool halo_slot(const DevWorld& W, int64_t c, int& d, int& x, bool& ghost) {
  const int X = W.world_x;
  if (c >= W.n) { const int64_t k = c - W.n; d = (int)(k / X); x = (int)(k - (int64_t)d * X); ghost = true; return true; }
  ghost = false;
  if (c < X) { d = 0; x = (int)c; return true; }
  if (c >= W.n - X) { d = 1; x = (int)(c - (W.n - X)); return true; }
  return false;
}
// a tile's cell is taken for round m's pick: occupied before round m - 1's
// resolve, or claimed in round m - 1 -- here, or by the neighbour on my edge
// row / on its own edge row (my ghost row): every claimed cell gets a winner,
// so this is the occupancy round m - 1's resolve leaves, read before that
// resolve (in the same launch) has written it.  Round 0 reads the ghost
// rows' occupancy straight from the received halo.
__device__ __forceinline__ bool tile_taken(const DevWorld& W, int64_t c, int m) {
  int d, x;
  bool ghost;
  const bool h = halo_slot(W, c, d, x, ghost);
  if (m == 0) return (h && ghost) ? halo_occ(W.h_recv[d], W.world_x)[x] != 0 : W.occ[c] != 0;
  if (W.occ[c] || W.claim_r[m - 1][c] != 0ull) return true;
  return h && halo_cl(W.h_recv[d], W.world_x, (m - 1) & 1, ghost ? 1 : 0)[x] != 0ull;
}
// round m's merged claim on cell t: mine, the neighbour's
__device__ __forceinline__ unsigned long long tile_merged(const DevWorld& W, int64_t t, int m) {
  unsigned long long v = W.claim_r[m][t];
  int d, x;
  bool ghost;
  if (halo_slot(W, t, d, x, ghost)) {
    const unsigned long long o = halo_cl(W.h_recv[d], W.world_x, m & 1, ghost ? 1 : 0)[x];
    if (o > v) v = o;
  }
  return v;
}

// The rest of a deferred divide (interp.hip, BI_FINAL), in two halves that
// run side by side in placement round 0's launch.  The offspring's RNG key
// (derived from the parent's key and divide count) is the pick's, which draws
// from it (finalize_key); the offspring's fitness (cPhenotype::DivideReset,
// merit / gestation time) and -- from the record of the parent's last divide
// of the update, the one whose sequence number is its final num_div -- the
// parent's merit, fitness, gestation time, copied / executed sizes and last
// task counts (main/cPhenotype.cc:824-1000) are the extra blocks'
// (finalize_phenotype), off the pick's dependency chain.  BI_FINAL stays set
// (a row is rewritten whole by its next divide): both halves test it.
__device__ __forceinline__ void finalize_key(const DevWorld& W, int64_t r, int parent) {
  int32_t* row = W.b_inh + r * BI_WORDS;
  if ((row[BI_FINAL] & 1) == 0) return;
  uint32_t clo, chi;
  derive_key(W.rng[parent], W.rng[W.n + parent], W.b_seq[r], 0x1B873593U, clo, chi);
  row[BI_RLO] = (int32_t)clo;
  row[BI_RHI] = (int32_t)chi;
}
// (every load it needs is issued before the first test: the record's row, its
// parent and sequence number, then the parent's divide count -- a chain of
// three dependent loads after the queue entry)
__device__ __forceinline__ void finalize_phenotype(const DevWorld& W, int64_t r) {
  static_assert(BI_LTASK == 12 && BI_FINAL == 11 && AVGPU_NUM_LOGIC_TASKS <= 12, "row quads");
  int32_t* row = W.b_inh + r * BI_WORDS;
  const int4* q = reinterpret_cast<const int4*>(row);
  const int4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4], q5 = q[5];
  const int parent = W.b_parent[r];
  const int seq = (int)W.b_seq[r];
  if ((q2.w & 1) == 0) return;                 // BI_FINAL
  const int nd = W.num_div[parent];
  const double merit = __hiloint2double(q0.y, q0.x);
  const int gt = q1.w;
  const double fit = __ddiv_rn(merit, (double)gt);
  const long long fb = __double_as_longlong(fit);
  row[BI_FITNESS] = (int32_t)fb;
  row[BI_FITNESS + 1] = (int32_t)(fb >> 32);
  if (seq == nd) {
    W.merit[parent] = merit;
    W.fitness[parent] = fit;
    W.gest_time[parent] = gt;
    W.child_copied[parent] = q1.y;
    W.executed[parent] = q1.z;
    const int lt[12] = {q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, q4.z, q4.w, q5.x, q5.y, q5.z, q5.w};
#pragma unroll
    for (int k = 0; k < AVGPU_NUM_LOGIC_TASKS; k++) W.last_task[(int64_t)k * W.n + parent] = lt[k];
  }
}

// ---- time-ordered placement (oracle/oracle.cc "3. Time-ordered placement";
// DESIGN.md 5) ----
// claim key: [63:48] time key (kill: t, empty: 0xFFFF - t), [47] kill,
// [46:32] the pick's draw >> 17, [31:8] the parent's GLOBAL cell id (tiles
// agree), [7:0] its divide number
__device__ __forceinline__ unsigned long long claim_key(uint32_t t, bool kill, uint32_t draw, int64_t gparent,
                                                        uint32_t seq) {
  const unsigned long long tk = kill ? (unsigned long long)(t & 0xFFFFu) : (unsigned long long)(0xFFFFu - (t & 0xFFFFu));
  return (tk << 48) | ((unsigned long long)(kill ? 1 : 0) << 47) | ((unsigned long long)(draw >> 17) << 32) |
         ((unsigned long long)(gparent & 0xFFFFFF) << 8) | (unsigned long long)(seq & 0xFF);
}
__device__ __forceinline__ bool key_kill(unsigned long long k) { return ((k >> 47) & 1ull) != 0ull; }
__device__ __forceinline__ uint32_t key_time(unsigned long long k) {
  const uint32_t tk = (uint32_t)(k >> 48);
  return key_kill(k) ? tk : 0xFFFFu - tk;
}
// record states (b_state)
enum : int8_t { BS_PENDING = 0, BS_WON = 1 /* 1 + round */, BS_KILL_LOST = 8 /* 8 + round */,
                BS_CANCELLED = -1, BS_NO_CELL = -2 /* - round: found no cell in that round */ };
__device__ __forceinline__ uint32_t rec_time(const DevWorld& W, int64_t r) {
  return BI_TIME(W.b_inh[r * BI_WORDS + BI_FINAL]);
}
__device__ __forceinline__ uint32_t owner_time(const DevWorld& W, int o) {
  return o >= 0 ? rec_time(W, o) : (uint32_t)((-2 - o) >> 2);
}
// a round's winner with time t takes its cell unless the cell's owner from an
// earlier round is later in time (that owner overwrote it)
__device__ __forceinline__ bool takes_cell(const DevWorld& W, int owner, uint32_t t) {
  return owner == -1 || owner_time(W, owner) <= t;
}
// the last round a record claimed in (-1: none) -- its claims are cleared at
// activation (round k's at b_tgt[k])
__device__ __forceinline__ int last_claim_round(int st) {
  if (st == BS_PENDING) return 3;
  if (st >= BS_WON && st < BS_WON + 4) return st - BS_WON;
  if (st >= BS_KILL_LOST && st < BS_KILL_LOST + 4) return st - BS_KILL_LOST;
  if (st <= BS_NO_CELL) return BS_NO_CELL - st - 1;
  return -1;
}

// PositionOffspring for record r in round m (main/cPopulation.cc:5353-5413):
// an empty neighbour (not taken) when PREFER_EMPTY, else any of the eight
// neighbours or the parent (ALLOW_PARENT); BIRTH_METHOD 3 with no empty
// neighbour: the parent's cell without a draw (:5407), placed only if
// ALLOW_PARENT (ActivateOffspring :706-713), else never (BS_NO_CELL).  The
// key records whether the target is taken (a kill).  taken(c): the round's
// occupancy -- round 0 occ (tiles: the ghost rows' received occupancy), round
// m > 0 also every cell claimed in round m - 1 (tile_m >= 0: here or by the
// neighbour, tile_taken).  Returns false for no cell.
__device__ __forceinline__ bool tile_taken(const DevWorld& W, int64_t c, int m);
// BIRTH_METHOD 1: the cell's organism's age; 2: cOrganism::CalcMeritRatio
// (main/cOrganism.cc:703-708, age / merit, or the age without a positive
// merit); an empty cell (a newborn's to be) 0 (oracle position_value)
__device__ __forceinline__ double position_value(const DevWorld& W, int c) {
  if (c >= W.n || !(W.ctl[c] & CTL_ALIVE)) return 0.0;
  const double age = (double)W.age[c];
  if (W.birth_method == 1) return age;
  const double m = W.merit[c];
  return m > 0.0 ? __ddiv_rn(age, m) : age;
}
// BIRTH_METHOD 4 (POSITION_OFFSPRING_FULL_SOUP_RANDOM, main/cPopulation.cc:
// 5297-5310; oracle soup_target): with PREFER_EMPTY one draw among the cells
// empty at placement start that this round has not taken (e_list, compacted
// before every round by k_empty_*: FindRandEmptyCell, :5650-5668, draws
// uniformly among the empty cells), else -- a full world, or every empty cell
// claimed by earlier births -- GetUInt(size); without PREFER_EMPTY
// GetUInt(size), redrawn while it is the parent and ALLOW_PARENT is 0.
// Single worlds only (capi refuses strip tiles).
template <bool TILE>
__device__ __forceinline__ bool place_pick_one(const DevWorld& W, int64_t r, int m) {
  const int parent = W.b_parent[r];
  if (m == 0) finalize_key(W, r, parent);   // round 0: the record's first draws
  const unsigned long long* prev = m > 0 ? W.claim_r[m - 1] : nullptr;
  auto taken = [&](int c) -> bool {
    if (TILE) return tile_taken(W, c, m);
    return W.occ[c] != 0 || (prev && prev[c] != 0ull);
  };
  if (!TILE && W.birth_method == 4) {
    int32_t* const inh = W.b_inh + (int64_t)r * BI_WORDS;
    const uint32_t lo = (uint32_t)inh[BI_RLO], hi = (uint32_t)inh[BI_RHI];
    uint32_t ctr = (uint32_t)inh[BI_RCTR];
    const uint32_t n = (uint32_t)W.n;
    int t = -1;
    if (W.prefer_empty) {
      const uint32_t ne = (uint32_t)W.e_blk[(W.n + 255) / 256];
      t = ne > 0u ? W.e_list[rng_below(lo, hi, ctr, ne)] : (int)rng_below(lo, hi, ctr, n);
    } else {
      t = (int)rng_below(lo, hi, ctr, n);
      while (!W.allow_parent && n > 1u && t == parent) t = (int)rng_below(lo, hi, ctr, n);
    }
    if (t == parent && !W.allow_parent) {              // ActivateOffspring drops it (:706-713)
      inh[BI_RCTR] = (int32_t)ctr;
      W.b_target[r] = -1;
      W.b_state[r] = (int8_t)(BS_NO_CELL - m);
      return false;
    }
    const unsigned long long key = claim_key(BI_TIME(inh[BI_FINAL]), taken(t), rng_next(lo, hi, ctr),
                                             W.cell0 + parent, W.b_seq[r]);
    inh[BI_RCTR] = (int32_t)ctr;
    W.b_target[r] = t;
    W.b_prio[r] = key;
    W.b_tgt[(int64_t)m * W.rcap + r] = t;
    return true;
  }
  int nbr[8];
  const int nn = neighbours(W, parent, nbr);
  int cand[9];
  int nc = 0;
  if (W.prefer_empty)
    for (int k = 0; k < nn; k++)
      if (!taken(nbr[k])) cand[nc++] = nbr[k];
  if (nc == 0 && (W.birth_method == 1 || W.birth_method == 2)) {
    // PositionAge / PositionMerit (main/cPopulation.cc:5416-5470): the parent
    // first, valued -1 without ALLOW_PARENT; a neighbour of a larger value
    // replaces the list, one of an equal value joins it (oracle place_pick)
    double best = W.allow_parent ? position_value(W, parent) : -1.0;
    cand[nc++] = parent;
    for (int k = 0; k < nn; k++) {
      const double v = position_value(W, nbr[k]);
      if (v > best) { best = v; nc = 0; cand[nc++] = nbr[k]; }
      else if (v == best) cand[nc++] = nbr[k];
    }
  } else if (nc == 0 && W.birth_method != 3) {
    for (int k = 0; k < nn; k++) cand[nc++] = nbr[k];
    if (W.allow_parent) cand[nc++] = parent;
  }
  if (nc == 0 && !W.allow_parent) {
    W.b_target[r] = -1;
    W.b_state[r] = (int8_t)(BS_NO_CELL - m);
    return false;
  }
  int32_t* const inh = W.b_inh + (int64_t)r * BI_WORDS;
  const uint32_t lo = (uint32_t)inh[BI_RLO], hi = (uint32_t)inh[BI_RHI];
  uint32_t ctr = (uint32_t)inh[BI_RCTR];
  const int t = nc > 0 ? cand[rng_below(lo, hi, ctr, (uint32_t)nc)] : parent;
  const unsigned long long key = claim_key(BI_TIME(inh[BI_FINAL]), taken(t), rng_next(lo, hi, ctr),
                                           W.cell0 + parent, W.b_seq[r]);
  inh[BI_RCTR] = (int32_t)ctr;
  W.b_target[r] = t;
  W.b_prio[r] = key;
  W.b_tgt[(int64_t)m * W.rcap + r] = t;
  return true;
}

// grid-stride over the birth queue (its length is only known on the device)
#define QUEUE_LOOP(i) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, _qn = queue_len(W); i < _qn; \
       i += (int64_t)gridDim.x * blockDim.x)
// BIRTH_METHOD 4 + PREFER_EMPTY: round m's candidates, ascending -- the cells
// empty at placement start (after the slices' deaths) and, for m > 0, not
// claimed in round m - 1 (FindRandEmptyCell's; oracle place_reset /
// soup_round_cells): per-256-cell counts, one block's exclusive scan over them
// (e_blk[nb]: the total), the scatter.  (Before round m's launch, occ holds
// the winners up to round m - 2; round m - 1's are in its claims.)
__device__ __forceinline__ bool soup_free(const DevWorld& W, int64_t c, int m) {
  return c < W.n && W.occ[c] == 0 && (m == 0 || W.claim_r[m - 1][c] == 0ull);
}
__global__ __launch_bounds__(256) void k_empty_count(DevWorld W, int m) {
  __shared__ int ws[4];
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool e = soup_free(W, c, m);
  const int cnt = __popcll(__ballot(e));
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) W.e_blk[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
__global__ __launch_bounds__(1024) void k_empty_scan(DevWorld W, int nb) {
  __shared__ int part[1024];
  const int per = (nb + 1023) / 1024;
  const int b0 = (int)threadIdx.x * per, b1 = min(nb, b0 + per);
  int sum = 0;
  for (int b = b0; b < b1; b++) sum += W.e_blk[b];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {          // inclusive scan of the runs' sums
    const int v = (int)threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = threadIdx.x > 0 ? part[threadIdx.x - 1] : 0;
  for (int b = b0; b < b1; b++) {
    const int v = W.e_blk[b];
    W.e_blk[b] = run;
    run += v;
  }
  if (threadIdx.x == 1023) W.e_blk[nb] = part[1023];
}
__global__ __launch_bounds__(256) void k_empty_scatter(DevWorld W, int m) {
  __shared__ int ws[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool e = soup_free(W, c, m);
  const unsigned long long bm = __ballot(e);
  if (lane == 0) ws[wv] = __popcll(bm);
  __syncthreads();
  int base = W.e_blk[blockIdx.x];
  for (int k = 0; k < wv; k++) base += ws[k];
  if (e) W.e_list[base + __popcll(bm & ((1ull << lane) - 1ull))] = (int)c;
}

// The divide mutations (k_place_pick_mut, k_tile_prep), by 256-thread blocks:
// block b of nb scans MUT_PER_BLOCK queue entries at a time -- lane k of each
// wave loads one entry's five edit words and both lengths -- and lists the
// ~10 % that have edits in LDS; the block's four waves then apply the list
// round robin, each genome from the words in hand (apply_edits_core).  A
// wave that applied its own 8 entries' edits ran up to ~5 genomes one after
// the other (the launch's longest wave, 36 us: profiles/r04f_split_*); the
// block's pool of 32 caps a wave at ~2.  (One entry per wave over 65536
// waves instead: 71 us for the fused launch, profiles/r04g_*.)
#define MUT_PER_WAVE 8
#define MUT_PER_BLOCK (4 * MUT_PER_WAVE)
__device__ __forceinline__ void mutation_block(const DevWorld& W, int64_t blk, int64_t nblk,
                                               uint8_t (*child)[TAPE_SLOT + 16]) {
  __shared__ int ml[MUT_PER_BLOCK][8];   // record (2 words), e0..e4, len0 | len << 16
  __shared__ int mn;
  const int nb = queue_len(W);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t q0 = blk * MUT_PER_BLOCK; q0 < nb; q0 += nblk * MUT_PER_BLOCK) {   // block-uniform
    if (threadIdx.x == 0) mn = 0;
    __syncthreads();
    const int64_t q = q0 + wv * MUT_PER_WAVE + lane;
    if (lane < MUT_PER_WAVE && q < nb) {
      const int64_t r = rec_of(W, q);
      int e[5];
#pragma unroll
      for (int k = 0; k < 5; k++) e[k] = W.b_edit[(int64_t)k * W.rcap + r];
      const int l0 = W.b_len0[r], l1 = W.b_len[r];
      int x = e[0] | e[1] | e[2] | e[3] | e[4];
      if (W.seg_any)
        for (int k = 0; k < NSEG; k++) x |= W.b_pcnt[(int64_t)k * W.rcap + r];
      if (x) {
        const int i = atomicAdd(&mn, 1);
        ml[i][0] = (int)(uint32_t)r; ml[i][1] = (int)(r >> 32);
#pragma unroll
        for (int k = 0; k < 5; k++) ml[i][2 + k] = e[k];
        ml[i][7] = l0 | (l1 << 16);
      }
    }
    __syncthreads();
    const int n = mn;
    for (int i = wv; i < n; i += 4) {
      const int64_t r = (int64_t)(uint32_t)ml[i][0] | ((int64_t)ml[i][1] << 32);
      const int e[5] = {ml[i][2], ml[i][3], ml[i][4], ml[i][5], ml[i][6]};
      apply_edits_core(W, r, e, ml[i][7] & 0xFFFF, ml[i][7] >> 16, child[wv]);
    }
    __syncthreads();
  }
}

// A single world's placement launch m = 1..3: round m - 1 resolved and round m
// picked (oracle run_update_impl).  Each round has its own claim array, so
// round m - 1's claims stay intact for the whole launch: a record whose key is
// the maximum won -- it occupies its cell and owns it unless the cell's owner
// from an earlier round is later in time; a lost kill claim was placed and
// overwritten by the later winner; a lost empty claim picks again, treating
// every cell claimed in round m - 1 as taken (each has a winner).
__global__ void k_place_round(DevWorld W, int m) {
  const unsigned long long* prev = W.claim_r[m - 1];
  unsigned long long* cur = W.claim_r[m];
  QUEUE_LOOP(q) {
    const int64_t r = rec_of(W, q);
    if (W.b_state[r] != BS_PENDING) continue;
    const int t = W.b_target[r];
    const unsigned long long key = W.b_prio[r];
    if (prev[t] == key) {                      // won round m-1
      W.b_state[r] = (int8_t)(BS_WON + m - 1);
      W.occ[t] = 1;
      if (takes_cell(W, W.owner[t], rec_time(W, r))) W.owner[t] = (int)r;
      continue;
    }
    if (key_kill(key)) { W.b_state[r] = (int8_t)(BS_KILL_LOST + m - 1); continue; }
    if (place_pick_one<false>(W, r, m)) atomicMax(&cur[W.b_target[r]], W.b_prio[r]);
  }
}
// Launch 0b of a single world: a record whose parent's cell was killed before
// its own birth time (a round-0 pick of an earlier birth landed there:
// killt[parent] > 2^16 - t) is cancelled -- the reference would have killed
// its parent before this divide; the others claim their round-0 targets.
__global__ void k_place_claim0(DevWorld W, long long* pred_out, long long pred_seq) {
  // the list rows are free after the main pass: the newborn pass's (k_activate)
  if (blockIdx.x == 0 && threadIdx.x < NUM_LISTS) W.class_count[threadIdx.x] = 0;
  // the update's last step: its predictor and organisms to the host (mapped
  // memory), which chooses the next update's steps from them
  if (pred_out && blockIdx.x == 0 && threadIdx.x == 0) {
    pred_out[0] = pacc_sum(W, 0);
    pred_out[1] = (long long)W.totals[1];
    pred_out[2] = densest_quarter(W);
    // then its sequence number, after them at system scope: the host polls it
    __threadfence_system();
    __hip_atomic_store(pred_out + 3, pred_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  QUEUE_LOOP(q) {
    const int64_t r = rec_of(W, q);
    if (W.b_state[r] != BS_PENDING) continue;
    const int p = W.b_parent[r];
    if (W.killt[p] > 0x10000u - rec_time(W, r)) { W.b_state[r] = BS_CANCELLED; continue; }
    atomicMax(&W.claim_r[0][W.b_target[r]], W.b_prio[r]);
  }
}
// Launch 0 of a single world's placement with the divide mutations beside it:
// blocks [0, pblocks) pick round 0 (a pick whose target is occupied is a kill:
// the cell's kill time, atomicMax of 2^16 - t); the next fblocks finalize the
// deferred divides' phenotype; the rest apply the edits (a wave per 8 queue
// entries, rewriting the ~10 % of genomes that have edits one after the
// other; 4 waves per block) -- placement reads no genome, so they are
// independent and share one launch instead of several latency-bound ones.
// (boff / nblocks: the launch's first logical block and the logical grid, for
// the AVGPU_SPLIT_PICK_MUT diagnostic build that times the three parts apart)
__global__ __launch_bounds__(256) void k_place_pick_mut(DevWorld W, int pblocks, int fblocks, int boff, int nblocks) {
  __shared__ uint8_t child[4][TAPE_SLOT + 16];
  const int nb = queue_len(W);
  const int bid = (int)blockIdx.x + boff;
  if (bid < pblocks) {
    for (int64_t i = (int64_t)bid * 256 + threadIdx.x; i < nb; i += (int64_t)pblocks * 256) {
      const int64_t r = rec_of(W, i);
      if (!place_pick_one<false>(W, r, 0)) continue;
      const unsigned long long key = W.b_prio[r];
      if (key_kill(key)) atomicMax(&W.killt[W.b_target[r]], 0x10000u - key_time(key));
    }
    return;
  }
  if (bid < pblocks + fblocks) {               // deferred divides' phenotype half
    for (int64_t i = (int64_t)(bid - pblocks) * 256 + threadIdx.x; i < nb; i += (int64_t)fblocks * 256)
      finalize_phenotype(W, rec_of(W, i));
    return;
  }
  pblocks += fblocks;
  mutation_block(W, bid - pblocks, nblocks - pblocks, child);
}


// ---- strip tiles' placement: one launch per round (DESIGN.md "Multi-GPU") ----
// k_tile_prep, after interpretation: blocks [0, mblocks) apply the divide
// mutations (as k_place_pick_mut's extra blocks); the rest walk the 2 x X
// halo cells: the ghost rows empty (occ, owner, every round's claims), the
// edge rows' occupancy into the send buffers and both parities' claim slots
// zeroed; fblocks more run the deferred divides' phenotype half
// (finalize_phenotype).  (k_allot initialised the tile's own cells.)
__global__ __launch_bounds__(256) void k_tile_prep(DevWorld W, int mblocks, int fblocks) {
  __shared__ uint8_t child[4][TAPE_SLOT + 16];
  if ((int)blockIdx.x >= mblocks && (int)blockIdx.x < mblocks + fblocks) {
    const int nb = queue_len(W);
    for (int64_t i = (int64_t)(blockIdx.x - mblocks) * 256 + threadIdx.x; i < nb; i += (int64_t)fblocks * 256)
      finalize_phenotype(W, rec_of(W, i));
    return;
  }
  if ((int)blockIdx.x < mblocks) {
    mutation_block(W, blockIdx.x, mblocks, child);
    return;
  }
  const int X = W.world_x;
  const int g = (blockIdx.x - mblocks - fblocks) * blockDim.x + threadIdx.x;
  if (g >= 2 * X) return;
  const int d = g / X, x = g - d * X;
  const int64_t gc = ghost_cell(W, d, x);
  W.occ[gc] = 0;
  W.owner[gc] = -1;
#pragma unroll
  for (int k = 0; k < 4; k++) W.claim_r[k][gc] = 0ull;
  uint8_t* b = W.h_send[d];
  halo_occ(b, X)[x] = W.occ[edge_cell(W, d, x)];
#pragma unroll
  for (int k = 0; k < 4; k++) halo_cl(b, X, k >> 1, k & 1)[x] = 0ull;
  halo_kt(b, X)[x] = 0u;
}

// Launch m of a tile's placement (oracle orc_tile_place / tile_launch), after
// the previous exchange: blocks [0, rblocks) take the records, the rest walk
// the 2 x X halo cells.
// m = 0: round 0's picks with their kill times (own cells: killt; ghost
//   cells: the halo's kill-time slots, read by the neighbour's launch 0b);
//   the halo cells import the ghost rows' occupancy.
// m = 1..3: round m - 1 resolved against the merged claims -- a halo cell
//   whose maximum came from the neighbour (an edge cell: its claims on my edge
//   row; a ghost cell: its own claims on its edge row) is that round's remote
//   winner's (owner REMOTE_OWNER(m - 1, t), by the time rule) and occupied;
//   a claimed ghost cell is occupied; a record that won takes its cell by the
//   time rule, a lost kill claim was placed and overwritten, a lost empty
//   claim picks round m (tile_taken: the occupancy that resolve leaves) --
//   and the send parity of round m + 1 is cleared (its last contents, round
//   m - 1's, went out before this launch).
// m = 4: the last resolve only, and the record buffers' headers cleared for
//   k_halo_pack.
__global__ __launch_bounds__(256) void k_tile_round(DevWorld W, int m, int rblocks) {
  const int X = W.world_x;
  if ((int)blockIdx.x < rblocks) {
    const int nb = queue_len(W);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nb; q += (int64_t)rblocks * blockDim.x) {
      const int64_t r = rec_of(W, q);
      if (W.b_state[r] != BS_PENDING) continue;
      if (m == 0) {
        if (!place_pick_one<true>(W, r, 0)) continue;
        const unsigned long long key = W.b_prio[r];
        if (!key_kill(key)) continue;
        const int t = W.b_target[r];
        const uint32_t kv = 0x10000u - key_time(key);
        if (t >= W.n) {
          const int64_t k = t - W.n;
          const int d = (int)(k / X), x = (int)(k - (int64_t)d * X);
          atomicMax(&halo_kt(W.h_send[d], X)[x], kv);
        } else {
          atomicMax(&W.killt[t], kv);
        }
        continue;
      }
      const int t = W.b_target[r];
      const unsigned long long key = W.b_prio[r];
      if (tile_merged(W, t, m - 1) == key) {   // won round m - 1
        W.b_state[r] = (int8_t)(BS_WON + m - 1);
        W.occ[t] = 1;
        if (takes_cell(W, W.owner[t], rec_time(W, r))) W.owner[t] = (int)r;
        continue;
      }
      if (key_kill(key)) { W.b_state[r] = (int8_t)(BS_KILL_LOST + m - 1); continue; }
      if (m < 4 && place_pick_one<true>(W, r, m)) {
        const int nt = W.b_target[r];
        const unsigned long long nk = W.b_prio[r];
        atomicMax(&W.claim_r[m][nt], nk);
        int d, x;
        bool ghost;
        if (halo_slot(W, nt, d, x, ghost)) atomicMax(&halo_cl(W.h_send[d], X, m & 1, ghost ? 0 : 1)[x], nk);
      }
    }
    return;
  }
  const int g = (blockIdx.x - rblocks) * blockDim.x + threadIdx.x;
  if (m == 4 && g < 2) {
    HaloHdr* hdr = reinterpret_cast<HaloHdr*>(W.r_send[g]);
    hdr->count = 0;
    hdr->arena_used = 0;
    hdr->overflow = 0;
  }
  if (g >= 2 * X) return;
  const int d = g / X, x = g - d * X;
  const int64_t gc = ghost_cell(W, d, x);
  if (m == 0) {
    W.occ[gc] = halo_occ(W.h_recv[d], X)[x];
    return;
  }
  const int p = (m - 1) & 1;
  const int64_t c = edge_cell(W, d, x);
  const unsigned long long rc = halo_cl(W.h_recv[d], X, p, 0)[x], rg = halo_cl(W.h_recv[d], X, p, 1)[x];
  const unsigned long long lg = W.claim_r[m - 1][gc];
  if (rc != 0ull && rc > W.claim_r[m - 1][c]) {
    const uint32_t tr = key_time(rc);
    if (takes_cell(W, W.owner[c], tr)) W.owner[c] = REMOTE_OWNER(m - 1, tr);
    W.occ[c] = 1;
  }
  if (rg != 0ull && rg > lg) {
    const uint32_t tr = key_time(rg);
    if (takes_cell(W, W.owner[gc], tr)) W.owner[gc] = REMOTE_OWNER(m - 1, tr);
  }
  if (lg != 0ull || rg != 0ull) W.occ[gc] = 1;
  if (m == 1 || m == 2) {                      // round m + 1's send parity = round m - 1's
    uint8_t* b = W.h_send[d];
    halo_cl(b, X, p, 0)[x] = 0ull;
    halo_cl(b, X, p, 1)[x] = 0ull;
  }
}
// Launch 0b of a tile (after the kill times' exchange): a record whose
// parent's cell was killed earlier -- by a pick here or, on an edge row, by
// the neighbour's (the halo's kill-time slot) -- is cancelled; the others
// claim their round-0 targets (and the halo send slots of parity 0).
__global__ __launch_bounds__(256) void k_tile_claim0(DevWorld W) {
  const int X = W.world_x;
  if (blockIdx.x == 0 && threadIdx.x < NUM_LISTS) W.class_count[threadIdx.x] = 0;
  QUEUE_LOOP(q) {
    const int64_t r = rec_of(W, q);
    if (W.b_state[r] != BS_PENDING) continue;
    const int p = W.b_parent[r];
    uint32_t kt = W.killt[p];
    int d, x;
    bool ghost;
    if (halo_slot(W, p, d, x, ghost)) kt = max(kt, halo_kt(W.h_recv[d], X)[x]);
    if (kt > 0x10000u - rec_time(W, r)) { W.b_state[r] = BS_CANCELLED; continue; }
    const int t = W.b_target[r];
    const unsigned long long key = W.b_prio[r];
    atomicMax(&W.claim_r[0][t], key);
    if (halo_slot(W, t, d, x, ghost)) atomicMax(&halo_cl(W.h_send[d], X, 0, ghost ? 0 : 1)[x], key);
  }
}

// ---- the batch step's newborns (oracle newborn_pass) ----
// An activated offspring first gives back (1 - t) of what its cell's replaced
// organism consumed in the step's main pass, then runs its own share of the
// step's remaining picks: Binomial(round(UD_s (1 - t)), merit / total) from a
// stateless draw of its global cell, in the newborn pass (interp.hip NB).
// The picks beyond what the replaced organism had left ((1 - t) of the
// instructions it ran) are the step's carry, taken from the next allotment.
__device__ __forceinline__ double nb_frac(uint32_t t) { return __dmul_rn((double)(0x10000u - t), 1.0 / 65536.0); }
__device__ __forceinline__ long long newborn_budget(const DevWorld& W, int64_t c, uint32_t t, double merit,
                                                    uint32_t key, long long uds, double total) {
  if (!(total > 0.0) || uds <= 0) return 0;
  const long long n = (long long)floor(__dadd_rn(__dmul_rn((double)uds, nb_frac(t)), 0.5));
  const double p = __ddiv_rn(sched_weight(merit, 0u), total);   // (oracle: sched_weight, no head start)
  const long long b = binom_draw(n, p, node_draw(W.seed_lo, W.seed_hi, key, SALT_NEWBORN, (uint64_t)(W.cell0 + c)));
  return min(b, (long long)(BUDGET_PRIM - 1));
}
__device__ __forceinline__ void newborn_credit(const DevWorld& W, int64_t c, uint32_t t) {
  const double f = nb_frac(t);
  for (int r = 0; r < W.n_res; r++) {
    const double v = W.cons[(int64_t)r * W.n + c];
    if (v == 0.0) continue;
    const double back = __dmul_rn(v, f);
    const ResParam& q = W.res_param[r];
    if (q.geometry != AVGPU_RES_GLOBAL) {
      double* p = W.res_amount + (int64_t)q.slot * W.n + c;
      *p = __dadd_rn(*p, back);
    } else {
      atomicAdd(W.res_cons + r, 0ull - (unsigned long long)__dmul_rn(back, RES_FIX));
    }
  }
}
// one newborn in cell c: credit, budget, carry; returns its list row (-1: no slice)
// (ran: W.ran[c], loaded by the caller ahead of the offspring's stores -- a
// load behind them would wait for all of them)
__device__ __forceinline__ int newborn_setup(const DevWorld& W, int64_t c, uint32_t t, double merit, int len,
                                             uint32_t key, long long uds, double total, long long& carry,
                                             unsigned long long& wasted, int ran) {
  if (W.env_resources) newborn_credit(W, c, t);
  const long long left = (long long)__dmul_rn((double)ran, nb_frac(t));
  const long long bud = newborn_budget(W, c, t, merit, key, uds, total);
  carry += bud - left;
  wasted += (unsigned long long)left;
  W.budget[c] = (int32_t)bud;
  return bud > 0 ? class_of(::need_of(len, CTL_ALIVE, W.size_range)) : -1;
}
// the wave's newborns into the newborn pass's lists (row 0: class 0, rows
// 1..3 the list classes), one atomic per row and wave
__device__ __forceinline__ void newborn_enqueue(const DevWorld& W, int cell, int row) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < NUM_CLASSES; k++) {
    const unsigned long long m = __ballot(row == k);
    if (!m) continue;
    int base = 0;
    if (lane == 0) base = atomicAdd(&W.class_count[k], (int)__popcll(m));
    base = __shfl(base, 0);
    if (row == k) W.class_list[(int64_t)k * W.n + base + (int)__popcll(m & ((1ull << lane) - 1ull))] = cell;
  }
}

// One lane per queued birth: the owners of cells inside this world are
// activated (ActivateOrganism + SetupOffspring; owners of ghost-row cells were
// shipped by k_halo_pack), with the head start 2^16 - t for their first
// allotment.  The record's fields are loaded before the ownership test
// (independent loads in flight together instead of a chain behind it).
// fused 1 (single world): round 3 is resolved here -- a round-3 winner owns
// its cell unless the owner from an earlier round is later in time; an
// earlier round's owner keeps it unless a round-3 winner (necessarily a
// kill claim: the cell was taken) is not earlier than it.  fused 2 (strip
// tiles): the owners are final (k_tile_round resolved round 3).  Either way
// each record clears the claims it made (round 3's, which this launch reads,
// are cleared by k_allot).  A record that does not own its cell was placed
// and overwritten (CNT_OVERWRITTEN), unless it was cancelled
// (CNT_CANCELLED: its parent died first) or found no cell (CNT_DROPPED).
#ifndef ACT_PRE
#define ACT_PRE 8    // 16-B quads of the offspring's genome k_activate loads ahead
#endif
__global__ __launch_bounds__(64) void k_activate(DevWorld W, int fused, uint32_t key, int sub, int nsub) {
  const int nb = queue_len(W);
  const int64_t ncell = W.n + (W.tiled ? 2 * (int64_t)W.world_x : 0);
  const int lane = threadIdx.x & 63;
  const double total = W.totals[2];
  const long long uds = sub_share((long long)W.totals[3], sub, nsub);
  unsigned long long born = 0, over = 0, canc = 0, nocell = 0, bad = 0, wasted = 0, nbs = 0;
  long long carry = 0;
  for (int64_t q0 = (int64_t)blockIdx.x * 64; q0 < nb; q0 += (int64_t)gridDim.x * 64) {
    const int64_t q = q0 + lane;
    int nrow = -1, ncell_nb = 0;
    do {
      if (q >= nb) break;
      const int64_t i = rec_of(W, q);
      // the genome's first 128 B, loaded before the claims decide whether the
      // record won (a dependent round trip less for the ~95 % that do; the
      // whole class-0 genome, 20 quads, measured no faster)
      const uint4* g4 = reinterpret_cast<const uint4*>(W.b_genome + i * TAPE_SLOT);
      uint4 pre[ACT_PRE];
#pragma unroll
      for (int u = 0; u < ACT_PRE; u++) pre[u] = g4[u];
      const int tgt = W.b_target[i];
      const int8_t st = W.b_state[i];
      Child b = child_of_record(W, i);
      // the replaced organism's instructions, loaded with the claim words
      const int ran = (tgt >= 0 && (int64_t)tgt < W.n) ? W.ran[tgt] : 0;
      const int lastr = last_claim_round(st);
      // the record's claims, round k's at b_tgt[k] (the last one its target);
      // a target out of range is a corrupt record: counted, never written
      bool ok = true;
      for (int k = 0; k <= lastr && k < 3; k++) {
        const int tk = (k == lastr && tgt >= 0) ? tgt : W.b_tgt[(int64_t)k * W.rcap + i];
        if (tk >= 0 && (int64_t)tk < ncell) W.claim_r[k][tk] = 0ull;
        else ok = false;
      }
      if (st == BS_CANCELLED) { canc++; break; }
      if (st <= BS_NO_CELL) { nocell++; break; }
      if (!ok || tgt < 0 || (int64_t)tgt >= ncell) { bad++; break; }
      const uint32_t t = 0x10000u - b.hs;
      bool won = false;
      if (fused == 2) {
        won = st >= BS_WON && st < BS_WON + 4 && W.owner[tgt] == (int)i;
      } else if (st == BS_PENDING) {
        won = W.claim_r[3][tgt] == W.b_prio[i] && takes_cell(W, W.owner[tgt], t);
      } else if (st >= BS_WON && st < BS_WON + 4) {
        const unsigned long long c3 = W.claim_r[3][tgt];
        won = W.owner[tgt] == (int)i && !(c3 != 0ull && key_time(c3) >= t);
      }
      if (!won) { over++; break; }
      if (b.len < 0 || b.len > AVGPU_MAX_GENOME) { bad++; break; }   // (k_halo_pack skips it too)
      if (tgt >= W.n) break;                   // sent to the neighbouring tile
      born++;
      b.hs = 0;                                // it runs its share of this step instead (newborn pass)
      setup_child_lane<ACT_PRE>(W, tgt, b, W.b_genome + i * TAPE_SLOT, pre);
      nrow = newborn_setup(W, tgt, t, b.merit, b.len, key, uds, total, carry, wasted, ran);
      ncell_nb = tgt;
    } while (0);
    nbs += nrow >= 0 ? 1ull : 0ull;
    newborn_enqueue(W, ncell_nb, nrow);
  }
  for (int off = 32; off > 0; off >>= 1) {
    born += __shfl_xor(born, off);
    over += __shfl_xor(over, off);
    canc += __shfl_xor(canc, off);
    nocell += __shfl_xor(nocell, off);
    bad += __shfl_xor(bad, off);
    wasted += __shfl_xor(wasted, off);
    nbs += __shfl_xor(nbs, off);
    carry += __shfl_xor(carry, off);
  }
  if (threadIdx.x == 0) {
    if (born) count_add(W, CNT_BIRTHS, born);
    if (over) count_add(W, CNT_OVERWRITTEN, over);
    if (canc) count_add(W, CNT_CANCELLED, canc);
    if (nocell) count_add(W, CNT_DROPPED, nocell);
    if (bad) count_add(W, CNT_BAD_RECORD, bad);
    if (wasted) count_add(W, CNT_WASTED, wasted);
    if (nbs) count_add(W, CNT_SLICES, nbs);
    if (carry) atomicAdd(reinterpret_cast<unsigned long long*>(W.sched + 1), (unsigned long long)carry);
  }
}

// Winners of ghost-row cells -> record buffer of that direction (one wave per
// queued birth; one record per ghost cell at most: its last winner here).
// The lanes of a wave test 64 queued births at once; the wave then packs the
// few that won a ghost cell one after the other (a wave per queued birth
// spent ~40 us per update on the test alone).
__global__ __launch_bounds__(64) void k_halo_pack(DevWorld W) {
  const int nb = queue_len(W);
  const int lane = threadIdx.x;
  const int X = W.world_x;
  unsigned long long sent = 0, lost = 0;
  for (int64_t q0 = (int64_t)blockIdx.x * 64; q0 < nb; q0 += (int64_t)gridDim.x * 64) {
    const int64_t q = q0 + lane;
    int64_t mine = -1;
    if (q < nb) {
      const int64_t i = rec_of(W, q);
      const int tgt = W.b_target[i];
      const int8_t st = W.b_state[i];
      // (a target past the ghost rows or a length out of range is a corrupt
      // record: counted in k_activate, which sees the same fields, never sent)
      if (st >= BS_WON && st < BS_WON + 4 && tgt >= W.n && (int64_t)tgt < W.n + 2 * (int64_t)X &&
          W.b_len[i] >= 0 && W.b_len[i] <= AVGPU_MAX_GENOME && W.owner[tgt] == (int)i)
        mine = i;
    }
    for (unsigned long long m = __ballot(mine >= 0); m; m &= m - 1ull) {
    const int64_t i = (int64_t)__shfl((long long)mine, __ffsll((long long)m) - 1);
    const int tgt = W.b_target[i];
    const int d = (tgt - (int)W.n) / X, col = (tgt - (int)W.n) - d * X;
    const int len = W.b_len[i];
    HaloHdr* hdr = reinterpret_cast<HaloHdr*>(W.r_send[d]);
    HaloRec* recs = reinterpret_cast<HaloRec*>(W.r_send[d] + sizeof(HaloHdr));
    uint8_t* arena = W.r_send[d] + sizeof(HaloHdr) + (int64_t)X * sizeof(HaloRec);
    int slot = 0, off = 0;
    if (lane == 0) {
      slot = atomicAdd(&hdr->count, 1);
      off = atomicAdd(&hdr->arena_used, (len + 3) & ~3);
    }
    slot = __shfl(slot, 0);
    off = __shfl(off, 0);
    const bool fits = (int64_t)off + len <= W.r_arena;
    if (lane == 0) {
      HaloRec r;
      r.col = col; r.round = W.b_state[i] - BS_WON; r.len = fits ? len : -1;
      const Child b = child_of_record(W, i);
      r.gen = b.gen; r.ccopied = b.ccopied; r.exec = b.exec; r.gest = b.gest;
      r.rng_lo = b.lo; r.rng_hi = b.hi; r.rng_ctr = b.ctr;
      r.off = off; r.t = 0x10000u - b.hs; r.merit = b.merit; r.fitness = b.fitness;
#pragma unroll
      for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) r.last_task[t] = b.ltask[t];
      r.pad2[0] = r.pad2[1] = r.pad2[2] = 0;
      recs[slot] = r;
      if (!fits) atomicAdd(&hdr->overflow, 1);
    }
    if (fits) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(W.b_genome + i * TAPE_SLOT);
      uint32_t* dst = reinterpret_cast<uint32_t*>(arena + off);
      for (int w = lane; w < (len + 3) / 4; w += 64) dst[w] = src[w];
      sent++;
    } else {
      lost++;
    }
    }
  }
  if (lane == 0) {
    if (sent) count_add(W, CNT_HALO_SENT, sent);
    if (lost) { count_add(W, CNT_HALO_LOST, lost); count_add(W, CNT_DROPPED, lost); }
  }
}

// Records received from direction d: the offspring owns its target cell when
// it was that cell's last winner (owner == REMOTE_OWNER(its round)).
__global__ __launch_bounds__(64) void k_activate_remote(DevWorld W, uint32_t key, int sub, int nsub) {
  const int lane = threadIdx.x;
  const double total = W.totals[2];
  const long long uds = sub_share((long long)W.totals[3], sub, nsub);
  long long carry = 0;
  unsigned long long wasted = 0, nbs = 0;
  const int X = W.world_x;
  // blocks [0, G/2) take the records from above, the rest those from below
  const int half = gridDim.x >> 1;
  const int d = (int)blockIdx.x >= half ? 1 : 0;
  const int b0 = (int)blockIdx.x - d * half;
  const HaloHdr* hdr = reinterpret_cast<const HaloHdr*>(W.r_recv[d]);
  const HaloRec* recs = reinterpret_cast<const HaloRec*>(W.r_recv[d] + sizeof(HaloHdr));
  const uint8_t* arena = W.r_recv[d] + sizeof(HaloHdr) + (int64_t)X * sizeof(HaloRec);
  const int nrec = min(hdr->count, X);
  unsigned long long born = 0, lost = 0;
  for (int q = b0; q < nrec; q += half) {
    const HaloRec r = recs[q];
    if (r.len < 0) continue;                  // lost at the sender (counted there)
    // fields used as indices / lengths are checked: a record the exchange
    // delivered damaged is counted (CNT_BAD_RECORD), never followed
    if (r.col < 0 || r.col >= X || r.len > AVGPU_MAX_GENOME || r.off < 0 || (r.off & 3) ||
        (int64_t)r.off + r.len > W.r_arena || r.round < 0 || r.round > 3) {
      if (lane == 0) count_add(W, CNT_BAD_RECORD, 1ull);
      continue;
    }
    const int64_t c = edge_cell(W, d, r.col);
    if (W.owner[c] != REMOTE_OWNER(r.round, r.t)) { lost++; continue; }   // overwritten by a later winner
    born++;
    Child b;
    b.len = r.len; b.gen = r.gen; b.ccopied = r.ccopied; b.exec = r.exec; b.gest = r.gest;
    b.hs = 0;                                  // it runs its share of this step (newborn pass)
    b.merit = r.merit; b.fitness = r.fitness; b.lo = r.rng_lo; b.hi = r.rng_hi; b.ctr = r.rng_ctr;
    b.ltask = recs[q].last_task; b.lstride = 1;
    const int ran = W.ran[c];
    setup_child<64>(W, c, b, reinterpret_cast<const uint32_t*>(arena + r.off), lane);
    if (lane == 0) {
      const int row = newborn_setup(W, c, r.t, r.merit, r.len, key, uds, total, carry, wasted, ran);
      if (row >= 0) {
        nbs++;
        const int slot = atomicAdd(&W.class_count[row], 1);
        W.class_list[(int64_t)row * W.n + slot] = (int)c;
      }
    }
  }
  if (lane == 0) {
    if (born) count_add(W, CNT_BIRTHS, born);
    if (lost) count_add(W, CNT_OVERWRITTEN, lost);
    if (wasted) count_add(W, CNT_WASTED, wasted);
    if (nbs) count_add(W, CNT_SLICES, nbs);
    if (carry) atomicAdd(reinterpret_cast<unsigned long long*>(W.sched + 1), (unsigned long long)carry);
  }
}

// ---- statistics: per-block partials, then one block ----
// partial slots: 0 orgs 1 merit 2 fitness 3 gestation 4 genome length 5 max fitness
// 6 generation 7 memory size 8..16 task organisms
#define NPART 24
#define NUSED (8 + AVGPU_NUM_LOGIC_TASKS)
#define NSTAT 45
__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}
// part layout [NPART][nb] so that k_stats_final reads it coalesced
__device__ __forceinline__ int wave_sum_i(int v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
// Integer-valued slots (organisms, gestation, genome length, generation,
// memory, task organisms) reduce as integers: their double sums are exact in
// any order, so the partials are the same numbers at a third of the shuffle
// work; the nine task flags go as one u64 of 7-bit lanes (<= 64 per wave).
__global__ __launch_bounds__(256) void k_stats_partial(DevWorld W, double* part) {
  __shared__ double s[4][NPART];
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double merit = 0.0, fit = 0.0;
  int iv[5] = {0, 0, 0, 0, 0};                 // slots 0 3 4 6 7
  unsigned long long tasks = 0;
  if (c < W.n && (W.ctl[c] & CTL_ALIVE)) {
    merit = W.merit[c];
    fit = W.fitness[c];
    iv[0] = 1;
    iv[1] = W.gest_time[c];
    iv[2] = W.birth_len[c];
    iv[3] = W.generation[c];
    iv[4] = W.mem_size[c];
#pragma unroll
    for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++)
      tasks |= (W.last_task[t * W.n + c] > 0 ? 1ull : 0ull) << (7 * t);
  }
  const double rm = wave_sum(merit), rf = wave_sum(fit), rx = wave_max(fit);
  int ri[5];
#pragma unroll
  for (int k = 0; k < 5; k++) ri[k] = wave_sum_i(iv[k]);
  const unsigned long long rt = wave_sum_u64(tasks);
  if (lane == 0) {
    s[wv][0] = (double)ri[0]; s[wv][1] = rm; s[wv][2] = rf; s[wv][3] = (double)ri[1];
    s[wv][4] = (double)ri[2]; s[wv][5] = rx; s[wv][6] = (double)ri[3]; s[wv][7] = (double)ri[4];
#pragma unroll
    for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) s[wv][8 + t] = (double)((rt >> (7 * t)) & 127ull);
  }
  __syncthreads();
  // only the NUSED slots carry data (the rest of the NPART rows are never
  // written and k_stats_final reports them as 0)
  if (threadIdx.x < NUSED) {
    const int k = threadIdx.x;
    double r = s[0][k];
    for (int q = 1; q < 4; q++) r = (k == 5) ? fmax(r, s[q][k]) : r + s[q][k];
    part[(int64_t)k * gridDim.x + blockIdx.x] = r;
  }
}

// out: [0..23] partial sums, 24 insts 25 deaths 26 divides 27 births 28 dropped
// 29 spills 30 cumulative insts 31 cumulative births 32 slices 33 lane steps.
// Block k < NPART reduces partial row k (256 lanes, fixed order: lane t sums
// entries t, t+256, ..., then a pairwise tree); block NPART sums the counter
// shards.
__global__ __launch_bounds__(256) void k_stats_final(DevWorld W, const double* part, int64_t nb,
                                                     double* out) {
  __shared__ double sd[256];
  constexpr int NG = 256 / CNT_STRIDE;          // groups of shards the block sums in parallel
  __shared__ unsigned long long cs[NG][CNT_STRIDE];
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  if (k >= NUSED && k < NPART) {
    if (tid == 0) out[k] = 0.0;
    return;
  }
  if (k < NPART) {
    const bool mx = k == 5;
    double acc = 0.0;
    for (int64_t b = tid; b < nb; b += 256) {
      const double o = part[(int64_t)k * nb + b];
      acc = mx ? fmax(acc, o) : acc + o;
    }
    sd[tid] = acc;
    __syncthreads();
    for (int stride = 128; stride >= 1; stride >>= 1) {
      if (tid < stride) sd[tid] = mx ? fmax(sd[tid], sd[tid + stride]) : sd[tid] + sd[tid + stride];
      __syncthreads();
    }
    if (tid == 0) out[k] = sd[0];
    return;
  }
  {
    const int slot = tid & (CNT_STRIDE - 1), g = tid / CNT_STRIDE;
    unsigned long long a = 0;
    for (int sh = g; sh < NSHARD; sh += NG) a += W.counters[sh * CNT_STRIDE + slot];
    cs[g][slot] = a;
  }
  __syncthreads();
  // the running sums take this update's counts once: here, or (statistics
  // never asked for) in the next reset_counts_block
  const bool fold = W.counters[CNT_CUM_FLAG] == 0ull;
  __syncthreads();
  if (tid < CNT_STRIDE) {
    unsigned long long t = 0;
    for (int g = 0; g < NG; g++) t += cs[g][tid];
    cs[0][tid] = t;
    if (tid == CNT_STRIDE - 1) W.counters[CNT_CUM_FLAG] = 1ull;
    else if (fold) W.counters[CNT_CUM_BASE + tid] += t;
  }
  __syncthreads();
  if (tid == 0) {
    out[24] = (double)cs[0][CNT_INSTS];
    out[25] = (double)cs[0][CNT_DEATHS];
    out[26] = (double)cs[0][CNT_DIVIDES];
    out[27] = (double)cs[0][CNT_BIRTHS];
    out[28] = (double)cs[0][CNT_DROPPED];
    out[29] = (double)cs[0][CNT_SPILLS];
    out[30] = (double)W.counters[CNT_CUM_INSTS];
    out[31] = (double)W.counters[CNT_CUM_BIRTHS];
    out[32] = (double)cs[0][CNT_SLICES];
    out[33] = (double)cs[0][CNT_LANESTEPS];
    out[34] = (double)cs[0][CNT_OVERWRITTEN];
    out[35] = (double)cs[0][CNT_CANCELLED];
    out[36] = (double)cs[0][CNT_WASTED];
    out[37] = __longlong_as_double(pacc_sum(W, 0));         // the predictor (bits)
    out[38] = __longlong_as_double(W.sched[1] + W.sched[2]); // the pick carry (bits)
    out[39] = W.totals[1];                                  // the organisms it is relative to
    out[40] = __longlong_as_double(densest_quarter(W));
    for (int q = 0; q < 4; q++) out[41 + q] = __longlong_as_double(quarter_count(W, q));   // (bits)
  }
}

}  // namespace

// ---------------------------------------------------------------------------
static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

void launch_set_orgs(const DevWorld& W, hipStream_t s, int64_t first, int64_t count,
                     const uint8_t* codes, const int32_t* offsets, const int32_t* lens,
                     const double* merits, const int32_t* inputs, int deterministic) {
  hipLaunchKernelGGL(k_set_orgs, dim3(nblk(count, 64)), dim3(64), 0, s, W, first, count, codes,
                     offsets, lens, merits, inputs, deterministic);
}

void launch_get_states(const DevWorld& W, hipStream_t s, int64_t first, int64_t count,
                       avgpu_cpu_state* states, uint8_t* codes, int cap) {
  hipLaunchKernelGGL(k_get_states, dim3(nblk(count, 64)), dim3(64), 0, s, W, first, count, states,
                     codes, cap);
}

void launch_state_digest(const DevWorld& W, hipStream_t s, int64_t first, int64_t count, uint64_t* d_out) {
  if (count <= 0) return;
  k_state_digest<<<(unsigned)((count + 127) / 128), 128, 0, s>>>(W, first, count, d_out);
}

void launch_get_census(const DevWorld& W, hipStream_t s, int64_t first, int64_t count, avgpu_census* d_out) {
  if (count <= 0) return;
  k_census<<<(unsigned)((count + 255) / 256), 256, 0, s>>>(W, first, count, d_out);
}
void launch_set_states(const DevWorld& W, hipStream_t s, int64_t first, int64_t count, const avgpu_cpu_state* in,
                       const uint8_t* codes, int cap) {
  hipLaunchKernelGGL(k_set_states, dim3((unsigned)((count + 127) / 128)), dim3(128), 0, s, W, first, count, in,
                     codes, cap);
}

void launch_classify_uniform(const DevWorld& W, hipStream_t s, int64_t first, int64_t count,
                             const int32_t* budget, int32_t uniform) {
  hipMemsetAsync(W.class_count, 0, sizeof(int32_t) * 8, s);
  hipLaunchKernelGGL(k_classify_uniform, dim3(nblk(count, 256)), dim3(256), 0, s, W, first, count,
                     budget, uniform);
}

static void launch_block_counts(const DevWorld& W, hipStream_t s, const double* part, const int32_t* alive,
                                int64_t nb, int ntiles, int L, double* totals, uint32_t update, int mode,
                                int sub = 0, int nsub = 1) {
  if (((int64_t)1 << L) <= TREE_LDS_P) {
    hipLaunchKernelGGL(k_block_counts<true>, dim3(1), dim3(1024), 0, s, W, part, alive, nb, ntiles, L, totals, update,
                       mode, 0, sub, nsub);
    return;
  }
  const int Lt = L - TREE_C_LOG;
  const int64_t K = (int64_t)1 << Lt;
  hipLaunchKernelGGL(k_tree_up, dim3((unsigned)K), dim3(1024), 0, s, W, part, alive, nb, ntiles, mode);
  // the K chunk roots' tree in LDS: K <= 4096 for any world of < 2^31 cells
  // (2^23 blocks at most, so K <= 2^11)
  hipLaunchKernelGGL(k_block_counts<true>, dim3(1), dim3(1024), 0, s, W, part, alive, nb, ntiles, Lt, totals,
                     update, mode, 1, sub, nsub);
  if (mode == 3) return;
  const int64_t b0 = mode == 1 ? W.cell0 / 256 : 0, nloc = (W.n + 255) / 256;
  const int64_t nk = ((b0 + nloc - 1) >> TREE_C_LOG) - (b0 >> TREE_C_LOG) + 1;
  hipLaunchKernelGGL(k_tree_down, dim3((unsigned)nk), dim3(1024), 0, s, W, part, alive, nb, ntiles, mode, K, update);
}

static int tree_levels(int64_t nbt) {
  int L = 0;
  while (((int64_t)1 << L) < nbt) L++;
  return L;
}

// totals: [0] total weight, [1] organisms (mode 3 of k_block_counts).
// scratch: (n+255)/256 doubles + as many int32 partials
void launch_merit_total(const DevWorld& W, hipStream_t s, double* totals, double* scratch) {
  const int64_t nb = (W.n + 255) / 256;
  int32_t* alive_partial = reinterpret_cast<int32_t*>(scratch + nb);
  hipLaunchKernelGGL(k_merit_partial, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, W, scratch, alive_partial,
                     (double*)nullptr, 0);
  launch_block_counts(W, s, scratch, alive_partial, nb, 1, tree_levels(nb), totals, 0u, 3);
}

// the update's counters, birth-queue and class-list lengths, zeroed by one
// launch instead of three fill packets (~10 us each on the queue)
__global__ __launch_bounds__(256) void k_reset_counts(DevWorld W) { reset_counts_block(W); }

// the allotment of a world whose block counts are in W.blk_count: budgets,
// class lists, occupancy; then the class-0 order
static void launch_allot(const DevWorld& W, hipStream_t s, const double* totals, hipEvent_t lists_ready,
                         uint32_t update, int tick = 1) {
  // (16 blocks per workgroup: the class lists take one global atomic per
  // class and 4096 cells -- with 1024-cell workgroups those atomics on three
  // addresses serialised to ~50 us per update, profiles/r04c_tail_per_update.txt)
  hipLaunchKernelGGL(k_allot, dim3(nblk(W.n, 4096)), dim3(1024), 0, s, W, totals, update, tick);
  // the class lists are complete: the aux streams of the list classes start
  // here, beside the window sort, so that their blocks take CUs before class 0
  // (with the sort folded into the allotment they start together with class 0
  // and end ~35 us after it: profiles/r02q_tail_per_update.txt).  With the
  // lists inside class 0's launch (mix_lists) there is no fork: an event
  // record here left ~14 us of dead time on the world's stream
  if (!mix_lists()) hipEventRecord(lists_ready, s);
  hipLaunchKernelGGL(k_window_order, dim3(nblk(W.n, 4096)), dim3(1024), 0, s, W);
}

// single world: block partials (k_merit_partial also zeroes the update's
// counters), the scheduler's top tree, the allotment, the class-0 order
void launch_world_begin(const DevWorld& W, hipStream_t s, double* totals, double* scratch,
                        hipEvent_t lists_ready, uint32_t update, int sub, int nsub) {
  const int64_t nb = (W.n + 255) / 256;
  int32_t* alive_partial = reinterpret_cast<int32_t*>(scratch + nb);
  if (sub == 0) launch_resources_begin(W, s);   // ProcessPreUpdate + the update's first DoUpdates
  hipLaunchKernelGGL(k_merit_partial, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, W, scratch, alive_partial,
                     (double*)nullptr, sub == 0 ? 1 : 2);
  launch_block_counts(W, s, scratch, alive_partial, nb, 1, tree_levels(nb), totals, update, 0, sub, nsub);
  launch_allot(W, s, totals, lists_ready, update, sub == 0 ? 1 : 0);
}

// a world whose totals were handed in (avgpu_update_totals + an all-reduce of
// every world's {total weight, organisms}, in totals[0..1]): its block
// partials, then this world's picks by cMultiProcessWorld's formula
// (k_block_counts mode 2).  reset: clear the update's counters here.
void launch_world_pre(const DevWorld& W, hipStream_t s, double* totals, double* scratch, hipEvent_t lists_ready,
                      uint32_t update, bool reset) {
  const int64_t nb = (W.n + 255) / 256;
  int32_t* alive_partial = reinterpret_cast<int32_t*>(scratch + nb);
  launch_resources_begin(W, s);   // ProcessPreUpdate + the update's first DoUpdates
  hipLaunchKernelGGL(k_merit_partial, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, W, scratch, alive_partial,
                     (double*)nullptr, reset ? 1 : 0);
  launch_block_counts(W, s, scratch, alive_partial, nb, 1, tree_levels(nb), totals, update, 2);
  launch_allot(W, s, totals, lists_ready, update);
}

// a strip tile: the top tree over every strip's gathered partials (mode 1),
// then the allotment (its partials' launch cleared the counters)
void launch_tile_pre(const DevWorld& W, hipStream_t s, const double* gathered, int ntiles, double* totals,
                     hipEvent_t lists_ready, uint32_t update, int sub, int nsub) {
  const int64_t nb = (W.n + 255) / 256;
  if (sub == 0) launch_resources_begin(W, s);
  launch_block_counts(W, s, gathered, nullptr, nb, ntiles, tree_levels(nb * ntiles), totals, update, 1, sub, nsub);
  launch_allot(W, s, totals, lists_ready, update, sub == 0 ? 1 : 0);
}

void launch_stats(const DevWorld& W, hipStream_t s, double* stats) {
  const int64_t nb = (W.n + 255) / 256;
  double* part = stats + NSTAT;
  hipLaunchKernelGGL(k_stats_partial, dim3((unsigned)nb), dim3(256), 0, s, W, part);
  hipLaunchKernelGGL(k_stats_final, dim3(NPART + 1), dim3(256), 0, s, W, part, nb, stats);
}

// k_activate: a lane per birth; 2048 waves cover 131k queued births per pass
static unsigned lane_grid(const DevWorld& W) { return (unsigned)std::min<int64_t>(nblk(W.rcap, 64), 2048); }
// placement kernels stride over the queue; 8 blocks of 256 per CU cover it
// (AVGPU_PLACE_GRID overrides the cap for sweeps)
static unsigned place_grid(const DevWorld& W) {
  static int cap = -1;
  if (cap < 0) {
    const char* e = getenv("AVGPU_PLACE_GRID");
    cap = e ? std::max(1, atoi(e)) : 2048;
  }
  return (unsigned)std::min<int64_t>(nblk(W.rcap, 256), cap);
}

static bool has_divide_mutations(const DevWorld& W) {
  return (W.th_div_mut | W.th_div_ins | W.th_div_del | W.th_div_slip | W.th_div_uni) != 0 || W.seg_any;
}
static unsigned mut_grid(const DevWorld& W) { return (unsigned)std::min<int64_t>(nblk(W.rcap, MUT_PER_WAVE), 8192); }

// after a serial-world update (its births are placed): resources, statistics
void launch_serial_post(const DevWorld& W, hipStream_t s, double* stats) {
  launch_resources_end(W, s);
  launch_stats(W, s, stats);
}

// the serial world's cPhenotype::IncAge tick (k_allot's, for the batch update)
__global__ void k_age_tick(DevWorld W) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < W.n && W.track_age && (W.ctl[c] & CTL_ALIVE)) W.age[c] += 1;
}
void launch_age_tick(const DevWorld& W, hipStream_t s) {
  hipLaunchKernelGGL(k_age_tick, dim3(nblk(W.n, 256)), dim3(256), 0, s, W);
}

void launch_reset_counts(const DevWorld& W, hipStream_t s) {
  hipLaunchKernelGGL(k_reset_counts, dim3(1), dim3(256), 0, s, W);
}

// Placement rounds alternate between the claim arrays claim / claim2 (round k
// claims into array k & 1 after zeroing its records' round k-1 claims; the
// last round's are zeroed by k_activate): no clearing launch per round.
void launch_world_post(const DevWorld& W, hipStream_t s, uint32_t key, int sub, int nsub, long long* pred_out,
                       long long pred_seq) {
  // the occupancy was initialised by k_allot_total; the divide mutations
  // ride in round 0's pick launch
  // round 0's pick (with the divide mutations beside it), then three launches
  // of resolve(m-1) + pick(m), then activation with round 3's resolve: 5
  // launches instead of 9 (k_place_round)
  const unsigned bb = place_grid(W);
  const int pm = has_divide_mutations(W) ? (int)((mut_grid(W) + 3) / 4) : 0;
  const int pf = (int)std::min<unsigned>(bb, 256u);   // finalize_phenotype blocks
  const int nbk = (int)bb + pf + pm;
  const bool soup = W.birth_method == 4 && W.prefer_empty;
  auto soup_cells = [&](int m) {                    // the soup's candidates of round m (k_empty_*)
    const int eb = (int)nblk(W.n, 256);
    hipLaunchKernelGGL(k_empty_count, dim3(eb), dim3(256), 0, s, W, m);
    hipLaunchKernelGGL(k_empty_scan, dim3(1), dim3(1024), 0, s, W, eb);
    hipLaunchKernelGGL(k_empty_scatter, dim3(eb), dim3(256), 0, s, W, m);
  };
  if (soup) soup_cells(0);
#ifdef AVGPU_SPLIT_PICK_MUT
  hipLaunchKernelGGL(k_place_pick_mut, dim3(bb), dim3(256), 0, s, W, (int)bb, pf, 0, nbk);
  hipLaunchKernelGGL(k_place_pick_mut, dim3(pf), dim3(256), 0, s, W, (int)bb, pf, (int)bb, nbk);
  if (pm) hipLaunchKernelGGL(k_place_pick_mut, dim3(pm), dim3(256), 0, s, W, (int)bb, pf, (int)bb + pf, nbk);
#else
  hipLaunchKernelGGL(k_place_pick_mut, dim3(nbk), dim3(256), 0, s, W, (int)bb, pf, 0, nbk);
#endif
  hipLaunchKernelGGL(k_place_claim0, dim3(bb), dim3(256), 0, s, W, pred_out, pred_seq);
  for (int m = 1; m < 4; m++) {
    if (soup) soup_cells(m);
    hipLaunchKernelGGL(k_place_round, dim3(bb), dim3(256), 0, s, W, m);
  }
  hipLaunchKernelGGL(k_activate, dim3(lane_grid(W)), dim3(64), 0, s, W, 1, key, sub, nsub);
}

// after the newborn pass (interp.hip): the step's global consumption settled,
// then (eager) the update's statistics
void launch_world_end(const DevWorld& W, hipStream_t s, double* stats, bool eager) {
  launch_resources_end(W, s);
  if (eager) launch_stats(W, s, stats);
}

// ---- strip tiles: the same update split around the halo exchanges ----
// (a strip tile's partials start its update: block 0 also clears the counters)
void launch_tile_partials(const DevWorld& W, hipStream_t s, double* out, int reset) {
  const int64_t nb = (W.n + 255) / 256;
  hipLaunchKernelGGL(k_merit_partial, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, W, out, (int32_t*)nullptr,
                     out + nb, reset);
}

// after interpretation: the divide mutations, the ghost rows emptied and the
// edge-row occupancy out (one launch, k_tile_prep)
void launch_tile_after_interpret(const DevWorld& W, hipStream_t s) {
  const unsigned hb = nblk(2 * (int64_t)W.world_x, 256);
  const int mb = has_divide_mutations(W) ? (int)((mut_grid(W) + 3) / 4) : 0;
  const int fb = (int)std::min<unsigned>(place_grid(W), 256u);   // finalize_phenotype blocks
  hipLaunchKernelGGL(k_tile_prep, dim3(mb + fb + hb), dim3(256), 0, s, W, mb, fb);
}

// phase 0: round 0's picks and kill times, or (round 1..3) k_tile_round:
//          resolve round - 1, pick round
// phase 3: (round 0) the cancellations and round 0's claims (k_tile_claim0)
// phase 1: (round 3) the last resolve, then the ghost-row winners packed into
//          the record buffers
// phase 2: (round 3) this tile's own winners activated -- while the records
//          travel; avgpu_tile_finish then activates the received ones
void launch_tile_place(const DevWorld& W, hipStream_t s, int round, int phase, uint32_t key, int sub, int nsub) {
  const unsigned bb = place_grid(W);
  const unsigned hb = nblk(2 * (int64_t)W.world_x, 256);
  if (phase == 0) {
    hipLaunchKernelGGL(k_tile_round, dim3(bb + hb), dim3(256), 0, s, W, round, (int)bb);
  } else if (phase == 3) {
    hipLaunchKernelGGL(k_tile_claim0, dim3(bb), dim3(256), 0, s, W);
  } else if (phase == 1) {
    hipLaunchKernelGGL(k_tile_round, dim3(bb + hb), dim3(256), 0, s, W, 4, (int)bb);
    hipLaunchKernelGGL(k_halo_pack, dim3(lane_grid(W)), dim3(64), 0, s, W);
  } else {
    hipLaunchKernelGGL(k_activate, dim3(lane_grid(W)), dim3(64), 0, s, W, 2, key, sub, nsub);
  }
}

void launch_tile_finish(const DevWorld& W, hipStream_t s, uint32_t key, int sub, int nsub) {
  const unsigned rb = (unsigned)std::max(1, std::min(W.world_x, 4096));
  hipLaunchKernelGGL(k_activate_remote, dim3(2 * rb), dim3(64), 0, s, W, key, sub, nsub);
}
