// capi.hip -- host side of the C-ABI declared in include/avida_gpu.h.
//
// The world object owns every device allocation (SoA organism state, tapes,
// birth queue, scratch) on one HIP device and one HIP stream.  Each entry
// point names the reference interface it replaces in the header.  There is no
// CPU execution path in this library: every state transition of the hot path
// runs in the kernels of interp.hip / world.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "device.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t _e = (x);                                                            \
    if (_e != hipSuccess) return fail(AVGPU_EHIP, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)
// A copy / fill of an API call on the world's stream, complete on return.  The
// world's streams are non-blocking: a null-stream hipMemcpy / hipMemset would
// neither wait for the kernels queued on them nor be waited for by them.
#define COPY_SYNC(ww, dst, src, bytes, kind)                                        \
  do {                                                                              \
    HIPCHK(hipMemcpyAsync((dst), (src), (bytes), (kind), (ww)->stream));           \
    HIPCHK(hipStreamSynchronize((ww)->stream));                                     \
  } while (0)
#define SET_SYNC(ww, dst, val, bytes)                                               \
  do {                                                                              \
    HIPCHK(hipMemsetAsync((dst), (val), (bytes), (ww)->stream));                    \
    HIPCHK(hipStreamSynchronize((ww)->stream));                                     \
  } while (0)

}  // namespace

struct avgpu_world {
  avgpu_cfg cfg;
  int device = 0;
  hipStream_t stream = nullptr;      // current stream (own or external)
  hipStream_t own_stream = nullptr;
  hipStream_t aux_stream[3] = {};   // [0] class 1, [1] classes 2 + 3 beside class 0 (world updates); [2] unused
  hipEvent_t ev_fork = nullptr, ev_join[3] = {};
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // event ring around interpreter phases (avgpu_last_kernel_ms,
  // avgpu_kernel_times): ev[i][0] before class 0, ev[i][k+1] after class k
  static const int RING = 512;
  hipEvent_t ring[RING][NUM_CLASSES + 1] = {};
  int ring_head = 0, ring_count = 0;
  // avgpu_set_timing: bracket every time_every-th interpretation (0: none)
  int time_every = 1;
  int64_t interp_calls = 0;
  double acc_ms = 0.0;
  double acc_class_ms[NUM_CLASSES] = {};
  int64_t acc_phases = 0;
  DevWorld W;
  DevWorld* d_W = nullptr;      // device copy of W read by k_interpret: one of d_Wv
  // two device copies (a world whose resources swap their buffers every
  // update alternates between two descriptors: after two updates neither
  // is uploaded again), uploaded in stream order from pinned staging
  DevWorld* d_Wv[2] = {};
  DevWorld pushedv[2];          // what d_Wv[k] holds
  bool validv[2] = {false, false};
  int cur_w = 0;
  DevWorld* h_stage = nullptr;  // [2] pinned
  hipEvent_t ev_stage[2] = {};  // the last upload from h_stage[k]
  std::vector<void*> allocs;
  // instruction set translation
  int n_ops = 0;
  uint8_t op2code[256];
  int16_t code2op[64];
  bool instset_loaded = false;
  int res_geom[AVGPU_MAX_RESOURCES] = {};
  std::vector<avgpu_resource> res_spec;       // avgpu_load_resources input (re-seeded by set_tile)
  std::vector<avgpu_cell_resource> cell_spec;
  bool env_loaded = false;
  // device scratch
  double* d_totals = nullptr;   // [8 + partials]
  double* d_stats = nullptr;    // [32 + partials]
  bool stats_stale = false;     // the last update ran without statistics (out == NULL)
  bool use_global = false;
  int64_t update = 0;
  float last_kernel_ms = 0.f;
  int64_t last_launches = 0;
  bool has_test_buffers = false;
  double* rec_buf = nullptr;    // RECORDED mode stream (avgpu_set_rng_mode)
  double* srec_buf[2] = {nullptr, nullptr};   // the serial world's recorded streams
  // strip tiles
  int ntiles_last = 0;
  bool tile_buffers = false;
  // batch steps: the last update's predictor and organisms
  // (coherent mapped host memory the update's last step writes, then pred_seq), the
  // host's copy, the steps the last update ran; strips: the current step
  long long* h_pred = nullptr;
  long long* d_pred = nullptr;   // its device address
  bool pred_pending = false;
  long long pred_seq = 0;       // the sequence number k_place_claim0 publishes with the predictor
  bool reaper_rebuild = false;  // the serial reaper queue is built again at the next serial update
  long long pred_acc = 0, pred_n = 0, pred_cnt = 0;
  int last_k = 1;
  int tile_sub = 0, tile_k = 1, tile_sub_next = 0;
  uint32_t tile_key = 0;

  template <typename T>
  int alloc(T** p, size_t count) {
    void* q = nullptr;
    size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) return fail(AVGPU_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    hipMemsetAsync(q, 0, bytes, stream);
    allocs.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
  }
};

namespace {

int setup_world(avgpu_world* w, int64_t n, bool test_buffers) {
  DevWorld& W = w->W;
  memset(&W, 0, sizeof(W));
  W.n = n;
  const avgpu_cfg& c = w->cfg;
  int rc = 0;
#define A(ptr, cnt) if ((rc = w->alloc(&W.ptr, (size_t)(cnt))) < 0) return rc
  A(xs, (size_t)n * XS_WORDS); A(ctl, n); A(mem_size, n); A(max_exec, n); A(age, n); A(birth_len, n); A(gkey, n); A(rng, 3 * n);
  A(budget, n); A(aclass, n); A(tape, (size_t)n * TAPE_SLOT);
  A(inputs, 3 * n); A(last_task, AVGPU_MAX_REACTIONS * n);
  A(cur_react, AVGPU_MAX_REACTIONS * n);
  A(merit, n); A(fitness, n); A(credit, n); A(gest_time, n); A(num_div, n);
  A(generation, n); A(copied, n); A(child_copied, n); A(executed, n);
  HIPCHK(hipMemsetAsync(W.aclass, ACLASS_NONE, n, w->stream));   // no slice allotted yet
  A(class_list, NUM_LISTS * n); A(order, n); A(sub_hist, (size_t)((n + 4095) / 4096) * SORT_BUCKETS); A(class_count, 8); A(counters, CNT_WORDS);
  // birth records: one primary record per cell + overflow for further
  // offspring of one slice (device.h); test worlds never enqueue births
  W.rcap = n + (test_buffers ? 16 : std::max<int64_t>(4096, n / 4));
  const int64_t R = W.rcap;
  A(b_count, 3); A(b_list, n); A(b_parent, R); A(b_seq, R); A(b_len, R); A(b_len0, R); A(b_edit, 5 * R);
  // DIV_MUT_PROB arena: three times the largest expected substitutions per
  // record plus 16 (offsets are int32); a fill past it is counted
  // (AVGPU_CNT_SUB_OVERFLOW), never written
  const double pmeans[5] = {c.divide_poisson_slip_mean, c.divide_poisson_mut_mean,
                            c.divide_poisson_ins_mean, c.divide_poisson_del_mean, c.divide_poisson_trans_mean};
  const double psite[6] = {c.div_mut_prob, c.div_ins_prob, c.div_del_prob, c.div_uniform_prob, c.div_slip_prob,
                           c.div_trans_prob};
  // data fills (SLIP_FILL_MODE 2 / 3, TRANS_FILL_MODE 1) keep their draws in
  // the arena, and the one-shot slip then goes there as a segment
  const bool sdata = c.slip_fill_mode == 2 || c.slip_fill_mode == 3, tdata = c.trans_fill_mode == 1;
  const double eslip = c.divide_slip_prob + c.divide_poisson_slip_mean + c.div_slip_prob * AVGPU_MAX_GENOME;
  const double etrans = c.divide_trans_prob + c.divide_poisson_trans_mean + c.div_trans_prob * AVGPU_MAX_GENOME;
  bool pois = false, site = c.divide_trans_prob > 0.0 || (sdata && eslip > 0.0);
  for (int q = 0; q < 5; q++) pois = pois || pmeans[q] > 0.0;
  for (int q = 0; q < 6; q++) site = site || psite[q] > 0.0;
  if (pois || site) {
    // arena words per record: 3x the largest expected count of each kind
    // (per site: a 2048-site offspring) + 16 each; offsets are int32
    const int tw = tdata ? 3 : 2, sw = sdata ? 2 : 1;
    int64_t k = 16 + tw + sw;    // + the one-shot translocation's and slip's words
    for (int q = 0; q < 6; q++)
      if (psite[q] > 0.0)
        k += (q == 5 ? tw : (q == 4 ? sw : 1)) * ((int64_t)std::ceil(AVGPU_MAX_GENOME * std::min(1.0, psite[q]) * 3.0) + 16);
    for (int q = 0; q < 5; q++)
      if (pmeans[q] > 0.0) k += (q == 4 ? tw : (q == 0 ? sw : 1)) * ((int64_t)std::ceil(3.0 * std::min(pmeans[q], 4096.0)) + 16);
    // fill words: a slip or translocation of an L-site insertion keeps L words
    // + L/32 of bit set; E[L] <= a sixth of the offspring (from, to uniform),
    // sized at 3x for an offspring of AVGPU_MAX_GENOME / 4 sites
    const double efill = (AVGPU_MAX_GENOME / 4.0) / 6.0 * (1.0 + 1.0 / 32.0) + 2.0;
    if (sdata && eslip > 0.0) k += (int64_t)std::ceil(3.0 * std::min(eslip, 4096.0) * efill) + 16;
    if (tdata && etrans > 0.0) k += (int64_t)std::ceil(3.0 * std::min(etrans, 4096.0) * efill) + 16;
    k = std::min<int64_t>(k, (int64_t)INT32_MAX / R);
    W.scap = R * k;
    A(b_subs, W.scap); A(b_pofs, NSEG * R); A(b_pcnt, NSEG * R);
  }
  W.seg_any = (pois || site) ? 1 : 0;
  W.pois_any = pois ? 1 : 0;
  for (int q = 0; q < 5; q++) W.pois_L[q] = pmeans[q] > 0.0 ? std::exp(-pmeans[q]) : 0.0;
  A(b_inh, (size_t)BI_WORDS * R); A(b_target, R); A(b_state, R);
  A(b_prio, R); A(b_genome, (size_t)R * TAPE_SLOT);
  // placement scratch with two ghost rows (strip tiles)
  // occupancy, owners and the four placement rounds' claims, each with the two
  // ghost rows a strip tile keeps after its n cells
  const int64_t ng = n + 2 * (int64_t)c.world_x;
  A(occ, ng); A(claim, ng); A(claim2, ng); A(owner, ng); A(killt, n); A(sdone, n); A(ran, n); A(sched, 12); A(pacc, NSHARD * PACC_STRIDE);
  W.claim_r[0] = W.claim; W.claim_r[1] = W.claim2;
  A(claim_r[2], ng); A(claim_r[3], ng); A(b_tgt, 4 * R);
  if (c.birth_method == 4) {
    A(e_list, n); A(e_blk, (n + 255) / 256 + 1); A(soup_perm, n);
    std::vector<int32_t> iota((size_t)n);
    for (int64_t i = 0; i < n; i++) iota[(size_t)i] = (int32_t)i;
    // on the world's stream, after alloc's zeroing memset (a plain hipMemcpy
    // runs on the null stream, which does not wait for the non-blocking one)
    HIPCHK(hipMemcpyAsync(W.soup_perm, iota.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice,
                          w->stream));
    HIPCHK(hipStreamSynchronize(w->stream));
  }
  if (test_buffers) {
    A(t_flags, (size_t)n * TAPE_SLOT); A(t_flags_len, n); A(t_child, (size_t)n * TAPE_SLOT);
    A(t_child_len, n);
  }
  A(rand_cum, 64); A(rand_code, 64); A(task_lut, 256); A(rand_lut, 256);
  A(react_tab, AVGPU_MAX_REACTIONS * RT_STRIDE); A(task_tab, 32);
  A(react_res, AVGPU_MAX_REACTIONS * RR_STRIDE); A(res_param, AVGPU_MAX_RESOURCES);
  A(res_global, AVGPU_MAX_RESOURCES); A(res_cons, AVGPU_MAX_RESOURCES);
  if ((rc = w->alloc(&w->d_Wv[0], 1)) || (rc = w->alloc(&w->d_Wv[1], 1))) return rc;
  w->d_W = w->d_Wv[0];
  w->validv[0] = w->validv[1] = false;
  const int64_t nb = (n + 255) / 256;
  if ((rc = w->alloc(&w->d_totals, (size_t)(8 + 2 * nb)))) return rc;
  W.totals = w->d_totals;
  // the scheduler's tree: block counts, the top tree's levels (a strip tile
  // regrows them for the whole world at avgpu_tile_begin)
  if ((rc = w->alloc(&W.blk_count, (size_t)nb))) return rc;
  W.tree_cap = 1;
  while (W.tree_cap < nb) W.tree_cap <<= 1;
  if ((rc = w->alloc(&W.tree_scr, (size_t)(2 * W.tree_cap)))) return rc;
  if ((rc = w->alloc(&W.tree_cnt, (size_t)(2 * W.tree_cap)))) return rc;
  if ((rc = w->alloc(&w->d_stats, (size_t)(45 + 24 * nb)))) return rc;
#undef A
  w->has_test_buffers = test_buffers;
  // config scalars
  W.world_x = c.world_x; W.world_y = c.world_y; W.geometry = c.world_geometry;
  W.ave_time_slice = c.ave_time_slice; W.slicing = c.slicing_method;
  W.base_merit_method = c.base_merit_method; W.base_const_merit = c.base_const_merit;
  W.default_bonus = c.default_bonus; W.size_range = c.offspring_size_range;
  W.min_copied_lines = c.min_copied_lines; W.min_exe_lines = c.min_exe_lines;
  W.merit_default_bonus = c.merit_default_bonus; W.required_bonus = c.required_bonus;
  W.inherit_merit = c.inherit_merit; W.require_allocate = c.require_allocate;
  W.alloc_method = c.alloc_method; W.max_label_exe = c.max_label_exe_size;
  W.cfg_min_genome = c.min_genome_size; W.cfg_max_genome = c.max_genome_size;
  W.max_genome = (!c.max_genome_size || c.max_genome_size > AVGPU_MAX_GENOME) ? AVGPU_MAX_GENOME : c.max_genome_size;
  W.min_genome = (!c.min_genome_size || c.min_genome_size < AVGPU_MIN_GENOME) ? AVGPU_MIN_GENOME : c.min_genome_size;
  W.death_method = c.death_method; W.age_limit = c.age_limit;
  W.prefer_empty = c.prefer_empty; W.allow_parent = c.allow_parent; W.birth_method = c.birth_method;
  // P(p) = u < p: a 32-bit counter draw x hits iff x < ceil(p 2^32)
  auto th = [](double p) -> uint64_t {
    if (!(p > 0.0)) return 0;
    if (p >= 1.0) return 1ull << 32;
    return (uint64_t)std::ceil(p * 4294967296.0);
  };
  W.th_copy_mut = th(c.copy_mut_prob);
  W.th_copy_ins = th(c.copy_ins_prob); W.p_copy_ins = c.copy_ins_prob;
  W.th_copy_del = th(c.copy_del_prob); W.p_copy_del = c.copy_del_prob;
  W.th_copy_uni = th(c.copy_uniform_prob); W.p_copy_uni = c.copy_uniform_prob;
  W.th_copy_slip = th(c.copy_slip_prob); W.p_copy_slip = c.copy_slip_prob;
  W.copy_ext = (W.th_copy_ins || W.th_copy_del || W.th_copy_uni || W.th_copy_slip) ? 1 : 0;
  W.th_div_mut = th(c.divide_mut_prob);
  W.th_div_ins = th(c.divide_ins_prob);
  W.th_div_del = th(c.divide_del_prob);
  W.th_div_slip = th(c.divide_slip_prob);
  W.th_div_uni = th(c.divide_uniform_prob);
  W.p_copy_mut = c.copy_mut_prob; W.p_div_mut = c.divide_mut_prob; W.p_div_ins = c.divide_ins_prob;
  W.p_div_del = c.divide_del_prob; W.p_div_slip = c.divide_slip_prob; W.p_div_uni = c.divide_uniform_prob;
  W.th_div_site = th(c.div_mut_prob);
  W.p_div_site = c.div_mut_prob;
  W.th_dsite[0] = th(c.div_ins_prob); W.p_dsite[0] = c.div_ins_prob;
  W.th_dsite[1] = th(c.div_del_prob); W.p_dsite[1] = c.div_del_prob;
  W.th_dsite[2] = th(c.div_uniform_prob); W.p_dsite[2] = c.div_uniform_prob;
  W.th_dsite[3] = th(c.div_slip_prob); W.p_dsite[3] = c.div_slip_prob;
  W.th_dsite[4] = th(c.div_trans_prob); W.p_dsite[4] = c.div_trans_prob;
  W.th_dtrans = th(c.divide_trans_prob); W.p_dtrans = c.divide_trans_prob;
  W.th_par_site = th(c.parent_mut_prob);
  W.p_par_site = c.parent_mut_prob;
  W.th_par_ins = th(c.parent_ins_prob); W.p_par_ins = c.parent_ins_prob;
  W.th_par_del = th(c.parent_del_prob); W.p_par_del = c.parent_del_prob;
  W.slip_fill_mode = c.slip_fill_mode;
  W.trans_fill_mode = c.trans_fill_mode;
  W.slip_copy_mode = c.slip_copy_mode;
  W.track_age = (c.birth_method == 1 || c.birth_method == 2) ? 1 : 0;
  W.rec = nullptr; W.rec_n = 0; W.rec_off = nullptr;
  W.seed_lo = (uint32_t)c.seed;
  W.seed_hi = (uint32_t)(c.seed >> 32);
  // interpreter slow-op batching (interp.hip); AVGPU_SLOW_BATCH overrides (tuning)
  W.slow_batch = 12;
  if (const char* e = getenv("AVGPU_SLOW_BATCH")) W.slow_batch = std::max(1, std::min(64, atoi(e)));
  // the newborn pass's own: 1 -- its duration is its longest newborn's, and a
  // parked lane waiting for a batch lengthens exactly that path (1.344 ->
  // 1.323 ms per update, profiles/r06g_ab_nbsb.txt)
  W.nb_slow_batch = 1;
  if (const char* e = getenv("AVGPU_NB_SLOW_BATCH")) W.nb_slow_batch = std::max(1, std::min(64, atoi(e)));
  W.row0 = 0;
  W.global_rows = c.world_y;
  W.rows = c.world_y;
  W.tiled = 0;
  W.cell0 = 0;
  // logic id -> task bitmask (main/cTaskLib.cc:511-575)
  static const int sets[9][6] = {
      {15, 51, 85, -1, -1, -1}, {63, 95, 119, -1, -1, -1}, {136, 160, 192, -1, -1, -1},
      {175, 187, 207, 221, 243, 245}, {238, 250, 252, -1, -1, -1}, {10, 12, 34, 48, 68, 80},
      {3, 5, 17, -1, -1, -1}, {60, 90, 102, -1, -1, -1}, {153, 165, 195, -1, -1, -1}};
  uint16_t lut[256] = {0};
  for (int t = 0; t < 9; t++)
    for (int k = 0; k < 6; k++)
      if (sets[t][k] >= 0) lut[sets[t][k]] |= (uint16_t)(1u << t);
  HIPCHK(hipMemcpyAsync(W.task_lut, lut, sizeof(lut), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  return 0;
}

// The avida.cfg values this path cannot run with the reference's semantics
// (main/cAvidaConfig.h): an empty string when the configuration is on the
// path, else the reason avgpu_create refuses it (AVGPU_EUNSUPPORTED).
std::string unsupported_cfg(const avgpu_cfg& c) {
  auto nz = [](double v) { return v != 0.0; };
  const bool slips = nz(c.divide_slip_prob) || nz(c.divide_poisson_slip_mean) || nz(c.div_slip_prob);
  if (slips && (c.slip_fill_mode < 0 || c.slip_fill_mode == 1 || c.slip_fill_mode > 4))
    return "SLIP_FILL_MODE 1 (nop-X) or an unknown mode";
  if (nz(c.copy_slip_prob) && c.slip_copy_mode != 0 && c.slip_copy_mode != 1)
    return "SLIP_COPY_MODE other than 0 (read-head jump) and 1 (memory slip)";
  if (nz(c.copy_slip_prob) && c.slip_copy_mode == 1 && c.slip_fill_mode != 0 && c.slip_fill_mode != 2 &&
      c.slip_fill_mode != 4)
    return "SLIP_COPY_MODE 1 with SLIP_FILL_MODE other than 0 (duplication), 2 (random), 4 (nop-C)";
  if ((nz(c.divide_trans_prob) || nz(c.divide_poisson_trans_mean) || nz(c.div_trans_prob)) &&
      (c.trans_fill_mode < 0 || c.trans_fill_mode > 1))
    return "TRANS_FILL_MODE other than 0 (duplication) / 1 (scrambled)";
  if (c.divide_poisson_slip_mean > 700.0 || c.divide_poisson_mut_mean > 700.0 ||
      c.divide_poisson_ins_mean > 700.0 || c.divide_poisson_del_mean > 700.0 ||
      c.divide_poisson_trans_mean > 700.0)
    return "DIVIDE_POISSON_*_MEAN above 700 (exp(-mean) underflows)";
  if (c.divide_method != 1) return "DIVIDE_METHOD other than 1 (split)";
  if (c.sub_updates < 0 || c.sub_updates > 64) return "sub_updates outside 0..64";
  if (c.sub_updates > 1 && c.slicing_method != 1) return "sub_updates > 1 with SLICING_METHOD other than 1";
  if (c.world_geometry != 1 && c.world_geometry != 2) return "WORLD_GEOMETRY other than 1 (grid) or 2 (torus)";
  if (c.slicing_method < 0 || c.slicing_method > 2) return "SLICING_METHOD other than 0, 1, 2";
  if (c.base_merit_method < 0 || c.base_merit_method > 5) return "BASE_MERIT_METHOD other than 0..5";
  if (c.birth_method < 0 || c.birth_method > 5)
    return "BIRTH_METHOD other than 0 (random neighbour), 1 (oldest), 2 (highest age / merit), 3 (empty only), "
           "4 (whole-world soup), 5 (eldest, serial world)";
  if ((c.birth_method == 1 || c.birth_method == 2) && !c.prefer_empty)
    return "BIRTH_METHOD 1 / 2 without PREFER_EMPTY (the reference reads the organism of an empty cell)";
  if (c.death_method < 0 || c.death_method > 2) return "DEATH_METHOD other than 0, 1, 2";
  if (c.alloc_method != 0 && c.alloc_method != 2) return "ALLOC_METHOD other than 0 (default) and 2 (random)";
  if (nz(c.point_mut_prob) || nz(c.point_ins_prob) || nz(c.point_del_prob) || nz(c.inst_point_mut_prob))
    return "POINT_MUT_PROB / POINT_INS_PROB / POINT_DEL_PROB / INST_POINT_MUT_PROB (cosmic-ray mutations)";
  if (nz(c.div_lgt_prob) || nz(c.divide_lgt_prob) || nz(c.divide_poisson_lgt_mean))
    return "DIV_LGT_PROB / DIVIDE_LGT_PROB / DIVIDE_POISSON_LGT_MEAN (lateral gene transfer)";
  if (nz(c.inject_mut_prob) || nz(c.inject_ins_prob) || nz(c.inject_del_prob)) return "INJECT_*_PROB";
  if (nz(c.meta_copy_mut) || nz(c.meta_std_dev)) return "META_COPY_MUT / META_STD_DEV";
  if (nz(c.death_prob)) return "DEATH_PROB";
  if (c.age_deviation != 0) return "AGE_DEVIATION";
  if (c.divide_failure_resets != 0) return "DIVIDE_FAILURE_RESETS";
  if (c.special_mut_line >= 0) return "SPECIAL_MUT_LINE";
  if (c.population_cap > 0) return "POPULATION_CAP";
  if (c.generation_inc_method != 1) return "GENERATION_INC_METHOD other than 1";
  if (c.reset_inputs_on_divide != 0) return "RESET_INPUTS_ON_DIVIDE";
  if (c.epigenetic_method != 0) return "EPIGENETIC_METHOD";
  if (c.min_cycles != 0) return "MIN_CYCLES";
  if (c.required_task < -1 || c.immunity_task < -1 || c.required_reaction < -1 || c.immunity_reaction < -1 ||
      c.required_task >= AVGPU_MAX_REACTIONS || c.immunity_task >= AVGPU_MAX_REACTIONS ||
      c.required_reaction >= 12 || c.immunity_reaction >= 12)
    return "REQUIRED_TASK / IMMUNITY_TASK outside the task library, REQUIRED_REACTION / IMMUNITY_REACTION "
           "beyond reaction 11";
  if (c.require_exact_copy != 0) return "REQUIRE_EXACT_COPY";
  if (c.fitness_method != 0) return "FITNESS_METHOD other than 0";
  if (c.juv_period != 0) return "JUV_PERIOD";
  if (c.no_mut_insts_len < 0 || c.no_mut_insts_len > 63 ||
      (size_t)c.no_mut_insts_len != strnlen(c.no_mut_insts, sizeof(c.no_mut_insts)))
    return "NO_MUT_INSTS longer than 63 symbols, or no_mut_insts_len not its length";
  if (c.test_fitness_measures != 0) return "REVERT_* / STERILIZE_* (Divide_TestFitnessMeasures1)";
  return std::string();
}

avgpu_world* create_world(const avgpu_cfg* cfg, int device, int64_t n, bool test_buffers) {
  if (!cfg) { fail(AVGPU_EINVAL, "cfg is NULL"); return nullptr; }
  {
    const std::string why = unsupported_cfg(*cfg);
    if (!why.empty()) {
      fail(AVGPU_EUNSUPPORTED, why + " is not on the GPU path");
      return nullptr;
    }
  }
  if (hipSetDevice(device) != hipSuccess) { fail(AVGPU_EHIP, "hipSetDevice failed"); return nullptr; }
  avgpu_world* w = new avgpu_world();
  w->cfg = *cfg;
  w->device = device;
  if (n <= 0) n = (int64_t)cfg->world_x * cfg->world_y;
  if (n <= 0 || n > (1ll << 30)) { delete w; fail(AVGPU_EINVAL, "bad cell count"); return nullptr; }
  // The list classes' aux streams get the higher priority: their blocks
  // become ready together with class 0's (both wait for k_allot_sort) and must
  // take their CUs first -- a class-3 block needs a whole CU's LDS, which a
  // CU full of class-0 blocks frees only when all of them have retired.
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  if (hipStreamCreateWithFlags(&w->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&w->aux_stream[0], hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&w->aux_stream[1], hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipEventCreateWithFlags(&w->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&w->ev_join[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&w->ev_join[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&w->ev_join[2], hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&w->ev0) != hipSuccess || hipEventCreate(&w->ev1) != hipSuccess ||
      hipHostMalloc((void**)&w->h_pred, 4 * sizeof(long long), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostMalloc((void**)&w->h_stage, 2 * sizeof(DevWorld), hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&w->ev_stage[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&w->ev_stage[1], hipEventDisableTiming) != hipSuccess ||
      hipHostGetDevicePointer((void**)&w->d_pred, w->h_pred, 0) != hipSuccess) {
    delete w; fail(AVGPU_EHIP, "stream/event creation failed"); return nullptr;
  }
  w->h_pred[0] = w->h_pred[1] = w->h_pred[2] = w->h_pred[3] = 0;
  w->stream = w->own_stream;
  for (int i = 0; i < avgpu_world::RING; i++) {
    for (int k = 0; k <= NUM_CLASSES; k++)
      if (hipEventCreate(&w->ring[i][k]) != hipSuccess) {
        fail(AVGPU_EHIP, "event creation failed"); return nullptr;
      }
  }
  for (int i = 0; i < 64; i++) w->code2op[i] = -1;
  if (setup_world(w, n, test_buffers) < 0) {
    std::string e = g_err;
    avgpu_destroy(w);
    g_err = e;
    return nullptr;
  }
  return w;
}

int copy_tables(avgpu_world* dst, const avgpu_world* src) {
  DevWorld& D = dst->W;
  const DevWorld& S = src->W;
  D.n_ops = S.n_ops; D.rand_total = S.rand_total; D.fill_code = S.fill_code;
  D.n_react = S.n_react;
  D.env_simple = S.env_simple; D.env_react_mask = S.env_react_mask; D.env_once_mask = S.env_once_mask;
  D.no_mut_mask = S.no_mut_mask;                       // (load_instset / load_env derive these)
  D.req_task = S.req_task; D.imm_task = S.imm_task; D.req_react = S.req_react; D.imm_react = S.imm_react;
  D.single_react = S.single_react; D.max_task_cnt = S.max_task_cnt; D.div_req = S.div_req;
  // the source's tables as its stream leaves them, into the destination on its own
  HIPCHK(hipStreamSynchronize(src->stream));
  HIPCHK(hipMemcpyAsync(D.task_tab, S.task_tab, 32 * sizeof(double), hipMemcpyDeviceToDevice, dst->stream));
  HIPCHK(hipMemcpyAsync(D.react_tab, S.react_tab, AVGPU_MAX_REACTIONS * RT_STRIDE * sizeof(int32_t),
                        hipMemcpyDeviceToDevice, dst->stream));
  HIPCHK(hipMemcpyAsync(D.rand_lut, S.rand_lut, 256, hipMemcpyDeviceToDevice, dst->stream));
  HIPCHK(hipMemcpyAsync(D.rand_cum, S.rand_cum, 64 * sizeof(int32_t), hipMemcpyDeviceToDevice, dst->stream));
  HIPCHK(hipMemcpyAsync(D.rand_code, S.rand_code, 64, hipMemcpyDeviceToDevice, dst->stream));
  HIPCHK(hipStreamSynchronize(dst->stream));
  dst->n_ops = src->n_ops;
  memcpy(dst->op2code, src->op2code, sizeof(dst->op2code));
  memcpy(dst->code2op, src->code2op, sizeof(dst->code2op));
  dst->instset_loaded = src->instset_loaded;
  dst->env_loaded = src->env_loaded;
  return 0;
}

int ready(avgpu_world* w) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  if (!w->instset_loaded) return fail(AVGPU_ESTATE, "avgpu_load_instset not called");
  if (!w->env_loaded) return fail(AVGPU_ESTATE, "avgpu_load_env not called");
  return 0;
}

int translate_genomes(avgpu_world* w, const uint8_t* genomes, const int32_t* lens, int64_t count,
                      std::vector<uint8_t>& codes, std::vector<int32_t>& offsets) {
  codes.clear();
  offsets.resize(count);
  size_t off = 0;
  for (int64_t i = 0; i < count; i++) {
    const int len = lens[i];
    if (len < 1 || len > AVGPU_MAX_GENOME) return fail(AVGPU_EINVAL, "genome length out of range");
    offsets[i] = (int32_t)codes.size();
    for (int k = 0; k < len; k++) {
      const uint8_t op = genomes[off + k];
      if (op >= w->n_ops) return fail(AVGPU_EINVAL, "genome op outside instruction set");
      codes.push_back(w->op2code[op]);
    }
    off += len;
    while (codes.size() & 3) codes.push_back(0);
  }
  if (codes.empty()) codes.push_back(0);
  return 0;
}

// the serial world's reaper queue (W.reaper: a ring of reaper_cap cells,
// positions [reaper_ix[0], reaper_ix[1]) from the rear), rear first
int reaper_read(avgpu_world* w, std::vector<int32_t>& q) {
  const DevWorld& W = w->W;
  int64_t ix[2];
  COPY_SYNC(w, ix, W.reaper_ix, sizeof(ix), hipMemcpyDeviceToHost);
  std::vector<int32_t> ring((size_t)W.reaper_cap);
  COPY_SYNC(w, ring.data(), W.reaper, ring.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
  if (ix[1] < ix[0] || ix[1] - ix[0] > W.reaper_cap) return fail(AVGPU_ESTATE, "reaper queue indices");
  q.clear();
  for (int64_t p = ix[0]; p < ix[1]; p++) q.push_back(ring[(size_t)(p % W.reaper_cap)]);
  return 0;
}
int reaper_write(avgpu_world* w, const std::vector<int32_t>& q) {
  const DevWorld& W = w->W;
  if ((int64_t)q.size() > W.reaper_cap) return fail(AVGPU_EUNSUPPORTED, "reaper queue longer than 2n + 64");
  std::vector<int32_t> ring((size_t)W.reaper_cap, 0);
  std::copy(q.begin(), q.end(), ring.begin());
  const int64_t ix[2] = {W.reaper_cap, W.reaper_cap + (int64_t)q.size()};   // position cap + k = slot k
  COPY_SYNC(w, W.reaper, ring.data(), ring.size() * sizeof(int32_t), hipMemcpyHostToDevice);
  COPY_SYNC(w, W.reaper_ix, ix, sizeof(ix), hipMemcpyHostToDevice);
  return 0;
}

// the queue as the reference has it after Setup and the injections of the
// living cells (oracle reaper_setup): cells 0..N-1 pushed, then every living
// cell in ascending order
int reaper_build(avgpu_world* w) {
  const DevWorld& W = w->W;
  std::vector<uint32_t> ctl((size_t)W.n);
  COPY_SYNC(w, ctl.data(), W.ctl, (size_t)W.n * sizeof(uint32_t), hipMemcpyDeviceToHost);
  std::vector<int32_t> q;
  for (int64_t c = 0; c < W.n; c++) q.push_back((int32_t)c);
  for (int64_t c = 0; c < W.n; c++) if (ctl[(size_t)c] & CTL_ALIVE) q.push_back((int32_t)c);
  w->reaper_rebuild = false;
  return reaper_write(w, q);
}

int set_orgs_impl(avgpu_world* w, int64_t first, int64_t count, const uint8_t* genomes,
                  const int32_t* lens, const double* merits, const int32_t* inputs, int det) {
  if (first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (count == 0) return 0;
  // a serial BIRTH_METHOD 5 world whose reaper queue exists: the injections'
  // queue entries (oracle reaper_inject; InjectGenome main/cPopulation.cc:
  // 6964-6968, ActivateOrganism :1358-1361), on the host (injection is rare)
  if (w->W.reaper && w->cfg.birth_method == 5 && !w->reaper_rebuild) {
    std::vector<uint32_t> ctl((size_t)count);
    COPY_SYNC(w, ctl.data(), w->W.ctl + first, (size_t)count * sizeof(uint32_t), hipMemcpyDeviceToHost);
    std::vector<int32_t> q;
    int qrc = reaper_read(w, q);
    if (qrc < 0) return qrc;
    for (int64_t i = 0; i < count; i++) {
      const int32_t c = (int32_t)(first + i);
      if (ctl[(size_t)i] & CTL_ALIVE) {
        for (size_t k = q.size(); k-- > 0;)      // the first entry from the front (the newest end)
          if (q[k] == c) { q.erase(q.begin() + (std::ptrdiff_t)k); break; }
      }
      q.push_back(c);
    }
    if ((qrc = reaper_write(w, q)) < 0) return qrc;
  }
  std::vector<uint8_t> codes;
  std::vector<int32_t> offsets;
  int rc = translate_genomes(w, genomes, lens, count, codes, offsets);
  if (rc < 0) return rc;
  uint8_t* d_codes = nullptr;
  int32_t *d_off = nullptr, *d_len = nullptr, *d_in = nullptr;
  double* d_m = nullptr;
  HIPCHK(hipMalloc(&d_codes, codes.size()));
  HIPCHK(hipMalloc(&d_off, count * sizeof(int32_t)));
  HIPCHK(hipMalloc(&d_len, count * sizeof(int32_t)));
  HIPCHK(hipMemcpyAsync(d_codes, codes.data(), codes.size(), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(d_off, offsets.data(), count * sizeof(int32_t), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(d_len, lens, count * sizeof(int32_t), hipMemcpyHostToDevice, w->stream));
  if (merits) {
    HIPCHK(hipMalloc(&d_m, count * sizeof(double)));
    HIPCHK(hipMemcpyAsync(d_m, merits, count * sizeof(double), hipMemcpyHostToDevice, w->stream));
  }
  if (inputs) {
    HIPCHK(hipMalloc(&d_in, 3 * count * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(d_in, inputs, 3 * count * sizeof(int32_t), hipMemcpyHostToDevice, w->stream));
  }
  launch_set_orgs(w->W, w->stream, first, count, d_codes, d_off, d_len, d_m, d_in, det);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(w->stream));
  hipFree(d_codes); hipFree(d_off); hipFree(d_len);
  if (d_m) hipFree(d_m);
  if (d_in) hipFree(d_in);
  return 0;
}

int drain_ring(avgpu_world* w, int keep) {
  while (w->ring_count > keep) {
    const int i = (w->ring_head - w->ring_count + avgpu_world::RING) % avgpu_world::RING;
    const int nk = class_timing_all() ? NUM_CLASSES : 1;   // class 0 only: 2 events
    HIPCHK(hipEventSynchronize(w->ring[i][nk]));
    for (int k = 0; k < nk; k++) {
      float f = 0.f;
      HIPCHK(hipEventElapsedTime(&f, w->ring[i][k], w->ring[i][k + 1]));
      w->acc_class_ms[k] += f;
      w->acc_ms += f;
    }
    w->acc_phases++;
    w->ring_count--;
  }
  return 0;
}

// point d_W at a device copy of the world descriptor equal to the host copy,
// uploading it into the other slot when neither holds it.  The upload is
// stream-ordered after every launch queued before it (the only readers of
// that slot: the aux streams of AVGPU_NO_MIX join the stream within their
// update, avgpu_set_stream synchronises), from pinned staging whose last
// upload is waited for -- no stream synchronisation on the update path
// (it cost ~30 us of idle GPU per configs[4] update, whose resource buffers
// swap every update).
int push_world(avgpu_world* w) {
  for (int k = 0; k < 2; k++)
    if (w->validv[k] && memcmp(&w->pushedv[k], &w->W, sizeof(DevWorld)) == 0) {
      w->cur_w = k;
      w->d_W = w->d_Wv[k];
      return 0;
    }
  const int k = 1 - w->cur_w;
  HIPCHK(hipEventSynchronize(w->ev_stage[k]));
  memcpy(&w->h_stage[k], &w->W, sizeof(DevWorld));
  HIPCHK(hipMemcpyAsync(w->d_Wv[k], &w->h_stage[k], sizeof(DevWorld), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipEventRecord(w->ev_stage[k], w->stream));
  memcpy(&w->pushedv[k], &w->W, sizeof(DevWorld));
  w->validv[k] = true;
  w->cur_w = k;
  w->d_W = w->d_Wv[k];
  return 0;
}

int interpret(avgpu_world* w, int mode, int64_t first, int64_t count, bool sorted = false) {
  int launches = 0;
  {
    const int prc = push_world(w);
    if (prc < 0) return prc;
  }
  int rc = drain_ring(w, avgpu_world::RING - 1);
  if (rc < 0) return rc;
  const bool timed = w->time_every > 0 && (w->interp_calls++ % w->time_every) == 0;
  const int i = w->ring_head;
  if (timed) HIPCHK(hipEventRecord(w->ring[i][0], w->stream));
  launch_interpret_classes(w->W, w->d_W, mode, w->stream, first, count, &launches,
                           timed ? &w->ring[i][1] : nullptr, sorted,
                           sorted ? w->aux_stream : nullptr, w->ev_fork, w->ev_join);
  HIPCHK(hipGetLastError());
  if (timed) {
    w->ring_head = (i + 1) % avgpu_world::RING;
    w->ring_count++;
  }
  w->last_launches = launches;
  return 0;
}

int update_run(avgpu_world* w, const double* dev_totals, avgpu_update_stats* out);

// An update's batch steps (oracle choose_k): avgpu_cfg.sub_updates
// when set; else the more of two rules over the last step's predictor: with E
// its weight term in mean weights per organism (the total weight's expected
// move within the update), ceil(E / 0.05) steps above E = 0.1; with D the
// fraction of organisms it expects to divide within the densest quarter of
// the update (a cohort in lock step; a steady state spreads its divides over
// the four), ceil(D / 0.15) steps above D = 0.3; one step otherwise, at most
// ADAPT_KMAX.
constexpr int ADAPT_KMAX = 16;
int choose_k(const avgpu_cfg& c, long long pred, long long n, bool handed_in, long long cnt) {
  if (c.sub_updates > 0) return c.sub_updates;
  if (handed_in || c.slicing_method != AVGPU_SLICE_PROBABILISTIC || n <= 0) return 1;
  const double a = (double)(pred < 0 ? -pred : pred), dn = (double)n;
  int k = 1;
  if (a > 104857.6 * dn) k = std::max(k, (int)std::ceil(a / (52428.8 * dn)));
  if ((double)cnt > 0.3 * dn) k = std::max(k, (int)std::ceil((double)cnt / (0.15 * dn)));
  return std::min(k, ADAPT_KMAX);
}

}  // namespace

// ===========================================================================
extern "C" {

const char* avgpu_last_error(void) { return g_err.c_str(); }

void avgpu_cfg_defaults(avgpu_cfg* c) {
  memset(c, 0, sizeof(*c));
  c->world_x = 60; c->world_y = 60; c->world_geometry = 2;
  c->ave_time_slice = 30; c->slicing_method = 1; c->base_merit_method = 4;
  c->base_const_merit = 100; c->default_bonus = 1.0;
  c->copy_mut_prob = 0.0075; c->divide_ins_prob = 0.05; c->divide_del_prob = 0.05;
  c->offspring_size_range = 2.0; c->min_copied_lines = 0.5; c->min_exe_lines = 0.5;
  c->require_allocate = 1; c->death_method = 2; c->age_limit = 20; c->alloc_method = 0;
  c->divide_method = 1; c->max_label_exe_size = 1; c->birth_method = 0; c->prefer_empty = 1;
  c->allow_parent = 1; c->test_cpu_time_mod = 20; c->inherit_merit = 1;
  c->seed = 101;
  // main/cAvidaConfig.h defaults of the refused knobs that are not 0
  c->special_mut_line = -1; c->generation_inc_method = 1;
  c->required_task = -1; c->immunity_task = -1;
  c->required_reaction = -1; c->immunity_reaction = -1;
  c->max_unique_task_count = -1;
}

avgpu_world* avgpu_create(const avgpu_cfg* cfg, int device, int64_t num_cells) {
  return create_world(cfg, device, num_cells, false);
}

int avgpu_check_cfg(const avgpu_cfg* cfg) {
  if (!cfg) return fail(AVGPU_EINVAL, "cfg is NULL");
  const std::string why = unsupported_cfg(*cfg);
  if (!why.empty()) return fail(AVGPU_EUNSUPPORTED, why + " is not on the GPU path");
  return 0;
}

int avgpu_destroy(avgpu_world* w) {
  if (!w) return 0;
  if (w->stream) hipStreamSynchronize(w->stream);
  if (w->own_stream) hipStreamSynchronize(w->own_stream);
  for (void* p : w->allocs) hipFree(p);
  if (w->rec_buf) hipFree(w->rec_buf);
  for (double* p : w->srec_buf) if (p) hipFree(p);
  if (w->ev0) hipEventDestroy(w->ev0);
  if (w->ev1) hipEventDestroy(w->ev1);
  for (int i = 0; i < avgpu_world::RING; i++) {
    for (int k = 0; k <= NUM_CLASSES; k++)
      if (w->ring[i][k]) hipEventDestroy(w->ring[i][k]);
  }
  if (w->own_stream) hipStreamDestroy(w->own_stream);
  for (int k = 0; k < 3; k++) {
    if (w->aux_stream[k]) { hipStreamSynchronize(w->aux_stream[k]); hipStreamDestroy(w->aux_stream[k]); }
    if (w->ev_join[k]) hipEventDestroy(w->ev_join[k]);
  }
  if (w->ev_fork) hipEventDestroy(w->ev_fork);
  if (w->h_pred) hipHostFree(w->h_pred);
  if (w->h_stage) hipHostFree(w->h_stage);
  for (int k = 0; k < 2; k++)
    if (w->ev_stage[k]) hipEventDestroy(w->ev_stage[k]);
  delete w;
  return 0;
}

int avgpu_set_stream(avgpu_world* w, void* hip_stream) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  HIPCHK(hipStreamSynchronize(w->stream));
  // NULL is the HIP null stream -- the stream PyTorch's default current
  // stream reports as 0 -- not the handle's own stream
  w->stream = reinterpret_cast<hipStream_t>(hip_stream);
  return 0;
}

int avgpu_sync(avgpu_world* w) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  HIPCHK(hipStreamSynchronize(w->stream));
  return 0;
}

int avgpu_load_instset(avgpu_world* w, int n, const uint8_t* handler_id, const int32_t* redundancy) {
  if (!w || n <= 0 || n > AVGPU_MAX_INST) return fail(AVGPU_EINVAL, "instruction set size");
  int32_t cum[64] = {0};
  uint8_t code[64] = {0};
  bool used[64] = {false};
  int32_t total = 0;
  for (int i = 0; i < 64; i++) w->code2op[i] = -1;
  for (int i = 0; i < n; i++) {
    const int h = handler_id[i];
    if (h < 0 || h >= AVGPU_H_COUNT) return fail(AVGPU_EINVAL, "unknown handler id");
    if (used[h]) return fail(AVGPU_EUNSUPPORTED, "handler mapped twice (non-injective instset)");
    if (h < 3 && h != i) return fail(AVGPU_EUNSUPPORTED, "nops must be ops 0..2 in A,B,C order");
    used[h] = true;
    total += redundancy ? redundancy[i] : 1;
    cum[i] = total;
    code[i] = (uint8_t)h;
    w->op2code[i] = (uint8_t)h;
    w->code2op[h] = (int16_t)i;
  }
  if (total <= 0) return fail(AVGPU_EINVAL, "zero total redundancy");
  // NO_MUT_INSTS over the handler codes the tapes hold (op i's symbol:
  // Instruction::GetSymbol, core/InstructionSequence.cc:69-106, its first
  // character -- '+', '-', '~', '?' past op 61)
  uint64_t nomut = 0;
  for (int i = 0; i < n; i++) {
    const int k = i % 62;
    const char sym = i >= 62 ? "+-~?"[std::min(i / 62, 4) - 1]
                             : (char)(k < 26 ? 'a' + k : (k < 52 ? 'A' + k - 26 : '0' + k - 52));
    if (memchr(w->cfg.no_mut_insts, sym, (size_t)w->cfg.no_mut_insts_len)) nomut |= 1ull << code[i];
  }
  w->W.no_mut_mask = nomut;
  w->n_ops = n;
  w->W.n_ops = n;
  w->W.rand_total = total;
  w->W.fill_code = code[0];
  HIPCHK(hipMemcpyAsync(w->W.rand_cum, cum, sizeof(cum), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(w->W.rand_code, code, sizeof(code), hipMemcpyHostToDevice, w->stream));
  // GetRandomInst as one table lookup when the weights fit (cpu/cInstSet.cc:83-88)
  uint8_t rlut[256];
  memset(rlut, 0, sizeof(rlut));
  if (total <= 256)
    for (int v = 0, i = 0; v < total; v++) {
      while (i < n - 1 && cum[i] <= v) i++;
      rlut[v] = code[i];
    }
  HIPCHK(hipMemcpyAsync(w->W.rand_lut, rlut, sizeof(rlut), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  w->instset_loaded = true;
  return 0;
}

int avgpu_load_env(avgpu_world* w, int nreact, const avgpu_reaction* r) {
  if (!w || nreact < 0 || nreact > AVGPU_MAX_REACTIONS) return fail(AVGPU_EINVAL, "reaction count");
  DevWorld& W = w->W;
  int32_t tab[AVGPU_MAX_REACTIONS * RT_STRIDE];
  memset(tab, 0, sizeof(tab));
  for (int i = 0; i < nreact; i++) {
    if (r[i].task < 0 || r[i].task >= AVGPU_NUM_LOGIC_TASKS) return fail(AVGPU_EINVAL, "task id");
    int32_t* t = tab + i * RT_STRIDE;
    t[RT_TASK] = r[i].task;
    t[RT_TYPE] = r[i].type;
    t[RT_MIN] = r[i].min_count;
    t[RT_MAX] = r[i].max_count;
    t[RT_HASREQ] = r[i].has_requisite;
    t[RT_USED] = 1;
    const double bonus = r[i].max_number * r[i].value;  // DoProcesses: consumed * value
    const double mult = (r[i].type == AVGPU_PROC_POW) ? std::pow(2.0, bonus) : bonus;
    memcpy(t + RT_MULT, &mult, 8);
    memcpy(t + RT_ADD, &bonus, 8);
  }
  W.n_react = nreact;
  // cOrganism::Divide_CheckViable's requirements (main/cOrganism.cc:788-919):
  // REQUIRED_TASK / IMMUNITY_TASK index the task library -- the distinct
  // tasks in the order of their first REACTION line (cTaskLib::AddTask) --,
  // the reaction knobs the reactions in environment order
  {
    int lib[AVGPU_MAX_REACTIONS], nlib = 0;
    for (int i = 0; i < nreact; i++) {
      bool seen = false;
      for (int k = 0; k < nlib; k++) seen = seen || lib[k] == r[i].task;
      if (!seen) lib[nlib++] = r[i].task;
    }
    const avgpu_cfg& c = w->cfg;
    auto task_of = [&](int t) { return t >= 0 && t < nlib ? lib[t] : -2; };
    W.req_task = c.required_task >= 0 ? task_of(c.required_task) : -1;
    W.imm_task = c.immunity_task >= 0 ? task_of(c.immunity_task) : -1;
    if (W.req_task == -2 || W.imm_task == -2)
      return fail(AVGPU_EUNSUPPORTED, "REQUIRED_TASK / IMMUNITY_TASK past the environment's task library");
    if (c.required_reaction >= nreact || c.immunity_reaction >= nreact)
      return fail(AVGPU_EUNSUPPORTED, "REQUIRED_REACTION / IMMUNITY_REACTION past the environment's reactions");
    if (c.require_single_reaction && nreact > 12)
      return fail(AVGPU_EUNSUPPORTED, "REQUIRE_SINGLE_REACTION with more than 12 reactions");
    W.req_react = c.required_reaction;
    W.imm_react = c.immunity_reaction;
    W.single_react = c.require_single_reaction ? 1 : 0;
    W.max_task_cnt = c.max_unique_task_count;
    W.div_req = (W.req_task >= 0 || (!W.single_react && W.req_react >= 0) || W.single_react ||
                 W.max_task_cnt > 0) ? 1 : 0;
  }
  // simple-environment fast path of the IO task check (interp.hip)
  double ttab[32];
  for (int t = 0; t < 16; t++) { ttab[t] = 1.0; ttab[16 + t] = 0.0; }
  bool simple = true;
  uint32_t rmask = 0, omask = 0;
  for (int i = 0; i < nreact; i++) {
    const int32_t* t = tab + i * RT_STRIDE;
    if (t[RT_TASK] != i) simple = false;
    if (t[RT_HASREQ]) {
      if (t[RT_MIN] > 0) simple = false;
      else if (t[RT_MAX] == 1) omask |= 1u << i;
      else if (t[RT_MAX] != INT32_MAX) simple = false;
    }
    rmask |= 1u << i;
    double m, a;
    memcpy(&m, t + RT_MULT, 8);
    memcpy(&a, t + RT_ADD, 8);
    if (t[RT_TYPE] == AVGPU_PROC_ADD) ttab[16 + i] = a; else ttab[i] = m;
  }
  // resource-bound processes (cEnvironment::DoProcesses): the general path
  double rr[AVGPU_MAX_REACTIONS * RR_STRIDE];
  memset(rr, 0, sizeof(rr));
  int uses = 0;
  uint32_t res_seen = 0, res_mask = 0;
  for (int i = 0; i < nreact; i++) {
    const int res = r[i].resource;       // 1 + index, 0 = infinite
    if (res == 0) continue;
    if (res < 0 || res > W.n_res) return fail(AVGPU_EINVAL, "reaction names an unknown resource");
    if (res_seen & (1u << (res - 1)))
      return fail(AVGPU_EUNSUPPORTED, "a resource consumed by two reactions is not on the GPU path");
    res_seen |= 1u << (res - 1);
    double* q = rr + i * RR_STRIDE;
    q[RR_RES] = (double)res;
    q[RR_SPATIAL] = w->res_geom[res - 1] != AVGPU_RES_GLOBAL ? 1.0 : 0.0;
    q[RR_DEPL] = r[i].depletable ? 1.0 : 0.0;
    q[RR_TYPE] = (double)r[i].type;
    q[RR_FRAC] = r[i].max_fraction > 1.0 ? 1.0 : r[i].max_fraction;
    q[RR_MIN] = r[i].min_number;
    q[RR_MAX] = r[i].max_number;
    q[RR_VALUE] = r[i].value;
    uses++;
    res_mask |= 1u << i;
  }
  W.env_resources = uses ? 1 : 0;
  W.env_res_mask = simple ? res_mask : 0u;   // the simple path indexes reactions by task
  HIPCHK(hipMemcpyAsync(W.react_res, rr, sizeof(rr), hipMemcpyHostToDevice, w->stream));
  W.env_simple = simple ? 1 : 0;
  W.env_react_mask = rmask;
  W.env_once_mask = omask;
  HIPCHK(hipMemcpyAsync(W.task_tab, ttab, sizeof(ttab), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(W.react_tab, tab, sizeof(tab), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  w->env_loaded = true;
  return 0;
}

int avgpu_set_org(avgpu_world* w, int64_t cell, const uint8_t* genome, int len, double merit,
                  const int32_t* inputs) {
  int rc = ready(w);
  if (rc < 0) return rc;
  const int32_t l = len;
  return set_orgs_impl(w, cell, 1, genome, &l, merit > 0 ? &merit : nullptr, inputs, 0);
}

int avgpu_set_orgs(avgpu_world* w, int64_t first, int64_t count, const uint8_t* genomes,
                   const int32_t* lens, const double* merits, const int32_t* inputs, int det) {
  int rc = ready(w);
  if (rc < 0) return rc;
  return set_orgs_impl(w, first, count, genomes, lens, merits, inputs, det);
}

int avgpu_kill(avgpu_world* w, int64_t cell) {
  if (!w || cell < 0 || cell >= w->W.n) return fail(AVGPU_EINVAL, "cell");
  uint32_t ctl = 0;
  COPY_SYNC(w, &ctl, w->W.ctl + cell, 4, hipMemcpyDeviceToHost);
  ctl &= ~CTL_ALIVE;
  COPY_SYNC(w, w->W.ctl + cell, &ctl, 4, hipMemcpyHostToDevice);
  return 0;
}

int avgpu_step(avgpu_world* w, int64_t first, int64_t count, const int32_t* budget,
               int32_t budget_uniform, int mode) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (mode < 0 || mode > 2) return fail(AVGPU_EINVAL, "mode");
  if (mode == AVGPU_MODE_TEST && !w->has_test_buffers)
    return fail(AVGPU_ESTATE, "TEST mode needs a test world (avgpu_test_genomes)");
  if (count == 0) return 0;
  // budgets are below 2^30 (bit 30 tags spilled slices on device, device.h)
  if (!budget && (budget_uniform < 0 || budget_uniform >= BUDGET_PRIM))
    return fail(AVGPU_EINVAL, "budget out of range [0, 2^30)");
  if (budget)
    for (int64_t i = 0; i < count; i++)
      if (budget[i] < 0 || budget[i] >= BUDGET_PRIM) return fail(AVGPU_EINVAL, "budget out of range [0, 2^30)");
  int32_t* d_b = nullptr;
  if (budget) {
    HIPCHK(hipMalloc(&d_b, count * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(d_b, budget, count * sizeof(int32_t), hipMemcpyHostToDevice, w->stream));
  }
  // the update's counters and queue lengths cleared -- an earlier update run
  // without statistics has its counts folded into the running sums first
  launch_reset_counts(w->W, w->stream);
  launch_classify_uniform(w->W, w->stream, first, count, d_b, budget_uniform);
  HIPCHK(hipGetLastError());
  rc = interpret(w, mode, first, count);
  if (d_b) { hipStreamSynchronize(w->stream); hipFree(d_b); }
  return rc;
}

// after launch_world_pre: the spatial step wrote res_amount_alt; later
// launches read the new amounts
static void after_resources_begin(avgpu_world* w) {
  DevWorld& W = w->W;
  if (res_stepped(W)) std::swap(W.res_amount, W.res_amount_alt);
  W.res_first = 0;
}

int avgpu_update_totals(avgpu_world* w, double* dev_totals) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (!dev_totals) return fail(AVGPU_EINVAL, "dev_totals is NULL");
  launch_merit_total(w->W, w->stream, dev_totals, w->d_totals + 8);
  HIPCHK(hipGetLastError());
  return 0;
}

int avgpu_update_run(avgpu_world* w, const double* dev_totals, avgpu_update_stats* out) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (w->cfg.birth_method == 5)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 5 (the reaper queue) runs on the serial world only");
  if (!dev_totals) return fail(AVGPU_EINVAL, "dev_totals is NULL");
  if (w->cfg.sub_updates > 1)
    return fail(AVGPU_EUNSUPPORTED, "sub_updates > 1 needs the world's own totals (no handed-in totals)");
  // every world's {total weight, organisms} -> this world's share of the
  // picks (cMultiProcessWorld::CalculateUpdateSize) and its allotment; one
  // batch step (choose_k: handed-in totals)
  if (dev_totals != w->d_totals)
    HIPCHK(hipMemcpyAsync(w->d_totals, dev_totals, 2 * sizeof(double), hipMemcpyDeviceToDevice, w->stream));
  w->pred_pending = false;
  launch_world_pre(w->W, w->stream, w->d_totals, w->d_totals + 8, w->ev_fork, (uint32_t)w->update);
  after_resources_begin(w);
  HIPCHK(hipGetLastError());
  rc = interpret(w, AVGPU_MODE_WORLD, 0, w->W.n, true);
  if (rc < 0) return rc;
  launch_world_post(w->W, w->stream, (uint32_t)w->update, 0, 1);
  launch_newborns(w->W, w->d_W, w->stream);
  // statistics only when asked for: a run without them (out == NULL) leaves
  // the reduction to avgpu_get_stats / avgpu_stats_vector, or skips it
  launch_world_end(w->W, w->stream, w->d_stats, out != nullptr);
  HIPCHK(hipGetLastError());
  w->last_k = 1;
  w->stats_stale = out == nullptr;
  w->update++;
  if (out) return avgpu_get_stats(w, out);
  return 0;
}

int avgpu_run_update(avgpu_world* w, avgpu_update_stats* out) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (w->cfg.birth_method == 5)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 5 (the reaper queue) runs on the serial world only");
  if (w->use_global) {                 // totals handed in (avgpu_update_totals / tiles)
    w->use_global = false;
    return avgpu_update_run(w, w->d_totals, out);
  }
  // K batch steps (choose_k: avgpu_cfg.sub_updates, or the
  // last update's predictor), each: total merit, allotment, class lists and
  // the class-0 order; interpretation; placement; the newborn pass.  The
  // predictor comes back by mapped memory from the last step's placement:
  // the host waits for it (here, at the next update) while the GPU runs the
  // rest of that update.
  if (w->pred_pending) {
    // the last step's placement launch published the predictor into
    // coherent mapped memory, then its sequence number (k_place_claim0): the
    // host polls that instead of an event on the stream (an event record
    // there left ~6 us of dead time per update before the next launch)
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(w->h_pred + 3, __ATOMIC_ACQUIRE) != w->pred_seq) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        HIPCHK(hipStreamSynchronize(w->stream));   // a fault surfaces here
        if (__atomic_load_n(w->h_pred + 3, __ATOMIC_ACQUIRE) != w->pred_seq)
          return fail(AVGPU_EHIP, "the batch-step predictor was never published");
      }
    }
    w->pred_acc = __atomic_load_n(w->h_pred + 0, __ATOMIC_ACQUIRE);
    w->pred_n = __atomic_load_n(w->h_pred + 1, __ATOMIC_ACQUIRE);
    w->pred_cnt = __atomic_load_n(w->h_pred + 2, __ATOMIC_ACQUIRE);
    w->pred_pending = false;
  }
  const int K = choose_k(w->cfg, w->pred_acc, w->pred_n, false, w->pred_cnt);
  for (int sub = 0; sub < K; sub++) {
    const uint32_t key = (uint32_t)w->update * (uint32_t)K + (uint32_t)sub;
    launch_world_begin(w->W, w->stream, w->d_totals, w->d_totals + 8, w->ev_fork, key, sub, K);
    if (sub == 0) after_resources_begin(w);
    HIPCHK(hipGetLastError());
    rc = interpret(w, AVGPU_MODE_WORLD, 0, w->W.n, true);
    if (rc < 0) return rc;
    const bool last = sub == K - 1;
    if (last) w->pred_seq++;
    launch_world_post(w->W, w->stream, key, sub, K, last ? w->d_pred : nullptr, w->pred_seq);
    launch_newborns(w->W, w->d_W, w->stream);
    // statistics only when asked for: a run without them (out == NULL) leaves
    // the reduction to avgpu_get_stats / avgpu_stats_vector, or skips it
    launch_world_end(w->W, w->stream, w->d_stats, out != nullptr && last);
    HIPCHK(hipGetLastError());
  }
  w->pred_pending = true;
  w->last_k = K;
  w->stats_stale = out == nullptr;
  w->update++;
  if (out) return avgpu_get_stats(w, out);
  return 0;
}

// the serial world's state, allocated on first use: merit sum tree,
// speculative credits, connection-list facings, the scheduler's and the
// context's counter streams (keyed by the seed, as the oracle's)
static int serial_alloc(avgpu_world* w) {
  DevWorld& W = w->W;
  if (W.stree) return 0;
  int rc;
  int64_t size = 1;
  while (size < W.n) size <<= 1;
  W.stree_size = size;
  if ((rc = w->alloc(&W.stree, (size_t)(2 * size))) < 0) return rc;
  if ((rc = w->alloc(&W.spec, (size_t)W.n)) < 0) return rc;
  if ((rc = w->alloc(&W.face, (size_t)W.n)) < 0) return rc;
  if ((rc = w->alloc(&W.grng, 3)) < 0) return rc;
  if ((rc = w->alloc(&W.sctx, 3)) < 0) return rc;
  if (w->cfg.birth_method == 5) {
    // the reaper queue (oracle reaper_setup): Setup's cells 0..N-1, then the
    // living cells in ascending order, each pushed at the front
    const int64_t cap = 2 * W.n + 64;
    if ((rc = w->alloc(&W.reaper, (size_t)cap)) < 0) return rc;
    if ((rc = w->alloc(&W.reaper_ix, 2)) < 0) return rc;
    W.reaper_cap = cap;
    if ((rc = reaper_build(w)) < 0) return rc;
  }
  uint32_t g[3] = {0, 0, 0}, x[3] = {0, 0, 0};
  const uint64_t seed = (uint64_t)w->cfg.seed;
  derive_key((uint32_t)seed, (uint32_t)(seed >> 32), 0x5CEDu, 0xC0FFEEu, g[0], g[1]);
  derive_key((uint32_t)seed, (uint32_t)(seed >> 32), 0xC7C7u, 0x5EED5u, x[0], x[1]);
  HIPCHK(hipMemcpyAsync(W.grng, g, sizeof(g), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(W.sctx, x, sizeof(x), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  return 0;
}

int avgpu_set_serial_streams(avgpu_world* w, const double* sched, int64_t n_sched, const double* ctx,
                             int64_t n_ctx) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  if ((sched && n_sched <= 0) || (ctx && n_ctx <= 0)) return fail(AVGPU_EINVAL, "empty stream");
  int rc = serial_alloc(w);
  if (rc < 0) return rc;
  DevWorld& W = w->W;
  HIPCHK(hipStreamSynchronize(w->stream));   // no queued serial update still reads them
  for (double** p : {&w->srec_buf[0], &w->srec_buf[1]})
    if (*p) { hipFree(*p); *p = nullptr; }
  W.srec_sched = nullptr; W.srec_sched_n = 0; W.srec_ctx = nullptr; W.srec_ctx_n = 0;
  if (sched) {
    HIPCHK(hipMalloc(&w->srec_buf[0], (size_t)n_sched * sizeof(double)));
    COPY_SYNC(w, w->srec_buf[0], sched, (size_t)n_sched * sizeof(double), hipMemcpyHostToDevice);
    W.srec_sched = w->srec_buf[0]; W.srec_sched_n = n_sched;
  }
  if (ctx) {
    HIPCHK(hipMalloc(&w->srec_buf[1], (size_t)n_ctx * sizeof(double)));
    COPY_SYNC(w, w->srec_buf[1], ctx, (size_t)n_ctx * sizeof(double), hipMemcpyHostToDevice);
    W.srec_ctx = w->srec_buf[1]; W.srec_ctx_n = n_ctx;
  }
  // both positions restart at 0 (counter streams: their counters)
  HIPCHK(hipMemsetAsync(W.grng + 2, 0, 4, w->stream));
  HIPCHK(hipMemsetAsync(W.sctx + 2, 0, 4, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  return 0;
}

int avgpu_get_serial_state(avgpu_world* w, avgpu_serial_state* st, int32_t* spec, uint8_t* face,
                           int32_t* soup_perm, int32_t* reaper, int64_t reaper_cap) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  const DevWorld& W = w->W;
  const int64_t n = W.n;
  const bool started = W.stree != nullptr;     // serial_alloc ran (a serial update, or a set state)
  uint32_t g[3] = {0, 0, 0}, x[3] = {0, 0, 0};
  if (started) {
    COPY_SYNC(w, g, W.grng, sizeof(g), hipMemcpyDeviceToHost);
    COPY_SYNC(w, x, W.sctx, sizeof(x), hipMemcpyDeviceToHost);
  }
  std::vector<int32_t> q;
  const bool have_q = W.reaper && !w->reaper_rebuild;
  if (have_q) {
    int rc = reaper_read(w, q);
    if (rc < 0) return rc;
  }
  if (st) {
    memset(st, 0, sizeof(*st));
    st->sched_pos = g[2];
    st->ctx_pos = x[2];
    st->reaper_len = have_q ? (int64_t)q.size() : -1;
    st->started = started ? 1 : 0;
  }
  if (spec) {
    std::vector<uint32_t> ctl((size_t)n);
    COPY_SYNC(w, ctl.data(), W.ctl, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (started) COPY_SYNC(w, spec, W.spec, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost);
    for (int64_t c = 0; c < n; c++)
      spec[c] = (started ? (spec[c] & 0xFFFF) : 0) | ((ctl[(size_t)c] & CTL_SPECDIE) ? 1 << 16 : 0);
  }
  if (face) {
    if (started) COPY_SYNC(w, face, W.face, (size_t)n, hipMemcpyDeviceToHost);
    else memset(face, 0, (size_t)n);
  }
  if (soup_perm) {
    if (W.soup_perm) COPY_SYNC(w, soup_perm, W.soup_perm, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost);
    else for (int64_t c = 0; c < n; c++) soup_perm[c] = (int32_t)c;
  }
  if (reaper && !q.empty()) {
    if (reaper_cap < (int64_t)q.size()) return fail(AVGPU_EINVAL, "reaper buffer too small");
    std::copy(q.begin(), q.end(), reaper);
  }
  return 0;
}

int avgpu_set_serial_state(avgpu_world* w, const avgpu_serial_state* st, const int32_t* spec, const uint8_t* face,
                           const int32_t* soup_perm, const int32_t* reaper) {
  if (!w || !st) return fail(AVGPU_EINVAL, "serial state");
  if (!st->started) return 0;
  DevWorld& W = w->W;
  const int64_t n = W.n, len = st->reaper_len;
  if (soup_perm) {
    std::vector<char> seen((size_t)n, 0);
    for (int64_t c = 0; c < n; c++) {
      if (soup_perm[c] < 0 || soup_perm[c] >= n || seen[(size_t)soup_perm[c]])
        return fail(AVGPU_EINVAL, "soup_perm is not a permutation of the cells");
      seen[(size_t)soup_perm[c]] = 1;
    }
  }
  if (len > 2 * n + 64) return fail(AVGPU_EINVAL, "reaper queue longer than 2n + 64");
  if (len > 0 && !reaper) return fail(AVGPU_EINVAL, "reaper queue");
  for (int64_t k = 0; k < len; k++)
    if (reaper[k] < 0 || reaper[k] >= n) return fail(AVGPU_EINVAL, "reaper queue cell out of range");
  int rc = serial_alloc(w);
  if (rc < 0) return rc;
  const uint32_t gp = (uint32_t)st->sched_pos, xp = (uint32_t)st->ctx_pos;
  COPY_SYNC(w, W.grng + 2, &gp, 4, hipMemcpyHostToDevice);
  COPY_SYNC(w, W.sctx + 2, &xp, 4, hipMemcpyHostToDevice);
  if (spec) {
    std::vector<int32_t> cr((size_t)n);
    std::vector<uint32_t> ctl((size_t)n);
    COPY_SYNC(w, ctl.data(), W.ctl, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    for (int64_t c = 0; c < n; c++) {
      cr[(size_t)c] = spec[c] & 0xFFFF;
      ctl[(size_t)c] = (ctl[(size_t)c] & ~CTL_SPECDIE) | (((spec[c] >> 16) & 1) ? CTL_SPECDIE : 0u);
    }
    COPY_SYNC(w, W.spec, cr.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice);
    COPY_SYNC(w, W.ctl, ctl.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (face) COPY_SYNC(w, W.face, face, (size_t)n, hipMemcpyHostToDevice);
  if (soup_perm && W.soup_perm) COPY_SYNC(w, W.soup_perm, soup_perm, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice);
  if (W.reaper) {
    if (len < 0) {
      w->reaper_rebuild = true;                      // built again at the next serial update
    } else {
      w->reaper_rebuild = false;
      if ((rc = reaper_write(w, std::vector<int32_t>(reaper, reaper + len))) < 0) return rc;
    }
  }
  return 0;
}

int avgpu_run_serial_updates(avgpu_world* w, int n, avgpu_update_stats* last) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (n < 0) return fail(AVGPU_EINVAL, "n_updates < 0");
  DevWorld& W = w->W;
  if (W.rec) return fail(AVGPU_EUNSUPPORTED, "the serial world takes its own two streams (avgpu_set_serial_streams), "
                                             "not per-organism recorded streams");
  if (W.tiled) return fail(AVGPU_EUNSUPPORTED, "the serial world runs single worlds, not strip tiles");
  if (W.birth_method == 1 || W.birth_method == 2)
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 1 / 2 run on the batch world, not the serial world");
  if ((rc = serial_alloc(w)) < 0) return rc;
  if (w->reaper_rebuild && (rc = reaper_build(w)) < 0) return rc;
  for (int u = 0; u < n; u++) {
    launch_reset_counts(W, w->stream);
    launch_age_tick(W, w->stream);
    launch_resources_begin(W, w->stream);
    after_resources_begin(w);
    if ((rc = push_world(w)) < 0) return rc;
    launch_serial_update(W, w->d_W, w->stream);
    launch_serial_post(W, w->stream, w->d_stats);
    HIPCHK(hipGetLastError());
    w->stats_stale = false;
    w->update++;
  }
  if (last) return avgpu_get_stats(w, last);
  return 0;
}

int avgpu_run_updates(avgpu_world* w, int n, avgpu_update_stats* last) {
  for (int i = 0; i < n; i++) {
    int rc = avgpu_run_update(w, nullptr);
    if (rc < 0) return rc;
  }
  if (last) return avgpu_get_stats(w, last);
  return 0;
}

int avgpu_get_stats(avgpu_world* w, avgpu_update_stats* out) {
  if (!w || !out) return fail(AVGPU_EINVAL, "args");
  double v[45];
  if (w->stats_stale) {
    launch_stats(w->W, w->stream, w->d_stats);
    HIPCHK(hipGetLastError());
    w->stats_stale = false;
  }
  HIPCHK(hipMemcpyAsync(v, w->d_stats, sizeof(v), hipMemcpyDeviceToHost, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  memset(out, 0, sizeof(*out));
  out->update = w->update - 1;
  out->num_organisms = (int64_t)v[0];
  out->sum_merit = v[1];
  out->sum_fitness = v[2];
  out->sum_gestation = v[3];
  out->sum_genome_length = v[4];
  out->max_fitness = v[5];
  out->ave_generation = v[0] > 0 ? v[6] / v[0] : 0.0;
  for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) out->task_orgs[t] = (int64_t)v[8 + t];
  out->insts_executed = (int64_t)v[24];
  out->deaths = (int64_t)v[25];
  out->divides = (int64_t)v[26];
  out->births = (int64_t)v[27];
  out->births_dropped = (int64_t)v[28];
  out->sum_mem_size = v[7];
  out->cum_insts_executed = (int64_t)v[30];
  out->cum_births = (int64_t)v[31];
  out->slices = (int64_t)v[32];
  out->lane_steps = (int64_t)v[33];
  out->births_overwritten = (int64_t)v[34];
  out->births_cancelled = (int64_t)v[35];
  out->seed = w->cfg.seed;
  out->insts_wasted = (int64_t)v[36];
  memcpy(&out->sched_pred, v + 37, 8);        // (int64 bits)
  memcpy(&out->sched_carry, v + 38, 8);
  out->sched_pred_n = (int64_t)v[39];
  memcpy(&out->sched_pred_cnt, v + 40, 8);
  for (int q = 0; q < 4; q++) memcpy(&out->sched_pred_bins[q], v + 41 + q, 8);
  out->sub_steps = w->last_k;
  return 0;
}

int avgpu_get_census(avgpu_world* w, int64_t first, int64_t count, avgpu_census* out) {
  if (!w || !out || first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (count == 0) return 0;
  avgpu_census* d = nullptr;
  HIPCHK(hipMalloc(&d, count * sizeof(avgpu_census)));
  launch_get_census(w->W, w->stream, first, count, d);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, d, count * sizeof(avgpu_census), hipMemcpyDeviceToHost, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  hipFree(d);
  return 0;
}

int avgpu_state_digests(avgpu_world* w, int64_t first, int64_t count, uint64_t* out) {
  if (!w || !out || first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (count == 0) return 0;
  uint64_t* d = nullptr;
  HIPCHK(hipMalloc(&d, count * sizeof(uint64_t)));
  launch_state_digest(w->W, w->stream, first, count, d);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, d, count * sizeof(uint64_t), hipMemcpyDeviceToHost, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  hipFree(d);
  return 0;
}

int avgpu_set_rng_mode(avgpu_world* w, int mode, const double* stream, int64_t n, const int64_t* offsets) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  DevWorld& W = w->W;
  HIPCHK(hipStreamSynchronize(w->stream));
  if (mode == AVGPU_RNG_COUNTER) {
    W.rec = nullptr;
    W.rec_n = 0;
    if (W.rec_off) SET_SYNC(w, W.rec_off, 0xFF, W.n * sizeof(int64_t));   // -1: counter streams
    return 0;
  }
  if (mode != AVGPU_RNG_RECORDED || !stream || n <= 0) return fail(AVGPU_EINVAL, "rng mode / stream");
  std::vector<int64_t> off(W.n, 0);
  if (offsets)
    for (int64_t c = 0; c < W.n; c++) {
      if (offsets[c] < 0 || offsets[c] > n) return fail(AVGPU_EINVAL, "stream offset outside the stream");
      off[c] = offsets[c];
    }
  if (w->rec_buf) { hipFree(w->rec_buf); w->rec_buf = nullptr; }
  HIPCHK(hipMalloc(&w->rec_buf, n * sizeof(double)));
  COPY_SYNC(w, w->rec_buf, stream, n * sizeof(double), hipMemcpyHostToDevice);
  if (!W.rec_off) {
    HIPCHK(hipMalloc(&W.rec_off, W.n * sizeof(int64_t)));
    w->allocs.push_back(W.rec_off);
  }
  COPY_SYNC(w, W.rec_off, off.data(), W.n * sizeof(int64_t), hipMemcpyHostToDevice);
  W.rec = w->rec_buf;
  W.rec_n = n;
  // every organism's position in its segment starts at 0
  SET_SYNC(w, W.rng + 2 * W.n, 0, W.n * sizeof(uint32_t));
  return 0;
}

int avgpu_set_genotype_keys(avgpu_world* w, int64_t first, int64_t count, const uint64_t* keys) {
  if (!w || !keys || first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (count == 0) return 0;
  HIPCHK(hipMemcpyAsync(w->W.gkey + first, keys, count * sizeof(uint64_t), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  return 0;
}

int avgpu_get_states(avgpu_world* w, int64_t first, int64_t count, avgpu_cpu_state* states,
                     uint8_t* mem_ops, uint8_t* mem_flags, int mem_cap) {
  if (!w || first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (count == 0) return 0;
  avgpu_cpu_state* d_s = nullptr;
  uint8_t* d_c = nullptr;
  const bool want_mem = mem_ops && mem_flags && mem_cap > 0;
  HIPCHK(hipMalloc(&d_s, count * sizeof(avgpu_cpu_state)));
  if (want_mem) {
    HIPCHK(hipMalloc(&d_c, (size_t)count * mem_cap));
    HIPCHK(hipMemsetAsync(d_c, 0, (size_t)count * mem_cap, w->stream));
  }
  launch_get_states(w->W, w->stream, first, count, d_s, d_c, mem_cap);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(states, d_s, count * sizeof(avgpu_cpu_state), hipMemcpyDeviceToHost, w->stream));
  std::vector<uint8_t> codes;
  if (want_mem) {
    codes.resize((size_t)count * mem_cap);
    HIPCHK(hipMemcpyAsync(codes.data(), d_c, codes.size(), hipMemcpyDeviceToHost, w->stream));
  }
  HIPCHK(hipStreamSynchronize(w->stream));
  hipFree(d_s);
  if (d_c) hipFree(d_c);
  if (want_mem) {
    for (int64_t i = 0; i < count; i++) {
      const int m = std::min(states[i].mem_size, mem_cap);
      for (int k = 0; k < mem_cap; k++) {
        const size_t o = (size_t)i * mem_cap + k;
        if (k < m) {
          const uint8_t b = codes[o];
          const int op = w->code2op[b & CODE_MASK];
          mem_ops[o] = (uint8_t)(op < 0 ? 255 : op);
          mem_flags[o] = (uint8_t)(((b & TF_COPIED) ? 0x01 : 0) | ((b & TF_EXEC) ? 0x04 : 0));
        } else {
          mem_ops[o] = 0;
          mem_flags[o] = 0;
        }
      }
    }
  }
  return 0;
}

int avgpu_set_states(avgpu_world* w, int64_t first, int64_t count, const avgpu_cpu_state* states,
                     const uint8_t* mem_ops, const uint8_t* mem_flags, int mem_cap) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (first < 0 || count < 0 || first + count > w->W.n) return fail(AVGPU_EINVAL, "cell range");
  if (!states || !mem_ops || !mem_flags || mem_cap <= 0) return fail(AVGPU_EINVAL, "states / memory");
  if (count == 0) return 0;
  std::vector<uint8_t> codes((size_t)count * mem_cap, 0);
  for (int64_t i = 0; i < count; i++) {
    const avgpu_cpu_state& st = states[i];
    if (st.mem_size < 0 || st.mem_size > AVGPU_MAX_GENOME || st.mem_size > mem_cap)
      return fail(AVGPU_EINVAL, "memory size outside the tape / mem_cap");
    for (int k = 0; k < st.mem_size; k++) {
      const size_t o = (size_t)i * mem_cap + k;
      if (mem_ops[o] >= w->n_ops) return fail(AVGPU_EINVAL, "op code outside the instruction set");
      codes[o] = (uint8_t)(w->op2code[mem_ops[o]] | ((mem_flags[o] & 0x01) ? TF_COPIED : 0) |
                           ((mem_flags[o] & 0x04) ? TF_EXEC : 0));
    }
  }
  avgpu_cpu_state* d_s = nullptr;
  uint8_t* d_c = nullptr;
  HIPCHK(hipMalloc(&d_s, count * sizeof(avgpu_cpu_state)));
  HIPCHK(hipMalloc(&d_c, codes.size()));
  HIPCHK(hipMemcpyAsync(d_s, states, count * sizeof(avgpu_cpu_state), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(d_c, codes.data(), codes.size(), hipMemcpyHostToDevice, w->stream));
  launch_set_states(w->W, w->stream, first, count, d_s, d_c, mem_cap);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(w->stream));
  hipFree(d_s);
  hipFree(d_c);
  return 0;
}

int avgpu_set_clock(avgpu_world* w, const avgpu_update_stats* last) {
  if (!w || !last) return fail(AVGPU_EINVAL, "args");
  double v[2] = {(double)last->cum_insts_executed, (double)last->cum_births};
  HIPCHK(hipMemcpyAsync(w->d_stats + 30, v, sizeof(v), hipMemcpyHostToDevice, w->stream));
  // the running sums k_stats_final adds each update to
  const unsigned long long ci = (unsigned long long)last->cum_insts_executed;
  const unsigned long long cb = (unsigned long long)last->cum_births;
  HIPCHK(hipMemcpyAsync(w->W.counters + CNT_CUM_INSTS, &ci, sizeof(ci), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemcpyAsync(w->W.counters + CNT_CUM_BIRTHS, &cb, sizeof(cb), hipMemcpyHostToDevice, w->stream));
  // the sums given are complete: the current shards are not folded in again
  static const unsigned long long one = 1ull;
  HIPCHK(hipMemcpyAsync(w->W.counters + CNT_CUM_FLAG, &one, sizeof(one), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  w->update = last->update + 1;
  // the scheduler's key (the world's RANDOM_SEED) comes with the clock; a
  // zero seed (stats from an older checkpoint, or not from avgpu_get_stats)
  // keeps the configured one
  if (last->seed != 0) {
    w->cfg.seed = last->seed;
    w->W.seed_lo = (uint32_t)last->seed;
    w->W.seed_hi = (uint32_t)(last->seed >> 32);
    // the serial world's two streams are keyed by the seed too (serial_alloc;
    // their positions stay)
    if (w->W.grng) {
      uint32_t g[2], x[2];
      derive_key((uint32_t)last->seed, (uint32_t)(last->seed >> 32), 0x5CEDu, 0xC0FFEEu, g[0], g[1]);
      derive_key((uint32_t)last->seed, (uint32_t)(last->seed >> 32), 0xC7C7u, 0x5EED5u, x[0], x[1]);
      HIPCHK(hipMemcpyAsync(w->W.grng, g, sizeof(g), hipMemcpyHostToDevice, w->stream));
      HIPCHK(hipMemcpyAsync(w->W.sctx, x, sizeof(x), hipMemcpyHostToDevice, w->stream));
      HIPCHK(hipStreamSynchronize(w->stream));
    }
  }
  // the batch-step predictor and the pick carry
  w->pred_acc = last->sched_pred;
  w->pred_n = last->sched_pred_n;
  w->pred_cnt = std::max(std::max(last->sched_pred_bins[0], last->sched_pred_bins[1]),
                          std::max(last->sched_pred_bins[2], last->sched_pred_bins[3]));
  w->pred_pending = false;
  const long long sv[5] = {0, 0, last->sched_carry, 0, 0};
  HIPCHK(hipMemcpyAsync(w->W.sched, sv, sizeof(sv), hipMemcpyHostToDevice, w->stream));
  // the predictor into shard 0 (device.h pacc_sum), the other shards zero
  std::vector<long long> pa(NSHARD * PACC_STRIDE, 0);
  pa[0] = last->sched_pred;
  pa[1] = (long long)((uint64_t)last->sched_pred_bins[0] | ((uint64_t)last->sched_pred_bins[1] << 32));
  pa[2] = (long long)((uint64_t)last->sched_pred_bins[2] | ((uint64_t)last->sched_pred_bins[3] << 32));
  HIPCHK(hipMemcpyAsync(w->W.pacc, pa.data(), pa.size() * sizeof(long long), hipMemcpyHostToDevice, w->stream));
  const double nv = (double)last->sched_pred_n;
  HIPCHK(hipMemcpyAsync(w->d_totals + 1, &nv, sizeof(nv), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  return 0;
}

int avgpu_test_genomes(avgpu_world* w, int n, const uint8_t* genomes, const int32_t* lens,
                       avgpu_test_result* results, char* executed_flags, int flags_cap,
                       uint8_t* offspring) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (n <= 0) return 0;
  avgpu_cfg tc = w->cfg;
  tc.copy_mut_prob = 0; tc.divide_mut_prob = 0; tc.divide_ins_prob = 0; tc.divide_del_prob = 0;
  avgpu_world* t = create_world(&tc, w->device, n, true);
  if (!t) return AVGPU_ENOMEM;
  if ((rc = copy_tables(t, w)) < 0) { avgpu_destroy(t); return rc; }
  if ((rc = set_orgs_impl(t, 0, n, genomes, lens, nullptr, nullptr, 1)) < 0) { avgpu_destroy(t); return rc; }
  std::vector<int32_t> budget(n);
  for (int i = 0; i < n; i++) budget[i] = w->cfg.test_cpu_time_mod * lens[i];
  if ((rc = avgpu_step(t, 0, n, budget.data(), 0, AVGPU_MODE_TEST)) < 0) { avgpu_destroy(t); return rc; }
  std::vector<avgpu_cpu_state> st(n);
  std::vector<uint8_t> ops((size_t)n * AVGPU_MAX_GENOME), fl((size_t)n * AVGPU_MAX_GENOME);
  if ((rc = avgpu_get_states(t, 0, n, st.data(), ops.data(), fl.data(), AVGPU_MAX_GENOME)) < 0) {
    avgpu_destroy(t); return rc;
  }
  std::vector<uint8_t> tflags((size_t)n * TAPE_SLOT), tchild((size_t)n * TAPE_SLOT);
  std::vector<int32_t> tflen(n), tclen(n);
  // (checked: a failed copy would hand back uninitialised flags and offspring)
  const hipError_t ce[4] = {
      hipMemcpyAsync(tflags.data(), t->W.t_flags, tflags.size(), hipMemcpyDeviceToHost, t->stream),
      hipMemcpyAsync(tchild.data(), t->W.t_child, tchild.size(), hipMemcpyDeviceToHost, t->stream),
      hipMemcpyAsync(tflen.data(), t->W.t_flags_len, n * 4, hipMemcpyDeviceToHost, t->stream),
      hipMemcpyAsync(tclen.data(), t->W.t_child_len, n * 4, hipMemcpyDeviceToHost, t->stream)};
  const hipError_t se = hipStreamSynchronize(t->stream);
  for (hipError_t e : {ce[0], ce[1], ce[2], ce[3], se})
    if (e != hipSuccess) {
      avgpu_destroy(t);
      return fail(AVGPU_EHIP, std::string("test_genomes copy: ") + hipGetErrorString(e));
    }
  size_t off = 0;
  for (int i = 0; i < n; i++) {
    avgpu_test_result& r = results[i];
    const avgpu_cpu_state& s = st[i];
    memset(&r, 0, sizeof(r));
    r.divided = s.num_divides > 0;
    r.copied_size = s.copied_size;
    r.executed_size = s.executed_size;
    r.gestation_time = s.gestation_time;
    r.genome_length = s.genome_length;
    r.time_used = s.time_used;
    r.merit = s.merit;
    r.fitness = s.fitness;
    for (int k = 0; k < AVGPU_MAX_REACTIONS; k++) r.task_count[k] = s.last_task_count[k];
    r.offspring_len = r.divided ? tclen[i] : 0;
    bool same = r.divided && tclen[i] == lens[i];
    for (int k = 0; same && k < lens[i]; k++)
      same = (w->code2op[tchild[(size_t)i * TAPE_SLOT + k]] == genomes[off + k]);
    r.copy_true = same;
    if (executed_flags && flags_cap > 0) {
      char* dst = executed_flags + (size_t)i * flags_cap;
      memset(dst, 0, flags_cap);
      if (r.divided) {
        const int m = std::min(tflen[i], flags_cap - 1);
        memcpy(dst, tflags.data() + (size_t)i * TAPE_SLOT, m);
      } else {
        const int m = std::min(s.mem_size, flags_cap - 1);
        for (int k = 0; k < m; k++) dst[k] = (fl[(size_t)i * AVGPU_MAX_GENOME + k] & 0x04) ? '+' : '-';
      }
    }
    if (offspring) {
      uint8_t* d = offspring + (size_t)i * AVGPU_MAX_GENOME;
      memset(d, 0, AVGPU_MAX_GENOME);
      for (int k = 0; k < r.offspring_len; k++)
        d[k] = (uint8_t)w->code2op[tchild[(size_t)i * TAPE_SLOT + k]];
    }
    off += lens[i];
  }
  avgpu_destroy(t);
  return 0;
}

int avgpu_stats_vector(avgpu_world* w, void** dev_ptr) {
  if (!w || !dev_ptr) return fail(AVGPU_EINVAL, "args");
  if (w->stats_stale) {           // the vector is complete once this stream reaches it
    launch_stats(w->W, w->stream, w->d_stats);
    HIPCHK(hipGetLastError());
    w->stats_stale = false;
  }
  *dev_ptr = w->d_stats;
  return 0;
}

int avgpu_set_global_totals(avgpu_world* w, double total_merit, int64_t total_orgs) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  double v[2] = {total_merit, (double)total_orgs};
  HIPCHK(hipMemcpyAsync(w->d_totals, v, sizeof(v), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  w->use_global = true;
  return 0;
}

// ---- resources (resources.hip; DESIGN.md "Resources") ----
// initial amounts of this world's cells (cResourceCount::Setup: RateAll(
// initial / size) + StateAll, main/cResourceCount.cc:323-328; SetCellList:
// Rate + State, main/cSpatialResCount.cc:216-231; a strip tile seeds its rows)
static int res_seed(avgpu_world* w) {
  DevWorld& W = w->W;
  HIPCHK(hipStreamSynchronize(w->stream));   // res_param may still be in flight
  const int64_t n = W.n, nglobal = (int64_t)W.world_x * W.world_y;
  const int nres = (int)w->res_spec.size();
  ResParam P[AVGPU_MAX_RESOURCES];
  COPY_SYNC(w, P, W.res_param, sizeof(P), hipMemcpyDeviceToHost);
  double glob[AVGPU_MAX_RESOURCES];
  memset(glob, 0, sizeof(glob));
  if (W.n_spatial) {
    std::vector<double> amt((size_t)W.n_spatial * n);
    for (int r = 0; r < nres; r++) {
      if (P[r].slot < 0) continue;
      const double per = w->res_spec[r].initial / (double)nglobal;
      for (int64_t c = 0; c < n; c++) amt[(size_t)P[r].slot * n + c] = 0.0 + per;
    }
    for (const avgpu_cell_resource& e : w->cell_spec) {
      const int64_t l = e.cell - W.cell0;
      if (e.cell >= 0 && e.cell < nglobal && l >= 0 && l < n) {
        double& a = amt[(size_t)P[e.resource].slot * n + l];
        a = a + (0.0 + e.initial);
      }
    }
    HIPCHK(hipMemcpyAsync(W.res_amount, amt.data(), amt.size() * sizeof(double), hipMemcpyHostToDevice, w->stream));
  }
  for (int r = 0; r < nres; r++) glob[r] = P[r].slot < 0 ? w->res_spec[r].initial : 0.0;
  HIPCHK(hipMemcpyAsync(W.res_global, glob, sizeof(glob), hipMemcpyHostToDevice, w->stream));
  HIPCHK(hipMemsetAsync(W.res_cons, 0, AVGPU_MAX_RESOURCES * sizeof(unsigned long long), w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  W.res_first = 1;
  return 0;
}

int avgpu_load_resources(avgpu_world* w, int nres, const avgpu_resource* res, int ncell,
                         const avgpu_cell_resource* cells) {
  if (!w || nres < 0 || nres > AVGPU_MAX_RESOURCES || ncell < 0 || (ncell && !cells) || (nres && !res))
    return fail(AVGPU_EINVAL, "resource arguments");
  DevWorld& W = w->W;
  int nsp = 0;
  ResParam P[AVGPU_MAX_RESOURCES];
  memset(P, 0, sizeof(P));
  for (int r = 0; r < nres; r++) {
    const avgpu_resource& q = res[r];
    if (q.geometry < 0 || q.geometry > 2) return fail(AVGPU_EINVAL, "resource geometry");
    if (q.initial < 0 || q.inflow < 0 || q.outflow < 0 || q.outflow > 1)
      return fail(AVGPU_EINVAL, "resource initial / inflow / outflow out of range");
    ResParam& p = P[r];
    p.geometry = q.geometry;
    p.slot = q.geometry == AVGPU_RES_GLOBAL ? -1 : nsp++;
    p.in_x1 = q.inflow_x1; p.in_x2 = q.inflow_x2; p.in_y1 = q.inflow_y1; p.in_y2 = q.inflow_y2;
    p.out_x1 = q.outflow_x1; p.out_x2 = q.outflow_x2; p.out_y1 = q.outflow_y1; p.out_y2 = q.outflow_y2;
    const double decay = 1.0 - q.outflow;                        // cPopulation.cc:440
    // Source: amount / cells of the inflow rectangle (cSpatialResCount.cc:341-353)
    const double boxcells = (double)(p.in_y2 - p.in_y1 + 1) * (double)(p.in_x2 - p.in_x1 + 1) * 1.0;
    p.in_share = q.inflow / boxcells;
    p.sink_frac = 1.0 - decay;
    p.has_sink = (p.out_x1 != AVGPU_RES_NONE && p.out_y1 != AVGPU_RES_NONE &&
                  p.out_x2 != AVGPU_RES_NONE && p.out_y2 != AVGPU_RES_NONE) ? 1 : 0;
    p.xdiffuse = q.xdiffuse; p.ydiffuse = q.ydiffuse; p.xgravity = q.xgravity; p.ygravity = q.ygravity;
    p.flows = (q.xdiffuse != 0.0 || q.ydiffuse != 0.0 || q.xgravity != 0.0 || q.ygravity != 0.0) ? 1 : 0;
    p.in_all = (p.in_x2 - p.in_x1 + 1 == W.world_x && p.in_y2 - p.in_y1 + 1 == W.world_y) ? 1 : 0;
    p.out_all = (p.out_x2 - p.out_x1 + 1 == W.world_x && p.out_y2 - p.out_y1 + 1 == W.world_y) ? 1 : 0;
    // precalc tables (cResourceCount.cc:336-345), the reference's own loop
    const double step_decay = std::pow(decay, 1.0 / 10000.0), step_inflow = q.inflow * (1.0 / 10000.0);
    double dp = 1.0, ip = 0.0;
    for (int i = 1; i <= 100; i++) {
      dp = dp * step_decay;
      ip = ip * step_decay + step_inflow;
      if (i == 99) { p.decay99 = dp; p.inflow99 = ip; }
    }
    p.decay100 = dp; p.inflow100 = ip;
    w->res_geom[r] = q.geometry;
    W.res_spatial_host[r] = q.geometry != AVGPU_RES_GLOBAL;
    W.res_flows_host[r] = (int8_t)p.flows;
    W.res_grav_host[r] = (int8_t)(q.xgravity != 0.0 || q.ygravity != 0.0);
    W.res_cells_host[r] = 0;
  }
  for (int i = 0; i < ncell; i++) {
    if (cells[i].resource < 0 || cells[i].resource >= nres || res[cells[i].resource].geometry == AVGPU_RES_GLOBAL)
      return fail(AVGPU_EINVAL, "CELL entry names a resource that is not spatial");
    W.res_cells_host[cells[i].resource] = 1;
  }
  const int64_t n = W.n;
  if ((int64_t)W.world_x * W.world_y >= (int64_t)1 << 31)
    return fail(AVGPU_EUNSUPPORTED, "resources need fewer than 2^31 cells in the world");
  if (nsp && !W.res_amount) {
    HIPCHK(hipMalloc(&W.res_amount, (size_t)AVGPU_MAX_RESOURCES * n * sizeof(double)));
    w->allocs.push_back(W.res_amount);
    HIPCHK(hipMalloc(&W.res_amount_alt, (size_t)AVGPU_MAX_RESOURCES * n * sizeof(double)));
    w->allocs.push_back(W.res_amount_alt);
    HIPCHK(hipMalloc(&W.res_delta, (size_t)(n + 64) * sizeof(double)));   // + k_res_step's junk lanes
    w->allocs.push_back(W.res_delta);
  }
  if (nres && !W.cons) {   // each cell's consumption in a step (newborn credit)
    HIPCHK(hipMalloc(&W.cons, (size_t)AVGPU_MAX_RESOURCES * n * sizeof(double)));
    w->allocs.push_back(W.cons);
    HIPCHK(hipMemsetAsync(W.cons, 0, (size_t)AVGPU_MAX_RESOURCES * n * sizeof(double), w->stream));
  }
  if (ncell) {
    if (W.res_cells) hipFree(W.res_cells);
    HIPCHK(hipMalloc(&W.res_cells, ncell * sizeof(avgpu_cell_resource)));
    HIPCHK(hipMemcpyAsync(W.res_cells, cells, ncell * sizeof(avgpu_cell_resource), hipMemcpyHostToDevice, w->stream));
  }
  W.n_res = nres;
  W.n_cellres = ncell;
  W.n_spatial = nsp;
  w->res_spec.assign(res, res + nres);
  w->cell_spec.assign(cells, cells + ncell);
  HIPCHK(hipMemcpyAsync(W.res_param, P, sizeof(P), hipMemcpyHostToDevice, w->stream));
  return res_seed(w);
}

int avgpu_set_resources(avgpu_world* w, const double* levels, const double* spatial) {
  if (!w || !levels) return fail(AVGPU_EINVAL, "args");
  DevWorld& W = w->W;
  double glob[AVGPU_MAX_RESOURCES];
  ResParam P[AVGPU_MAX_RESOURCES];
  COPY_SYNC(w, glob, W.res_global, sizeof(glob), hipMemcpyDeviceToHost);
  COPY_SYNC(w, P, W.res_param, sizeof(P), hipMemcpyDeviceToHost);
  for (int r = 0; r < W.n_res; r++) {
    if (P[r].slot < 0) { glob[r] = levels[r]; continue; }
    if (!spatial) return fail(AVGPU_EINVAL, "spatial resources need their grids");
    COPY_SYNC(w, W.res_amount + (size_t)P[r].slot * W.n, spatial + (size_t)r * W.n, W.n * sizeof(double),
              hipMemcpyHostToDevice);
  }
  COPY_SYNC(w, W.res_global, glob, sizeof(glob), hipMemcpyHostToDevice);
  SET_SYNC(w, W.res_cons, 0, AVGPU_MAX_RESOURCES * sizeof(unsigned long long));
  W.res_first = 0;
  return 0;
}

int avgpu_get_resources(avgpu_world* w, double* levels, double* spatial) {
  if (!w || !levels) return fail(AVGPU_EINVAL, "args");
  DevWorld& W = w->W;
  double glob[AVGPU_MAX_RESOURCES];
  ResParam P[AVGPU_MAX_RESOURCES];
  COPY_SYNC(w, glob, W.res_global, sizeof(glob), hipMemcpyDeviceToHost);
  COPY_SYNC(w, P, W.res_param, sizeof(P), hipMemcpyDeviceToHost);
  std::vector<double> row(W.n);
  for (int r = 0; r < W.n_res; r++) {
    if (P[r].slot < 0) {
      levels[r] = glob[r];
      if (spatial) memset(spatial + (size_t)r * W.n, 0, W.n * sizeof(double));
      continue;
    }
    COPY_SYNC(w, row.data(), W.res_amount + (size_t)P[r].slot * W.n, W.n * sizeof(double),
              hipMemcpyDeviceToHost);
    double sum = 0.0;                                   // cStats::PrintResourceData order
    for (int64_t c = 0; c < W.n; c++) sum += row[c];
    levels[r] = sum;
    if (spatial) memcpy(spatial + (size_t)r * W.n, row.data(), W.n * sizeof(double));
  }
  return 0;
}

// ---- strip tiles (DESIGN.md "Multi-GPU") ----
int avgpu_set_tile(avgpu_world* w, int64_t row0, int64_t arena_bytes) {
  if (w && (w->cfg.birth_method == 1 || w->cfg.birth_method == 2))
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 1 / 2 on strip tiles (the ghost rows carry no age or merit)");
  if (w && (w->cfg.birth_method == 4 || w->cfg.birth_method == 5))
    return fail(AVGPU_EUNSUPPORTED, "BIRTH_METHOD 4 / 5 on strip tiles (a soup birth may land in any strip)");
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  DevWorld& W = w->W;
  const int64_t X = W.world_x;
  if (X <= 0 || W.n % X) return fail(AVGPU_EINVAL, "tile cells must be whole rows of WORLD_X");
  const int64_t rows = W.n / X;
  if (rows < 2) return fail(AVGPU_EINVAL, "a tile needs at least 2 rows");
  if (W.n % 256) return fail(AVGPU_EINVAL, "tile cells must be a multiple of 256 (merit blocks)");
  if (row0 < 0 || row0 + rows > W.global_rows)
    return fail(AVGPU_EINVAL, "tile rows outside WORLD_Y (the global row count)");
  if (arena_bytes <= 0) arena_bytes = std::max<int64_t>(256 * 1024, X * 256);
  arena_bytes = (arena_bytes + 15) / 16 * 16;
  W.row0 = (int32_t)row0;
  W.rows = (int32_t)rows;
  W.tiled = rows < W.global_rows ? 1 : 0;
  W.cell0 = row0 * X;
  W.r_arena = arena_bytes;
  w->tile_buffers = false;
  W.rs_send[0] = W.rs_send[1] = W.rs_recv[0] = W.rs_recv[1] = nullptr;
  if (W.n_res) return res_seed(w);   // this strip's share of the initial amounts
  return 0;
}

int avgpu_tile_res_bytes(avgpu_world* w, int64_t* bytes) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  if (bytes) *bytes = (int64_t)w->W.n_spatial * w->W.world_x * (int64_t)sizeof(double);
  return 0;
}

int avgpu_set_tile_res_buffers(avgpu_world* w, void* send_up, void* send_down, void* recv_up,
                               void* recv_down) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  if (!w->W.tiled) return fail(AVGPU_ESTATE, "avgpu_set_tile did not make this world a strip tile");
  if (w->W.n_spatial && (!send_up || !send_down || !recv_up || !recv_down))
    return fail(AVGPU_EINVAL, "NULL tile resource buffer");
  DevWorld& W = w->W;
  W.rs_send[0] = (double*)send_up; W.rs_send[1] = (double*)send_down;
  W.rs_recv[0] = (double*)recv_up; W.rs_recv[1] = (double*)recv_down;
  return 0;
}

int avgpu_tile_res_cons(avgpu_world* w, uint64_t* dev_out) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (!dev_out) return fail(AVGPU_EINVAL, "dev_out is NULL");
  HIPCHK(hipMemcpyAsync(dev_out, w->W.res_cons, AVGPU_MAX_RESOURCES * sizeof(unsigned long long),
                        hipMemcpyDeviceToDevice, w->stream));
  int g = 0;
  for (int r = 0; r < w->W.n_res; r++) g += w->res_geom[r] == AVGPU_RES_GLOBAL;
  return g;
}

int avgpu_tile_res_settle(avgpu_world* w, const uint64_t* dev_sum) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (!dev_sum) return fail(AVGPU_EINVAL, "dev_sum is NULL");
  launch_resources_settle(w->W, w->stream, (const unsigned long long*)dev_sum);
  HIPCHK(hipGetLastError());
  return 0;
}

int avgpu_tile_buffer_bytes(avgpu_world* w, int64_t* partial_bytes, int64_t* halo_b, int64_t* record_b) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  if (partial_bytes) *partial_bytes = tile_part_stride((w->W.n + 255) / 256) * (int64_t)sizeof(double);
  if (halo_b) *halo_b = halo_bytes(w->W.world_x);
  if (record_b) *record_b = record_bytes(w->W.world_x, w->W.r_arena);
  return 0;
}

int avgpu_set_tile_buffers(avgpu_world* w, void* halo_send_up, void* halo_send_down, void* halo_recv_up,
                           void* halo_recv_down, void* rec_send_up, void* rec_send_down,
                           void* rec_recv_up, void* rec_recv_down) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  if (!w->W.tiled) return fail(AVGPU_ESTATE, "avgpu_set_tile did not make this world a strip tile");
  void* p[8] = {halo_send_up, halo_send_down, halo_recv_up, halo_recv_down,
                rec_send_up, rec_send_down, rec_recv_up, rec_recv_down};
  for (int i = 0; i < 8; i++)
    if (!p[i]) return fail(AVGPU_EINVAL, "NULL tile buffer");
  DevWorld& W = w->W;
  W.h_send[0] = (uint8_t*)p[0]; W.h_send[1] = (uint8_t*)p[1];
  W.h_recv[0] = (uint8_t*)p[2]; W.h_recv[1] = (uint8_t*)p[3];
  W.r_send[0] = (uint8_t*)p[4]; W.r_send[1] = (uint8_t*)p[5];
  W.r_recv[0] = (uint8_t*)p[6]; W.r_recv[1] = (uint8_t*)p[7];
  w->tile_buffers = true;
  return 0;
}

static int tile_ready(avgpu_world* w) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (!w->W.tiled || !w->tile_buffers) return fail(AVGPU_ESTATE, "not a strip tile with registered buffers");
  return 0;
}

int avgpu_tile_partials(avgpu_world* w, double* dev_out) {
  int rc = ready(w);
  if (rc < 0) return rc;
  if (!dev_out) return fail(AVGPU_EINVAL, "dev_out is NULL");
  // a strip's first step of an update clears the update's counters, a later
  // step its queues only (the counts add up over the update)
  launch_tile_partials(w->W, w->stream, dev_out, w->W.tiled ? (w->tile_sub_next == 0 ? 1 : 2) : 0);
  if (w->W.tiled) launch_resources_pack(w->W, w->stream);
  HIPCHK(hipGetLastError());
  return 0;
}

// the update's batch steps from every strip's predictor (the gathered
// partials' tails) and the organisms of the last step (the same on every strip)
int avgpu_tile_steps(avgpu_world* w, const double* dev_gathered, int ntiles, int* k_out) {
  int rc = tile_ready(w);
  if (rc < 0) return rc;
  if (!dev_gathered || ntiles < 1 || !k_out) return fail(AVGPU_EINVAL, "gathered partials / k_out");
  const int64_t nb = (w->W.n + 255) / 256, stride = tile_part_stride(nb);
  std::vector<double> tail((size_t)(6 * ntiles));
  for (int k = 0; k < ntiles; k++)
    HIPCHK(hipMemcpyAsync(tail.data() + 6 * k, dev_gathered + k * stride + 2 * nb, 6 * sizeof(double),
                          hipMemcpyDeviceToHost, w->stream));
  double n = 0.0;
  HIPCHK(hipMemcpyAsync(&n, w->d_totals + 1, sizeof(double), hipMemcpyDeviceToHost, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  long long sum = 0, bins[4] = {0, 0, 0, 0};
  for (int k = 0; k < ntiles; k++) {
    long long v;
    memcpy(&v, tail.data() + 6 * k, 8);
    sum += v;
    for (int q = 0; q < 4; q++) {
      long long c;
      memcpy(&c, tail.data() + 6 * k + 2 + q, 8);
      bins[q] += c;
    }
  }
  const long long dens = std::max(std::max(bins[0], bins[1]), std::max(bins[2], bins[3]));
  *k_out = choose_k(w->cfg, sum, (long long)n, false, dens);
  return 0;
}

int avgpu_tile_begin_step(avgpu_world* w, const double* dev_gathered, int ntiles, int sub, int K) {
  int rc = tile_ready(w);
  if (rc < 0) return rc;
  if (w->W.n_spatial && !w->W.rs_recv[0])
    return fail(AVGPU_ESTATE, "spatial resources need avgpu_set_tile_res_buffers");
  if (!dev_gathered || ntiles < 1) return fail(AVGPU_EINVAL, "gathered partials");
  if (K < 1 || K > 64 || sub < 0 || sub >= K) return fail(AVGPU_EINVAL, "batch step sub of K");
  if (K > 1 && w->cfg.slicing_method != AVGPU_SLICE_PROBABILISTIC)
    return fail(AVGPU_EUNSUPPORTED, "batch steps > 1 need SLICING_METHOD 1");
  // the scheduler's top tree spans every strip's blocks
  {
    int64_t P = 1;
    const int64_t nbt = ((w->W.n + 255) / 256) * (int64_t)ntiles;
    while (P < nbt) P <<= 1;
    if (P > w->W.tree_cap) {   // (the smaller buffers stay in the world's allocations)
      if ((rc = w->alloc(&w->W.tree_scr, (size_t)(2 * P))) < 0) return rc;
      if ((rc = w->alloc(&w->W.tree_cnt, (size_t)(2 * P))) < 0) return rc;
      w->W.tree_cap = P;
      const int prc = push_world(w);
      if (prc < 0) return prc;
    }
  }
  // (the counters were cleared by avgpu_tile_partials' launch at step 0)
  const uint32_t key = (uint32_t)w->update * (uint32_t)K + (uint32_t)sub;
  launch_tile_pre(w->W, w->stream, dev_gathered, ntiles, w->d_totals, w->ev_fork, key, sub, K);
  if (sub == 0) after_resources_begin(w);
  HIPCHK(hipGetLastError());
  rc = interpret(w, AVGPU_MODE_WORLD, 0, w->W.n, true);
  if (rc < 0) return rc;
  launch_tile_after_interpret(w->W, w->stream);
  HIPCHK(hipGetLastError());
  w->ntiles_last = ntiles;
  w->tile_sub = sub; w->tile_k = K; w->tile_key = key;
  w->tile_sub_next = sub + 1 < K ? sub + 1 : 0;
  return 0;
}

int avgpu_tile_begin(avgpu_world* w, const double* dev_gathered, int ntiles) {
  return avgpu_tile_begin_step(w, dev_gathered, ntiles, 0, 1);
}

int avgpu_tile_place(avgpu_world* w, int round, int phase) {
  int rc = tile_ready(w);
  if (rc < 0) return rc;
  if (round < 0 || round > 3 || phase < 0 || phase > 3 || (phase >= 1 && phase <= 2 && round != 3) ||
      (phase == 3 && round != 0))
    return fail(AVGPU_EINVAL, "round 0..3 with phase 0, round 0 with phase 3; phases 1, 2 after round 3");
  launch_tile_place(w->W, w->stream, round, phase, w->tile_key, w->tile_sub, w->tile_k);
  HIPCHK(hipGetLastError());
  return 0;
}

int avgpu_tile_finish(avgpu_world* w, avgpu_update_stats* out) {
  int rc = tile_ready(w);
  if (rc < 0) return rc;
  // the received offspring, the step's newborn pass; after the update's last
  // step its statistics
  launch_tile_finish(w->W, w->stream, w->tile_key, w->tile_sub, w->tile_k);
  launch_newborns(w->W, w->d_W, w->stream);
  HIPCHK(hipGetLastError());
  if (w->tile_sub + 1 < w->tile_k) return 0;
  if (out) launch_stats(w->W, w->stream, w->d_stats);
  HIPCHK(hipGetLastError());
  w->stats_stale = out == nullptr;
  w->last_k = w->tile_k;
  w->update++;
  if (out) return avgpu_get_stats(w, out);
  return 0;
}

int avgpu_last_step_insts(avgpu_world* w, int64_t* insts) {
  if (!w || !insts) return fail(AVGPU_EINVAL, "args");
  std::vector<unsigned long long> v(NSHARD * CNT_STRIDE);
  HIPCHK(hipMemcpyAsync(v.data(), w->W.counters, v.size() * 8, hipMemcpyDeviceToHost, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  unsigned long long s = 0;
  for (int sh = 0; sh < NSHARD; sh++) s += v[sh * CNT_STRIDE + CNT_INSTS];
  *insts = (int64_t)s;
  return 0;
}

int avgpu_last_kernel_ms(avgpu_world* w, double* ms, int64_t* launches) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  int rc = drain_ring(w, 0);
  if (rc < 0) return rc;
  if (ms) *ms = w->acc_ms;
  if (launches) *launches = w->acc_phases;
  w->acc_ms = 0.0;
  w->acc_phases = 0;
  for (int k = 0; k < NUM_CLASSES; k++) w->acc_class_ms[k] = 0.0;
  return 0;
}

int avgpu_set_timing(avgpu_world* w, int every) {
  if (!w || every < 0) return fail(AVGPU_EINVAL, "every < 0");
  w->time_every = every;
  w->interp_calls = 0;
  return 0;
}

int avgpu_kernel_times(avgpu_world* w, double* class_ms, int64_t* phases) {
  if (!w) return fail(AVGPU_EINVAL, "NULL world");
  int rc = drain_ring(w, 0);
  if (rc < 0) return rc;
  if (class_ms)
    for (int k = 0; k < NUM_CLASSES; k++) class_ms[k] = w->acc_class_ms[k];
  if (phases) *phases = w->acc_phases;
  w->acc_ms = 0.0;
  w->acc_phases = 0;
  for (int k = 0; k < NUM_CLASSES; k++) w->acc_class_ms[k] = 0.0;
  return 0;
}

int avgpu_counters(avgpu_world* w, int cumulative, int64_t* out, int n) {
  if (!w || !out || n < 0) return fail(AVGPU_EINVAL, "args");
  if (n > AVGPU_NUM_COUNTERS) n = AVGPU_NUM_COUNTERS;
  std::vector<unsigned long long> v(CNT_WORDS);
  HIPCHK(hipMemcpyAsync(v.data(), w->W.counters, v.size() * 8, hipMemcpyDeviceToHost, w->stream));
  HIPCHK(hipStreamSynchronize(w->stream));
  for (int k = 0; k < n; k++) {
    unsigned long long s = 0;
    // (an update run without statistics has its counts still in the shards)
    if (!cumulative || v[CNT_CUM_FLAG] == 0ull)
      for (int sh = 0; sh < NSHARD; sh++) s += v[sh * CNT_STRIDE + k];
    if (cumulative) s += v[CNT_CUM_BASE + k];
    out[k] = (int64_t)s;
  }
  return 0;
}

}  // extern "C"
