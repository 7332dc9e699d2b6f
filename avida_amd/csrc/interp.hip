// interp.hip -- k_interpret: the batched heads-CPU interpreter for gfx950.
//
// Replaces the serial loop Avida2Driver::Run -> cPopulation::ProcessStep ->
// cHardwareCPU::SingleProcess (targets/avida/Avida2Driver.cc:111-116,
// main/cPopulation.cc:5698-5788, cpu/cHardwareCPU.cc:908-1058).
//
// One organism per wavefront lane; 64-thread workgroups (one wave each).
// On-chip state for the whole time slice:
//   VGPRs : registers, heads, label, counters, RNG stream, IO buffers, cell
//           inputs, merit bonus, task counts, fault count;
//   LDS   : the memory tape (S + 4 bytes per lane; the 4-byte pad rotates
//           lanes across banks), both 10-deep stacks ([row][lane], conflict
//           free), and the block-shared tables (logic-id -> task mask,
//           mutation weights).
// HBM is touched only to stage state in/out, by h-divide (offspring, phenotype
// reset) and by fire-and-forget reaction-count atomics.  Divide appends the
// mutated offspring to a birth queue; IO runs the logic-9 task check fused.
// Lanes whose next h-alloc would outgrow their LDS slot stop before it
// ("spill") and are appended, with their remaining budget, to the next size
// class, which is launched afterwards on the same stream.
#include <cstdlib>

#include "device.h"
#include "births.h"

#pragma clang fp contract(off)

namespace {

// Decode tables over canonical handler ids (include/avida_gpu.h).
// Ops that call FindModifiedRegister/FindModifiedHead (cpu/cHardwareCPU.cc:1622-1672):
#define OPB(x) (1u << (x))
constexpr uint32_t MOD_OPS =
    OPB(AVGPU_H_IF_N_EQU) | OPB(AVGPU_H_IF_LESS) | OPB(AVGPU_H_POP) | OPB(AVGPU_H_PUSH) |
    OPB(AVGPU_H_SWAP) | OPB(AVGPU_H_SHIFT_R) | OPB(AVGPU_H_SHIFT_L) | OPB(AVGPU_H_INC) |
    OPB(AVGPU_H_DEC) | OPB(AVGPU_H_ADD) | OPB(AVGPU_H_SUB) | OPB(AVGPU_H_NAND) | OPB(AVGPU_H_IO) |
    OPB(AVGPU_H_MOV_HEAD) | OPB(AVGPU_H_JMP_HEAD) | OPB(AVGPU_H_GET_HEAD) | OPB(AVGPU_H_SET_FLOW);
// their default register/head (2 bits per op): BX for register ops and IO,
// HEAD_IP for the head ops, CX for set-flow
constexpr uint64_t DEF_OPS =
    (1ull << (2 * AVGPU_H_IF_N_EQU)) | (1ull << (2 * AVGPU_H_IF_LESS)) | (1ull << (2 * AVGPU_H_POP)) |
    (1ull << (2 * AVGPU_H_PUSH)) | (1ull << (2 * AVGPU_H_SWAP)) | (1ull << (2 * AVGPU_H_SHIFT_R)) |
    (1ull << (2 * AVGPU_H_SHIFT_L)) | (1ull << (2 * AVGPU_H_INC)) | (1ull << (2 * AVGPU_H_DEC)) |
    (1ull << (2 * AVGPU_H_ADD)) | (1ull << (2 * AVGPU_H_SUB)) | (1ull << (2 * AVGPU_H_NAND)) |
    (1ull << (2 * AVGPU_H_IO)) | (2ull << (2 * AVGPU_H_SET_FLOW));
// ops executed by the branch-free block
constexpr uint32_t FAST_OPS =
    OPB(AVGPU_H_NOP_A) | OPB(AVGPU_H_NOP_B) | OPB(AVGPU_H_NOP_C) | OPB(AVGPU_H_IF_N_EQU) |
    OPB(AVGPU_H_IF_LESS) | OPB(AVGPU_H_SWAP_STK) | OPB(AVGPU_H_SWAP) | OPB(AVGPU_H_SHIFT_R) |
    OPB(AVGPU_H_SHIFT_L) | OPB(AVGPU_H_INC) | OPB(AVGPU_H_DEC) | OPB(AVGPU_H_ADD) |
    OPB(AVGPU_H_SUB) | OPB(AVGPU_H_NAND) | OPB(AVGPU_H_MOV_HEAD) | OPB(AVGPU_H_JMP_HEAD) |
    OPB(AVGPU_H_GET_HEAD) | OPB(AVGPU_H_SET_FLOW);
// fast ops that write reg[r]
constexpr uint32_t WR_OPS =
    OPB(AVGPU_H_SWAP) | OPB(AVGPU_H_SHIFT_R) | OPB(AVGPU_H_SHIFT_L) | OPB(AVGPU_H_INC) |
    OPB(AVGPU_H_DEC) | OPB(AVGPU_H_ADD) | OPB(AVGPU_H_SUB) | OPB(AVGPU_H_NAND);
#undef OPB

// bytes of the tape word starting at site w4 that lie in [from, to)
__device__ __forceinline__ uint32_t byte_mask(int w4, int from, int to) {
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) m |= (w4 + q >= from && w4 + q < to) ? (0xFFu << (8 * q)) : 0u;
  return m;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// The world descriptor is read through a device pointer rather than passed by
// value: as a by-value kernel argument its ~70 pointers and scalars were all
// held in SGPRs and spilled into VGPR lanes (hundreds of v_readlane in the
// loop); through the pointer each field is a scalar load at its use.
//
// One 64-organism chunk: class 0 = cells first + 64*chunk + lane (dense
// sweep), classes 1..3 = entries 64*chunk + lane of the class list.
// cEnvironment::DoProcesses, finite resource (main/cEnvironment.cc:1660-1724):
// the organism's own cell (spatial; ModifyCell applies at once) or the
// update's global level (consumption summed in 2^-32 units, subtracted at the
// update's end).  Returns whether the process paid (rc counts it).
__device__ __forceinline__ bool consume_resource(const DevWorld& W, const double* rr, int64_t N, int64_t cell,
                                                 double& mult, double& addb, bool wcons) {
  const int slot = (int)rr[RR_RES] - 1;
  const bool spatial = rr[RR_SPATIAL] != 0.0;
  double* cellp = W.res_amount + (int64_t)W.res_param[slot].slot * N + cell;
  const double level = spatial ? *cellp : W.res_global[slot];
  double consumed = (level == 0.0) ? 0.0 : __dmul_rn(level, rr[RR_FRAC]);
  if (consumed > rr[RR_MAX]) consumed = rr[RR_MAX];
  if (consumed < rr[RR_MIN]) consumed = 0.0;
  if (consumed == 0.0) return false;
  consumed = fmin(consumed, level);
  if (rr[RR_DEPL] != 0.0) {
    if (spatial) *cellp = __dsub_rn(level, consumed);
    else atomicAdd(W.res_cons + slot, (unsigned long long)__dmul_rn(consumed, RES_FIX));
    // the cell's consumption this step (a newborn that replaces the organism
    // gives back its share after the birth: world.hip newborn_credit)
    if (wcons) { double* cp = W.cons + (int64_t)slot * N + cell; *cp = __dadd_rn(*cp, consumed); }
  }
  const double bon = __dmul_rn(consumed, rr[RR_VALUE]);
  const int ty = (int)rr[RR_TYPE];
  if (ty == AVGPU_PROC_ADD) addb = __dadd_rn(addb, bon);
  else if (ty == AVGPU_PROC_MULT) mult = __dmul_rn(mult, bon);
  else mult = __dmul_rn(mult, det_exp2(bon));
  return true;
}

// The branch-free ops -- register ALU, swap, conditionals, head moves -- of
// one instruction (op with its register / head r); returns m_advance_ip.
__device__ __forceinline__ bool fast_op(const int op, const int r, int& r0, int& r1, int& r2, int& ip, int& rh,
                                        int& wh, int& fh, uint32_t& ctl, const int M) {
  const int rn = (r == 2) ? 0 : r + 1;                    // FindNextRegister :1676
  const int ra = (r == 0) ? r0 : ((r == 1) ? r1 : r2);
  const int rb = (rn == 0) ? r0 : ((rn == 1) ? r1 : r2);
  int res = ~(r1 & r2);                                                  // nand :3018
  res = (op == AVGPU_H_ADD) ? (int)((uint32_t)r1 + (uint32_t)r2) : res;  // add :2959
  res = (op == AVGPU_H_SUB) ? (int)((uint32_t)r1 - (uint32_t)r2) : res;  // sub :2968
  res = (op == AVGPU_H_INC) ? (int)((uint32_t)ra + 1u) : res;            // inc :2864
  res = (op == AVGPU_H_DEC) ? (int)((uint32_t)ra - 1u) : res;            // dec :2871
  res = (op == AVGPU_H_SHIFT_R) ? (ra >> 1) : res;                       // shift-r :2806
  res = (op == AVGPU_H_SHIFT_L) ? (int)((uint32_t)ra << 1) : res;        // shift-l :2813
  res = (op == AVGPU_H_SWAP) ? rb : res;                                 // swap :2742
  const bool wr = (WR_OPS & (1u << op)) != 0u;
  const bool sw = op == AVGPU_H_SWAP;
  // head ops: head id = nop-mod or IP (mov-head :6809, jmp-head :6859, get-head :6907)
  const int hv = (r == 0) ? ip : ((r == 1) ? rh : wh);
  const bool hw = op == AVGPU_H_MOV_HEAD || op == AVGPU_H_JMP_HEAD;
  int hnew = fh;                                                         // mov-head: Set(FLOW), no adjust
  if (op == AVGPU_H_JMP_HEAD) hnew = head_adjust((int)((uint32_t)hv + (uint32_t)r2), M);
  r0 = (wr && r == 0) ? res : ((sw && rn == 0) ? ra : r0);
  r1 = (wr && r == 1) ? res : ((sw && rn == 1) ? ra : r1);
  r2 = (wr && r == 2) ? res : ((sw && rn == 2) ? ra : r2);
  r2 = (op == AVGPU_H_GET_HEAD) ? hv : r2;
  rh = (hw && r == 1) ? hnew : rh;
  wh = (hw && r == 2) ? hnew : wh;
  if (op == AVGPU_H_SET_FLOW) fh = head_adjust(ra, M);                   // set-flow :7270
  if (hw && r == 0) ip = hnew;
  // if-n-equ :2190 / if-less :2235 skip the next instruction
  const bool skip = (op == AVGPU_H_IF_N_EQU && ra == rb) || (op == AVGPU_H_IF_LESS && ra >= rb);
  if (skip) ip = head_wrap(ip + 1, M);
  ctl ^= (op == AVGPU_H_SWAP_STK) ? CTL_CURSTK : 0u;                     // swap-stk :2739
  return !(op == AVGPU_H_MOV_HEAD && r == 0);
}

// configs[4]'s deferred rewards (interpret_chunk's IO block): up to 3 queued
// events of 9 task bits per lane, the count in bits 30..31.  Applies every
// lane's events in order, each rank by rank -- every lane takes its lowest
// remaining task, so an organism applies its tasks in ascending order with
// consume_resource's arithmetic; a reaction's settings and its resource's
// grid row come by scalar loads, one step per distinct task of the rank, and
// the rank's cell levels go out together.  Runs with the whole wave.
template <bool GTAB>
__device__ __forceinline__ void res_flush(const DevWorld& W, const int64_t N, const int64_t cell, uint32_t& rpq,
                                          double& bonus, int (&rc)[AVGPU_MAX_REACTIONS], const uint32_t ttab,
                                          const double* tmul, const double* tadd, const uint32_t k_env_res_mask,
                                          const bool wcons) {
  while (__ballot(rpq != 0u) != 0ull) {
    const uint32_t ev = rpq & 0x1FFu;
    double mult = 1.0, addb = 0.0;
    uint32_t paid = ev, rem = ev;
    while (__ballot(rem != 0u) != 0ull) {
      const bool has = rem != 0u;
      const int t = has ? __ffs(rem) - 1 : 0;
      const bool isres = has && ((k_env_res_mask >> t) & 1u);
      // (the lane shuffles run with the whole wave active: a ds_bpermute
      // reads 0 from an inactive source lane)
      const double fm = GTAB ? __hiloint2double(__shfl((int)ttab, 2 * t + 1), __shfl((int)ttab, 2 * t)) : 1.0;
      const double fa = GTAB ? __hiloint2double(__shfl((int)ttab, 33 + 2 * t), __shfl((int)ttab, 32 + 2 * t)) : 0.0;
      if (has && !isres) {
        mult = __dmul_rn(mult, GTAB ? fm : tmul[t]);
        addb = __dadd_rn(addb, GTAB ? fa : tadd[t]);
      }
      double frac = 0.0, rmin = 0.0, rmax = 0.0, rval = 0.0;
      double* lvp = nullptr;
      int rty = 0, rslot = 0;
      bool rdepl = false, rsp = false;
      for (uint64_t need = __ballot(isres); need;) {
        const int tu = __builtin_amdgcn_readlane(t, __ffsll((long long)need) - 1);
        const double* rr = W.react_res + tu * RR_STRIDE;     // wave-uniform: scalar loads
        const int slot = (int)rr[RR_RES] - 1;
        const bool sp = rr[RR_SPATIAL] != 0.0;
        const bool mine = isres && t == tu;
        if (mine) {
          frac = rr[RR_FRAC]; rmin = rr[RR_MIN]; rmax = rr[RR_MAX]; rval = rr[RR_VALUE];
          rty = (int)rr[RR_TYPE]; rdepl = rr[RR_DEPL] != 0.0; rsp = sp; rslot = slot;
          lvp = sp ? W.res_amount + (int64_t)W.res_param[slot].slot * N + cell : W.res_global + slot;
        }
        need &= ~__ballot(mine);
      }
      if (isres) {
        const double level = *lvp;
        double consumed = (level == 0.0) ? 0.0 : __dmul_rn(level, frac);
        if (consumed > rmax) consumed = rmax;
        if (consumed < rmin) consumed = 0.0;
        if (consumed == 0.0) {
          paid &= ~(1u << t);
        } else {
          consumed = fmin(consumed, level);
          if (rdepl) {
            if (rsp) *lvp = __dsub_rn(level, consumed);
            else atomicAdd(W.res_cons + rslot, (unsigned long long)__dmul_rn(consumed, RES_FIX));
            if (wcons) { double* cp = W.cons + (int64_t)rslot * N + cell; *cp = __dadd_rn(*cp, consumed); }
          }
          const double bon = __dmul_rn(consumed, rval);
          if (rty == AVGPU_PROC_ADD) addb = __dadd_rn(addb, bon);
          else if (rty == AVGPU_PROC_MULT) mult = __dmul_rn(mult, bon);
          else mult = __dmul_rn(mult, det_exp2(bon));
        }
      }
      rem &= rem - 1u;
    }
    if (ev) {
#pragma unroll
      for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) rc[q] += (paid >> q) & 1u;
      bonus = __dadd_rn(__dmul_rn(bonus, mult), addb);         // cPhenotype.cc:1645-1646
    }
    const uint32_t n = rpq >> 30;
    rpq = n > 1u ? (((rpq & 0x07FFFFFFu) >> 9) | ((n - 1u) << 30)) : 0u;
  }
}

__host__ __device__ constexpr int tape_stride(int S) { return S == CLASS0_SIZE ? S : S + 16; }

// The adaptive sub-step predictor's term of one organism at the end of its
// slice (oracle pred_term, the same IEEE operations): an
// organism expected to divide within the next update's share of picks is
// counted in the quarter of the update its divide is expected in (q, -1
// none) and moves the total weight by twice its merit's change at the divide
// (its own and its offspring's, which replaces a relative of about its old
// merit) from that point on, in mean weights, 2^-20 fixed point.
__device__ __forceinline__ long long pred_term(const DevWorld& W, int cell, int tu, int gs, int blen, int dcop,
                                               int dexe, double bonus, int& q) {
  const double total = W.totals[2], n = W.totals[1];
  if (!(total > 0.0) || !(n > 0.0)) return 0;
  const double wbar = __ddiv_rn(total, n);
  const double wi = W.merit[cell];
  if (!(wi > 0.0) || !(wi <= 1.7976931348623157e308) || !(wbar > 0.0)) return 0;
  const double e = __ddiv_rn(__dmul_rn((double)W.ave_time_slice, wi), wbar);
  const int gt = W.gest_time[cell];
  const int G = gt > 0 ? gt : blen;
  const double r = (double)(G - (tu - gs));
  if (!(r <= __dmul_rn(e, 1.25))) return 0;
  const double t = r <= 0.0 ? 0.0 : fmin(__ddiv_rn(r, e), 1.0);
  q = min(3, (int)__dmul_rn(t, 4.0));
  int sz = blen;
  if (sz > dcop) sz = dcop;
  if (sz > dexe) sz = dexe;
  const double m = gt > 0 ? wi : __dmul_rn((double)sz, bonus);
  double term = __ddiv_rn(__dmul_rn(__dadd_rn(__dsub_rn(m, wi), __dsub_rn(m, wi)), __dsub_rn(1.0, t)), wbar);
  if (!(term <= 1.0e6)) term = 1.0e6;
  if (!(term >= -1.0e6)) term = -1.0e6;
  return (long long)__dmul_rn(term, 1048576.0);
}

// divide-mutation edits (Divide_DoMutations, applied in order): kind | a << 3 | b << 15
enum { E_SLIP = 1, E_POINT = 2, E_INS = 3, E_DEL = 4, E_TRANS = 5 };
__device__ __forceinline__ int edit_word(int kind, int a, int b) { return kind | (a << 3) | (b << 15); }

// serial != 0: a step of the serial world (k_serial_update), lane 0 running
// cell `first` for the reference's ProcessStepSpeculative
// (main/cPopulation.cc:5740-5788) with every draw from the world's context
// stream (DevWorld::sctx / srec_ctx) -- serial = 1: the one non-speculative
// SingleProcess; an offspring is left in the cell's primary record, placed by
// the caller at once (inside the h-divide, as ActivateOffspring does); serial
// = 2: the speculative run, up to 32 instructions, each rejected before IO or
// h-divide (cpu/cHardwareCPU.cc:961-968); one that reaches the age limit sets
// m_spec_die (:1045-1049: not counted, the organism stays until its next
// pick, CTL_SPECDIE).  Returns, for the running lane: instructions executed |
// divides << 16 | birth << 24 | spec death << 25.
// C0W: the class-0 sweep of a world update, with the class and the mode known
// at compile time -- the test-CPU and list-row code drops out of the hot loop;
// SIMPLE: the environment's reactions are the simple form (env_simple) with
// no finite resource, so the general reaction path drops out as well; DEF:
// the allocation, divide and merit knobs at the reference's defaults
// (def_knobs, capi.hip), so their other branches drop out; RES: with SIMPLE,
// the simple reactions consume finite resources (configs[4]) -- without it
// the resource walk drops out of the simple path
// MIX: a list-class chunk run in class 0's 320-site block (k_interpret's
// mixed launch): each organism takes kslot consecutive 320-B slots (class 1:
// 3, class 2: 5, class 3: 7), 64 / kslot organisms per block; the slot size,
// the staging granules per organism and the spill capacity are runtime
// NB: the newborn pass of a batch step (oracle newborn_pass):
// class 0 takes its organisms from list row 0 (k_activate), and a viable
// h-divide is not run -- its cycle is taken back and the slice ends before it.
// pred: a world update's main pass, whose slices add their sub-step
// predictor terms (pred_term) to W.pacc (its block's shard) and count the
// organisms expected to divide within the next update by quarter there.
template <int S, bool REC, bool C0W = false, bool SIMPLE = false, bool DEF = false, bool RES = false,
          bool MIX = false, bool NB = false>
__device__ __forceinline__ int interpret_chunk(const DevWorld* __restrict__ Wp, int cls_arg, int mode_arg,
                                               int64_t first, int64_t count, int64_t chunk,
                                               uint32_t* __restrict__ lds32, bool sorted, int row,
                                               int lpw, int serial = 0, int kslot = 1, int direct = -2,
                                               bool pred = false) {
  const DevWorld& W = *Wp;
  const int cls = C0W ? 0 : cls_arg;
  const int mode = C0W ? (int)AVGPU_MODE_WORLD : mode_arg;
  // per-lane tape stride: a whole number of 16-byte quads (16-B LDS-DMA).
  // The fetch / label / search windows read up to 16 bytes past a site; what
  // they read beyond the organism's memory is masked off.  Classes 1-3 keep a
  // 16-byte pad; class 0 has none -- a window past lane L's slot reads lane
  // L+1's tape (lane 63's: past the block's LDS, which reads as 0) -- so that
  // its block (tapes only, 20 KiB) fits 8 times in a CU.
  constexpr int STRIDE0 = tape_stride(S);
  // staging granule: 16-B quads (dwords for a stride that is not a whole
  // number of quads; device.h CLASS0_SIZE on why class 0 is not)
  constexpr int GRAN = (STRIDE0 % 16 == 0) ? 16 : 4;
  constexpr int QUADS0 = STRIDE0 / GRAN;
  constexpr int TAPE_WORDS = 64 * STRIDE0 / 4;
  // per-organism slot, granules and capacity (MIX: kslot slots of S sites)
  const int STRIDE = MIX ? STRIDE0 * kslot : STRIDE0;
  const int QUADS = MIX ? QUADS0 * kslot : QUADS0;
  const int Scap = MIX ? min(S * kslot, AVGPU_MAX_GENOME) : S;
  // class 0 keeps the two stacks in VGPRs (sv[]): without their 5 KiB of LDS a
  // block needs 26 KiB and 6 blocks fit a CU instead of 5
  constexpr bool VSTK = (S == CLASS0_SIZE);
  constexpr int STK_WORDS = VSTK ? 0 : 2 * AVGPU_STACK_SIZE * 64;
  // one __shared__ object: tapes | stacks | task LUT (256 x u16) | rand_cum (64 x i32) |
  // rand_code (64 B) | rand_lut (256 B) | reactions (16 x RT_STRIDE words) |
  // task bonus factors (16 doubles) | task bonus addends (16 doubles)
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);
  int32_t* stk = reinterpret_cast<int32_t*>(lds32 + TAPE_WORDS);
  uint32_t* tab = lds32 + TAPE_WORDS + STK_WORDS;
  // class 0 keeps no table in LDS: its 20 KiB are the tapes (8 blocks per CU;
  // with the task and random-instruction LUTs beside 336-site tapes a block
  // needed 22.25 KiB and 7 fitted, 4 % slower per update).  It reads them from
  // global memory by loads that wait for themselves (a compiler-visible
  // vector load made the IO path wait on vmcnt(0) at its join, i.e. for every
  // store the wave still had in flight), the rest through uniform loads.
  constexpr bool GTAB = (S == CLASS0_SIZE);
  constexpr bool GLUT = GTAB;
  // the list classes' tables are in LDS; said so explicitly, or an access
  // through a generic pointer is a flat load, whose wait also drains every
  // outstanding global store of the wave
  typedef const __attribute__((address_space(3))) uint16_t lds_u16_t;
  typedef const __attribute__((address_space(3))) uint8_t lds_u8_t;
  lds_u16_t* lut = (lds_u16_t*)(tab);
  const int32_t* rcum = GTAB ? W.rand_cum : reinterpret_cast<const int32_t*>(tab + 128);
  const uint8_t* rcode = GTAB ? W.rand_code : reinterpret_cast<const uint8_t*>(tab + 192);
  lds_u8_t* rlut = (lds_u8_t*)(tab + (GTAB ? 128 : 208));
  const int32_t* rtab = GTAB ? W.react_tab : reinterpret_cast<const int32_t*>(tab + 272);
  // per-task bonus factor / addend of the simple-environment path (16 + 16 doubles)
  const double* tmul = GTAB ? W.task_tab
                            : reinterpret_cast<const double*>(tab + 272 + AVGPU_MAX_REACTIONS * RT_STRIDE);
  const double* tadd = tmul + 16;

  // class 0 reads the cumulative random-instruction weights and codes from
  // global memory (rare paths) by loads that wait for themselves: a
  // compiler-visible load there left an outstanding-load wait at the join
  // with the LDS path, i.e. every copy mutation drained the wave's stores
  auto tab_i32 = [&](const int32_t* p) -> int32_t { return GTAB ? (int32_t)ld_sync_u32(p) : *p; };
  auto tab_u8 = [&](const uint8_t* p) -> uint32_t { return GTAB ? ld_sync_u8(p) : (uint32_t)*p; };
  const int lane = threadIdx.x;
  const int64_t N = W.n;
  int cell = -1;
  int M = 0;
  if (serial) {
    if (lane == 0) {
      cell = (int)first;
      M = W.mem_size[cell];
    }
  } else if (NB && cls == 0) {
    // the newborn pass's class-0 organisms: list row 0 (k_activate)
    const int64_t idx = chunk * 64 + lane;
    if (idx < W.class_count[0]) {
      cell = W.class_list[idx];
      M = W.mem_size[cell];
    }
  } else if (cls == 0) {
    // dense sweep: in cell order, or (world updates) through the
    // budget-sorted windows of k_window_order
    const int64_t c = sorted ? (chunk * 64 + lane < count ? (int64_t)W.order[chunk * 64 + lane] : first + count)
                             : first + chunk * 64 + lane;
    // the cell's slice is class 0 by k_allot's tag (device.h aclass), not by
    // its live size: list classes may be rewriting their cells concurrently
    if (c < first + count && W.aclass[c] == 0) {
      cell = (int)c;
      M = W.mem_size[c];
    }
  } else if (MIX && direct != -2) {
    // the organisms a class-0 wave spilled, continued by the same wave
    // (k_interpret): the lane's cell, -1 for none
    if (direct >= 0) {
      cell = direct;
      M = W.mem_size[direct];
    }
  } else {
    // list rows: lpw entries per wave (lanes >= lpw idle)
    const int lcount = W.class_count[row];
    const int64_t base = chunk * lpw;
    if (base >= lcount) return 0;
    const int idx = (int)base + lane;
    if (lane < lpw && idx < lcount) {
      cell = W.class_list[(int64_t)row * N + idx];
      M = W.mem_size[cell];
    }
  }
  const bool active = cell >= 0;
  if (!__any(active)) return 0;
  const bool fresh = active && (W.ctl[cell] & CTL_FRESH);
#ifdef AVGPU_PHASE_CLOCKS
  const uint64_t clk0 = __builtin_amdgcn_s_memtime();
  int it_fast = 0, it_copy = 0, it_slow = 0, it_loop = 0;   // it_loop: loop iterations (wave-uniform)
  // loop cycles by block: decode, fast, copy, switch, wave phase, advance
  uint64_t cb[6] = {0, 0, 0, 0, 0, 0};
  uint64_t clast = 0;
  // slow-switch cycles by case: pop, push, IO, h-alloc, h-divide, h-search,
  // if-label, and the stretch from the copy block to the switch
  uint64_t cc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // + IO's second half: task lookup, rewards
#define CK(k) do { const uint64_t _n = __builtin_amdgcn_s_memtime(); cb[k] += _n - clast; clast = _n; } while (0)
#define CKC(k) do { const uint64_t _n = __builtin_amdgcn_s_memtime(); cc[k] += _n - clast; clast = _n; } while (0)
#elif defined(AVGPU_ISA_MARKS)
#define CK(k) asm volatile("; @MARK CK" #k)
#define CKC(k) asm volatile("; @MARK CKC" #k)
#else
#define CK(k) do { } while (0)
#define CKC(k) do { } while (0)
#endif
  const int m_in = M;

  // ---- block-shared tables ----
  if (!GTAB) {
    uint32_t* l32 = tab;
    const uint32_t* g_lut = reinterpret_cast<const uint32_t*>(W.task_lut);
    l32[lane] = g_lut[lane];
    l32[64 + lane] = g_lut[64 + lane];
    l32[128 + lane] = (uint32_t)W.rand_cum[lane];
    if (lane < 16) l32[192 + lane] = reinterpret_cast<const uint32_t*>(W.rand_code)[lane];
    l32[208 + lane] = reinterpret_cast<const uint32_t*>(W.rand_lut)[lane];
    for (int k = lane; k < AVGPU_MAX_REACTIONS * RT_STRIDE; k += 64) l32[272 + k] = (uint32_t)W.react_tab[k];
    l32[272 + AVGPU_MAX_REACTIONS * RT_STRIDE + lane] = reinterpret_cast<const uint32_t*>(W.task_tab)[lane];
  }
  // ---- stage tapes and stacks into LDS by LDS-DMA.  The 64 tapes form one
  // lane-linear image of 64 x QUADS granules (granule i = organism i / QUADS,
  // part i % QUADS), so each global_load_lds moves 64 granules (1 KiB of
  // quads, 256 B of dwords) with per-lane sources; all copies are in flight
  // together and retired by one wait ----
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  // a serial step runs lane 0 only: its quads are the image's first QUADS
  const int qits = serial ? (QUADS0 + 63) / 64 : QUADS0;   // MIX: the same 64 x QUADS0 granule image
  // class 0: unrolled so that the shuffles of several quads are in flight
  // together (one LDS round trip per quad otherwise); the list classes' 49 /
  // 97 / 129-quad loops stay rolled (code size)
  constexpr int QUNR = (S == CLASS0_SIZE) ? (QUADS0 % 7 == 0 ? 7 : 5) : 1;
#pragma unroll QUNR
  for (int it = 0; it < qits; it++) {
    const int i = it * 64 + lane;
    const int j = i / QUADS, q = i - j * QUADS;
    const int c = __shfl(cell, j);
    const int m = __shfl(M, j);
    if (c >= 0 && q * GRAN < m) {
      void* src = (void*)(W.tape + (int64_t)c * TAPE_SLOT + q * GRAN);
      if constexpr (GRAN == 16) __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(lds32 + it * 256), 16, 0, 0);
      else __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(lds32 + it * 64), 4, 0, 0);
    }
  }
  // stacks: class 0's into VGPRs with the execution record below; the list
  // classes' from the record into LDS, one word per lane and entry
  int32_t* const xrec = W.xs + (int64_t)(cell < 0 ? 0 : cell) * XS_WORDS;
  int32_t sv[2 * AVGPU_STACK_SIZE];
#pragma unroll
  for (int k = 0; k < 2 * AVGPU_STACK_SIZE; k++) {
    if (VSTK) {
      sv[k] = 0;
    } else if (active && !fresh) {
      __builtin_amdgcn_global_load_lds((void*)(xrec + XS_STACK + k), (lds_ptr_t)(stk + k * 64), 4, 0, 0);
    } else {
      stk[k * 64 + lane] = 0;
    }
  }

  // (MIX: lanes past the block's 64 / kslot organisms never touch their tape;
  // they point at lane 0's)
  uint8_t* T = lds + ((MIX && lane * kslot >= 64) ? 0 : lane) * STRIDE;

  // ---- hot state into registers ----
  int r0 = 0, r1 = 0, r2 = 0, ip = 0, rh = 0, wh = 0, fh = 0;
  uint32_t ctl = 0, rl = 0, klo = 0, khi = 0, kct = 0;
  uint32_t olo = 0, ohi = 0;     // the organism's own key (its offspring's keys derive from it)
  int cyc = 0, tu = 0, gs = 0, mx = 0, blen = 0, budget = 0, errs = 0, sdone = 0;
  int in0 = 0, in1 = 0, in2 = 0, intot = 0, inptr = 0, inp0 = 0, inp1 = 0, inp2 = 0;
  int outv = 0, outtot = 0;
  double bonus = 0.0;
  int tc[AVGPU_NUM_LOGIC_TASKS];
#pragma unroll
  for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] = 0;
  // divide bookkeeping kept on chip so that no global load or store is
  // compiler-visible inside the loop (written back after it if a divide happened)
  int dexe = 0, dcop = 0, dnd = 0, dgen = 0;
  // cur_reaction_count: reactions 0..11 from the execution record (the
  // running count), 12..15 counted since slice start / last reset (added to
  // their cur_react rows at write-back)
  int rc[AVGPU_MAX_REACTIONS];
  uint32_t nzm = 0;              // tasks with a non-zero count this gestation
#pragma unroll
  for (int q = 0; q < AVGPU_MAX_REACTIONS; q++) rc[q] = 0;
  bool didv = false, prim = false, prim0 = false;
  int sbirth = 0;                // serial step: an offspring is in the primary record
  int sdie = 0;                  // serial speculative run: m_spec_die
  int ndrop = 0, noversize = 0;
  if (active) {
    // written at birth (setup_child) or by the previous slice
    ctl = W.ctl[cell];
    mx = W.max_exec[cell]; blen = W.birth_len[cell];
    klo = W.rng[cell]; khi = W.rng[N + cell]; kct = W.rng[2 * N + cell];
    olo = klo; ohi = khi;
    if (serial) { klo = W.sctx[0]; khi = W.sctx[1]; kct = W.sctx[2]; }   // the context stream
    budget = W.budget[cell];
    prim = (budget & BUDGET_PRIM) != 0;   // a spilled slice already used its primary record
    budget &= ~BUDGET_PRIM;
    // a spill row continues a slice: the instructions it ran before it spilled
    // (birth times count from the slice's start)
    if (row > NUM_CLASSES - 1) sdone = W.sdone[cell];
    if (serial) { budget = serial == 1 ? 1 : 32; prim = false; }
    inp0 = W.inputs[cell]; inp1 = W.inputs[N + cell]; inp2 = W.inputs[2 * N + cell];
    dexe = W.executed[cell]; dcop = W.copied[cell]; dgen = W.generation[cell];
    bonus = W.default_bonus;
  }
  static_assert(AVGPU_NUM_LOGIC_TASKS == 9 && 2 * AVGPU_STACK_SIZE == 20, "execution record layout");
  if (active && !fresh) {
    // the execution record (device.h XS_*): 16-byte loads of its own lines
    const int4* xr = reinterpret_cast<const int4*>(xrec);
    const int4 x0 = xr[0], x1 = xr[1], x2 = xr[2], x3 = xr[3], x4 = xr[4], x5 = xr[5], x6 = xr[6], x7 = xr[7];
    r0 = x0.x; r1 = x0.y; r2 = x0.z; ip = x0.w;
    rh = x1.x; wh = x1.y; fh = x1.z; rl = (uint32_t)x1.w;
    cyc = x2.x; tu = x2.y; gs = x2.z; errs = x2.w;
    in0 = x3.x; in1 = x3.y; in2 = x3.z; intot = x3.w;
    inptr = x4.x; outv = x4.y; outtot = x4.z;
    bonus = __hiloint2double(x5.y, x5.x);
    tc[0] = x5.z; tc[1] = x5.w; tc[2] = x6.x; tc[3] = x6.y; tc[4] = x6.z; tc[5] = x6.w;
    tc[6] = x7.x; tc[7] = x7.y; tc[8] = x7.z;
    if (VSTK) {
#pragma unroll
      for (int j = 0; j < 5; j++) {
        const int4 v = xr[8 + j];
        sv[4 * j] = v.x; sv[4 * j + 1] = v.y; sv[4 * j + 2] = v.z; sv[4 * j + 3] = v.w;
      }
    }
    static_assert(XS_REACT == 52 && XS_NREACT == 12, "execution record: reaction counts");
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int4 v = xr[13 + j];
      rc[4 * j] = v.x; rc[4 * j + 1] = v.y; rc[4 * j + 2] = v.z; rc[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) nzm |= (tc[q] > 0 ? 1u : 0u) << q;
    dnd = W.num_div[cell];
  }
  prim0 = prim;
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), visible to the compiler's waitcnt tracking
  __syncthreads();
#ifdef AVGPU_PHASE_CLOCKS
  const uint64_t clk1 = __builtin_amdgcn_s_memtime();
#endif

  // the lane's run state as bits of one int (F_DEAD | F_STOP | F_SPILL): as
  // three bools, each was a lane mask in SGPRs that every join of the
  // divergent loop body merged with its own s_andn2 / s_and / s_or triple
  enum { F_DEAD = 1, F_STOP = 2, F_SPILL = 4 };
  int fl = (active && (ctl & CTL_ALIVE)) ? 0 : F_DEAD;
  const bool alive0 = fl == 0;
  int executed = 0, divides = 0;

  // world scalars the loop uses, read once: through the descriptor pointer
  // each use was an s_load + lgkmcnt wait inside the loop
  const double k_size_range = DEF ? 2.0 : W.size_range;
  const int k_require_allocate = DEF ? 1 : W.require_allocate, k_alloc_method = DEF ? 0 : W.alloc_method;
  const uint64_t k_th_copy_mut = W.th_copy_mut;
  const int k_copy_ext = DEF ? 0 : W.copy_ext;
  const uint64_t k_no_mut = DEF ? 0ull : W.no_mut_mask;   // NO_MUT_INSTS (checkNoMutList)
  const uint64_t k_th_copy_ins = DEF ? 0ull : W.th_copy_ins, k_th_copy_del = DEF ? 0ull : W.th_copy_del;
  const uint64_t k_th_copy_uni = DEF ? 0ull : W.th_copy_uni, k_th_copy_slip = DEF ? 0ull : W.th_copy_slip;
  const int k_slip_whole = DEF ? 0 : W.slip_copy_mode;
  const int k_rand_total = W.rand_total, k_n_ops = W.n_ops, k_n_react = W.n_react;
  const bool k_rand_lut = DEF || k_rand_total <= 256;   // GetRandomInst from the LUT
  // RECORDED streams (include/avida_gpu.h "random streams"): the organism's
  // k-th draw is rbase[k]; REC = false compiles the counter path only
  const double* rbase = nullptr;
  int64_t rlim = 0;
  bool rover = false;
  if (REC && active) {
    if (serial) {
      rbase = W.srec_ctx; rlim = W.srec_ctx_n;      // the serial world's recorded context stream
    } else {
      const int64_t off = W.rec_off[cell];
      if (off >= 0) { rbase = W.rec + off; rlim = W.rec_n - off; }
    }
  }
  // the reference's draws on a uniform u (Apto::RNG P / GetUInt)
  auto rd = [&]() -> double {
    const uint32_t k = kct++;
    if ((int64_t)k < rlim) return rbase[k];
    rover = true;
    return 0.0;
  };
  auto draw_p = [&](uint64_t th, double p) -> bool {
    if (REC && rbase) return rd() < p;
    return rng_p(klo, khi, kct, th);
  };
  auto draw_below = [&](uint32_t n) -> uint32_t {
    if (REC && rbase) { const uint32_t v = (uint32_t)(rd() * (double)n); return v < n ? v : n - 1u; }
    return rng_below(klo, khi, kct, n);
  };
  const int k_env_simple = SIMPLE ? 1 : W.env_simple, k_max_label_exe = DEF ? 1 : W.max_label_exe;
  const int k_env_resources = W.env_resources;
  const uint32_t k_env_res_mask = (SIMPLE && !RES) ? 0u : W.env_res_mask;
  const uint32_t k_env_react_mask = W.env_react_mask, k_env_once_mask = W.env_once_mask;
  // cInstSet::GetRandomInst (cpu/cInstSet.cc:83-88) from the LDS tables
  auto rand_code = [&]() -> uint8_t {
    const uint32_t r = draw_below((uint32_t)k_rand_total);
    if (k_rand_lut) return GLUT ? (uint8_t)sgather_u8(W.rand_lut, r) : rlut[r];
    int i = 0;
    while (i < k_n_ops - 1 && tab_i32(rcum + i) <= (int32_t)r) i++;
    return (uint8_t)tab_u8(rcode + i);
  };

#define GETREG(i) ((i) == 0 ? r0 : ((i) == 1 ? r1 : r2))
#define SETREG(i, v) do { const int _v = (v); if ((i) == 0) r0 = _v; else if ((i) == 1) r1 = _v; else r2 = _v; } while (0)
#define GETHEAD(i) ((i) == 0 ? ip : ((i) == 1 ? rh : ((i) == 2 ? wh : fh)))
#define SETHEAD(i, v) do { const int _v = (v); if ((i) == 0) ip = _v; else if ((i) == 1) rh = _v; else if ((i) == 2) wh = _v; else fh = _v; } while (0)

  // Requests for the O(memory) parts of heavy instructions -- the divide's
  // flag counts, offspring copy and flag clearing, h-alloc's fill, h-search's
  // label scan.  A lane decodes such an instruction and posts a request; the
  // whole wave then serves the requests one lane at a time, 64 sites per
  // instruction (DESIGN.md "Cooperative heavy ops").  Run per lane, every
  // iteration of the wave paid for the longest such loop of any of its lanes.
  const int RQ_NONE = 0, RQ_DIVIDE = 1, RQ_FILL = 2, RQ_SEARCH = 3;
  const uint32_t fill4 = (uint32_t)W.fill_code * 0x01010101u;
  // Slow ops (stack, IO, h-alloc, h-divide, h-search, if-label) are batched:
  // a lane that decodes one parks (the decode is committed: counters,
  // executed flags, modifier) and keeps its op; the wave runs the divergent
  // slow switch only once W.slow_batch lanes are parked, or when no unparked
  // lane can step any more.  Each organism still executes its own
  // instructions in order -- only the interleaving across lanes changes.
  int pop = -1, pr = 0;                                       // parked op, its register
  int io_id = -2;                                             // IO's logic id (-1: none; -2: no IO this step)
  // class 0's task LUT (256 x u16) spread over the wave: lane j holds entries 4j .. 4j+3
  uint32_t tl0 = 0u, tl1 = 0u;
  // and its per-task bonus factors / addends (32 doubles): lane j holds word j,
  // read by v_readlane at a wave-uniform task index
  uint32_t ttab = 0u;
  if (GLUT) {
    const uint32_t* g_lut = reinterpret_cast<const uint32_t*>(W.task_lut);
    tl0 = g_lut[2 * lane];
    tl1 = g_lut[2 * lane + 1];
    ttab = reinterpret_cast<const uint32_t*>(W.task_tab)[lane];
  }
  const uint32_t* T32 = reinterpret_cast<const uint32_t*>(T);
  const int slow_batch = NB ? W.nb_slow_batch : W.slow_batch;
  uint32_t rpq = 0u;        // configs[4]'s queued reward events (res_flush)

  while (true) {
    const bool run = fl == 0 && budget > 0 && pop < 0;
    if (!__any(run || pop >= 0)) break;                       // wave-uniform loop
#ifdef AVGPU_PHASE_CLOCKS
    if (clast == 0) clast = __builtin_amdgcn_s_memtime();
    it_loop++;
    CK(5);
#endif
    bool adv = true;                                          // m_advance_ip
    bool stepped = false;
    if (run) {
      // ---- SingleProcess (cpu/cHardwareCPU.cc:908-1058) ----
      const int ipa = head_adjust(ip, M);                     // ip.Adjust() :952
      // fetch window: sites ipa .. ipa+4 in two independent word reads, and
      // h-copy's two sites read with it (one LDS round trip per iteration
      // instead of two; used only if the op is h-copy)
      const int rha = head_adjust(rh, M), wha = head_adjust(wh, M);
      const uint64_t fwin = ((uint64_t)T32[(ipa >> 2) + 1] << 32) | (uint64_t)T32[ipa >> 2];
      const int src_byte = T[rha], dst_byte = T[wha];
      const uint32_t fsh = (uint32_t)(ipa & 3) * 8u;
      const int cur_byte = (int)((fwin >> fsh) & 0xFFu);
      const int op = cur_byte & CODE_MASK;                    // fetch :959
      if (op == AVGPU_H_H_ALLOC) {
        // would this allocation outgrow the LDS slot?  (spill check; the
        // instruction is then executed by the next size class)
        const int cur = M;
        int alloc = (int)(k_size_range * cur);
        if (alloc > AVGPU_MAX_GENOME - cur) alloc = AVGPU_MAX_GENOME - cur;
        const int nsz = cur + alloc;
        const bool ok = !(k_require_allocate && (ctl & CTL_MAL)) && alloc >= 1 &&
                        nsz <= AVGPU_MAX_GENOME && nsz >= AVGPU_MIN_GENOME &&
                        alloc <= (int)(cur * k_size_range) && cur <= (int)(alloc * k_size_range);
        if (ok && nsz > Scap) { fl |= F_SPILL; ip = ipa; }
      }
      // serial step: the speculative run ends before IO / h-divide
      // (cHardwareCPU::SingleProcess stall instructions, cpu/cHardwareCPU.cc:961-968)
      if (serial == 2 && (op == AVGPU_H_IO || op == AVGPU_H_H_DIVIDE)) fl |= F_STOP;
    if (fl == 0) {
    stepped = true;
    cyc++;                                                    // IncCPUCyclesUsed :929
    tu++;                                                     // IncTimeUsed :930
    ip = ipa;
    T[ip] = (uint8_t)(cur_byte | TF_EXEC);                    // SetFlagExecuted :996
    executed++;
    budget--;
    const int nbyte = (int)((fwin >> (fsh + 8u)) & 0xFFu);
    const int nxt = (ip + 1 < M) ? (nbyte & CODE_MASK) : CODE_ERROR;  // GetNextInst
    // ---- FindModifiedRegister / FindModifiedHead (:1622-1672), applied once
    // for every op that takes a nop modifier: r = nop-mod or the op's default ----
    const uint32_t obit = 1u << op;
    const bool mod = ((MOD_OPS & obit) != 0u) && nxt < 3;
    const int r = mod ? nxt : (int)((DEF_OPS >> (2 * op)) & 3ull);
    if (mod) { ip = ip + 1; T[ip] = (uint8_t)(nbyte | TF_EXEC); }
#ifdef AVGPU_PHASE_CLOCKS
    it_fast += __ballot((FAST_OPS & obit) != 0u) != 0ull;
    it_copy += __ballot(op == AVGPU_H_H_COPY) != 0ull;
#endif
    CK(0);
    if (FAST_OPS & obit) adv = fast_op(op, r, r0, r1, r2, ip, rh, wh, fh, ctl, M);
    CK(1);
    if (op == AVGPU_H_H_COPY) {                               // :7130 Inst_HeadCopy
      rh = rha;
      wh = wha;
      int v = src_byte & CODE_MASK;
      const uint32_t kct_h = kct, rl_h = rl;                  // rewound if the copy spills (below)
      // ReadInst (:1459-1466)
      if (v < 3) {
        const int len = rl & 15;
        if (len < AVGPU_MAX_LABEL) rl = (rl & ~15u) | (uint32_t)(len + 1) | ((uint32_t)v << (4 + 2 * len));
      } else {
        rl = 0;
      }
      // TestCopyMut: no draw at rate 0 (main/cMutationRates.h:112)
      // (the rare mutated copy behind a wave-uniform test, so that the
      // common path falls through instead of branching around it)
      const bool cmut = mode != AVGPU_MODE_TEST && k_th_copy_mut && draw_p(k_th_copy_mut, W.p_copy_mut);
      if (__builtin_expect(__ballot(cmut) != 0ull, 0)) {
        // a listed read instruction keeps itself (no GetRandomInst draw, :7144)
        if (cmut && !((k_no_mut >> v) & 1ull)) v = rand_code();
      }
      // the write head's executed flag: as read, or just set if it is the IP
      const int wex = (wh == ip) ? TF_EXEC : (dst_byte & TF_EXEC);
      T[wh] = (uint8_t)(wex | TF_COPIED | v);
      // COPY_INS / DEL / UNIFORM / SLIP (:7153-7161, each drawing only at a
      // non-zero rate, in that order): the memory grows or shrinks at the
      // write head (cCPUMemory::Insert / Remove, cpu/cCPUMemory.cc:103-138;
      // doUniformCopyMutation cpu/cHardwareBase.cc:597-612), or the read head
      // jumps (SLIP_COPY_MODE 0).  A copy whose memory would outgrow this size
      // class's LDS slot is rewound -- counter, label, written site, cycle --
      // and the organism spills to the next class, which draws the same
      // numbers again; at AVGPU_MAX_GENOME sites an insertion is skipped
      // (counted), as in the oracle.
      bool cspill = false;
      if (!DEF && k_copy_ext && mode != AVGPU_MODE_TEST) {
        int e_ins = -1, e_uni = -1, e_slip = -1;
        bool e_del = false;
        if (k_th_copy_ins && draw_p(k_th_copy_ins, W.p_copy_ins)) e_ins = rand_code();
        if (k_th_copy_del) e_del = draw_p(k_th_copy_del, W.p_copy_del);
        if (k_th_copy_uni && draw_p(k_th_copy_uni, W.p_copy_uni)) e_uni = (int)draw_below((uint32_t)(2 * k_n_ops + 1));
        const bool e_slp = k_th_copy_slip && draw_p(k_th_copy_slip, W.p_copy_slip);
        // NO_MUT_INSTS: the uniform mutation leaves a listed write-head
        // instruction (doUniformCopyMutation, cpu/cHardwareBase.cc:597-612),
        // the one at the write head after the insertion / deletion above (a
        // head past the end reads none)
        if (e_uni >= 0 && k_no_mut) {
          const bool ins = e_ins >= 0 && M < AVGPU_MAX_GENOME;
          const bool del = e_del && M + (ins ? 1 : 0) > 1;
          int at;
          if (ins) at = del ? v : e_ins;                        // the inserted site, or (removed again) the written one
          else if (del) at = wh + 1 < M ? (T[wh + 1] & CODE_MASK) : -1;
          else at = v;
          if (at >= 0 && ((k_no_mut >> at) & 1ull)) e_uni = -1;
        }
        const bool ev = e_ins >= 0 || e_del || e_uni >= 0 || e_slp;
        if (__builtin_expect(__ballot(ev) != 0ull, 0)) {
          if (ev) {
            // the size the memory passes through: a slot that cannot hold it
            // (below the largest genome) makes the copy spill
            int mx_sz = M + (e_ins >= 0 ? 1 : 0);
            if (e_uni > k_n_ops) mx_sz = max(mx_sz, M + (e_ins >= 0 ? 1 : 0) - (e_del ? 1 : 0) + 1);
            // SLIP_COPY_MODE 1 (oracle slip_memory): the slip's `to` is the
            // next draw, from the size the edits above leave (their caps
            // included); its result size joins the check
            int s_to = -1;
            if (e_slp && k_slip_whole) {
              int Mp = M;
              if (e_ins >= 0 && Mp < AVGPU_MAX_GENOME) Mp++;
              if (e_del && Mp > 1) Mp--;
              if (e_uni == k_n_ops && Mp > 1) Mp--;
              else if (e_uni > k_n_ops && Mp < AVGPU_MAX_GENOME) Mp++;
              s_to = (int)draw_below((uint32_t)(wh == 0 ? Mp : Mp + 1));
              if (Mp + wh - s_to <= AVGPU_MAX_GENOME) mx_sz = max(mx_sz, Mp + wh - s_to);
            }
            if (mx_sz > Scap && Scap < AVGPU_MAX_GENOME) {
              T[wh] = (uint8_t)dst_byte;                       // undo the write, then the step
              T[ipa] = (uint8_t)cur_byte;
              kct = kct_h; rl = rl_h;
              cyc--; tu--; executed--; budget++;
              ip = ipa;
              cspill = true;
            } else {
              int ncap = 0;
              auto ins_at = [&](int pos, int code) {
                if (M >= AVGPU_MAX_GENOME) { ncap++; return; }
                for (int i = M; i > pos; i--) T[i] = T[i - 1];
                T[pos] = (uint8_t)code;                        // new site: flags 0
                M++;
              };
              auto del_at = [&](int pos) {
                if (M <= 1) { ncap++; return; }
                if (pos > M - 1) pos = M - 1;                  // Remove(size) drops the last site
                for (int i = pos; i < M - 1; i++) T[i] = T[i + 1];
                M--;
              };
              if (e_ins >= 0) ins_at(wh, e_ins);
              if (e_del) del_at(wh);
              if (e_uni >= 0) {
                if (e_uni < k_n_ops) {
                  if (wh < M) T[wh] = (uint8_t)((T[wh] & ~CODE_MASK) | (int)tab_u8(rcode + e_uni));   // SetInst
                } else if (e_uni == k_n_ops) {
                  del_at(wh);
                } else {
                  ins_at(wh, (int)tab_u8(rcode + e_uni - k_n_ops - 1));
                }
              }
              if (e_slp && !k_slip_whole) e_slip = (int)draw_below((uint32_t)M);   // read_head.Set(GetInt(size))
              if (e_slip >= 0) rh = e_slip;
              if (s_to >= 0) {                                 // the memory slip at the write head
                const int from = wh, ins = from - s_to, Mn = M + ins;
                if (Mn > AVGPU_MAX_GENOME) {
                  ncap++;
                } else if (ins > 0) {                          // only codes move; flags stay per position
                  for (int j = Mn - 1; j >= from + ins; j--) {
                    const int cd = T[j - ins] & CODE_MASK;
                    T[j] = (uint8_t)(j < M ? ((T[j] & ~CODE_MASK) | cd) : cd);
                  }
                  const int sfm = W.slip_fill_mode;
                  for (int i = 0; i < ins; i++) {
                    const int j = from + i;
                    const int cd = sfm == 0 ? (T[s_to + i] & CODE_MASK) : sfm == 2 ? rand_code() : 2;   // nop-C
                    T[j] = (uint8_t)(j < M ? ((T[j] & ~CODE_MASK) | cd) : cd);
                  }
                  M = Mn;
                } else if (ins < 0) {
                  for (int j = from; j < Mn; j++) T[j] = (uint8_t)((T[j] & ~CODE_MASK) | (T[j - ins] & CODE_MASK));
                  M = Mn;
                }
              }
              if (ncap) count_add(W, CNT_MEM_CAP, (unsigned long long)ncap);
            }
          }
        }
      }
      if (cspill) {
        fl |= F_SPILL;
        stepped = false;
      } else if (!DEF && k_copy_ext) {
        rh = head_adjust(rh + 1, M);
        wh = head_adjust(wh + 1, M);
      } else {
        rh = head_wrap(rh + 1, M);
        wh = head_wrap(wh + 1, M);
      }
    }
    // if-label (:6914 Inst_IfLabel) from the fetch window when its label ends
    // inside the window (the copy loop's short labels): no park, no label
    // read.  The window holds sites ipa+1 .. ipa+avail; a label that may run
    // past them parks and reads its own 16-byte window in the slow phase.
    bool lab_done = false;
    if (op == AVGPU_H_IF_LABEL && k_max_label_exe == 1) {
      const int base = ip + 1;
      const int avail = 7 - (ipa & 3);
      const uint64_t w = fwin >> (fsh + 8u);                // site base in byte 0
      const uint64_t cl = w & 0x3F3F3F3F3F3F3F3Full;
      const uint64_t nl = (cl + 0x7D7D7D7D7D7D7D7Dull) & 0x8080808080808080ull;   // non-nop bytes
      const int run = nl ? (int)(__ffsll((long long)nl) - 8) >> 3 : 8;
      const int lim = min(AVGPU_MAX_LABEL, M - base);
      if (run < avail || lim <= avail) {
        lab_done = true;
        const int len = max(min(run, lim), 0);
        uint64_t v = cl & 0x0303030303030303ull;
        v = (v | (v >> 6)) & 0x000F000F000F000Full;
        v = (v | (v >> 12)) & 0x000000FF000000FFull;
        v = (v | (v >> 24)) & 0xFFFFull;
        const uint32_t lmask = (1u << (2 * len)) - 1u;
        const uint32_t lab = (uint32_t)v & lmask;
        const uint32_t dl = lab & 0x55555u, dh = (lab >> 1) & 0x55555u;
        const uint32_t rot = ((~dl & ~dh & 0x55555u) | (dl << 1)) & lmask;   // Rotate(1, NUM_NOPS)
        if (len > 0) T[base] = (uint8_t)((uint32_t)w | TF_EXEC);         // the label's first site (MAX_LABEL_EXE_SIZE 1)
        ip += len;
        if (((uint32_t)len | (rot << 4)) != rl) ip = head_wrap(ip + 1, M);
      }
    }
    CK(2);
    if (!(FAST_OPS & obit) && op != AVGPU_H_H_COPY && !lab_done) { pop = op; pr = r; stepped = false; }   // park
    }  // !spill
    }  // run
    if (stepped && !(fl & F_STOP)) {
      if (adv) ip = head_wrap(ip + 1, M);                     // ip.Advance() :1013
      if (mx > 0 && tu >= mx) {                               // death :1045-1049
        if (serial == 2) { sdie = 1; fl |= F_STOP; executed--; }   // m_spec_die: not counted
        else fl |= F_DEAD;
      }
    }
    // ---- slow phase ----
    const int npark = __popcll(__ballot(pop >= 0));
    if (npark == 0) continue;
    if (npark < slow_batch && __any(fl == 0 && budget > 0 && pop < 0)) continue;
#ifdef AVGPU_PHASE_CLOCKS
    it_slow++;
#endif
    {
    int rq = RQ_NONE, qa = 0, qb = 0;
    bool adv = true;
    const bool sstep = pop >= 0;
    if (sstep) {
      const int op = pop, r = pr;
      CKC(7);
      switch (op) {
      case AVGPU_H_POP:                                       // :2698, cCPUStack::Pop
      case AVGPU_H_PUSH: {                                    // :2705, cCPUStack::Push
        // one case for both, so that a wave's pops and pushes share one pass
        // over the register stacks: Push moves the pointer down and stores,
        // Pop reads, clears and moves it up
        const bool push = op == AVGPU_H_PUSH;
        const int k = (ctl & CTL_CURSTK) ? 1 : 0;
        int sp = k ? CTL_SP1(ctl) : CTL_SP0(ctl);
        if (push) sp = (sp == 0) ? AVGPU_STACK_SIZE - 1 : sp - 1;
        const int nv = push ? GETREG(r) : 0;
        int v = 0;
        if (VSTK) {
          const int idx = k * AVGPU_STACK_SIZE + sp;
#pragma unroll
          for (int i = 0; i < 2 * AVGPU_STACK_SIZE; i++) {
            v = (i == idx) ? sv[i] : v;
            sv[i] = (i == idx) ? nv : sv[i];
          }
        } else {
          int32_t* slot = stk + (k * AVGPU_STACK_SIZE + sp) * 64 + lane;
          v = *slot;
          *slot = nv;
        }
        if (!push) {
          sp = (sp + 1 == AVGPU_STACK_SIZE) ? 0 : sp + 1;
          SETREG(r, v);
        }
        ctl = k ? ((ctl & ~0xF0u) | ((uint32_t)sp << 4)) : ((ctl & ~0xFu) | (uint32_t)sp);
        CKC(0);
        break; }
      case AVGPU_H_IO: {                                      // :4188 Inst_TaskIO
        const int out = GETREG(r);
        // cOrganism::DoOutput -> cTaskLib::SetupTests (main/cTaskLib.cc:369-448)
        outv = out;
        outtot++;
        const int num = intot < 3 ? intot : 3;
        const uint32_t a = num > 0 ? (uint32_t)in0 : 0u;
        const uint32_t b = num > 1 ? (uint32_t)in1 : 0u;
        const uint32_t c = num > 2 ? (uint32_t)in2 : 0u;
        const uint32_t o = (uint32_t)out;
        // logic id (cTaskLib::SetupTests, main/cTaskLib.cc:395-440): per input
        // combination p the output bits where the inputs spell p are all 1
        // (logic[p] = 1), all 0 (0), mixed (no id) or absent (-1); missing
        // inputs repeat the lower half; id = sum logic[p] 2^p.  In bit masks:
        // "ones" / "zeros" seen per p, present P = ones | zeros, and with
        // every logic[p] in {-1, 0, 1}, id = ones - (~P & 0xFF).  With three
        // inputs and every combination present -- always, for SetupInputs'
        // 0x0F/0x33/0x55 top bytes -- that is just the "ones" mask.
        uint32_t ones = 0u, zeros = 0u;
#pragma unroll
        for (int p = 0; p < 8; p++) {
          const uint32_t m = ((p & 1) ? a : ~a) & ((p & 2) ? b : ~b) & ((p & 4) ? c : ~c);
          ones |= min(o & m, 1u) << p;
          zeros |= min(~o & m, 1u) << p;
        }
        // a missing input is 0, so the combinations that need it are absent
        // and their bits are clear: the copies below only fill empty bits
        uint32_t lo = ones, pr = ones | zeros;
        if (num < 1) { lo |= (lo & 1u) << 1; pr |= (pr & 1u) << 1; }
        if (num < 2) { lo |= (lo & 3u) << 2; pr |= (pr & 3u) << 2; }
        if (num < 3) { lo |= (lo & 15u) << 4; pr |= (pr & 15u) << 4; }
        const int id = (int)lo - (int)(~pr & 0xFFu);
        // the task lookup, the rewards and the input follow the switch, with
        // the whole wave converged (io_id: the logic id, or -1 for none)
        io_id = ((ones & zeros) == 0u && id >= 0) ? id : -1;
        CKC(2);
        break; }
      case AVGPU_H_H_ALLOC: {                                 // :3294 Inst_MaxAlloc -> Allocate_Main :1707
        const int cur = M;
        int alloc = (int)(k_size_range * cur);
        if (alloc > AVGPU_MAX_GENOME - cur) alloc = AVGPU_MAX_GENOME - cur;
        const int nsz = cur + alloc;
        const bool ok = !(k_require_allocate && (ctl & CTL_MAL)) && alloc >= 1 &&
                        nsz <= AVGPU_MAX_GENOME && nsz >= AVGPU_MIN_GENOME &&
                        alloc <= (int)(cur * k_size_range) && cur <= (int)(alloc * k_size_range);
        if (!ok) { errs++; break; }                           // cOrganism::Fault
        if (k_alloc_method == 2) {
          for (int i = cur; i < nsz; i++) T[i] = rand_code();
        } else {
          rq = RQ_FILL; qa = cur; qb = nsz;                   // new sites = op 0 (wave fill below)
        }
        M = nsz;
        ctl |= CTL_MAL;
        r0 = cur;
        CKC(3);
        break; }
      case AVGPU_H_H_DIVIDE: {                                // :6961 -> :6942 -> Divide_Main :1775
        ip = head_adjust(ip, M); rh = head_adjust(rh, M); wh = head_adjust(wh, M); fh = head_adjust(fh, M);
        const int div = rh;
        const int child_end = (wh == 0) ? M : wh;
        const int child = child_end - div;
        // Divide_CheckViable (cpu/cHardwareBase.cc:140-289): sizes here, the
        // executed / copied line counts in the wave phase below
        const int min_size = max(AVGPU_MIN_GENOME, (int)(blen / k_size_range));
        const int max_size = min(AVGPU_MAX_GENOME, (int)(blen * k_size_range));
        bool ok = child >= min_size && child <= max_size && div >= min_size && div <= max_size;
        if (!DEF && ok && W.cfg_min_genome && (child < W.cfg_min_genome || div < W.cfg_min_genome)) ok = false;
        if (!DEF && ok && W.cfg_max_genome && (child > W.cfg_max_genome || div > W.cfg_max_genome)) ok = false;
        if (ok) { rq = RQ_DIVIDE; qa = div; qb = child; }
        CKC(4);
        break; }
      case AVGPU_H_H_SEARCH:                                  // :7245 Inst_HeadSearch
      case AVGPU_H_IF_LABEL: {                                // :6914 Inst_IfLabel
        // ReadLabel (:1484-1502), branch free: the up to 10 sites after IP
        // come from one 16-byte window; a byte is a nop iff its code < 3,
        // i.e. (code + 0x7D) has bit 7 clear (codes are <= 0x3F, no carries)
        const int base = ip + 1;
        const int w0 = base >> 2;
        const uint32_t bsh = (uint32_t)(base & 3) * 8u;
        uint64_t lo64 = ((uint64_t)T32[w0 + 1] << 32) | (uint64_t)T32[w0];
        uint64_t hi64 = ((uint64_t)T32[w0 + 3] << 32) | (uint64_t)T32[w0 + 2];
        if (bsh) { lo64 = (lo64 >> bsh) | (hi64 << (64u - bsh)); hi64 >>= bsh; }
        const uint64_t K3F = 0x3F3F3F3F3F3F3F3Full, K7D = 0x7D7D7D7D7D7D7D7Dull, K80 = 0x8080808080808080ull;
        const uint64_t cl = lo64 & K3F, ch = hi64 & K3F;
        const uint64_t nl = (cl + K7D) & K80, nh = (ch + K7D) & K80;
        int len = nl ? (int)(__ffsll((long long)nl) - 8) >> 3 : 8 + (nh ? (int)(__ffsll((long long)nh) - 8) >> 3 : 8);
        len = min(len, min(AVGPU_MAX_LABEL, M - base));
        len = max(len, 0);
        // 2-bit nop codes of bytes 0..7 packed (SWAR), bytes 8, 9 after them
        uint64_t v = cl & 0x0303030303030303ull;
        v = (v | (v >> 6)) & 0x000F000F000F000Full;
        v = (v | (v >> 12)) & 0x000000FF000000FFull;
        v = (v | (v >> 24)) & 0xFFFFull;
        uint32_t lab = (uint32_t)v | ((uint32_t)(ch & 3u) << 16) | ((uint32_t)((ch >> 8) & 3u) << 18);
        const uint32_t lmask = (1u << (2 * len)) - 1u;
        lab &= lmask;
        // executed flags of the label's first sites, from the window's own bytes
        // (no LDS read-modify-write round trip)
        for (int k = 0; k < min(len, k_max_label_exe); k++)
          T[base + k] = (uint8_t)(((k < 8 ? (lo64 >> (8 * k)) : (hi64 >> (8 * (k - 8)))) & 0xFFull) | TF_EXEC);
        ip += len;
        // Rotate(1, NUM_NOPS): per 2-bit digit 0->1, 1->2, 2->0
        const uint32_t dl = lab & 0x55555u, dh = (lab >> 1) & 0x55555u;
        const uint32_t rot = ((~dl & ~dh & 0x55555u) | (dl << 1)) & lmask;
        if (op == AVGPU_H_IF_LABEL) {
          const uint32_t packed = (uint32_t)len | (rot << 4);
          if (packed != rl) ip = head_adjust(ip + 1, M);
          CKC(6);
          break;
        }
        if (len > 0) { rq = RQ_SEARCH; qa = len; qb = (int)rot; CKC(5); break; }   // label scan below
        r1 = 0;                                               // empty label: found = IP
        r2 = 0;
        fh = head_adjust(ip + 1, M);
        CKC(5);
        break; }
      default:
        break;
    }
    }
    // ---- IO, second half (converged): cTaskLib's logic id -> task mask,
    // cEnvironment::TestOutput / TestRequisites / DoProcesses
    // (main/cEnvironment.cc:1314-1406, :1408-1503, :1610-1760), then
    // GetNextInput + DoInput.  Class 0 holds its task LUT spread over the
    // wave's lanes (tl0 / tl1) and reads it by lane shuffles, and its per-task
    // bonus factors (ttab) by v_readlane at a wave-uniform task: a vector load
    // here waited (vmcnt) for every store the wave still had in flight, and a
    // scalar load per task present cost a memory round trip each.
    if (__ballot(io_id >= -1) != 0ull) {
      const bool io = io_id >= -1;
      uint32_t tmask = 0u;
      if (GLUT) {
        const int sl = io_id >= 0 ? (io_id >> 2) : 0;
        const uint32_t a0 = (uint32_t)__shfl((int)tl0, sl), a1 = (uint32_t)__shfl((int)tl1, sl);
        const uint32_t wv = (io_id & 2) ? a1 : a0;
        tmask = io_id >= 0 ? (wv >> ((io_id & 1) * 16)) & 0xFFFFu : 0u;
      } else if (io_id >= 0) {
        tmask = lut[io_id];
      }
      CKC(8);
      if (k_env_simple) {
        // reaction i rewards task i, requisites at most "max_count=1"
        // (capi.hip avgpu_load_env): the firing set is a bit operation and
        // the bonus factors multiply in reaction order (ascending bits)
        uint32_t done = io ? (tmask & k_env_react_mask & ~(k_env_once_mask & nzm)) : 0u;
        if (__ballot(done != 0u) != 0ull) {
          double mult = 1.0, addb = 0.0;
          uint32_t paid = done;
          if (k_env_res_mask != 0u) {
            // finite resources (configs[4]): the event is queued and its
            // bonus, reaction counts and consumption applied at the next
            // flush (res_flush: before a divide of the lane, when its queue is
            // full, at the slice's end) -- nothing else reads them, and only
            // this organism draws on its cell in the slice, so the order of
            // every level, bonus and count is unchanged; the wave pays one
            // memory round trip per flushed rank instead of one per IO
            if (done) {
              const uint32_t n = rpq >> 30;
              rpq = (rpq & 0x07FFFFFFu) | (done << (9 * n)) | ((n + 1u) << 30);
#pragma unroll
              for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] += (done >> q) & 1u;
              nzm |= done;
            }
            done = 0u;
          } else
          for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) {   // wave-uniform t
            const bool dt = (done >> t) & 1u;
            if (__ballot(dt) == 0ull) continue;
            {
              const double fm = GTAB ? __hiloint2double(__builtin_amdgcn_readlane((int)ttab, 2 * t + 1),
                                                        __builtin_amdgcn_readlane((int)ttab, 2 * t)) : tmul[t];
              const double fa = GTAB ? __hiloint2double(__builtin_amdgcn_readlane((int)ttab, 33 + 2 * t),
                                                        __builtin_amdgcn_readlane((int)ttab, 32 + 2 * t)) : tadd[t];
              if (dt) { mult = __dmul_rn(mult, fm); addb = __dadd_rn(addb, fa); }
            }
          }
          if (done) {
#pragma unroll
            for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) {
              tc[q] += (done >> q) & 1u;
              rc[q] += (paid >> q) & 1u;
            }
            nzm |= done;
            bonus = __dadd_rn(__dmul_rn(bonus, mult), addb);   // cPhenotype.cc:1645-1646
          }
        }
      } else if (io && tmask) {
        uint32_t done = 0;
        double mult = 1.0, addb = 0.0;
#pragma unroll
        for (int i = 0; i < AVGPU_MAX_REACTIONS; i++) {
          if (i >= k_n_react) break;
          const int32_t* rt = rtab + i * RT_STRIDE;           // uniform LDS reads
          const int t = rt[RT_TASK];
          int cnt = 0;
#pragma unroll
          for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) cnt = (q == t) ? tc[q] : cnt;
          const bool fire = rt[RT_USED] && ((tmask >> t) & 1u) &&
                            !(rt[RT_HASREQ] && (cnt < rt[RT_MIN] || cnt >= rt[RT_MAX]));
          if (fire) {
            done |= 1u << t;                                  // MarkTask precedes the processes
            const double* rr = W.react_res + i * RR_STRIDE;   // uniform (scalar) loads
            if (!k_env_resources || rr[RR_RES] == 0.0) {      // infinite resource
              if (rt[RT_TYPE] == AVGPU_PROC_ADD)
                addb = __dadd_rn(addb, *reinterpret_cast<const double*>(rt + RT_ADD));
              else
                mult = __dmul_rn(mult, *reinterpret_cast<const double*>(rt + RT_MULT));
              rc[i]++;
            } else if (consume_resource(W, rr, N, cell, mult, addb, mode == AVGPU_MODE_WORLD)) {
              rc[i]++;
            }
          }
        }
        if (done) {
#pragma unroll
          for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] += (done >> q) & 1u;
          nzm |= done;
          bonus = __dadd_rn(__dmul_rn(bonus, mult), addb);     // cPhenotype.cc:1645-1646
        }
      }
      CKC(9);
      if (io) {
        // GetNextInput (main/cOrganism.h:249 -> cPopulationCell.h:214-218) + DoInput
        const int p = inptr >= 3 ? 0 : inptr;
        const int in = p == 0 ? inp0 : (p == 1 ? inp1 : inp2);
        inptr = p + 1;
        in2 = in1; in1 = in0; in0 = in;
        intot++;
        SETREG(pr, in);
      }
      io_id = -2;
    }
    CK(3);

    // a divide reads the bonus and resets the counts: apply its queued rewards first
    if (k_env_res_mask != 0u && __ballot(rpq != 0u && (rq == RQ_DIVIDE || (rpq >> 30) == 3u)) != 0ull)
      res_flush<GTAB>(W, N, cell, rpq, bonus, rc, ttab, tmul, tadd, k_env_res_mask, mode == AVGPU_MODE_WORLD);
    // ---- wave phase: serve the posted requests, one lane at a time ----
    unsigned long long pend = __ballot(rq != RQ_NONE);
    while (pend) {
      const int L = __ffsll((long long)pend) - 1;            // wave-uniform
      pend &= pend - 1ull;
      const int kind = __shfl(rq, L);
      const int a = __shfl(qa, L), b = __shfl(qb, L);
      uint32_t* TL32 = lds32 + L * (STRIDE / 4);
      const uint8_t* TL = lds + L * STRIDE;
      if (kind == RQ_FILL) {
        // Allocate_Main: new sites [a, b) get op 0 (ALLOC_METHOD 0/1)
        for (int w = (a >> 2) + lane; (w << 2) < b; w += 64) {
          const uint32_t keep = byte_mask(w << 2, a, b);
          TL32[w] = (TL32[w] & ~keep) | (fill4 & keep);
        }
      } else if (kind == RQ_SEARCH) {
        // FindLabel(0) -> FindLabel_Forward(label, memory, 0) (:1177-1295).
        // The reference probes every label_size sites and, inside a probed
        // nop run, tests every offset; every maximal nop run that can hold the
        // label is probed except a run that ends exactly at label_size.  Its
        // answer is therefore the smallest offset o whose label_size sites
        // spell the label (all nops) and that is not that unprobed run
        // (o > 0, or site label_size is a nop).  Lane t tests the window that
        // ends at site base + t.
        const int len = a;
        const uint32_t rot = (uint32_t)b;
        const int ML = __shfl(M, L);
        const bool run0_ok = len < ML && (TL[len] & CODE_MASK) < 3;
        int fpos = -1;
        for (int base = 0; base < ML && fpos < 0; base += 64) {
          const int j = base + lane;
          bool m = j < ML && j >= len - 1 && (j != len - 1 || run0_ok);
          if (m) {
            const int st = j - len + 1;
            const int w0 = st >> 2;
            const uint64_t lo64 = ((uint64_t)TL32[w0 + 1] << 32) | (uint64_t)TL32[w0];
            const uint64_t hi64 = ((uint64_t)TL32[w0 + 3] << 32) | (uint64_t)TL32[w0 + 2];
            const int b0 = st & 3;
            for (int i = 0; i < len; i++) {
              const int k = b0 + i;
              const uint32_t cc = (uint32_t)(((k < 8) ? (lo64 >> (8 * k)) : (hi64 >> (8 * (k - 8)))) & CODE_MASK);
              m = m && cc == ((rot >> (2 * i)) & 3u);
            }
          }
          const unsigned long long bm = __ballot(m);
          if (bm) fpos = base + __ffsll((long long)bm);        // first site after the label
        }
        if (lane == L) {
          const int found = fpos >= 0 ? head_adjust(fpos - 1, M) : ip;
          r1 = found - ip;
          r2 = len;
          fh = head_adjust(found + 1, M);
        }
      } else {
        // ---- Divide_Main (:1775-1843) for lane L ----
        const int div = a, child = b;
        // calcExecutedSize (cpu/cHardwareBase.cc:130-138), calcCopiedSize (cpu/cHardwareCPU.cc:1765-1772)
        int ne = 0, nc = 0;
        for (int w = lane; (w << 2) < div + child; w += 64) {
          const uint32_t v = TL32[w];
          ne += __popc(v & (TF_EXEC * 0x01010101u) & byte_mask(w << 2, 0, div));
          nc += __popc(v & (TF_COPIED * 0x01010101u) & byte_mask(w << 2, div, div + child));
        }
        // both counts (<= AVGPU_MAX_GENOME each) in one reduction: halves of one word
        const int both = wave_sum_i32(ne | (nc << 16));
        const int exe = both & 0xFFFF, cop = both >> 16;
        int okw = 0, rec = -1, len = 0, e0 = 0, e1 = 0, e2 = 0, e3 = 0, e4 = 0;   // edits: slip mut ins del uniform
        int pcnt[NSEG] = {0}, pofs[NSEG] = {0};   // variable-count edit segments in b_subs (device.h)
        if (lane == L) {
          // The world parameters and phenotype arrays this block uses, loaded
          // together and made opaque (OPQ): the asm stores below are
          // scheduling barriers, and the compiler re-issued each invariant
          // scalar load just before its use -- one load-to-use wait per field.
          double p_min_exe = DEF ? 0.5 : W.min_exe_lines, p_min_cop = DEF ? 0.5 : W.min_copied_lines;
          double p_req = DEF ? 0.0 : W.required_bonus;
          double p_mdb = DEF ? 0.0 : W.merit_default_bonus, p_defb = DEF ? 1.0 : W.default_bonus;
          int p_inherit = DEF ? 1 : W.inherit_merit, p_bmm = DEF ? 4 : W.base_merit_method;
          int p_bcm = W.base_const_merit;
          double* g_merit = W.merit;
          double* g_fitness = W.fitness;
          int32_t* g_gest = W.gest_time;
          int32_t* g_ccop = W.child_copied;
          int32_t* g_exec = W.executed;
          int32_t* g_ltask = W.last_task;
          OPQ(p_bcm);
          if (!DEF) { OPQ(p_min_exe); OPQ(p_min_cop); OPQ(p_req); OPQ(p_defb); OPQ(p_mdb); OPQ(p_inherit); OPQ(p_bmm); }
          OPQ(g_merit); OPQ(g_fitness); OPQ(g_gest); OPQ(g_ccop); OPQ(g_exec); OPQ(g_ltask);
          bool ok = exe >= (int)(div * p_min_exe) && cop >= (int)(child * p_min_cop);
          double bon = bonus;
          if (ok) {  // cOrganism::Divide_CheckViable (main/cOrganism.cc:788-919)
            if (bon < p_req) ok = false;
            if (!DEF && W.div_req) {
              // the required task unless the immunity task was done, the
              // required reaction likewise (no stolen reactions on this
              // path), at most MAX_UNIQUE_TASK_COUNT distinct tasks, with
              // REQUIRE_SINGLE_REACTION some reaction (:826-880)
              int nt = 0, ct_req = 0, ct_imm = 0, cr_req = 0, cr_imm = 0, any = 0;
#pragma unroll
              for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) {
                nt += tc[q] > 0 ? 1 : 0;
                ct_req = q == W.req_task ? tc[q] : ct_req;
                ct_imm = q == W.imm_task ? tc[q] : ct_imm;
              }
#pragma unroll
              for (int q = 0; q < 12; q++) {
                cr_req = q == W.req_react ? rc[q] : cr_req;
                cr_imm = q == W.imm_react ? rc[q] : cr_imm;
                any |= rc[q];
              }
              if (W.req_task >= 0 && ct_req == 0 && (W.imm_task < 0 || ct_imm == 0)) ok = false;
              if (!W.single_react && W.req_react >= 0 && cr_req == 0 && (W.imm_react < 0 || cr_imm == 0)) ok = false;
              if (W.max_task_cnt > 0 && nt > W.max_task_cnt) ok = false;
              if (W.single_react && any == 0) ok = false;
            }
            const double base0 = (double)size_merit(p_bmm, p_bcm, blen, dcop, dexe);
            double b0 = bon;
            if (p_mdb != 0.0) b0 = p_mdb;
            double off_merit = __dmul_rn(base0, b0);
            if (p_inherit == 0) off_merit = base0;
            if (off_merit == 0.0) ok = false;
          }
          if (NB && ok) {
            // the newborn pass ends before a viable divide: the instruction's
            // cycle is taken back (its executed flag stays -- it is set again
            // when the divide runs) and the slice stops with the IP on it
            ok = false;
            fl |= F_STOP;
            cyc--; tu--; executed--;
          }
          if (ok) {
            okw = 1;
            dexe = exe;                                       // SetLinesExecuted
            const int nd = dnd + 1;
            // DivideReset / TestDivideReset (main/cPhenotype.cc:824-1000, :1064-1180)
            const double base = (double)size_merit(p_bmm, p_bcm, blen, dcop, exe);
            if (p_mdb != 0.0) bon = p_mdb;
            double merit = __dmul_rn(base, bon);
            if (p_inherit == 0) merit = base;
            const int gt = tu - gs;
            // The parent's phenotype (merit, fitness, gestation time, copied /
            // executed size, last task counts) and the offspring's fitness and
            // RNG key: a world slice at the default knobs leaves them to
            // finalize_key / finalize_phenotype (world.hip, placement round 0: SIMT over the
            // records, where here one lane at a time ran them with the wave
            // waiting); otherwise, or without a record, they are stored here.
            const bool defer = DEF && mode == AVGPU_MODE_WORLD && !serial;
            auto parent_phenotype = [&]() {
              const double fit = __ddiv_rn(__dmul_rn(base, bon), (double)gt);
              // write-only fields go out now (fire and forget) rather than
              // being held in registers to the end of the slice
              st_async_u64(g_merit + cell, (uint64_t)__double_as_longlong(merit));
              st_async_u64(g_fitness + cell, (uint64_t)__double_as_longlong(fit));
              st_async_u32(g_gest + cell, (uint32_t)gt);
              st_async_u32(g_ccop + cell, (uint32_t)cop);     // SetLinesCopied
              st_async_u32(g_exec + cell, (uint32_t)exe);
#pragma unroll
              for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++)
                st_async_u32(g_ltask + (int64_t)q * N + cell, (uint32_t)tc[q]);
            };
            if (!defer) parent_phenotype();
            gs = tu;
            dnd = nd;
            const int gen = dgen + 1;
            dgen = gen;
            didv = true;
            errs = 0;
            bonus = p_defb;
            cyc = 0;
            nzm = 0;
#pragma unroll
            for (int i = 0; i < AVGPU_MAX_REACTIONS; i++) rc[i] = i < k_n_react ? 0 : rc[i];
            len = child;
            if (mode == AVGPU_MODE_TEST) {
              st_async_u32(W.t_flags_len + cell, (uint32_t)div);
              st_async_u32(W.t_child_len + cell, (uint32_t)child);
              fl |= F_STOP;
            } else {
              // Divide_DoMutations (cpu/cHardwareBase.cc:296-569) in the
              // reference's order of draws (oracle divide_mutations): slip,
              // mut, ins, del always draw; uniform only at a non-zero rate.
              // The offspring is this lane's child sites under up to 5 edits,
              // one fixed slot per kind (e0 .. e4, 0 = none) in the order applied.
              uint64_t t_slip = W.th_div_slip, t_mut = W.th_div_mut, t_ins = W.th_div_ins;
              uint64_t t_del = W.th_div_del, t_uni = DEF ? 0ull : W.th_div_uni;
              double q_slip = W.p_div_slip, q_mut = W.p_div_mut, q_ins = W.p_div_ins;
              double q_del = W.p_div_del, q_uni = W.p_div_uni;
              int g_max = W.max_genome, g_min = W.min_genome;
              OPQ(t_slip); OPQ(t_mut); OPQ(t_ins); OPQ(t_del);
              if (!DEF) OPQ(t_uni);
              OPQ(q_slip); OPQ(q_mut); OPQ(q_ins); OPQ(q_del); OPQ(q_uni); OPQ(g_max); OPQ(g_min);
              // NumDividePoisson* (main/cMutationRates.h:137-144; Apto's
              // GetRandPoisson restated as in the oracle: multiply uniforms
              // until the product falls below exp(-mean)), each kind's edits
              // right after its one-shot test, in an arena segment (WORLD)
              const bool segs = !DEF && W.seg_any;
              // the longest the offspring gets while its edits apply: edit
              // words hold 12-bit positions, so an offspring that passes 4095
              // sites on the way is dropped as oversize (the oracle too)
              int lmax = len;
              const bool pois = !DEF && W.pois_any;
              auto draw_u = [&]() -> double {
                if (REC && rbase) return rd();
                return (double)rng_next(klo, khi, kct) * 2.3283064365386963e-10;
              };
              auto npois = [&](int k) -> int {
                const double Lk = W.pois_L[k];
                if (!(Lk > 0.0)) return 0;
                double x = draw_u();
                int n = 0;
                while (x >= Lk && n < 4096) { x = __dmul_rn(x, draw_u()); n++; }
                return n;
              };
              // GetRandBinomial(len, p): one P(p) per site (oracle binom)
              auto nbinom = [&](uint64_t th, double p) -> int {
                int n = 0;
                for (int i = 0; i < len; i++) n += draw_p(th, p) ? 1 : 0;
                return n;
              };
              // reserve n words of segment k / write its i-th edit (WORLD only)
              // (a full arena stops taking reservations, so its int32 fill
              // cannot wrap: a reservation refused is placed at scap, i.e. it
              // overflows below)
              auto preserve = [&](int k, int n) {
                if (n > 0 && mode == AVGPU_MODE_WORLD)
                  pofs[k] = (int64_t)__atomic_load_n(W.b_count + 2, __ATOMIC_RELAXED) >= W.scap
                                ? (int)W.scap : atomicAdd(W.b_count + 2, n);
              };
              auto pput = [&](int k, int i, int ew) {
                if (mode == AVGPU_MODE_WORLD && pofs[k] >= 0 && (int64_t)pofs[k] + i < W.scap) W.b_subs[pofs[k] + i] = ew;
              };
              // Data fills (SLIP_FILL_MODE 2 / 3, TRANS_FILL_MODE 1): after a
              // slip's or translocation's from / to (/ ins_loc) draws, its L
              // fill draws in the reference's order (:636-665, :721-741):
              // GetRandomInst per site (2), or GetInt(L - i) per site with the
              // scrambled walk over copied_so_far (3, translocation 1).  The
              // interpreter resolves them into the arena (WORLD): codes, or
              // the source site of each filled site in the sequence before the
              // edit -- a scrambled translocation that reads a site it already
              // filled takes that site's source.  A bit set of L bits after
              // the L words marks the indices taken.  Other modes only draw.
              const int sfm = DEF ? 0 : W.slip_fill_mode, tfm = DEF ? 0 : W.trans_fill_mode;
              const bool sdata = sfm == 2 || sfm == 3, tdata = tfm == 1;
              bool ftrunc = false;
              auto fill_draws = [&](int kind, int L, int to, int ins_loc) -> int {
                if (L <= 0) return -1;
                const int nbw = kind == 2 ? 0 : (L + 31) >> 5;
                int off = -1;
                if (mode == AVGPU_MODE_WORLD) {
                  if ((int64_t)__atomic_load_n(W.b_count + 2, __ATOMIC_RELAXED) < W.scap) {
                    const int o = atomicAdd(W.b_count + 2, L + nbw);
                    if ((int64_t)o + L + nbw <= W.scap) off = o;
                  }
                  if (off < 0) ftrunc = true;
                }
                int32_t* f = off >= 0 ? W.b_subs + off : nullptr;
                uint32_t* bits = f ? reinterpret_cast<uint32_t*>(f + L) : nullptr;
                if (bits)
                  for (int q = 0; q < nbw; q++) bits[q] = 0u;
                for (int i = 0; i < L; i++) {
                  if (kind == 2) {
                    const int v = rand_code();
                    if (f) f[i] = v;
                    continue;
                  }
                  int rem = (int)draw_below((uint32_t)(L - i));
                  if (!f) continue;
                  int wd = 0;                              // the rem-th index not taken
                  while (true) {
                    const int fr = 32 - __popc(bits[wd]);
                    if (rem < fr) break;
                    rem -= fr;
                    wd++;
                  }
                  uint32_t z = ~bits[wd];
                  for (int q = 0; q < rem; q++) z &= z - 1u;
                  const int bit = __ffs((int)z) - 1;
                  bits[wd] |= 1u << bit;
                  int src = to + wd * 32 + bit;
                  if (kind == 5 && src >= ins_loc && src < ins_loc + i) src = f[src - ins_loc];
                  f[i] = src;
                }
                return off;
              };
              auto slip_edit = [&](int k, int i) {   // doSlipMutation :621-694 into segment k
                const int from = (int)draw_below((uint32_t)len + 1u);
                const int to = from == 0 ? (int)draw_below((uint32_t)len) : (int)draw_below((uint32_t)len + 1u);
                if (sdata) {
                  const int fo = fill_draws(sfm, from - to, to, 0);
                  pput(k, 2 * i, edit_word(E_SLIP, from, to));
                  pput(k, 2 * i + 1, fo);
                } else {
                  pput(k, i, edit_word(E_SLIP, from, to));
                }
                len += from - to;
                lmax = max(lmax, len);
              };
              const int sw = sdata ? 2 : 1, tw = tdata ? 3 : 2;   // words per slip / translocation
              auto uniform_edit = [&]() -> int {   // doUniformMutation :572-595
                const int mut = (int)draw_below((uint32_t)(2 * k_n_ops + 1));
                int ew = 0;
                if (mut < k_n_ops) {
                  ew = edit_word(E_POINT, (int)draw_below((uint32_t)len), (int)tab_u8(rcode + mut));
                } else if (mut == k_n_ops) {
                  if (len != g_min) { ew = edit_word(E_DEL, (int)draw_below((uint32_t)len), 0); len--; }
                } else if (len != g_max) {
                  ew = edit_word(E_INS, (int)draw_below((uint32_t)len + 1u), (int)tab_u8(rcode + mut - k_n_ops - 1));
                  len++;
                  lmax = max(lmax, len);
                }
                return ew;
              };
              if (draw_p(t_slip, q_slip)) {          // doSlipMutation :621-694
                if (segs && sdata) {                   // as a segment, with its fill
                  preserve(SEG_OSLIP, 2);
                  slip_edit(SEG_OSLIP, 0);
                  pcnt[SEG_OSLIP] = 2;
                } else {
                  const int from = (int)draw_below((uint32_t)len + 1u);
                  const int to = from == 0 ? (int)draw_below((uint32_t)len) : (int)draw_below((uint32_t)len + 1u);
                  if (sdata) fill_draws(sfm, from - to, to, 0);   // (no arena: the draws only)
                  e0 = edit_word(E_SLIP, from, to);
                  len += from - to;
                  lmax = max(lmax, len);
                }
              }
              if (pois) {                            // Poisson slips :318-320
                const int n = npois(0);
                preserve(SEG_PSLIP, sw * n);
                for (int i = 0; i < n; i++) slip_edit(SEG_PSLIP, i);
                pcnt[SEG_PSLIP] = sw * n;
              }
              if (segs && W.th_dsite[3]) {           // slips per site :323-327
                const int n = nbinom(W.th_dsite[3], W.p_dsite[3]);
                preserve(SEG_SSLIP, sw * n);
                for (int i = 0; i < n; i++) slip_edit(SEG_SSLIP, i);
                pcnt[SEG_SSLIP] = sw * n;
              }
              // translocations (doTransMutation :700-760): from, to, then the
              // insertion site on the size before it, then the fill's draws
              auto trans_edit = [&](int k, int i) {
                const int from = (int)draw_below((uint32_t)len + 1u);
                const int to = from == 0 ? (int)draw_below((uint32_t)len) : (int)draw_below((uint32_t)len + 1u);
                const int ins_loc = (int)draw_below((uint32_t)len + 1u);
                pput(k, tw * i, edit_word(E_TRANS, ins_loc, to));
                pput(k, tw * i + 1, from);
                if (tdata) pput(k, tw * i + 2, fill_draws(5, from - to, to, ins_loc));
                len += from - to;
                lmax = max(lmax, len);
              };
              if (segs && W.th_dtrans && draw_p(W.th_dtrans, W.p_dtrans)) {   // one-shot :331
                preserve(SEG_TTRANS, tw);
                trans_edit(SEG_TTRANS, 0);
                pcnt[SEG_TTRANS] = tw;
              }
              if (pois) {                            // Poisson translocations :334-335
                const int n = npois(4);
                preserve(SEG_PTRANS, tw * n);
                for (int i = 0; i < n; i++) trans_edit(SEG_PTRANS, i);
                pcnt[SEG_PTRANS] = tw * n;
              }
              if (segs && W.th_dsite[4]) {           // translocations per site :338-342
                const int n = nbinom(W.th_dsite[4], W.p_dsite[4]);
                preserve(SEG_STRANS, tw * n);
                for (int i = 0; i < n; i++) trans_edit(SEG_STRANS, i);
                pcnt[SEG_STRANS] = tw * n;
              }
              if (draw_p(t_mut, q_mut)) {
                const int line = (int)draw_below((uint32_t)len);
                e1 = edit_word(E_POINT, line, rand_code());
              }
              if (pois) {                            // Poisson substitutions :383-391
                const int n = npois(1);
                preserve(SEG_PMUT, n);
                for (int i = 0; i < n; i++) {
                  const int line = (int)draw_below((uint32_t)len);
                  pput(SEG_PMUT, i, edit_word(E_POINT, line, rand_code()));
                }
                pcnt[SEG_PMUT] = n;
              }
              if (draw_p(t_ins, q_ins) && len < g_max) {
                const int line = (int)draw_below((uint32_t)len + 1u);
                e2 = edit_word(E_INS, line, rand_code());
                len++;
                lmax = max(lmax, len);
              }
              if (pois) {                            // Poisson insertions :404-413
                const int n = npois(2);
                preserve(SEG_PINS, n);
                int used = 0;
                for (int i = 0; i < n && len < g_max; i++) {
                  const int line = (int)draw_below((uint32_t)len + 1u);
                  pput(SEG_PINS, i, edit_word(E_INS, line, rand_code()));
                  len++;
                  lmax = max(lmax, len);
                  used++;
                }
                pcnt[SEG_PINS] = used;
              }
              if (draw_p(t_del, q_del) && len > g_min) {
                e3 = edit_word(E_DEL, (int)draw_below((uint32_t)len), 0);
                len--;
              }
              if (pois) {                            // Poisson deletions :426-435
                const int n = npois(3);
                preserve(SEG_PDEL, n);
                int used = 0;
                for (int i = 0; i < n && len > g_min; i++) {
                  pput(SEG_PDEL, i, edit_word(E_DEL, (int)draw_below((uint32_t)len), 0));
                  len--;
                  used++;
                }
                pcnt[SEG_PDEL] = used;
              }
              if (t_uni && draw_p(t_uni, q_uni)) e4 = uniform_edit();
              // the per-site kinds (cpu/cHardwareBase.cc:447-503), each only at
              // a non-zero rate, in the reference's order: substitutions,
              // insertions (all sites drawn, sorted, inserted from the highest
              // down), deletions, uniform mutations
              if (segs && W.th_div_site) {
                const int n = nbinom(W.th_div_site, W.p_div_site);
                preserve(SEG_SMUT, n);
                for (int i = 0; i < n; i++) {
                  const int site = (int)draw_below((uint32_t)len);
                  pput(SEG_SMUT, i, edit_word(E_POINT, site, rand_code()));
                }
                pcnt[SEG_SMUT] = n;
              }
              if (segs && W.th_dsite[0]) {
                int n = nbinom(W.th_dsite[0], W.p_dsite[0]);
                if (n + len > g_max) n = g_max - len;
                if (n > 0) {
                  preserve(SEG_SINS, n);
                  const bool keep = mode == AVGPU_MODE_WORLD && (int64_t)pofs[SEG_SINS] + n <= W.scap;
                  int32_t* seg = W.b_subs + pofs[SEG_SINS];
                  for (int i = 0; i < n; i++) {
                    const int site = (int)draw_below((uint32_t)len + 1u);
                    if (keep) {                // insertion sort, highest first
                      int j = i;
                      while (j > 0 && seg[j - 1] < site) { seg[j] = seg[j - 1]; j--; }
                      seg[j] = site;
                    }
                  }
                  for (int i = 0; i < n; i++) {
                    const int code = rand_code();
                    if (keep) seg[i] = edit_word(E_INS, seg[i], code);
                  }
                  len += n;
                  lmax = max(lmax, len);
                  pcnt[SEG_SINS] = n;
                }
              }
              if (segs && W.th_dsite[1]) {
                int n = nbinom(W.th_dsite[1], W.p_dsite[1]);
                if (len - n < g_min) n = len - g_min;
                if (n > 0) {
                  preserve(SEG_SDEL, n);
                  for (int i = 0; i < n; i++) {
                    pput(SEG_SDEL, i, edit_word(E_DEL, (int)draw_below((uint32_t)len), 0));
                    len--;
                  }
                  pcnt[SEG_SDEL] = n;
                }
              }
              if (segs && W.th_dsite[2]) {
                const int n = nbinom(W.th_dsite[2], W.p_dsite[2]);
                preserve(SEG_SUNI, n);
                for (int i = 0; i < n; i++) pput(SEG_SUNI, i, uniform_edit());
                pcnt[SEG_SUNI] = n;
              }
              // a segment that did not fit the arena (its edits were not all
              // written): the offspring cannot be rebuilt, so it is dropped
              // (counted in CNT_SUB_OVERFLOW and CNT_DROPPED; tests require 0)
              bool truncated = false;
              if (ftrunc) { count_add(W, CNT_SUB_OVERFLOW, 1ull); truncated = true; }   // a fill found the arena full
              if (segs && mode == AVGPU_MODE_WORLD)
#pragma unroll
                for (int k = 0; k < NSEG; k++)
                  if (pcnt[k] > 0 && ((int64_t)pofs[k] < 0 || (int64_t)pofs[k] + pcnt[k] > W.scap)) {
                    count_add(W, CNT_SUB_OVERFLOW, (unsigned long long)pcnt[k]);
                    truncated = true;
                  }
              // (the parent's own mutations -- Divide_DoMutations' last draws,
              // cpu/cHardwareBase.cc:508-565 -- follow the child's copy-out below:
              // insertions shift the sites the child still occupies)
              // record (WORLD): the cell's primary record for the slice's
              // first offspring, an overflow record (atomic) for any further
              // one; an offspring a slip grew past the largest genome is dropped
              if (mode == AVGPU_MODE_WORLD && (len > AVGPU_MAX_GENOME || lmax > 4095)) {
                ndrop++;
                noversize++;
              } else if (mode == AVGPU_MODE_WORLD && truncated) {
                ndrop++;
              } else if (mode == AVGPU_MODE_WORLD) {
              rec = cell;
              if (prim) {
                rec = (int)min((int64_t)W.n + atomicAdd(W.b_count + 1, 1), W.rcap);
                if (rec >= W.rcap) { rec = -1; ndrop++; }
              }
              prim = true;
              }
              if (serial && rec >= 0) sbirth = 1;      // placed by the caller before any speculation
              if (defer && rec < 0) parent_phenotype();   // no record to carry it
              if (rec >= 0) {
                uint32_t clo = 0u, chi = 0u;
                if (!defer) derive_key(olo, ohi, (uint32_t)nd, 0x1B873593U, clo, chi);
                // the record arrays, loaded together (see OPQ above)
                int32_t* b_parent = W.b_parent;
                uint32_t* b_seq = W.b_seq;
                int32_t* b_len = W.b_len;
                int32_t* b_len0 = W.b_len0;
                int32_t* b_edit = W.b_edit;
                int8_t* b_state = W.b_state;
                int32_t* b_target = W.b_target;
                int32_t* b_inh = W.b_inh;
                int64_t rcap = W.rcap;
                OPQ(b_parent); OPQ(b_seq); OPQ(b_len); OPQ(b_len0); OPQ(b_edit);
                OPQ(b_state); OPQ(b_target); OPQ(b_inh); OPQ(rcap);
                st_async_u32(b_parent + rec, (uint32_t)cell);
                st_async_u32(b_seq + rec, (uint32_t)nd);
                st_async_u32(b_len + rec, (uint32_t)len);
                st_async_u32(b_len0 + rec, (uint32_t)child);   // the placement launch edits the copy
                st_async_u32(b_edit + rec, (uint32_t)e0);
                st_async_u32(b_edit + rcap + rec, (uint32_t)e1);
                st_async_u32(b_edit + 2 * rcap + rec, (uint32_t)e2);
                st_async_u32(b_edit + 3 * rcap + rec, (uint32_t)e3);
                st_async_u32(b_edit + 4 * rcap + rec, (uint32_t)e4);
                if (!DEF && W.seg_any)
#pragma unroll
                  for (int k = 0; k < NSEG; k++) {
                    W.b_pofs[(int64_t)k * rcap + rec] = pofs[k];
                    W.b_pcnt[(int64_t)k * rcap + rec] = pcnt[k];
                  }
                // the inherited phenotype: one 128-B row, 16-B stores (device.h BI_*)
                // (deferred: fitness and key left to world.hip's finalize_*, BI_FINAL bit 0)
                int32_t* irow = b_inh + (int64_t)rec * BI_WORDS;
                const long long mb = __double_as_longlong(merit);
                const long long fb = defer ? 0ll : __double_as_longlong(__ddiv_rn(__dmul_rn(base, bon), (double)gt));
                st_async_b128(irow, (uint32_t)mb, (uint32_t)(mb >> 32), (uint32_t)fb, (uint32_t)(fb >> 32));
                st_async_b128(irow + 4, (uint32_t)gen, (uint32_t)cop, (uint32_t)exe, (uint32_t)gt);
                // birth time t = k / (b + 1) in 1/2^16 (oracle birth_time): k the
                // slice's instructions so far, the h-divide included; b its budget
                const int kdone = sdone + executed;
                const uint32_t tb = (uint32_t)__ddiv_rn(__dmul_rn((double)kdone, 65536.0),
                                                        (double)((int64_t)kdone + budget + 1));
                st_async_b128(irow + 8, clo, chi, 0u, (defer ? 1u : 0u) | (tb << 16));
                st_async_b128(irow + 12, (uint32_t)tc[0], (uint32_t)tc[1], (uint32_t)tc[2], (uint32_t)tc[3]);
                st_async_b128(irow + 16, (uint32_t)tc[4], (uint32_t)tc[5], (uint32_t)tc[6], (uint32_t)tc[7]);
                st_async_b128(irow + 20, (uint32_t)tc[8], 0u, 0u, 0u);
                st_async_u8(b_state + rec, 0u);
                st_async_u32(b_target + rec, 0xFFFFFFFFu);
              }
            }
#pragma unroll
            for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] = 0;
            divides++;
            // parent: Resize(div), Reset (:813-900), ClearFlags (:1839); no IP advance
            M = div;
            r0 = r1 = r2 = 0;
            ip = rh = wh = fh = 0;
            ctl = CTL_ALIVE;
            rl = 0;
            adv = false;
          }
        }
        okw = __shfl(okw, L);
        if (okw) {
          rec = __shfl(rec, L); len = __shfl(len, L);
          const int cell_l = __shfl(cell, L);
          if (mode == AVGPU_MODE_TEST) {
            // test-CPU snapshots: executed flags of the parent part, the offspring
            uint8_t* fl = W.t_flags + (int64_t)cell_l * TAPE_SLOT;
            uint8_t* ch = W.t_child + (int64_t)cell_l * TAPE_SLOT;
            for (int w = lane; (w << 2) < div; w += 64) {
              uint32_t wd = 0;
#pragma unroll
              for (int q = 0; q < 4; q++)
                wd |= (uint32_t)((TL[4 * w + q] & TF_EXEC) ? '+' : '-') << (8 * q);
              st_async_u32(fl + 4 * w, wd);
            }
            for (int w = lane; (w << 2) < child; w += 64) {
              uint32_t wd = 0;
#pragma unroll
              for (int q = 0; q < 4; q++) wd |= (uint32_t)(TL[div + 4 * w + q] & CODE_MASK) << (8 * q);
              st_async_u32(ch + 4 * w, wd);
            }
          } else if (mode == AVGPU_MODE_WORLD && rec >= 0) {
            // the unmutated child, 4 sites per lane; its divide mutations are
            // applied by k_place_pick_mut / k_tile_prep (world.hip) before placement, from
            // the edits stored with the record -- keeping the per-site edit
            // composition out of this kernel's registers
            uint8_t* g = W.b_genome + (int64_t)rec * TAPE_SLOT;
            const uint32_t dsh = (uint32_t)(div & 3) * 8u;
            for (int w = lane; (w << 2) < child; w += 64) {
              const int a = (div >> 2) + w;                 // aligned words around sites div+4w ..
              const uint32_t lo = TL32[a], hi = TL32[a + 1];
              const uint32_t v = dsh ? ((lo >> dsh) | (hi << (32u - dsh))) : lo;
              st_async_u32(g + 4 * w, v & 0x3F3F3F3Fu & byte_mask(w << 2, 0, child));
            }
          }
          // Parent Substitution / Insert / Deletion Mutations (per site)
          // (cpu/cHardwareBase.cc:508-565) on the parent's memory, already cut
          // to the divide point, in lane L's LDS tape: the last draws of
          // Divide_DoMutations, so drawing them after the child's copy-out
          // keeps the reference's order.  Insertions: all sites drawn
          // (GetUInt(size + 1)), sorted, inserted from the highest down with
          // a GetRandomInst each, capped at the largest genome; deletions capped
          // at the smallest; new sites have flags 0 (cleared below anyway).
          if (!DEF && mode != AVGPU_MODE_TEST && lane == L && (W.th_par_site || W.th_par_ins || W.th_par_del)) {
            int g_max = W.max_genome, g_min = W.min_genome;
            if (W.th_par_site) {
              int npar = 0;
              for (int i = 0; i < M; i++) npar += draw_p(W.th_par_site, W.p_par_site) ? 1 : 0;
              for (int i = 0; i < npar; i++) {
                const int site = (int)draw_below((uint32_t)M);
                T[site] = (uint8_t)((T[site] & ~CODE_MASK) | rand_code());
              }
            }
            if (W.th_par_ins) {
              int nins = 0;
              for (int i = 0; i < M; i++) nins += draw_p(W.th_par_ins, W.p_par_ins) ? 1 : 0;
              if (nins + M > g_max) nins = g_max - M;
              // the sorted sites sit in the last 4 * nins bytes of the slot
              // and the parent grows below them: M + 5 * nins <= S.  A parent
              // near its slot's end keeps the insertions that fit (the rest
              // counted in CNT_MEM_CAP; the oracle has no slot, tests require 0)
              const int nfit = (Scap - M) / 5;
              if (nins > nfit) {
                count_add(W, CNT_MEM_CAP, (unsigned long long)(nins - nfit));
                nins = nfit;
              }
              if (nins > 0) {
                // (the child's copy-out has read those bytes)
                int32_t* srt = reinterpret_cast<int32_t*>(T + Scap - 4 * nins);
                for (int i = 0; i < nins; i++) {
                  const int site = (int)draw_below((uint32_t)M + 1u);
                  int j = i;
                  while (j > 0 && srt[j - 1] > site) { srt[j] = srt[j - 1]; j--; }
                  srt[j] = site;
                }
                for (int i = nins - 1; i >= 0; i--) {
                  const int pos = srt[i];
                  const int code = rand_code();
                  for (int k = M; k > pos; k--) T[k] = T[k - 1];
                  T[pos] = (uint8_t)code;
                  M++;
                }
              }
            }
            if (W.th_par_del) {
              int ndel = 0;
              for (int i = 0; i < M; i++) ndel += draw_p(W.th_par_del, W.p_par_del) ? 1 : 0;
              if (M - ndel < g_min) ndel = M - g_min;
              for (int i = 0; i < ndel; i++) {
                const int site = (int)draw_below((uint32_t)M);
                for (int k = site; k < M - 1; k++) T[k] = T[k + 1];
                M--;
              }
            }
          }
          // parent ClearFlags over its remaining sites, empty stacks
          const int pmem = __shfl(M, L);
          for (int w = lane; (w << 2) < pmem; w += 64) TL32[w] &= 0x3F3F3F3Fu;
          if (VSTK) {
            if (lane == L) {
#pragma unroll
              for (int i = 0; i < 2 * AVGPU_STACK_SIZE; i++) sv[i] = 0;
            }
          } else if (lane < 2 * AVGPU_STACK_SIZE) {
            stk[lane * 64 + L] = 0;
          }
        }
      }
    }

    if (sstep && !(fl & F_STOP)) {
      if (adv) ip = head_adjust(ip + 1, M);                   // ip.Advance() :1013
      if (mx > 0 && tu >= mx) {                               // death :1045-1049
        if (serial == 2) { sdie = 1; fl |= F_STOP; executed--; }
        else fl |= F_DEAD;
      }
    }
    pop = -1;
    CK(4);
    }
  }
#undef CK
#undef CKC
#undef GETREG
#undef SETREG
#undef GETHEAD
#undef SETHEAD

  if (k_env_res_mask != 0u)
    res_flush<GTAB>(W, N, cell, rpq, bonus, rc, ttab, tmul, tadd, k_env_res_mask, mode == AVGPU_MODE_WORLD);
  // ---- write back ----
#ifdef AVGPU_PHASE_CLOCKS
  const uint64_t clk2 = __builtin_amdgcn_s_memtime();
#endif
  __syncthreads();
  if (active) {
    // the execution record: words 0..51 in 13 16-byte stores (whole 32-B
    // sectors of the cell's own lines)
    int4* xw = reinterpret_cast<int4*>(xrec);
    const long long bb = __double_as_longlong(bonus);
    xw[0] = make_int4(r0, r1, r2, ip);
    xw[1] = make_int4(rh, wh, fh, (int)rl);
    xw[2] = make_int4(cyc, tu, gs, errs);
    xw[3] = make_int4(in0, in1, in2, intot);
    xw[4] = make_int4(inptr, outv, outtot, 0);
    xw[5] = make_int4((int)(uint32_t)bb, (int)(bb >> 32), tc[0], tc[1]);
    xw[6] = make_int4(tc[2], tc[3], tc[4], tc[5]);
    xw[7] = make_int4(tc[6], tc[7], tc[8], 0);
#pragma unroll
    for (int j = 0; j < 5; j++)
      xw[8 + j] = VSTK ? make_int4(sv[4 * j], sv[4 * j + 1], sv[4 * j + 2], sv[4 * j + 3])
                       : make_int4(stk[(4 * j) * 64 + lane], stk[(4 * j + 1) * 64 + lane],
                                   stk[(4 * j + 2) * 64 + lane], stk[(4 * j + 3) * 64 + lane]);
#pragma unroll
    for (int j = 0; j < 3; j++) xw[13 + j] = make_int4(rc[4 * j], rc[4 * j + 1], rc[4 * j + 2], rc[4 * j + 3]);
    const bool alive = !(fl & F_DEAD);
    const bool spill = (fl & F_SPILL) != 0;
    if (!alive) ctl &= ~CTL_ALIVE;
    // a death frees the cell for this update's placement (k_allot_total
    // marked the living cells occupied)
    if (mode == AVGPU_MODE_WORLD && alive0 && !alive) W.occ[cell] = 0;
    W.ctl[cell] = (ctl & ~CTL_FRESH) | (sdie ? CTL_SPECDIE : 0u);
    W.mem_size[cell] = M;
    if (serial) W.sctx[2] = kct;                             // the context stream moved on
    else W.rng[2 * N + cell] = kct;
    W.budget[cell] = spill ? (budget | (prim ? BUDGET_PRIM : 0)) : 0;
    if (spill && mode == AVGPU_MODE_WORLD) W.sdone[cell] = sdone + executed;
    // the slice's instructions (a newborn replacing this organism gives the
    // step back the share after its birth: world.hip newborn_setup)
    if (!NB && !spill && mode == AVGPU_MODE_WORLD && !serial) W.ran[cell] = sdone + executed;
    // merit, fitness, gestation time, copied / executed sizes and last-task
    // counts were stored at the divide (st_async)
    // (a fresh organism's zero rows are stored here rather than at activation:
    // k_activate is bound by its scattered stores, class 0 is not)
    if (didv || fresh) { W.num_div[cell] = dnd; W.generation[cell] = dgen; }
    if (!DEF && didv && W.track_age) W.age[cell] = 0;        // DivideReset (main/cPhenotype.cc:950)
    // (a deferred divide's executed size: a spill row continuing this slice
    // in the same update reads it at its staging)
    if (didv) W.executed[cell] = dexe;
    if (fresh) {
#pragma unroll
      for (int q = AVGPU_NUM_LOGIC_TASKS; q < AVGPU_MAX_REACTIONS; q++) W.last_task[(int64_t)q * N + cell] = 0;
      if (!didv) W.child_copied[cell] = 0;   // last_task: the parent's, set at activation
    }
    // cur_reaction_count: reset at a divide, counted since (or added to the
    // stored counts when no divide happened in this slice)
#pragma unroll
    for (int i = XS_NREACT; i < AVGPU_MAX_REACTIONS; i++) {
      int32_t* p = W.cur_react + (int64_t)i * N + cell;
      if (i < W.n_react) {
        if (didv || fresh) *p = rc[i];
        else if (rc[i]) *p += rc[i];
      } else if (fresh) {
        *p = 0;
      }
    }
    if (spill) {
      // a class-0 world slice continues in the same wave (k_interpret), the
      // others in the spill row of class cls+1
      if (!(C0W && cls == 0)) {
        const int slot = atomicAdd(&W.class_count[3 + cls + 1], 1);
        W.class_list[(int64_t)(3 + cls + 1) * N + slot] = cell;
      }
      count_add(W, CNT_SPILLS, 1ull);
    }
  }
  // tapes back to HBM: the same lane-linear image, one granule per lane
#pragma unroll QUNR
  for (int it = 0; it < qits; it++) {
    const int i = it * 64 + lane;
    const int j = i / QUADS, q = i - j * QUADS;
    const int c = __shfl(cell, j);
    const int m = __shfl(M, j);
    if (c >= 0 && q * GRAN < m) {
      if (GRAN == 16) {
        const uint4 v = reinterpret_cast<const uint4*>(lds32)[i];
        *reinterpret_cast<uint4*>(W.tape + (int64_t)c * TAPE_SLOT + q * 16) = v;
      } else {
        *reinterpret_cast<uint32_t*>(W.tape + (int64_t)c * TAPE_SLOT + q * 4) = lds32[i];
      }
    }
  }
  if (serial) return executed | (divides << 16) | (sbirth << 24) | (sdie << 25);
  // ---- primary birth records -> birth queue (wavefront ballot + prefix) ----
  {
    const bool fresh = prim && !prim0;
    const unsigned long long bm = __ballot(fresh);
    if (bm) {
      int base = 0;
      if (lane == 0) base = atomicAdd(W.b_count, (int)__popcll(bm));
      base = __shfl(base, 0);
      if (fresh) W.b_list[base + (int)__popcll(bm & ((1ull << lane) - 1ull))] = cell;
    }
  }
  // the sub-step predictor (oracle pred_term): an organism that ran this
  // step's main pass to its slice's end, alive, without a divide in it
  if (pred) {
    long long pt = 0;
    int q = -1;
    if (active && !(fl & (F_DEAD | F_SPILL)) && alive0 && gs <= tu - executed - sdone)
      pt = pred_term(W, cell, tu, gs, blen, dcop, dexe, bonus, q);
    for (int off = 32; off > 0; off >>= 1) pt += __shfl_xor(pt, off);
    unsigned long long* pa = reinterpret_cast<unsigned long long*>(W.pacc) + (blockIdx.x & (NSHARD - 1)) * PACC_STRIDE;
    if (lane == 0 && pt) atomicAdd(pa, (unsigned long long)pt);
    // the quarter counts, two per 64-bit word: two atomics per wave
    const unsigned long long q01 = (unsigned long long)__popcll(__ballot(q == 0)) |
                                   ((unsigned long long)__popcll(__ballot(q == 1)) << 32);
    const unsigned long long q23 = (unsigned long long)__popcll(__ballot(q == 2)) |
                                   ((unsigned long long)__popcll(__ballot(q == 3)) << 32);
    if (lane == 0 && q01) atomicAdd(pa + 1, q01);
    if (lane == 0 && q23) atomicAdd(pa + 2, q23);
  }
  // counters: one atomic per wave
  unsigned long long e = (unsigned long long)executed;
  int dead = (active && (fl & F_DEAD)) ? 1 : 0;
  int dv = divides;
  int mxe = executed;
  int sl = active ? 1 : 0;
  int sites = active ? m_in + M : 0;
  int nover = noversize, nrover = rover ? 1 : 0;
  for (int off = 32; off > 0; off >>= 1) {
    ndrop += __shfl_down(ndrop, off);
    nover += __shfl_down(nover, off);
    if (REC) nrover += __shfl_down(nrover, off);
    e += __shfl_down(e, off);
    dead += __shfl_down(dead, off);
    dv += __shfl_down(dv, off);
    mxe = max(mxe, __shfl_down(mxe, off));
    sl += __shfl_down(sl, off);
    sites += __shfl_down(sites, off);
  }
  if (lane == 0) {
    count_add(W, CNT_LANESTEPS, 64ull * (unsigned long long)mxe);   // issued lane-steps
    count_add(W, CNT_INSTS, e);
    if (dead) count_add(W, CNT_DEATHS, (unsigned long long)dead);
    if (dv) count_add(W, CNT_DIVIDES, (unsigned long long)dv);
    if (ndrop) count_add(W, CNT_DROPPED, (unsigned long long)ndrop);
    if (nover) count_add(W, CNT_OVERSIZE, (unsigned long long)nover);
    if (REC && nrover) count_add(W, CNT_REC_OVER, (unsigned long long)nrover);
    if (S == CLASS0_SIZE && !NB) {   // everything the class-0 launch runs: its windows, list blocks, in-wave spills
      count_add(W, CNT_C0_SLICES, (unsigned long long)sl);
      count_add(W, CNT_C0_SITES, (unsigned long long)sites);
    }
  }
#ifdef AVGPU_PHASE_CLOCKS
  {
    const uint64_t clk3 = __builtin_amdgcn_s_memtime();
    for (int off = 32; off > 0; off >>= 1) {
      it_fast = max(it_fast, __shfl_down(it_fast, off));
      it_copy = max(it_copy, __shfl_down(it_copy, off));
      it_slow = max(it_slow, __shfl_down(it_slow, off));
    }
    if (lane == 0 && cls == 0) {
      count_add(W, CNT_CLK_STAGE, clk1 - clk0);
      count_add(W, CNT_CLK_LOOP, clk2 - clk1);
      count_add(W, CNT_CLK_WB, clk3 - clk2);
      count_add(W, CNT_ITERS, (unsigned long long)it_loop);
      count_add(W, CNT_IT_FAST, (unsigned long long)it_fast);
      count_add(W, CNT_IT_COPY, (unsigned long long)it_copy);
      count_add(W, CNT_IT_SLOW, (unsigned long long)it_slow);
      count_add(W, CNT_WAVES, 1ull);
      for (int k = 0; k < 6; k++) count_add(W, CNT_CB0 + k, cb[k]);
      for (int k = 0; k < 10; k++) count_add(W, CNT_CASE0 + k, cc[k]);
    }
  }
#endif
  // a class-0 world slice that spilled: its cell + 1, for the wave to continue
  return (C0W && cls == 0 && active && (fl & F_SPILL)) ? cell + 1 : 0;
}

// class 0 must keep 2 waves per SIMD (its LDS admits 7 blocks per CU): the
// second bound caps it at 256 registers (VGPR + AGPR)
// The mixed class-0 launch (nmix > 0, world updates): its first nmix blocks
// run the list classes 1 / 2 / 3 in class-0 blocks (MIX_B1 / MIX_B2 / MIX_B3
// blocks, each a grid-stride over its list in chunks of 64 / kslot
// organisms), the rest are class 0 -- one launch, so the list classes need no
// aux stream, no fork / join events and no head start on class 0.
#define MIX_B1 512
#define MIX_B2 16
#define MIX_B3 8
#define MIX_BLOCKS (MIX_B1 + MIX_B2 + MIX_B3)
static_assert(MIX_BLOCKS % 8 == 0, "class 0's XCD mapping needs whole rounds of 8 blocks");
// `sorted`: bit 0 the class-0 sweep follows the budget-sorted windows, bit 1
// a world update's main pass (its slices add the sub-step predictor); NB: the
// newborn pass (class 0 over list row 0, a grid-stride)
template <int S, bool REC, bool C0W = false, bool SIMPLE = false, bool DEF = false, bool RES = false, bool NB = false>
__global__ __launch_bounds__(64, (S == CLASS0_SIZE) ? 2 : 1) void k_interpret(const DevWorld* __restrict__ Wp, int cls, int row, int mode,
                                                  int64_t first, int64_t count, int sorted_arg, int lpw, int nmix = 0) {
  constexpr int TAB_WORDS = 128 + 64 + 16 + 64 + AVGPU_MAX_REACTIONS * RT_STRIDE + 64;
  // class 0: stacks in VGPRs, tables in global memory -- only the tapes in LDS
  constexpr int STK = (S == CLASS0_SIZE) ? 0 : 2 * AVGPU_STACK_SIZE * 64;
  constexpr int TAB = (S == CLASS0_SIZE) ? 0 : TAB_WORDS;     // class 0: tapes only
  __shared__ __attribute__((aligned(16))) uint32_t lds32[64 * tape_stride(S) / 4 + STK + TAB];
  const int sorted = sorted_arg & 1;
  const bool pred = (sorted_arg & 2) != 0;
  if (cls == 0) {
    if (S == CLASS0_SIZE && C0W && (int)blockIdx.x < nmix) {
      const int b = blockIdx.x;
      const int lc = b < MIX_B1 ? 1 : (b < MIX_B1 + MIX_B2 ? 2 : 3);
      const int b0 = lc == 1 ? 0 : (lc == 2 ? MIX_B1 : MIX_B1 + MIX_B2);
      const int nb = lc == 1 ? MIX_B1 : (lc == 2 ? MIX_B2 : MIX_B3);
      const int kslot = lc == 1 ? 3 : (lc == 2 ? 5 : 7);      // 960 / 1600 / 2240 B >= 768 / 1536 / 2048 sites
      const int per = 64 / kslot;
      const int lcount = Wp->class_count[lc];
      for (int64_t chunk = b - b0; chunk * per < lcount; chunk += nb) {
        interpret_chunk<S, REC, false, SIMPLE, DEF, RES, true, NB>(Wp, lc, mode, first, count, chunk, lds32, false, lc,
                                                                    per, 0, kslot, -2, pred);
        __syncthreads();
      }
      return;
    }
    const int64_t bx = (int64_t)blockIdx.x - nmix, gx = (int64_t)gridDim.x - nmix;
    // one class-0 chunk, then (world slices) the wave's own spills
    auto run_chunk = [&](int64_t chunk) {
      const int sp = interpret_chunk<S, REC, C0W, SIMPLE, DEF, RES, false, NB>(Wp, 0, mode, first, count, chunk, lds32,
                                                                               sorted, 0, 64, 0, 1, -2, pred) - 1;
      if (S == CLASS0_SIZE && C0W) {
        // Organisms whose h-alloc (or copy) outgrew their 320-site slot: this
        // wave continues them at once in 3-slot (960-site) lanes of its own
        // block's LDS -- their state was written back by this wave, so a
        // workgroup-scope fence makes it visible to the re-staging -- instead of
        // a spill row after class 0 (~55 organisms per update, 66 us after
        // class 0, latency-bound on the longest).  A slice that outgrows 960
        // sites goes on to the class-2 spill row.
        uint64_t m = __ballot(sp >= 0);
        if (m) {
          const int nsp = __popcll(m);
          int mine = -1;
          for (int j = 0; m; j++, m &= m - 1) {
            const int c = __shfl(sp, __ffsll((long long)m) - 1);
            if ((int)threadIdx.x == j) mine = c;
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
          __syncthreads();
          constexpr int PER3 = 64 / 3;
          for (int g = 0; g < nsp; g += PER3) {
            const int d = __shfl(mine, (g + (int)threadIdx.x) & 63);
            const int direct = ((int)threadIdx.x < PER3 && g + (int)threadIdx.x < nsp) ? d : -1;
            interpret_chunk<S, REC, false, SIMPLE, DEF, RES, true, NB>(Wp, 1, mode, first, count, 0, lds32, false, 4,
                                                                        PER3, 0, 3, direct, pred);
            __syncthreads();
          }
        }
      }
    };
    if (NB) {
      // the newborn pass: a grid-stride over list row 0
      const int ncount = Wp->class_count[0];
      for (int64_t chunk = bx; chunk * 64 < ncount; chunk += gx) {
        run_chunk(chunk);
        __syncthreads();
      }
      return;
    }
    // sorted windows: the 32 chunks of a window run on one XCD (blocks are
    // dealt to the 8 XCDs round robin), so its state lines meet in one L2
    int64_t chunk = bx;
    if (sorted && (gx & 7) == 0) chunk = (bx & 7) * (gx >> 3) + (bx >> 3);
    run_chunk(chunk);
    return;
  }
  if (C0W) return;
  // list classes: grid-stride over the list (its length is known on device
  // only); with cls < 0, rows row and row + 1 in one launch (their organisms
  // fit this class's tape slots: classes 2 + 3 beside class 0, spill rows 5 + 6)
  const int nrows = cls < 0 ? 2 : 1;
  for (int r = row; r < row + nrows; r++) {
    const int rc = cls >= 0 ? cls : (r <= 3 ? r : r - 3);
    const int lcount = Wp->class_count[r];
    for (int64_t chunk = blockIdx.x; chunk * lpw < lcount; chunk += gridDim.x) {
      interpret_chunk<S, REC, false, SIMPLE, DEF, RES, false, NB>(Wp, rc, mode, first, count, chunk, lds32, false, r,
                                                                   lpw, 0, 1, -2, pred);
      __syncthreads();
    }
  }
}

// ---- the serial world (oracle orc_run_serial_updates) ----
// Avida2Driver::Run's update with the reference's own schedule: UD = 30 x
// living organisms picks, each a merit-weighted draw of one cell from the
// scheduler's stream (cPopulation::ScheduleOrganism over a cWeightedIndex sum
// tree, tools/cWeightedIndex.cc:49-115); a picked organism with speculative
// credit spends one, otherwise it runs ProcessStepSpeculative
// (main/cPopulation.cc:5740-5788, interpret_chunk serial step) and an
// offspring is placed at once (ActivateOffspring / PositionOffspring,
// main/cPopulation.cc:621-952, :5185-5414) into a neighbour drawn from the
// same stream.  One wave per world: the picks are sequential by definition;
// the wave shares the tree walks, genome copies and the interpreter's staging.

// the sum tree's leaf for x: the binary descent of SerialSched::find, five
// levels per round -- lanes fetch the 62 nodes below p in parallel, then the
// walk runs in registers (same comparisons and subtractions, same order)
__device__ __forceinline__ int64_t stree_find(const double* tree, int64_t size, double x) {
  const int lane = threadIdx.x & 63;
  int depth = 0;
  for (int64_t s = size; s > 1; s >>= 1) depth++;
  int64_t p = 1;
  int dp = 0;
  while (dp < depth) {
    const int lv = min(5, depth - dp);
    const int h = lane + 2;                     // subtree heap index of this lane's node
    const int d = 31 - __clz(h);
    double v = 0.0;
    if (h < (2 << lv) && d <= lv) v = tree[(p << d) + (h - (1 << d))];
    int k = 1;
    for (int l = 0; l < lv; l++) {
      const double left = __shfl(v, 2 * k - 2);
      if (x < left) {
        k = 2 * k;
      } else {
        x = __dsub_rn(x, left);
        k = 2 * k + 1;
      }
    }
    p = (p << lv) + (k - (1 << lv));
    dp += lv;
  }
  return p - size;
}

// SerialSched::set: leaf = v, then every node on its path to the root as the
// sum of its two children (left + right); the siblings are fetched at once
__device__ __forceinline__ void stree_set(double* tree, int64_t size, int64_t i, double v) {
  const int lane = threadIdx.x & 63;
  int depth = 0;
  for (int64_t s = size; s > 1; s >>= 1) depth++;
  const int64_t leaf = size + i;
  double sib = 0.0;
  if (lane < depth) sib = tree[(leaf >> lane) ^ 1];
  double cur = v, mine = 0.0;
  for (int k = 0; k < depth; k++) {
    const double sk = __shfl(sib, k);
    cur = ((leaf >> k) & 1) ? __dadd_rn(sk, cur) : __dadd_rn(cur, sk);
    if (lane == k) mine = cur;
  }
  if (lane == 0) tree[leaf] = v;
  if (lane < depth) tree[leaf >> (lane + 1)] = mine;
  __threadfence_block();
}

// The reference's connection list of a cell (oracle conn_base;
// tools/cTopology.h:40-55: Push() prepends, so the list runs W, SW, S, SE, E,
// NE, N, NW; build_grid drops the wrapped entries, keeping the order)
__device__ __forceinline__ int conn_base(const DevWorld& W, int cell, int* out) {
  constexpr int DX[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, DY[8] = {0, 1, 1, 1, 0, -1, -1, -1};
  const int X = W.world_x, Y = W.world_y;
  const int x = cell % X, y = cell / X;
  int n = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int nx = x + DX[k], ny = y + DY[k];
    if (W.geometry == 1 && (nx < 0 || nx >= X || ny < 0 || ny >= Y)) continue;
    out[n++] = ((ny + Y) % Y) * X + (nx + X) % X;
  }
  return n;
}

// the serial world's context stream: GetUInt(n) of its next draw (counter, or
// the recorded srec_ctx); ct is its position
__device__ __forceinline__ uint32_t sctx_below(const DevWorld& W, uint32_t& ct, uint32_t n, bool& over) {
  if (W.srec_ctx) {
    double u = 0.0;
    if ((int64_t)ct < W.srec_ctx_n) u = W.srec_ctx[ct]; else over = true;
    ct++;
    const uint32_t v = (uint32_t)(u * (double)n);
    return v < n ? v : n - 1u;
  }
  return rng_below(W.sctx[0], W.sctx[1], ct, n);
}

template <int S, bool REC>
__global__ __launch_bounds__(64, 1) void k_serial_update(const DevWorld* __restrict__ Wp) {
  constexpr int TAB_WORDS = 128 + 64 + 16 + 64 + AVGPU_MAX_REACTIONS * RT_STRIDE + 64;
  __shared__ __attribute__((aligned(16))) uint32_t lds32[64 * tape_stride(S) / 4 + 2 * AVGPU_STACK_SIZE * 64 + TAB_WORDS];
  __shared__ __attribute__((aligned(16))) uint8_t child[TAPE_SLOT + 16];
  const DevWorld& W = *Wp;
  const int lane = threadIdx.x;
  const int64_t n = W.n, size = W.stree_size;
  double* tree = W.stree;
  // the tree over this update's merits (every cell's SerialSched::set)
  int na = 0;
  for (int64_t c = lane; c < size; c += 64) {
    const bool live = c < n && (W.ctl[c] & CTL_ALIVE);
    tree[size + c] = live ? W.merit[c] : 0.0;
    na += live ? 1 : 0;
  }
  __threadfence_block();
  for (int64_t lo = size >> 1; lo >= 1; lo >>= 1) {
    for (int64_t q = lo + lane; q < 2 * lo; q += 64) tree[q] = __dadd_rn(tree[2 * q], tree[2 * q + 1]);
    __threadfence_block();
  }
  for (int off = 32; off > 0; off >>= 1) na += __shfl_xor(na, off);
  const int64_t ud = (int64_t)W.ave_time_slice * na;   // cWorld::CalculateUpdateSize
  const uint32_t glo = W.grng[0], ghi = W.grng[1];
  uint32_t gct = W.grng[2];
  unsigned long long picks = 0, deaths = 0, divides = 0, births = 0, dropped = 0, over = 0;
  for (int64_t i = 0; i < ud; i++) {
    const double tot = tree[1];
    if (!(tot > 0.0)) break;
    // the scheduler's draw (its own stream: main/cPopulation.cc:7341-7346)
    double u;
    if (W.srec_sched) {
      u = (int64_t)gct < W.srec_sched_n ? W.srec_sched[gct] : 0.0;
      over += (int64_t)gct < W.srec_sched_n ? 0 : 1;
      gct++;
    } else {
      u = __dmul_rn((double)rng_next(glo, ghi, gct), 1.0 / 4294967296.0);
    }
    const int64_t c = stree_find(tree, size, __dmul_rn(u, tot));
    const uint32_t ctl = W.ctl[c];
    if (!(ctl & CTL_ALIVE)) continue;
    picks++;
    const int sp = W.spec[c];
    if (sp > 0) {                                 // a speculatively executed step
      if (lane == 0) W.spec[c] = sp - 1;
      __threadfence_block();
      continue;
    }
    if (ctl & CTL_SPECDIE) {                      // SingleProcess: m_spec_die -> Die (cpu/cHardwareCPU.cc:917-921)
      if (lane == 0) W.ctl[c] = ctl & ~(CTL_ALIVE | CTL_SPECDIE);
      __threadfence_block();
      stree_set(tree, size, c, 0.0);
      deaths++;
      continue;
    }
    // the one non-speculative SingleProcess
    const int r = __shfl(interpret_chunk<S, REC>(Wp, 1, AVGPU_MODE_WORLD, c, 1, 0, lds32, false, 0, 64, 1), 0);
    __builtin_amdgcn_s_waitcnt(0);              // the step's stores (some outside the compiler's view)
    __threadfence_block();
    divides += (r >> 16) & 0xFF;
    bool replaced = false;
    if ((r >> 24) & 1) {
      // ActivateOffspring inside the h-divide (main/cPopulation.cc:621-960)
      apply_edits_wave(W, c, child);
      int t = -1, face_t = -1;
      int32_t in3[3] = {0, 0, 0};
      int alive_n = 0;
      if (W.birth_method == 4 && W.prefer_empty) {   // num_organisms, for FindRandEmptyCell
        int a = 0;
        for (int64_t q = lane; q < W.n; q += 64) a += (W.ctl[q] & CTL_ALIVE) ? 1 : 0;
        alive_n = wave_sum_i32(a);
      }
      if (lane == 0) {
        uint32_t ct = W.sctx[2];
        bool ov = false;
        if (W.birth_method == 4) {
          // FULL_SOUP_RANDOM (oracle serial_soup): FindRandEmptyCell on the
          // persistent empty_cell_id_array, else GetUInt(size)
          const uint32_t n = (uint32_t)W.n;
          t = -1;
          if (W.prefer_empty) {
            if (alive_n < (int)n) {
              uint32_t ws = n;
              uint32_t idx = sctx_below(W, ct, ws, ov);
              int cc = W.soup_perm[idx];
              bool found = true;
              while (W.ctl[cc] & CTL_ALIVE) {
                --ws;
                const int sw = W.soup_perm[ws];
                W.soup_perm[ws] = cc;
                W.soup_perm[idx] = sw;
                if (ws == 1) { found = false; break; }
                idx = sctx_below(W, ct, ws, ov);
                cc = W.soup_perm[idx];
              }
              if (found) t = cc;
            }
            if (t < 0) t = (int)sctx_below(W, ct, n, ov);
          } else {
            t = (int)sctx_below(W, ct, n, ov);
            while (!W.allow_parent && n > 1u && t == (int)c) t = (int)sctx_below(W, ct, n, ov);
          }
        } else if (W.birth_method == 5) {
          // FULL_SOUP_ELDEST (oracle serial_eldest): the reaper queue's rear
          // cell; the parent's, without ALLOW_PARENT, goes back to the rear
          const int64_t C = W.reaper_cap;
          int64_t R = W.reaper_ix[0];
          t = W.reaper[R % C];
          R++;
          if (!W.allow_parent && t == (int)c && R < W.reaper_ix[1]) {
            t = W.reaper[R % C];                                  // PopRear, then PushRear(parent)
            W.reaper[R % C] = (int)c;                             // into the slot it freed
          }
          W.reaper_ix[0] = R;
        } else {
          // PositionOffspring on the rotated connection list (oracle serial_target)
          int base[8], conn[8], found[9];
          const int nb = conn_base(W, (int)c, base);
          const int f = nb ? W.face[c] % nb : 0;
          for (int k = 0; k < nb; k++) conn[k] = base[(f + k) % nb];
          int nf = 0;
          if (W.prefer_empty)
            for (int k = 0; k < nb; k++)
              if (!(W.ctl[conn[k]] & CTL_ALIVE)) { for (int q = nf; q > 0; q--) found[q] = found[q - 1]; found[0] = conn[k]; nf++; }
          if (nf == 0 && W.birth_method == 0) {
            if (W.allow_parent) found[nf++] = (int)c;
            for (int k = 0; k < nb; k++) found[nf++] = conn[k];
          }
          t = nf == 0 ? (int)c : found[sctx_below(W, ct, (uint32_t)nf, ov)];
        }
        if (t == (int)c && !W.allow_parent) t = -1;            // target_cells[i] = -1 (:706-712)
        if (t >= 0) {
          // ActivateOrganism -> SetupInputs random (main/cEnvironment.cc:1268-1271)
          in3[0] = (15 << 24) + (int)sctx_below(W, ct, 1u << 24, ov);
          in3[1] = (51 << 24) + (int)sctx_below(W, ct, 1u << 24, ov);
          in3[2] = (85 << 24) + (int)sctx_below(W, ct, 1u << 24, ov);
          // Rotate(parent_cell) (:935-944), for the local birth methods only
          // (birth_method < NUM_LOCAL_POSITION_OFFSPRING = 4, :938)
          if (t != (int)c && W.birth_method < 4) {
            int tb[8];                                          // (not adjacent: a full turn, no change)
            const int ntb = conn_base(W, t, tb);
            for (int k = 0; k < ntb; k++) if (tb[k] == (int)c && face_t < 0) face_t = k;
          }
        }
        W.sctx[2] = ct;
        over += ov ? 1 : 0;
      }
      t = __shfl(t, 0);
#pragma unroll
      for (int k = 0; k < 3; k++) in3[k] = __shfl(in3[k], 0);
      if (t < 0) {
        dropped++;
      } else {
        const bool parent_alive = t != (int)c;
        const bool killed = (W.ctl[t] & CTL_ALIVE) != 0;
        if (parent_alive) stree_set(tree, size, c, W.merit[c]);   // AdjustSchedule(parent) :933
        Child b = child_of_record(W, c);
        b.inputs = in3;                                          // from the context stream (lane 0's)
        b.hs = 0;                                                // placed at once: no head start
        setup_child<64>(W, t, b, reinterpret_cast<const uint32_t*>(W.b_genome + c * TAPE_SLOT), lane);
        __threadfence_block();
        if (lane == 0) {
          W.spec[t] = 0;                                         // InsertOrganism resets the credit
          if (parent_alive && face_t >= 0) W.face[t] = (uint8_t)face_t;
          if (W.birth_method == 5) {                             // ActivateOrganism: Push(target) (:1358-1361)
            const int64_t F = W.reaper_ix[1];
            W.reaper[F % W.reaper_cap] = t;
            W.reaper_ix[1] = F + 1;
          }
        }
        __threadfence_block();
        stree_set(tree, size, t, b.merit);
        births++;
        deaths += killed ? 1 : 0;
        replaced = !parent_alive;
      }
    }
    if (replaced) continue;                       // the parent died in its own step: no speculation
    if (!(W.ctl[c] & CTL_ALIVE)) { stree_set(tree, size, c, 0.0); deaths++; continue; }
    // the speculative run (ProcessStepSpeculative, main/cPopulation.cc:5758-5766)
    const int r2 = __shfl(interpret_chunk<S, REC>(Wp, 1, AVGPU_MODE_WORLD, c, 1, 0, lds32, false, 0, 64, 2), 0);
    __builtin_amdgcn_s_waitcnt(0);
    __threadfence_block();
    if (lane == 0) W.spec[c] = r2 & 0xFFFF;
    __threadfence_block();
  }
  if (lane == 0) {
    W.grng[2] = gct;
    count_add(W, CNT_INSTS, picks);
    if (deaths) count_add(W, CNT_DEATHS, deaths);
    if (divides) count_add(W, CNT_DIVIDES, divides);
    if (births) count_add(W, CNT_BIRTHS, births);
    if (dropped) count_add(W, CNT_DROPPED, dropped);
    if (over) count_add(W, CNT_REC_OVER, over);
  }
}

}  // namespace

// lanes per wave of the spill rows (AVGPU_SPILL_LPW overrides for sweeps)
static int spill_lpw() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("AVGPU_SPILL_LPW");
    const int x = e ? atoi(e) : 0;
    v = (x >= 1 && x <= 64) ? x : 1;
  }
  return v;
}

// timing events around class 0 only (default) or after every class
// (AVGPU_CLASS_TIMING=1, diagnostics): each timed event record costs ~10 us
// of queue time, and the three spill-row launches sit on the update's
// critical path
bool class_timing_all() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("AVGPU_CLASS_TIMING");
    v = (e && atoi(e) == 1) ? 1 : 0;
  }
  return v == 1;
}

// the knobs the DEF instantiation fixes, at the reference's defaults
// (avgpu_cfg_defaults; main/cAvidaConfig.h)
// AVGPU_NO_MIX=1: the list classes on their own aux-stream launches (A/B)
bool mix_lists() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("AVGPU_NO_MIX");
    v = (e && atoi(e) == 1) ? 0 : 1;
  }
  return v == 1;
}

static bool def_knobs(const DevWorld& W) {
  return W.alloc_method != 2 && W.require_allocate == 1 && W.max_label_exe == 1 && W.cfg_min_genome == 0 &&
         W.cfg_max_genome == 0 && W.merit_default_bonus == 0.0 && W.inherit_merit == 1 &&
         W.base_merit_method == 4 && W.th_div_uni == 0 && !W.seg_any && W.th_par_site == 0 && W.th_par_ins == 0 &&
         W.th_par_del == 0 && W.size_range == 2.0 && W.min_exe_lines == 0.5 &&
         W.min_copied_lines == 0.5 && W.required_bonus == 0.0 && W.default_bonus == 1.0 && W.rand_total <= 256 &&
         !W.copy_ext && !W.track_age && W.no_mut_mask == 0 && !W.div_req;
}

// NB: the newborn pass of a world update (launch_newborns): the same launches
// over the organisms k_activate listed -- class 0 from list row 0 by a
// grid-stride of NB_BLOCKS blocks, the list classes in its leading blocks,
// then the spill rows.  A world update's main pass (sorted) adds the sub-step
// predictor (bit 1 of the kernels' `sorted` argument).
#define NB_BLOCKS 2048
template <bool REC, bool NB>
static void launch_classes(const DevWorld& W, const DevWorld* dW, int mode, hipStream_t s,
                           int64_t first, int64_t count, int* launches, hipEvent_t* after_class,
                           bool sorted, hipStream_t* aux, hipEvent_t ev_fork, hipEvent_t* ev_join) {
  const int pfl = (!NB && sorted && mode == AVGPU_MODE_WORLD) ? 2 : 0;
  const int srt = ((!NB && sorted && first == 0 && count == W.n) ? 1 : 0) | pfl;
  const bool tall = class_timing_all();
  const unsigned blocks = NB ? (unsigned)NB_BLOCKS : (unsigned)((count + 63) / 64);
  // list classes: a capped grid strides over the list (length known on the
  // device only).  The caps follow the blocks a CU holds (LDS: 3 of class 1,
  // 1 of classes 2 / 3) and the lists' usual lengths (class 1 ~1 %, classes
  // 2 / 3 and the spill rows tens of organisms): a 2048-block grid of
  // 132-KiB class-3 blocks costs 8 dispatch rounds even when its list is
  // empty.
  const unsigned lb = std::min(blocks, 768u);
  const unsigned lb_small = std::min(blocks, 256u);
  // classes 2 / 3 beside class 0: a handful of blocks.  Each of their blocks
  // needs most of a CU's LDS (99 / 132 KiB), so a 256-block grid queued behind
  // the running class-0 blocks for most of class 0's duration (rocprof: 0.52
  // ms average k_interpret<2048> with lists of tens of organisms) and took
  // CUs away from it as their blocks dispatched one by one.
  const unsigned lb_c2 = std::min(blocks, 8u), lb_c3 = std::min(blocks, 4u);
  if (blocks == 0) {
    if (after_class)
      for (int k = 0; k < 4; k++) hipEventRecord(after_class[k], s);
    return;
  }
  // Organisms k_allot put in classes 1..3 (list rows 1..3) do not depend on
  // class 0; with an aux stream they run beside it and fill the CUs its tail
  // leaves idle.  Spills (rows 4..6) run after both, in class order.
  // list classes and spill rows of a world update at the simple environment
  // and default knobs: the same specialised interpreter as class 0's (SIMPLE,
  // DEF) -- the spill rows run alone after class 0, latency-bound on their
  // longest slice, so every instruction of the generic paths is on the
  // update's critical path
  // (DEF defers the divide's phenotype work to placement round 0: only world
  // updates run placement -- avgpu_step(MODE_WORLD) takes the general path)
  // (RES: the same with finite resources behind the simple reactions, configs[4])
  const bool fast = (NB || sorted) && mode == AVGPU_MODE_WORLD && W.env_simple && def_knobs(W);
  const bool res = W.env_res_mask != 0u;
  auto row = [&](int S, dim3 grid, hipStream_t st, int cls, int r, int lpw) {
#define ROW_LAUNCH(SZ) \
    do { if (fast && res) hipLaunchKernelGGL((k_interpret<SZ, REC, false, true, true, true, NB>), grid, dim3(64), 0, st, dW, cls, r, mode, first, count, pfl, lpw); \
         else if (fast) hipLaunchKernelGGL((k_interpret<SZ, REC, false, true, true, false, NB>), grid, dim3(64), 0, st, dW, cls, r, mode, first, count, pfl, lpw); \
         else hipLaunchKernelGGL((k_interpret<SZ, REC, false, false, false, false, NB>), grid, dim3(64), 0, st, dW, cls, r, mode, first, count, pfl, lpw); } while (0)
    if (S == CLASS1_SIZE) ROW_LAUNCH(CLASS1_SIZE);
    else if (S == CLASS2_SIZE) ROW_LAUNCH(CLASS2_SIZE);
    else ROW_LAUNCH(CLASS3_SIZE);
#undef ROW_LAUNCH
  };
  auto list = [&](int k, hipStream_t st) {
    if (k == 1) row(CLASS1_SIZE, dim3(lb), st, 1, 1, 64);
    if (k == 2) row(CLASS2_SIZE, dim3(lb_c2), st, 2, 2, 64);
    if (k == 3) row(CLASS3_SIZE, dim3(lb_c3), st, 3, 3, 64);
    // classes 2 + 3 in one launch of class 3's slots: both start at the fork,
    // before class 0's blocks fill the CUs (a class-3 block launched behind
    // class 2 waited ~0.5 ms for a CU with all of its LDS free)
    if (k == 23) row(CLASS3_SIZE, dim3(lb_c2 + lb_c3), st, -1, 2, 64);
  };
  // Two aux streams (class 1; classes 2 + 3, which are short): with the
  // world's stream that is three HIP streams, so they keep distinct hardware
  // queues (GPU_MAX_HW_QUEUES = 4); a third aux stream shared a queue with
  // the world's stream and serialised class 3 in front of class 0.  The aux
  // lists start after k_allot, beside the window sort, so that they take their
  // CUs before class 0 and end well inside it (forked after the sort they only
  // got CUs as class-0 waves retired and ended ~40-55 us after class 0).
  // the list classes inside class 0's launch (MIX_BLOCKS leading blocks):
  // sorted world updates, unless AVGPU_NO_MIX=1 (A/B)
  const bool mix = NB || (aux && mix_lists());
  const int nmix = mix ? MIX_BLOCKS : 0;
  const unsigned cblocks = blocks + (unsigned)nmix;
  if (!NB && aux && !mix) {
    // ev_fork: recorded by launch_world_pre right after k_allot built the lists
    for (int k = 0; k < 2; k++) hipStreamWaitEvent(aux[k], ev_fork, 0);
    list(1, aux[0]);
    list(2, aux[1]);
    list(3, aux[1]);
    // one join for the world's stream: aux 0 takes in aux 1 (classes 2 + 3,
    // short) off the critical path; each wait queued on the world's stream
    // costs ~10 us of dead time there even when its event has long completed
    hipEventRecord(ev_join[1], aux[1]);
    hipStreamWaitEvent(aux[0], ev_join[1], 0);
    hipEventRecord(ev_join[0], aux[0]);
  }
  if (fast && res)
    hipLaunchKernelGGL((k_interpret<CLASS0_SIZE, REC, true, true, true, true, NB>), dim3(cblocks), dim3(64), 0, s, dW, 0, 0, mode, first, count, srt, 64, nmix);
  else if (fast)
    hipLaunchKernelGGL((k_interpret<CLASS0_SIZE, REC, true, true, true, false, NB>), dim3(cblocks), dim3(64), 0, s, dW, 0, 0, mode, first, count, srt, 64, nmix);
  else if (mode == AVGPU_MODE_WORLD && W.env_simple && W.env_res_mask == 0u)
    hipLaunchKernelGGL((k_interpret<CLASS0_SIZE, REC, true, true, false, false, NB>), dim3(cblocks), dim3(64), 0, s, dW, 0, 0, mode, first, count, srt, 64, nmix);
  else if (mode == AVGPU_MODE_WORLD)
    hipLaunchKernelGGL((k_interpret<CLASS0_SIZE, REC, true, false, false, false, NB>), dim3(cblocks), dim3(64), 0, s, dW, 0, 0, mode, first, count, srt, 64, nmix);
  else if (!NB)
    hipLaunchKernelGGL((k_interpret<CLASS0_SIZE, REC>), dim3(blocks), dim3(64), 0, s, dW, 0, 0, mode, first, count, srt, 64);
  if (after_class) hipEventRecord(after_class[0], s);
  // Spill rows run after class 0, alone on the chip and latency-bound on their
  // longest remaining slice; spread over waves (spill_lpw lanes each), a
  // wave's iterations no longer pay for its other lanes' divergent paths.
  // Row 4 holds only class-0 organisms (those that outgrew its slots), so it
  // starts right behind class 0, and the joins with the aux streams (their
  // lists ended inside class 0) are queued while it runs instead of in front
  // of it (~17 us per update of event waits on the critical path).
  const int slpw = spill_lpw();
  // row 4 (class 0's spills): a world launch's class-0 waves continue their
  // own spills (k_interpret, C0W), other launches run the row
  const bool c0w = mode == AVGPU_MODE_WORLD;
  if (mix) {
    // no join: the lists ran in class 0's launch
  } else if (aux) {
    if (!c0w) row(CLASS1_SIZE, dim3(lb_small), s, 1, 4, slpw);
    hipStreamWaitEvent(s, ev_join[0], 0);
  } else {
    for (int k = 1; k <= 3; k++) list(k, s);
    if (!c0w) row(CLASS1_SIZE, dim3(lb_small), s, 1, 4, slpw);
  }
  if (after_class && tall) hipEventRecord(after_class[1], s);
  // spill rows 5 + 6 (beyond classes 1 / 2) in one launch of class 3's slots
  // (all three spill rows in one class-3 launch after the join measured 8 us
  // slower per update than these two launches: row 4's organisms ran slower
  // in class 3's slots than the saved launch gap)
  row(CLASS3_SIZE, dim3(std::min(lb_small, 64u)), s, -1, 5, slpw);
  if (after_class && tall) { hipEventRecord(after_class[2], s); hipEventRecord(after_class[3], s); }
  if (launches) *launches += 5;
}

// RECORDED streams launch the REC instantiations (device.h DevWorld::rec)
void launch_interpret_classes(const DevWorld& W, const DevWorld* dW, int mode, hipStream_t s,
                              int64_t first, int64_t count, int* launches, hipEvent_t* after_class,
                              bool sorted, hipStream_t* aux, hipEvent_t ev_fork, hipEvent_t* ev_join) {
  if (W.rec)
    launch_classes<true, false>(W, dW, mode, s, first, count, launches, after_class, sorted, aux, ev_fork, ev_join);
  else
    launch_classes<false, false>(W, dW, mode, s, first, count, launches, after_class, sorted, aux, ev_fork, ev_join);
}

// the newborn pass of a world update's batch step (after k_activate)
void launch_newborns(const DevWorld& W, const DevWorld* dW, hipStream_t s) {
  if (W.rec)
    launch_classes<true, true>(W, dW, AVGPU_MODE_WORLD, s, 0, W.n, nullptr, nullptr, false, nullptr, nullptr, nullptr);
  else
    launch_classes<false, true>(W, dW, AVGPU_MODE_WORLD, s, 0, W.n, nullptr, nullptr, false, nullptr, nullptr, nullptr);
}

// one serial-world update (launch_world_post's statistics follow it)
void launch_serial_update(const DevWorld& W, const DevWorld* dW, hipStream_t s) {
  if (W.srec_ctx) hipLaunchKernelGGL((k_serial_update<CLASS3_SIZE, true>), dim3(1), dim3(64), 0, s, dW);
  else hipLaunchKernelGGL((k_serial_update<CLASS3_SIZE, false>), dim3(1), dim3(64), 0, s, dW);
}
