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
#include "device.h"

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

// popcount of `bitmask`-selected flag bits over tape sites [from, to)
__device__ __forceinline__ int count_flag(const uint8_t* T, int from, int to, uint32_t bit) {
  const uint32_t* T32 = reinterpret_cast<const uint32_t*>(T);
  const uint32_t m4 = bit * 0x01010101u;
  int n = 0;
  int i = from;
  for (; i < to && (i & 3); i++) n += (T[i] & bit) ? 1 : 0;
  const int wend = to >> 2;
  int w = i >> 2;
  for (; w + 4 <= wend; w += 4) {
    const uint32_t a = T32[w], b = T32[w + 1], c = T32[w + 2], d = T32[w + 3];
    n += __popc(a & m4) + __popc(b & m4) + __popc(c & m4) + __popc(d & m4);
  }
  for (; w < wend; w++) n += __popc(T32[w] & m4);
  for (i = max(i, wend << 2); i < to; i++) n += (T[i] & bit) ? 1 : 0;
  return n;
}

template <int S>
__global__ __launch_bounds__(64) void k_interpret(DevWorld W, int cls, int mode, int64_t first,
                                                  int64_t count) {
  constexpr int STRIDE = S + 4;
  constexpr int TAPE_WORDS = 64 * STRIDE / 4;
  constexpr int STK_WORDS = 2 * AVGPU_STACK_SIZE * 64;
  // one __shared__ object: tapes | stacks | task LUT (256 x u16) | rand_cum (64 x i32) | rand_code (64 B)
  __shared__ uint32_t lds32[TAPE_WORDS + STK_WORDS + 128 + 64 + 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);
  int32_t* stk = reinterpret_cast<int32_t*>(lds32 + TAPE_WORDS);
  const uint16_t* lut = reinterpret_cast<const uint16_t*>(lds32 + TAPE_WORDS + STK_WORDS);
  const int32_t* rcum = reinterpret_cast<const int32_t*>(lds32 + TAPE_WORDS + STK_WORDS + 128);
  const uint8_t* rcode = reinterpret_cast<const uint8_t*>(lds32 + TAPE_WORDS + STK_WORDS + 192);

  const int lane = threadIdx.x;
  const int64_t N = W.n;
  int cell = -1;
  int M = 0;
  if (cls == 0) {
    // dense sweep in cell order: coalesced state loads, no list
    const int64_t c = first + (int64_t)blockIdx.x * 64 + lane;
    if (c < first + count) {
      const uint32_t c0 = W.ctl[c];
      const int m0 = W.mem_size[c];
      if ((c0 & CTL_ALIVE) && W.budget[c] > 0 && class_of(need_of(m0, c0, W.size_range)) == 0) {
        cell = (int)c;
        M = m0;
      }
    }
  } else {
    const int lcount = W.class_count[cls];
    const int base = blockIdx.x * 64;
    if (base >= lcount) return;
    const int idx = base + lane;
    if (idx < lcount) {
      cell = W.class_list[(int64_t)cls * N + idx];
      M = W.mem_size[cell];
    }
  }
  const bool active = cell >= 0;
  if (!__any(active)) return;
#ifdef AVGPU_PHASE_CLOCKS
  const uint64_t clk0 = __builtin_amdgcn_s_memtime();
  int it_fast = 0, it_copy = 0, it_slow = 0;
#endif
  const int m_in = M;

  // ---- block-shared tables ----
  {
    uint32_t* l32 = lds32 + TAPE_WORDS + STK_WORDS;
    const uint32_t* g_lut = reinterpret_cast<const uint32_t*>(W.task_lut);
    l32[lane] = g_lut[lane];
    l32[64 + lane] = g_lut[64 + lane];
    l32[128 + lane] = (uint32_t)W.rand_cum[lane];
    if (lane < 16) l32[192 + lane] = reinterpret_cast<const uint32_t*>(W.rand_code)[lane];
  }
  // ---- stage tapes and stacks into LDS by LDS-DMA (global_load_lds_dword:
  // per-lane source, lane-linear destination); all copies are in flight
  // together and retired by the single wait below ----
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  for (int j = 0; j < 64; j++) {
    const int c = __shfl(cell, j);
    const int m = __shfl(M, j);
    if (c < 0) continue;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(W.tape + (int64_t)c * TAPE_SLOT);
    const int words = (m + 3) >> 2;
    for (int k = 0; k * 64 < words; k++) {
      if (k * 64 + lane < words)
#ifdef AVGPU_NO_LDS_DMA
        lds32[j * (STRIDE / 4) + k * 64 + lane] = src[k * 64 + lane];
#else
        __builtin_amdgcn_global_load_lds((void*)(src + k * 64 + lane),
                                         (lds_ptr_t)(lds32 + j * (STRIDE / 4) + k * 64), 4, 0, 0);
#endif
    }
  }
#pragma unroll
  for (int k = 0; k < 2 * AVGPU_STACK_SIZE; k++) {
    if (active)
#ifdef AVGPU_NO_LDS_DMA
      stk[k * 64 + lane] = W.stack[(int64_t)k * N + cell];
#else
      __builtin_amdgcn_global_load_lds((void*)(W.stack + (int64_t)k * N + cell),
                                       (lds_ptr_t)(stk + k * 64), 4, 0, 0);
#endif
    else
      stk[k * 64 + lane] = 0;
  }

  uint8_t* T = lds + lane * STRIDE;

  // ---- hot state into registers ----
  int r0 = 0, r1 = 0, r2 = 0, ip = 0, rh = 0, wh = 0, fh = 0;
  uint32_t ctl = 0, rl = 0, klo = 0, khi = 0, kct = 0;
  int cyc = 0, tu = 0, gs = 0, mx = 0, blen = 0, budget = 0, errs = 0;
  int in0 = 0, in1 = 0, in2 = 0, intot = 0, inptr = 0, inp0 = 0, inp1 = 0, inp2 = 0;
  int outv = 0, outtot = 0;
  double bonus = 0.0;
  int tc[AVGPU_NUM_LOGIC_TASKS];
#pragma unroll
  for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] = 0;
  if (active) {
    r0 = W.reg[cell]; r1 = W.reg[N + cell]; r2 = W.reg[2 * N + cell];
    ip = W.head[cell]; rh = W.head[N + cell]; wh = W.head[2 * N + cell]; fh = W.head[3 * N + cell];
    ctl = W.ctl[cell]; rl = W.rlabel[cell];
    cyc = W.cycles[cell]; tu = W.time_used[cell]; gs = W.gest_start[cell];
    mx = W.max_exec[cell]; blen = W.birth_len[cell];
    klo = W.rng[cell]; khi = W.rng[N + cell]; kct = W.rng[2 * N + cell];
    budget = W.budget[cell];
    errs = W.errors[cell];
    in0 = W.inbuf[cell]; in1 = W.inbuf[N + cell]; in2 = W.inbuf[2 * N + cell];
    intot = W.in_total[cell]; inptr = W.in_ptr[cell];
    inp0 = W.inputs[cell]; inp1 = W.inputs[N + cell]; inp2 = W.inputs[2 * N + cell];
    outv = W.outbuf[cell]; outtot = W.out_total[cell];
    bonus = W.cur_bonus[cell];
#pragma unroll
    for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] = W.cur_task[(int64_t)q * N + cell];
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), visible to the compiler's waitcnt tracking
  __syncthreads();
#ifdef AVGPU_PHASE_CLOCKS
  const uint64_t clk1 = __builtin_amdgcn_s_memtime();
#endif

  bool alive = active && (ctl & CTL_ALIVE);
  bool stop = false, spill = false;
  int executed = 0, divides = 0;

  // cInstSet::GetRandomInst (cpu/cInstSet.cc:83-88) from the LDS tables
  auto rand_code = [&]() -> uint8_t {
    const uint32_t r = rng_below(klo, khi, kct, (uint32_t)W.rand_total);
    int i = 0;
    while (i < W.n_ops - 1 && rcum[i] <= (int32_t)r) i++;
    return rcode[i];
  };

#define GETREG(i) ((i) == 0 ? r0 : ((i) == 1 ? r1 : r2))
#define SETREG(i, v) do { const int _v = (v); if ((i) == 0) r0 = _v; else if ((i) == 1) r1 = _v; else r2 = _v; } while (0)
#define GETHEAD(i) ((i) == 0 ? ip : ((i) == 1 ? rh : ((i) == 2 ? wh : fh)))
#define SETHEAD(i, v) do { const int _v = (v); if ((i) == 0) ip = _v; else if ((i) == 1) rh = _v; else if ((i) == 2) wh = _v; else fh = _v; } while (0)

  while (alive && budget > 0) {
    // ---- SingleProcess (cpu/cHardwareCPU.cc:908-1058) ----
    const int ipa = head_adjust(ip, M);                       // ip.Adjust() :952
    // fetch window: sites ipa .. ipa+4 in two independent word reads
    const uint32_t* T32 = reinterpret_cast<const uint32_t*>(T);
    const uint64_t fwin = ((uint64_t)T32[(ipa >> 2) + 1] << 32) | (uint64_t)T32[ipa >> 2];
    const uint32_t fsh = (uint32_t)(ipa & 3) * 8u;
    const int cur_byte = (int)((fwin >> fsh) & 0xFFu);
    const int op = cur_byte & CODE_MASK;                      // fetch :959
    if (op == AVGPU_H_H_ALLOC) {
      // would this allocation outgrow the LDS slot?  (spill check; the
      // instruction is then executed by the next size class)
      const int cur = M;
      int alloc = (int)(W.size_range * cur);
      if (alloc > AVGPU_MAX_GENOME - cur) alloc = AVGPU_MAX_GENOME - cur;
      const int nsz = cur + alloc;
      const bool ok = !(W.require_allocate && (ctl & CTL_MAL)) && alloc >= 1 &&
                      nsz <= AVGPU_MAX_GENOME && nsz >= AVGPU_MIN_GENOME &&
                      alloc <= (int)(cur * W.size_range) && cur <= (int)(alloc * W.size_range);
      if (ok && nsz > S) { spill = true; ip = ipa; break; }
    }
    cyc++;                                                    // IncCPUCyclesUsed :929
    tu++;                                                     // IncTimeUsed :930
    ip = ipa;
    T[ip] = (uint8_t)(cur_byte | TF_EXEC);                    // SetFlagExecuted :996
    executed++;
    budget--;
    bool adv = true;                                          // m_advance_ip
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
    it_slow += __ballot(!(FAST_OPS & obit) && op != AVGPU_H_H_COPY) != 0ull;
#endif

    if (FAST_OPS & obit) {
      // ---- branch-free ops: register ALU, swap, conditionals, head moves ----
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
      const bool wr = (WR_OPS & obit) != 0u;
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
      adv = !(op == AVGPU_H_MOV_HEAD && r == 0);
      // if-n-equ :2190 / if-less :2235 skip the next instruction
      const bool skip = (op == AVGPU_H_IF_N_EQU && ra == rb) || (op == AVGPU_H_IF_LESS && ra >= rb);
      if (skip) ip = head_adjust(ip + 1, M);
      ctl ^= (op == AVGPU_H_SWAP_STK) ? CTL_CURSTK : 0u;                     // swap-stk :2739
    } else if (op == AVGPU_H_H_COPY) {                        // :7130 Inst_HeadCopy
      rh = head_adjust(rh, M);
      wh = head_adjust(wh, M);
      int v = T[rh] & CODE_MASK;
      // ReadInst (:1459-1466)
      if (v < 3) {
        const int len = rl & 15;
        if (len < AVGPU_MAX_LABEL) rl = (rl & ~15u) | (uint32_t)(len + 1) | ((uint32_t)v << (4 + 2 * len));
      } else {
        rl = 0;
      }
      if (mode != AVGPU_MODE_TEST && W.th_copy_mut && rng_p(klo, khi, kct, W.th_copy_mut))
        v = rand_code();
      T[wh] = (uint8_t)((T[wh] & TF_EXEC) | TF_COPIED | v);
      rh = head_adjust(rh + 1, M);
      wh = head_adjust(wh + 1, M);
    } else switch (op) {
      case AVGPU_H_POP: {                                     // :2698, cCPUStack::Pop
        const int k = (ctl & CTL_CURSTK) ? 1 : 0;
        int sp = k ? CTL_SP1(ctl) : CTL_SP0(ctl);
        int32_t* slot = stk + (k * AVGPU_STACK_SIZE + sp) * 64 + lane;
        const int v = *slot;
        *slot = 0;
        sp = (sp + 1 == AVGPU_STACK_SIZE) ? 0 : sp + 1;
        ctl = k ? ((ctl & ~0xF0u) | ((uint32_t)sp << 4)) : ((ctl & ~0xFu) | (uint32_t)sp);
        SETREG(r, v);
        break; }
      case AVGPU_H_PUSH: {                                    // :2705, cCPUStack::Push
        const int k = (ctl & CTL_CURSTK) ? 1 : 0;
        int sp = k ? CTL_SP1(ctl) : CTL_SP0(ctl);
        sp = (sp == 0) ? AVGPU_STACK_SIZE - 1 : sp - 1;
        stk[(k * AVGPU_STACK_SIZE + sp) * 64 + lane] = GETREG(r);
        ctl = k ? ((ctl & ~0xF0u) | ((uint32_t)sp << 4)) : ((ctl & ~0xFu) | (uint32_t)sp);
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
        int lo[8];
        bool bad = false;
#pragma unroll
        for (int p = 0; p < 8; p++) {
          const uint32_t m = ((p & 1) ? a : ~a) & ((p & 2) ? b : ~b) & ((p & 4) ? c : ~c);
          const uint32_t v = o & m;
          lo[p] = (m == 0u) ? -1 : (v == m ? 1 : 0);
          bad |= (m != 0u) && (v != m) && (v != 0u);
        }
        if (num < 1) lo[1] = lo[0];
        if (num < 2) { lo[2] = lo[0]; lo[3] = lo[1]; }
        if (num < 3) { lo[4] = lo[0]; lo[5] = lo[1]; lo[6] = lo[2]; lo[7] = lo[3]; }
        int id = 0;
#pragma unroll
        for (int p = 0; p < 8; p++) id += lo[p] * (1 << p);
        const uint32_t tmask = (!bad && id >= 0 && id < 256) ? lut[id] : 0u;
        if (tmask) {
          // cEnvironment::TestOutput / TestRequisites / DoProcesses
          // (main/cEnvironment.cc:1314-1406, :1408-1503, :1610-1760)
          uint32_t done = 0;
          double mult = 1.0, addb = 0.0;
          for (int i = 0; i < W.n_react; i++) {
            const int t = W.react_task[i];                    // uniform
            if (!((tmask >> t) & 1u)) continue;
            int cnt = 0;
#pragma unroll
            for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) cnt = (q == t) ? tc[q] : cnt;
            if (W.react_hasreq[i] && (cnt < W.react_min[i] || cnt >= W.react_max[i])) continue;
            done |= 1u << t;
            if (W.react_type[i] == AVGPU_PROC_ADD) addb = __dadd_rn(addb, W.react_add[i]);
            else mult = __dmul_rn(mult, W.react_mult[i]);
            atomicAdd(&W.cur_react[(int64_t)i * N + cell], 1);  // no return: no wait
          }
          if (done) {
#pragma unroll
            for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) tc[q] += (done >> q) & 1u;
            bonus = __dadd_rn(__dmul_rn(bonus, mult), addb);   // cPhenotype.cc:1645-1646
          }
        }
        // GetNextInput (main/cOrganism.h:249 -> cPopulationCell.h:214-218) + DoInput
        const int p = inptr >= 3 ? 0 : inptr;
        const int in = p == 0 ? inp0 : (p == 1 ? inp1 : inp2);
        inptr = p + 1;
        in2 = in1; in1 = in0; in0 = in;
        intot++;
        SETREG(r, in);
        break; }
      case AVGPU_H_H_ALLOC: {                                 // :3294 Inst_MaxAlloc -> Allocate_Main :1707
        const int cur = M;
        int alloc = (int)(W.size_range * cur);
        if (alloc > AVGPU_MAX_GENOME - cur) alloc = AVGPU_MAX_GENOME - cur;
        const int nsz = cur + alloc;
        const bool ok = !(W.require_allocate && (ctl & CTL_MAL)) && alloc >= 1 &&
                        nsz <= AVGPU_MAX_GENOME && nsz >= AVGPU_MIN_GENOME &&
                        alloc <= (int)(cur * W.size_range) && cur <= (int)(alloc * W.size_range);
        if (!ok) { errs++; break; }                           // cOrganism::Fault
        if (W.alloc_method == 2) {
          for (int i = cur; i < nsz; i++) T[i] = rand_code();
        } else {
          const uint32_t f = W.fill_code;
          int i = cur;
          for (; i < nsz && (i & 3); i++) T[i] = (uint8_t)f;
          const uint32_t f4 = f * 0x01010101u;
          for (; i + 4 <= nsz; i += 4) *reinterpret_cast<uint32_t*>(T + i) = f4;
          for (; i < nsz; i++) T[i] = (uint8_t)f;
        }
        M = nsz;
        ctl |= CTL_MAL;
        r0 = cur;
        break; }
      case AVGPU_H_H_DIVIDE: {                                // :6961 -> :6942 -> Divide_Main :1775
        ip = head_adjust(ip, M); rh = head_adjust(rh, M); wh = head_adjust(wh, M); fh = head_adjust(fh, M);
        const int div = rh;
        const int child_end = (wh == 0) ? M : wh;
        const int child = child_end - div;
        // Divide_CheckViable (cpu/cHardwareBase.cc:140-289)
        const int min_size = max(AVGPU_MIN_GENOME, (int)(blen / W.size_range));
        const int max_size = min(AVGPU_MAX_GENOME, (int)(blen * W.size_range));
        bool ok = child >= min_size && child <= max_size && div >= min_size && div <= max_size;
        if (ok && W.cfg_min_genome && (child < W.cfg_min_genome || div < W.cfg_min_genome)) ok = false;
        if (ok && W.cfg_max_genome && (child > W.cfg_max_genome || div > W.cfg_max_genome)) ok = false;
        int exe = 0, cop = 0;
        if (ok) {                                             // calcExecutedSize (cpu/cHardwareBase.cc:130-138)
          exe = count_flag(T, 0, div, TF_EXEC);
          ok = exe >= (int)(div * W.min_exe_lines);
        }
        if (ok) {                                             // calcCopiedSize (cpu/cHardwareCPU.cc:1765-1772)
          cop = count_flag(T, div, div + child, TF_COPIED);
          ok = cop >= (int)(child * W.min_copied_lines);
        }
        double bon = bonus;
        int old_exe = 0, copied = 0;
        if (ok) {  // cOrganism::Divide_CheckViable (main/cOrganism.cc:788-919)
          if (bon < W.required_bonus) ok = false;
          old_exe = W.executed[cell];
          copied = W.copied[cell];
          const double base0 = (double)calc_size_merit(W, blen, copied, old_exe);
          double b0 = bon;
          if (W.merit_default_bonus != 0.0) b0 = W.merit_default_bonus;
          double off_merit = __dmul_rn(base0, b0);
          if (W.inherit_merit == 0) off_merit = base0;
          if (off_merit == 0.0) ok = false;
        }
        if (!ok) break;                                       // AdjustHeads again: no-op
        W.executed[cell] = exe;                               // SetLinesExecuted
        W.child_copied[cell] = cop;                           // SetLinesCopied
        // ---- offspring ----
        const int nd = W.num_div[cell] + 1;
        if (mode == AVGPU_MODE_TEST) {
          uint8_t* fl = W.t_flags + (int64_t)cell * TAPE_SLOT;
          for (int i = 0; i < div; i++) fl[i] = (T[i] & TF_EXEC) ? '+' : '-';
          W.t_flags_len[cell] = div;
          uint8_t* ch = W.t_child + (int64_t)cell * TAPE_SLOT;
          for (int i = 0; i < child; i++) ch[i] = T[div + i] & CODE_MASK;
          W.t_child_len[cell] = child;
          stop = true;
        }
        // DivideReset / TestDivideReset (main/cPhenotype.cc:824-1000, :1064-1180)
        const double base = (double)calc_size_merit(W, blen, copied, exe);
        if (W.merit_default_bonus != 0.0) bon = W.merit_default_bonus;
        double merit = __dmul_rn(base, bon);
        if (W.inherit_merit == 0) merit = base;
        const int gt = tu - gs;
        const double fit = __ddiv_rn(__dmul_rn(base, bon), (double)gt);
        W.merit[cell] = merit;
        W.gest_time[cell] = gt;
        W.fitness[cell] = fit;
        gs = tu;
        W.num_div[cell] = nd;
        const int gen = W.generation[cell] + 1;
        W.generation[cell] = gen;
        errs = 0;
        bonus = W.default_bonus;
        cyc = 0;
#pragma unroll
        for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) {
          W.last_task[(int64_t)q * N + cell] = tc[q];
          tc[q] = 0;
        }
        for (int i = 0; i < W.n_react; i++) W.cur_react[(int64_t)i * N + cell] = 0;
        if (mode == AVGPU_MODE_WORLD) {
          // Divide_DoMutations (cpu/cHardwareBase.cc:296-569), default subset
          int len = child;
          int mline = -1, iline = -1, dline = -1;
          uint8_t mcode = 0, icode = 0;
          if (W.th_div_mut && rng_p(klo, khi, kct, W.th_div_mut)) {
            mline = (int)rng_below(klo, khi, kct, (uint32_t)len);
            mcode = rand_code();
          }
          if (W.th_div_ins && rng_p(klo, khi, kct, W.th_div_ins) && len < W.max_genome) {
            iline = (int)rng_below(klo, khi, kct, (uint32_t)len + 1);
            icode = rand_code();
            len++;
          }
          if (W.th_div_del && rng_p(klo, khi, kct, W.th_div_del) && len > W.min_genome) {
            dline = (int)rng_below(klo, khi, kct, (uint32_t)len);
            len--;
          }
          const int slot = atomicAdd(W.b_count, 1);
          if (slot < W.bcap) {
            uint32_t* g32 = reinterpret_cast<uint32_t*>(W.b_genome + (int64_t)slot * TAPE_SLOT);
            for (int j0 = 0; j0 < len; j0 += 4) {
              uint32_t word = 0;
#pragma unroll
              for (int b = 0; b < 4; b++) {
                const int j = j0 + b;
                const int k2 = (dline >= 0 && j >= dline) ? j + 1 : j;       // index before the deletion
                int v;
                if (iline >= 0 && k2 == iline) v = icode;
                else {
                  const int k1 = (iline >= 0 && k2 > iline) ? k2 - 1 : k2;  // before the insertion
                  v = (k1 == mline) ? mcode : (T[div + k1] & CODE_MASK);
                }
                word |= (j < len ? (uint32_t)v : 0u) << (8 * b);
              }
              g32[j0 >> 2] = word;
            }
            W.b_parent[slot] = cell;
            W.b_seq[slot] = (uint32_t)nd;
            W.b_len[slot] = len;
            W.b_merit[slot] = merit;
            W.b_fitness[slot] = fit;
            W.b_gen[slot] = gen;
            W.b_ccopied[slot] = cop;
            W.b_exec[slot] = exe;
            W.b_gest[slot] = gt;
            uint32_t clo, chi;
            derive_key(klo, khi, (uint32_t)nd, 0x1B873593U, clo, chi);
            W.b_rng[slot] = clo;
            W.b_rng[W.bcap + slot] = chi;
            W.b_rng[2 * W.bcap + slot] = 0;
            W.b_state[slot] = 0;
            W.b_target[slot] = -1;
          } else {
            count_add(W, CNT_DROPPED, 1ull);
          }
        }
        divides++;
        // parent: Resize(div), Reset (:813-900), ClearFlags (:1839); no IP advance
        M = div;
        r0 = r1 = r2 = 0;
        ip = rh = wh = fh = 0;
#pragma unroll
        for (int k = 0; k < 2 * AVGPU_STACK_SIZE; k++) stk[k * 64 + lane] = 0;
        ctl = CTL_ALIVE;
        rl = 0;
        {
          uint32_t* W32 = reinterpret_cast<uint32_t*>(T);
          for (int w = 0; w < ((div + 3) >> 2); w++) W32[w] &= 0x3F3F3F3Fu;  // ClearFlags (beyond div: unused)
        }
        adv = false;
        break; }
      case AVGPU_H_H_SEARCH:                                  // :7245 Inst_HeadSearch
      case AVGPU_H_IF_LABEL: {                                // :6914 Inst_IfLabel
        // ReadLabel (:1484-1502): the up to 10 sites after IP come from one
        // 16-byte window (4 independent word reads)
        uint32_t lab = 0;
        int len = 0;
        {
          const int base = ip + 1;
          const int w0 = base >> 2;
          const uint64_t lo64 = ((uint64_t)T32[w0 + 1] << 32) | (uint64_t)T32[w0];
          const uint64_t hi64 = ((uint64_t)T32[w0 + 3] << 32) | (uint64_t)T32[w0 + 2];
          const int b0 = base & 3;
          while (len < AVGPU_MAX_LABEL) {
            const int p = base + len;
            if (p >= M) break;
            const int k = b0 + len;
            const int cc = (int)(((k < 8) ? (lo64 >> (8 * k)) : (hi64 >> (8 * (k - 8)))) & CODE_MASK);
            if (cc >= 3) break;
            lab |= (uint32_t)cc << (2 * len);
            len++;
            if (len <= W.max_label_exe) T[p] |= TF_EXEC;
          }
          ip += len;
        }
        // Rotate(1, NUM_NOPS)
        uint32_t rot = 0;
        for (int i = 0; i < len; i++) {
          uint32_t nv = ((lab >> (2 * i)) & 3u) + 1u;
          if (nv >= 3u) nv -= 3u;
          rot |= nv << (2 * i);
        }
        if (op == AVGPU_H_IF_LABEL) {
          const uint32_t packed = (uint32_t)len | (rot << 4);
          if (packed != rl) ip = head_adjust(ip + 1, M);
          break;
        }
        // FindLabel(0) -> FindLabel_Forward(label, memory, 0) (:1177-1295).
        // The reference probes every label_size sites and, inside a probed nop
        // run, tests every offset; every maximal nop run that can hold the
        // label is probed except a run that ends exactly at label_size.  Its
        // answer is therefore the smallest offset o whose label_size sites
        // spell the label (all nops) and that is not that unprobed run
        // (o > 0, or site label_size is a nop).  A rolling 2-bit window over
        // 16-site word batches finds it (DESIGN.md "h-search").
        int found = ip;
        if (len > 0) {
          uint32_t lab_rev = 0;
          for (int i = 0; i < len; i++) lab_rev |= ((rot >> (2 * i)) & 3u) << (2 * (len - 1 - i));
          const uint32_t msk = (len == 16) ? 0xFFFFFFFFu : ((1u << (2 * len)) - 1u);
          const bool run0_ok = len < M && (T[len] & CODE_MASK) < 3;
          uint32_t wnd = 0xFFFFFFFFu;
          int fpos = -1;
          for (int w = 0; (w << 2) < M && fpos < 0; w += 4) {
            const uint32_t q0 = T32[w], q1 = T32[w + 1], q2 = T32[w + 2], q3 = T32[w + 3];
#pragma unroll
            for (int b = 0; b < 16; b++) {
              const uint32_t q = (b < 4) ? q0 : (b < 8) ? q1 : (b < 12) ? q2 : q3;
              const int j = (w << 2) + b;
              uint32_t cc = (q >> (8 * (b & 3))) & CODE_MASK;
              cc = cc < 3u ? cc : 3u;
              wnd = (wnd << 2) | cc;
              if (fpos < 0 && j < M && (wnd & msk) == lab_rev && (j != len - 1 || run0_ok)) fpos = j + 1;
            }
          }
          if (fpos >= 0) found = head_adjust(fpos - 1, M);
        }
        r1 = found - ip;
        r2 = len;
        fh = head_adjust(found + 1, M);
        break; }
      default:
        break;
    }
    if (stop) break;
    if (adv) ip = head_adjust(ip + 1, M);                     // ip.Advance() :1013
    if (mx > 0 && tu >= mx) alive = false;                    // death :1045-1049
  }
#undef GETREG
#undef SETREG
#undef GETHEAD
#undef SETHEAD

  // ---- write back ----
#ifdef AVGPU_PHASE_CLOCKS
  const uint64_t clk2 = __builtin_amdgcn_s_memtime();
#endif
  __syncthreads();
  if (active) {
    W.reg[cell] = r0; W.reg[N + cell] = r1; W.reg[2 * N + cell] = r2;
    W.head[cell] = ip; W.head[N + cell] = rh; W.head[2 * N + cell] = wh; W.head[3 * N + cell] = fh;
    if (!alive) ctl &= ~CTL_ALIVE;
    W.ctl[cell] = ctl; W.rlabel[cell] = rl;
    W.mem_size[cell] = M;
    W.cycles[cell] = cyc; W.time_used[cell] = tu; W.gest_start[cell] = gs;
    W.rng[2 * N + cell] = kct;
    W.budget[cell] = spill ? budget : 0;
    W.errors[cell] = errs;
    W.inbuf[cell] = in0; W.inbuf[N + cell] = in1; W.inbuf[2 * N + cell] = in2;
    W.in_total[cell] = intot; W.in_ptr[cell] = inptr;
    W.outbuf[cell] = outv; W.out_total[cell] = outtot;
    W.cur_bonus[cell] = bonus;
#pragma unroll
    for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++) W.cur_task[(int64_t)q * N + cell] = tc[q];
#pragma unroll
    for (int k = 0; k < 2 * AVGPU_STACK_SIZE; k++) W.stack[(int64_t)k * N + cell] = stk[k * 64 + lane];
    if (spill) {
      const int slot = atomicAdd(&W.class_count[cls + 1], 1);
      W.class_list[(int64_t)(cls + 1) * N + slot] = cell;
      count_add(W, CNT_SPILLS, 1ull);
    }
  }
  for (int j = 0; j < 64; j++) {
    const int c = __shfl(cell, j);
    const int m = __shfl(M, j);
    if (c < 0) continue;
    uint32_t* dst = reinterpret_cast<uint32_t*>(W.tape + (int64_t)c * TAPE_SLOT);
    const uint32_t* src = lds32 + j * (STRIDE / 4);
    const int words = (m + 3) >> 2;
    for (int w = lane; w < words; w += 64) dst[w] = src[w];
  }
  // counters: one atomic per wave
  unsigned long long e = (unsigned long long)executed;
  int dead = (active && !alive) ? 1 : 0;
  int dv = divides;
  int mxe = executed;
  int sl = active ? 1 : 0;
  int sites = active ? m_in + M : 0;
  for (int off = 32; off > 0; off >>= 1) {
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
    if (cls == 0) {
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
      count_add(W, CNT_ITERS, (unsigned long long)mxe);
      count_add(W, CNT_IT_FAST, (unsigned long long)it_fast);
      count_add(W, CNT_IT_COPY, (unsigned long long)it_copy);
      count_add(W, CNT_IT_SLOW, (unsigned long long)it_slow);
      count_add(W, CNT_WAVES, 1ull);
    }
  }
#endif
}

}  // namespace

void launch_interpret_classes(const DevWorld& W, int mode, hipStream_t s, int64_t first,
                              int64_t count, int* launches, hipEvent_t* after_class) {
  const unsigned blocks = (unsigned)((count + 63) / 64);
  if (blocks > 0) {
    hipLaunchKernelGGL(k_interpret<CLASS0_SIZE>, dim3(blocks), dim3(64), 0, s, W, 0, mode, first, count);
    if (after_class) hipEventRecord(after_class[0], s);
    hipLaunchKernelGGL(k_interpret<768>, dim3(blocks), dim3(64), 0, s, W, 1, mode, first, count);
    if (after_class) hipEventRecord(after_class[1], s);
    hipLaunchKernelGGL(k_interpret<1536>, dim3(blocks), dim3(64), 0, s, W, 2, mode, first, count);
    if (after_class) hipEventRecord(after_class[2], s);
    hipLaunchKernelGGL(k_interpret<2048>, dim3(blocks), dim3(64), 0, s, W, 3, mode, first, count);
    if (launches) *launches += 4;
  } else if (after_class) {
    for (int k = 0; k < 3; k++) hipEventRecord(after_class[k], s);
  }
  if (after_class) hipEventRecord(after_class[3], s);
}
