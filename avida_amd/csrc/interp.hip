// interp.hip -- k_interpret: the batched heads-CPU interpreter for gfx950.
//
// Replaces the serial loop Avida2Driver::Run -> cPopulation::ProcessStep ->
// cHardwareCPU::SingleProcess (targets/avida/Avida2Driver.cc:111-116,
// main/cPopulation.cc:5698-5788, cpu/cHardwareCPU.cc:908-1058).
//
// One organism per wavefront lane; 64-thread workgroups (one wave each).  The
// lane's memory tape is staged into LDS (S + 4 bytes per lane, the 4-byte pad
// rotates lanes across banks), all architectural hot state lives in VGPRs, and
// the cold state (stacks, IO buffers, task counters, bonus) is accessed in
// place in HBM only by the instructions that use it.  Divide appends the
// mutated offspring to a birth queue; IO runs the logic-9 task check fused.
// Lanes whose next h-alloc would outgrow their LDS slot stop before it
// ("spill") and are appended, with their remaining budget, to the next size
// class, which is launched afterwards on the same stream.
#include "device.h"

#pragma clang fp contract(off)

namespace {

template <int S>
__global__ __launch_bounds__(64) void k_interpret(DevWorld W, int cls, int mode, int64_t first,
                                                  int64_t count) {
  constexpr int STRIDE = S + 4;
  __shared__ uint32_t lds32[64 * STRIDE / 4];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds32);

  const int lane = threadIdx.x;
  const int64_t N = W.n;
  int cell = -1;
  int M = 0;
  if (cls == 0) {
    // dense sweep in cell order: coalesced hot-state loads, no list
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

  // ---- stage the tapes into LDS (each tape copied by the whole wave) ----
  for (int j = 0; j < 64; j++) {
    const int c = __shfl(cell, j);
    const int m = __shfl(M, j);
    if (c < 0) continue;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(W.tape + (int64_t)c * TAPE_SLOT);
    uint32_t* dst = lds32 + j * (STRIDE / 4);
    const int words = (m + 3) >> 2;
    for (int w = lane; w < words; w += 64) dst[w] = src[w];
  }
  __syncthreads();

  uint8_t* T = lds + lane * STRIDE;

  // ---- hot state into registers ----
  int r0 = 0, r1 = 0, r2 = 0, ip = 0, rh = 0, wh = 0, fh = 0;
  uint32_t ctl = 0, rl = 0, klo = 0, khi = 0, kct = 0;
  int cyc = 0, tu = 0, gs = 0, mx = 0, blen = 0, budget = 0;
  if (active) {
    r0 = W.reg[cell]; r1 = W.reg[N + cell]; r2 = W.reg[2 * N + cell];
    ip = W.head[cell]; rh = W.head[N + cell]; wh = W.head[2 * N + cell]; fh = W.head[3 * N + cell];
    ctl = W.ctl[cell]; rl = W.rlabel[cell];
    cyc = W.cycles[cell]; tu = W.time_used[cell]; gs = W.gest_start[cell];
    mx = W.max_exec[cell]; blen = W.birth_len[cell];
    klo = W.rng[cell]; khi = W.rng[N + cell]; kct = W.rng[2 * N + cell];
    budget = W.budget[cell];
  }
  bool alive = active && (ctl & CTL_ALIVE);
  bool stop = false, spill = false;
  int executed = 0, divides = 0;

#define GETREG(i) ((i) == 0 ? r0 : ((i) == 1 ? r1 : r2))
#define SETREG(i, v) do { const int _v = (v); if ((i) == 0) r0 = _v; else if ((i) == 1) r1 = _v; else r2 = _v; } while (0)
#define GETHEAD(i) ((i) == 0 ? ip : ((i) == 1 ? rh : ((i) == 2 ? wh : fh)))
#define SETHEAD(i, v) do { const int _v = (v); if ((i) == 0) ip = _v; else if ((i) == 1) rh = _v; else if ((i) == 2) wh = _v; else fh = _v; } while (0)

  while (alive && budget > 0) {
    // ---- SingleProcess (cpu/cHardwareCPU.cc:908-1058) ----
    const int ipa = head_adjust(ip, M);                       // ip.Adjust() :952
    const int op = T[ipa] & CODE_MASK;                        // fetch :959
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
    T[ip] |= TF_EXEC;                                         // SetFlagExecuted :996
    executed++;
    budget--;
    bool adv = true;                                          // m_advance_ip
    const int nxt = (ip + 1 < M) ? (T[ip + 1] & CODE_MASK) : CODE_ERROR;  // GetNextInst
    // FindModifiedRegister / FindModifiedHead (:1622-1672)
#define FMOD(def) ((nxt < 3) ? (ip = ip + 1, T[ip] |= TF_EXEC, nxt) : (def))

    switch (op) {
      case AVGPU_H_NOP_A: case AVGPU_H_NOP_B: case AVGPU_H_NOP_C:
        break;
      case AVGPU_H_IF_N_EQU: {                                // :2190
        const int a = FMOD(1); const int b = (a + 1) % 3;
        if (GETREG(a) == GETREG(b)) ip = head_adjust(ip + 1, M);
        break; }
      case AVGPU_H_IF_LESS: {                                 // :2235
        const int a = FMOD(1); const int b = (a + 1) % 3;
        if (GETREG(a) >= GETREG(b)) ip = head_adjust(ip + 1, M);
        break; }
      case AVGPU_H_POP: {                                     // :2698, cCPUStack::Pop
        const int r = FMOD(1);
        const int k = (ctl & CTL_CURSTK) ? 1 : 0;
        int sp = k ? CTL_SP1(ctl) : CTL_SP0(ctl);
        int32_t* slot = W.stack + ((int64_t)(k * AVGPU_STACK_SIZE + sp)) * N + cell;
        const int v = *slot;
        *slot = 0;
        sp = (sp + 1 == AVGPU_STACK_SIZE) ? 0 : sp + 1;
        ctl = k ? ((ctl & ~0xF0u) | ((uint32_t)sp << 4)) : ((ctl & ~0xFu) | (uint32_t)sp);
        SETREG(r, v);
        break; }
      case AVGPU_H_PUSH: {                                    // :2705, cCPUStack::Push
        const int r = FMOD(1);
        const int k = (ctl & CTL_CURSTK) ? 1 : 0;
        int sp = k ? CTL_SP1(ctl) : CTL_SP0(ctl);
        sp = (sp == 0) ? AVGPU_STACK_SIZE - 1 : sp - 1;
        W.stack[((int64_t)(k * AVGPU_STACK_SIZE + sp)) * N + cell] = GETREG(r);
        ctl = k ? ((ctl & ~0xF0u) | ((uint32_t)sp << 4)) : ((ctl & ~0xFu) | (uint32_t)sp);
        break; }
      case AVGPU_H_SWAP_STK:                                  // :2739
        ctl ^= CTL_CURSTK;
        break;
      case AVGPU_H_SWAP: {                                    // :2742
        const int a = FMOD(1); const int b = (a + 1) % 3;
        const int va = GETREG(a), vb = GETREG(b);
        SETREG(a, vb); SETREG(b, va);
        break; }
      case AVGPU_H_SHIFT_R: { const int r = FMOD(1); SETREG(r, GETREG(r) >> 1); break; }
      case AVGPU_H_SHIFT_L: { const int r = FMOD(1); SETREG(r, (int)((uint32_t)GETREG(r) << 1)); break; }
      case AVGPU_H_INC: { const int r = FMOD(1); SETREG(r, (int)((uint32_t)GETREG(r) + 1u)); break; }
      case AVGPU_H_DEC: { const int r = FMOD(1); SETREG(r, (int)((uint32_t)GETREG(r) - 1u)); break; }
      case AVGPU_H_ADD: { const int r = FMOD(1); SETREG(r, (int)((uint32_t)r1 + (uint32_t)r2)); break; }
      case AVGPU_H_SUB: { const int r = FMOD(1); SETREG(r, (int)((uint32_t)r1 - (uint32_t)r2)); break; }
      case AVGPU_H_NAND: { const int r = FMOD(1); SETREG(r, ~(r1 & r2)); break; }
      case AVGPU_H_IO: {                                      // :4188 Inst_TaskIO
        const int r = FMOD(1);
        const int out = GETREG(r);
        // cOrganism::DoOutput -> cTaskLib::SetupTests (main/cTaskLib.cc:369-448)
        W.outbuf[cell] = out;
        W.out_total[cell] += 1;
        const int i0 = W.inbuf[cell], i1 = W.inbuf[N + cell], i2 = W.inbuf[2 * N + cell];
        const int tot = W.in_total[cell];
        const int num = tot < 3 ? tot : 3;
        const uint32_t a = num > 0 ? (uint32_t)i0 : 0u;
        const uint32_t b = num > 1 ? (uint32_t)i1 : 0u;
        const uint32_t c = num > 2 ? (uint32_t)i2 : 0u;
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
        const uint32_t tmask = (!bad && id >= 0 && id < 256) ? W.task_lut[id] : 0u;
        if (tmask) {
          // cEnvironment::TestOutput / TestRequisites / DoProcesses
          // (main/cEnvironment.cc:1314-1406, :1408-1503, :1610-1760)
          uint32_t done = 0;
          double mult = 1.0, addb = 0.0;
          for (int i = 0; i < W.n_react; i++) {
            const int t = W.react_task[i];
            if (!((tmask >> t) & 1u)) continue;
            const int cnt = W.cur_task[(int64_t)t * N + cell];
            if (W.react_hasreq[i] && (cnt < W.react_min[i] || cnt >= W.react_max[i])) continue;
            done |= 1u << t;
            if (W.react_type[i] == AVGPU_PROC_ADD) addb = __dadd_rn(addb, W.react_add[i]);
            else mult = __dmul_rn(mult, W.react_mult[i]);
            W.cur_react[(int64_t)i * N + cell] += 1;
          }
          if (done) {
            for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++)
              if ((done >> t) & 1u) W.cur_task[(int64_t)t * N + cell] += 1;
            const double bon = W.cur_bonus[cell];
            W.cur_bonus[cell] = __dadd_rn(__dmul_rn(bon, mult), addb);  // cPhenotype.cc:1645-1646
          }
        }
        // GetNextInput (main/cOrganism.h:249 -> cPopulationCell.h:214-218) + DoInput
        int p = W.in_ptr[cell];
        if (p >= 3) p = 0;
        const int in = W.inputs[(int64_t)p * N + cell];
        W.in_ptr[cell] = p + 1;
        W.inbuf[2 * N + cell] = i1;
        W.inbuf[N + cell] = i0;
        W.inbuf[cell] = in;
        W.in_total[cell] = tot + 1;
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
        if (!ok) { W.errors[cell] += 1; break; }
        if (W.alloc_method == 2) {
          for (int i = cur; i < nsz; i++) T[i] = random_code(W, klo, khi, kct);
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
        if (ok) {
          for (int i = 0; i < div; i++) exe += (T[i] >> 7);
          ok = exe >= (int)(div * W.min_exe_lines);
        }
        if (ok) {
          for (int i = div; i < div + child; i++) cop += (T[i] >> 6) & 1;
          ok = cop >= (int)(child * W.min_copied_lines);
        }
        double bonus = 0.0;
        int old_exe = 0, copied = 0;
        if (ok) {  // cOrganism::Divide_CheckViable (main/cOrganism.cc:788-919)
          bonus = W.cur_bonus[cell];
          if (bonus < W.required_bonus) ok = false;
          old_exe = W.executed[cell];
          copied = W.copied[cell];
          const double base0 = (double)calc_size_merit(W, blen, copied, old_exe);
          double b0 = bonus;
          if (W.merit_default_bonus != 0.0) b0 = W.merit_default_bonus;
          double off_merit = __dmul_rn(base0, b0);
          if (W.inherit_merit == 0) off_merit = base0;
          if (off_merit == 0.0) ok = false;
        }
        if (!ok) break;                                       // AdjustHeads again: no-op
        W.executed[cell] = exe;                               // SetLinesExecuted
        W.child_copied[cell] = cop;                           // SetLinesCopied
        // ---- offspring ----
        int nd = W.num_div[cell] + 1;
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
        if (W.merit_default_bonus != 0.0) bonus = W.merit_default_bonus;
        double merit = __dmul_rn(base, bonus);
        if (W.inherit_merit == 0) merit = base;
        const int gt = tu - gs;
        const double fit = __ddiv_rn(__dmul_rn(base, bonus), (double)gt);
        W.merit[cell] = merit;
        W.gest_time[cell] = gt;
        W.fitness[cell] = fit;
        gs = tu;
        W.num_div[cell] = nd;
        const int gen = W.generation[cell] + 1;
        W.generation[cell] = gen;
        W.errors[cell] = 0;
        W.cur_bonus[cell] = W.default_bonus;
        cyc = 0;
        for (int t = 0; t < AVGPU_NUM_LOGIC_TASKS; t++) {
          W.last_task[(int64_t)t * N + cell] = W.cur_task[(int64_t)t * N + cell];
          W.cur_task[(int64_t)t * N + cell] = 0;
        }
        for (int i = 0; i < W.n_react; i++) W.cur_react[(int64_t)i * N + cell] = 0;
        if (mode == AVGPU_MODE_WORLD) {
          // Divide_DoMutations (cpu/cHardwareBase.cc:296-569), default subset
          int len = child;
          int mline = -1, iline = -1, dline = -1;
          uint8_t mcode = 0, icode = 0;
          if (W.th_div_mut && rng_p(klo, khi, kct, W.th_div_mut)) {
            mline = (int)rng_below(klo, khi, kct, (uint32_t)len);
            mcode = random_code(W, klo, khi, kct);
          }
          if (W.th_div_ins && rng_p(klo, khi, kct, W.th_div_ins) && len < W.max_genome) {
            iline = (int)rng_below(klo, khi, kct, (uint32_t)len + 1);
            icode = random_code(W, klo, khi, kct);
            len++;
          }
          if (W.th_div_del && rng_p(klo, khi, kct, W.th_div_del) && len > W.min_genome) {
            dline = (int)rng_below(klo, khi, kct, (uint32_t)len);
            len--;
          }
          const int slot = atomicAdd(W.b_count, 1);
          if (slot < W.bcap) {
            uint8_t* g = W.b_genome + (int64_t)slot * TAPE_SLOT;
            for (int j = 0; j < len; j++) {
              int k2 = (dline >= 0 && j >= dline) ? j + 1 : j;       // index before the deletion
              int v;
              if (iline >= 0 && k2 == iline) v = icode;
              else {
                const int k1 = (iline >= 0 && k2 > iline) ? k2 - 1 : k2;  // before the insertion
                v = (k1 == mline) ? mcode : (T[div + k1] & CODE_MASK);
              }
              g[j] = (uint8_t)v;
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
        for (int k = 0; k < 2 * AVGPU_STACK_SIZE; k++) W.stack[(int64_t)k * N + cell] = 0;
        ctl = CTL_ALIVE;
        rl = 0;
        for (int i = 0; i < div; i++) T[i] &= CODE_MASK;
        adv = false;
        break; }
      case AVGPU_H_H_COPY: {                                  // :7130 Inst_HeadCopy
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
          v = random_code(W, klo, khi, kct);
        T[wh] = (uint8_t)((T[wh] & TF_EXEC) | TF_COPIED | v);
        rh = head_adjust(rh + 1, M);
        wh = head_adjust(wh + 1, M);
        break; }
      case AVGPU_H_H_SEARCH:                                  // :7245 Inst_HeadSearch
      case AVGPU_H_IF_LABEL: {                                // :6914 Inst_IfLabel
        // ReadLabel (:1484-1502)
        uint32_t lab = 0;
        int len = 0;
        while (len < AVGPU_MAX_LABEL) {
          const int p = ip + 1;
          if (p >= M) break;
          const int cc = T[p] & CODE_MASK;
          if (cc >= 3) break;
          ip = p;
          lab |= (uint32_t)cc << (2 * len);
          len++;
          if (len <= W.max_label_exe) T[ip] |= TF_EXEC;
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
        // FindLabel(0) -> FindLabel_Forward(label, memory, 0) (:1177-1295)
        int found = ip;
        if (len > 0) {
          int pos = len;
          int fpos = -1;
          while (pos < M) {
            if ((T[pos] & CODE_MASK) < 3) {
              int sp0 = pos, ep = pos + 1;
              while (sp0 > 0 && (T[sp0 - 1] & CODE_MASK) < 3) sp0--;
              while (ep < M && (T[ep] & CODE_MASK) < 3) ep++;
              const int max_off = (ep - sp0) - len + 1;
              int off = sp0;
              bool hit = false;
              for (; off < sp0 + max_off; off++) {
                int mm = 0;
                for (; mm < len; mm++)
                  if ((int)((rot >> (2 * mm)) & 3u) != (T[off + mm] & CODE_MASK)) break;
                if (mm == len) { hit = true; break; }
              }
              if (hit) { fpos = len + off; break; }
              pos = ep;
            }
            pos += len;
          }
          if (fpos >= 0) found = head_adjust(fpos - 1, M);
        }
        r1 = found - ip;
        r2 = len;
        fh = head_adjust(found + 1, M);
        break; }
      case AVGPU_H_MOV_HEAD: {                                // :6809
        const int h = FMOD(0);
        SETHEAD(h, fh);
        if (h == 0) adv = false;
        break; }
      case AVGPU_H_JMP_HEAD: {                                // :6859
        const int h = FMOD(0);
        SETHEAD(h, head_adjust((int)((uint32_t)GETHEAD(h) + (uint32_t)r2), M));
        break; }
      case AVGPU_H_GET_HEAD: {                                // :6907
        const int h = FMOD(0);
        r2 = GETHEAD(h);
        break; }
      case AVGPU_H_SET_FLOW: {                                // :7270
        const int r = FMOD(2);
        fh = head_adjust(GETREG(r), M);
        break; }
      default:
        break;
    }
#undef FMOD
    if (stop) break;
    if (adv) ip = head_adjust(ip + 1, M);                     // ip.Advance() :1013
    if (mx > 0 && tu >= mx) alive = false;                    // death :1045-1049
  }
#undef GETREG
#undef SETREG
#undef GETHEAD
#undef SETHEAD

  // ---- write back ----
  if (active) {
    W.reg[cell] = r0; W.reg[N + cell] = r1; W.reg[2 * N + cell] = r2;
    W.head[cell] = ip; W.head[N + cell] = rh; W.head[2 * N + cell] = wh; W.head[3 * N + cell] = fh;
    if (!alive) ctl &= ~CTL_ALIVE;
    W.ctl[cell] = ctl; W.rlabel[cell] = rl;
    W.mem_size[cell] = M;
    W.cycles[cell] = cyc; W.time_used[cell] = tu; W.gest_start[cell] = gs;
    W.rng[2 * N + cell] = kct;
    W.budget[cell] = spill ? budget : 0;
    if (spill) {
      const int slot = atomicAdd(&W.class_count[cls + 1], 1);
      W.class_list[(int64_t)(cls + 1) * N + slot] = cell;
      count_add(W, CNT_SPILLS, 1ull);
    }
  }
  __syncthreads();
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
  for (int off = 32; off > 0; off >>= 1) {
    e += __shfl_down(e, off);
    dead += __shfl_down(dead, off);
    dv += __shfl_down(dv, off);
  }
  if (lane == 0) {
    count_add(W, CNT_INSTS, e);
    if (dead) count_add(W, CNT_DEATHS, (unsigned long long)dead);
    if (dv) count_add(W, CNT_DIVIDES, (unsigned long long)dv);
  }
}

}  // namespace

void launch_interpret_classes(const DevWorld& W, int mode, hipStream_t s, int64_t first,
                              int64_t count, int* launches) {
  const unsigned blocks = (unsigned)((count + 63) / 64);
  if (blocks == 0) return;
  hipLaunchKernelGGL(k_interpret<CLASS0_SIZE>, dim3(blocks), dim3(64), 0, s, W, 0, mode, first, count);
  hipLaunchKernelGGL(k_interpret<768>, dim3(blocks), dim3(64), 0, s, W, 1, mode, first, count);
  hipLaunchKernelGGL(k_interpret<1536>, dim3(blocks), dim3(64), 0, s, W, 2, mode, first, count);
  hipLaunchKernelGGL(k_interpret<2048>, dim3(blocks), dim3(64), 0, s, W, 3, mode, first, count);
  if (launches) *launches += 4;
}
