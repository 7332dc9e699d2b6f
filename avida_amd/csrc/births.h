// births.h -- offspring helpers shared by the placement kernels (world.hip)
// and the serial world (interp.hip): the neighbourhood, the divide-mutation
// edits, and ActivateOrganism / SetupOffspring of a record into a cell.
// Paths are relative to avida-core/source/ of the reference.
#pragma once
#include "device.h"

namespace {

// ---- birth placement (cPopulation::PositionOffspring restated) ----
// neighbour k of cell in fixed order NW N NE W E SW S SE (tools/cTopology.h).
// Tiled worlds map the rows above / below the strip to the ghost rows
// [n, n+X) / [n+X, n+2X) of occ / claim / owner.
__device__ __forceinline__ int neighbours(const DevWorld& W, int cell, int* out) {
  const int X = W.world_x, R = W.rows;
  const int x = cell % X, y = cell / X;
  int n = 0;
  for (int dy = -1; dy <= 1; dy++)
    for (int dx = -1; dx <= 1; dx++) {
      if (dx == 0 && dy == 0) continue;
      int nx = x + dx, ny = y + dy;
      if (W.geometry == 1) {
        if (nx < 0 || nx >= X) continue;
      } else {
        nx = (nx + X) % X;
      }
      if (ny >= 0 && ny < R) {
        out[n++] = ny * X + nx;
      } else if (!W.tiled) {
        if (W.geometry == 1) continue;
        ny = (ny + R) % R;
        out[n++] = ny * X + nx;
      } else {
        const int gy = W.row0 + ny;
        if (W.geometry == 1 && (gy < 0 || gy >= W.global_rows)) continue;
        out[n++] = (int)W.n + (ny < 0 ? 0 : X) + nx;
      }
    }
  return n;
}

// Divide_DoMutations' edits (cpu/cHardwareBase.cc:296-569), drawn in the
// interpreter in the reference's order and stored with the birth record
// (interp.hip): one wave per queued offspring that has any rewrites its
// genome -- site j of the mutated child is traced back through the edits
// (last first, the variable-count segments in b_subs included) to a site of
// the unmutated child or to a value an edit wrote.
// Runs before placement, so halo records and activation see final genomes.
// one edit word undone: site src of the genome after the edit -> the site it
// came from before it, or the value the edit wrote (val >= 0); slips go
// through slip_back
__device__ __forceinline__ void edit_back(int ew, int& src, int& val) {
  if (ew == 0 || val >= 0) return;
  const int kind = ew & 7, a = (ew >> 3) & 0xFFF, b = (ew >> 15) & 0xFFF;
  if (kind == 2) {                         // point (E_POINT)
    if (src == a) val = b;
  } else if (kind == 3) {                  // insertion (E_INS)
    if (src == a) val = b; else if (src > a) src--;
  } else if (kind == 4) {                  // deletion (E_DEL)
    if (src >= a) src++;
  }
}
// a slip undone (doSlipMutation, cpu/cHardwareBase.cc:621-694) from a to b:
// a site of the filled insertion [a, 2a - b) takes its SLIP_FILL_MODE fill --
// 0 duplication (site b + k), 4 nop-C, and the data fills (fill != nullptr:
// the slip's L words in the arena) 2 random codes, 3 scrambled source sites
__device__ __forceinline__ void slip_back(int ew, int sfm, const int32_t* fill, int& src, int& val) {
  if (ew == 0 || val >= 0) return;
  const int a = (ew >> 3) & 0xFFF, b = (ew >> 15) & 0xFFF;
  if (a > b && src >= a && src < 2 * a - b) {
    if (sfm == 4) { val = AVGPU_H_NOP_C; return; }
    if (sfm == 2 && fill) { val = fill[src - a]; return; }
    if (sfm == 3 && fill) { src = fill[src - a]; return; }
  }
  if (src >= a) src = b + (src - a);
}
// a translocation undone (doTransMutation, cpu/cHardwareBase.cc:700-760):
// w0 = E_TRANS | ins_loc << 3 | to << 15, w1 = from; fill (TRANS_FILL_MODE 1)
// the inserted sites' source sites, scrambling and its read-backs resolved
// by the interpreter
__device__ __forceinline__ void trans_back(int w0, int w1, const int32_t* fill, int& src, int val) {
  if (val >= 0) return;
  const int ins = (w0 >> 3) & 0xFFF, to = (w0 >> 15) & 0xFFF, L = w1 - to;
  if (L > 0) {
    if (src >= ins + L) src -= L;
    else if (src >= ins) src = fill ? fill[src - ins] : to + (src - ins);
  } else if (L < 0 && src >= ins) {
    src -= L;
  }
}
// applied order (device.h SEG_*): e0, segments 0-5 (slips, translocations),
// e1, segment 6, e2, the other segments (pcnt[k] words at subs + pofs[k]).
// sfm / tfm: SLIP_FILL_MODE / TRANS_FILL_MODE; with a data fill (2, 3 / 1)
// a slip takes two words (edit, fill offset) and a translocation three.
__device__ __forceinline__ int mut_source(int j, const int* e, int sfm, int tfm, int& val, const int32_t* subs,
                                          const int* pofs, const int* pcnt) {
  constexpr int first[5] = {SEG_OSLIP, SEG_PMUT, SEG_PINS, SEG_PDEL, SEG_SMUT};
  constexpr int last[5] = {SEG_STRANS, SEG_PMUT, SEG_PINS, SEG_PDEL, SEG_SUNI};
  const bool sdata = sfm == 2 || sfm == 3;
  const int tw = tfm == 1 ? 3 : 2;
  int src = j;
  val = -1;
#pragma unroll
  for (int k = 4; k >= 0; k--) {
#pragma unroll
    for (int g = last[k]; g >= first[k]; g--) {
      if (g >= SEG_TTRANS && g <= SEG_STRANS) {
        for (int i = pcnt[g] - tw; i >= 0 && val < 0; i -= tw) {
          const int fo = tw == 3 ? subs[pofs[g] + i + 2] : -1;
          trans_back(subs[pofs[g] + i], subs[pofs[g] + i + 1], fo >= 0 ? subs + fo : nullptr, src, val);
        }
      } else if (g <= SEG_SSLIP && sdata) {
        for (int i = pcnt[g] - 2; i >= 0 && val < 0; i -= 2) {
          const int fo = subs[pofs[g] + i + 1];
          slip_back(subs[pofs[g] + i], sfm, fo >= 0 ? subs + fo : nullptr, src, val);
        }
      } else if (g <= SEG_SSLIP) {
        for (int i = pcnt[g] - 1; i >= 0 && val < 0; i--) slip_back(subs[pofs[g] + i], sfm, nullptr, src, val);
      } else {
        for (int i = pcnt[g] - 1; i >= 0 && val < 0; i--) edit_back(subs[pofs[g] + i], src, val);
      }
    }
    if (k == 0) slip_back(e[0], sfm, nullptr, src, val);
    else edit_back(e[k], src, val);
  }
  return src;
}

// LDS written by some lanes of a wave, then read by others: wait for the
// wave's own LDS traffic (no block barrier -- the mutation waves of one
// workgroup run different numbers of records)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The divide-mutation edits of record r applied to its child genome by one
// wave (k_apply_mutations; the serial world per birth): a no-op when the
// record has none.  child: LDS scratch of TAPE_SLOT + 16 bytes.
// apply_edits_core: the same with the record's five edit words and lengths
// already in hand (the mutation scan loads them with the queue entry, so a
// genome costs one dependent round trip -- its own words -- instead of three)
__device__ __forceinline__ void apply_edits_core(const DevWorld& W, int64_t r, const int* e, int len0, int len,
                                                 uint8_t* child) {
  const int lane = threadIdx.x & 63;
  const int sfm = W.slip_fill_mode, tfm = W.trans_fill_mode;
  int pofs[NSEG], pcnt[NSEG], np = 0;   // variable-count edit segments
#pragma unroll
  for (int k = 0; k < NSEG; k++) {
    pofs[k] = W.seg_any ? W.b_pofs[(int64_t)k * W.rcap + r] : 0;
    pcnt[k] = W.seg_any ? W.b_pcnt[(int64_t)k * W.rcap + r] : 0;
    np |= pcnt[k];
  }
  if ((e[0] | e[1] | e[2] | e[3] | e[4] | np) == 0) return;   // wave-uniform
  uint32_t* g32 = reinterpret_cast<uint32_t*>(W.b_genome + r * TAPE_SLOT);
  uint32_t* c32 = reinterpret_cast<uint32_t*>(child);
  for (int w = lane; (w << 2) < len0; w += 64) c32[w] = g32[w];
  wave_lds_sync();
  for (int w = lane; (w << 2) < len; w += 64) {
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int j = 4 * w + k;
      int val;
      const int src = mut_source(j, e, sfm, tfm, val, W.b_subs, pofs, pcnt);
      const uint32_t v = val >= 0 ? (uint32_t)val : (uint32_t)child[src];
      word |= (j < len ? v : 0u) << (8 * k);
    }
    g32[w] = word;
  }
  wave_lds_sync();
}
__device__ __forceinline__ void apply_edits_wave(const DevWorld& W, int64_t r, uint8_t* child) {
  int e[5];
#pragma unroll
  for (int k = 0; k < 5; k++) e[k] = W.b_edit[(int64_t)k * W.rcap + r];
  apply_edits_core(W, r, e, W.b_len0[r], W.b_len[r], child);
}

// ActivateOrganism (main/cPopulation.cc:1320-1340) + SetupOffspring
// (main/cPhenotype.cc:349-420) of one offspring into cell c by one wave.  The
// organism is marked CTL_FRESH: its zero / default fields (registers, heads,
// stacks, IO buffers, counters, task and reaction counts, bonus) are implied
// by the bit instead of stored -- they sit in ~90 SoA rows, one scattered
// store each -- and its first slice writes them back.  What is stored here,
// one field per lane: the genome, its length and the phenotype it inherits.
struct Child {
  int len, gen, ccopied, exec, gest;
  double merit, fitness;
  uint32_t lo, hi, ctr;
  const int32_t* ltask;   // the parent's last task counts, ltask[q * lstride]
  int64_t lstride;
  const int32_t* inputs = nullptr;   // the cell inputs, drawn by the caller (serial world), or
                                     // nullptr: SetupInputs from the offspring's own stream
  uint32_t hs = 0;                   // head start (CTL_HS: 2^16 - birth time; 0 in the serial world)
};
// Run by a group of G lanes (G = 64: a wave, 32: a half-wave); `lane` is the
// lane's index inside its group.
template <int G>
__device__ __forceinline__ void setup_child(const DevWorld& W, int64_t c, const Child& b,
                                            const uint32_t* src, int lane) {
  static_assert(G == 32 || G == 64, "group = wave or half-wave");
  const int64_t N = W.n;
  const int len = b.len;
  uint32_t* dst = reinterpret_cast<uint32_t*>(W.tape + c * TAPE_SLOT);
  uint64_t gsum = 0;
  for (int w = lane; w < (len + 3) / 4; w += G) {
    const uint32_t v = src[w];
    dst[w] = v;
    gsum += gk_word(v, w, len);
  }
  for (int off = G / 2; off > 0; off >>= 1) gsum += __shfl_xor(gsum, off);
  if (lane == 0) W.gkey[c] = gk_final(gsum, len);
  switch (lane) {
    case 0: W.ctl[c] = CTL_ALIVE | CTL_FRESH | (b.hs << CTL_HS_SHIFT); break;
    case 1: W.mem_size[c] = len; break;
    case 2: {
      int mx = 0;
      if (W.death_method > 0) { mx = W.age_limit; if (W.death_method == 2) mx *= len; if (mx < 1) mx = 1; }
      W.max_exec[c] = mx;
      break; }
    case 3: W.birth_len[c] = len; break;
    case 4: W.merit[c] = b.merit; break;
    case 5: W.fitness[c] = b.fitness; break;
    case 6: W.credit[c] = 0.0; break;
    case 7: W.gest_time[c] = b.gest; break;
    case 8: W.generation[c] = b.gen; break;
    case 9: W.copied[c] = b.ccopied; break;
    case 10: W.executed[c] = b.exec; break;
    case 11: {
      uint32_t ctr = b.ctr;
      // cEnvironment::SetupInputs random (main/cEnvironment.cc:1268-1271)
      if (b.inputs) {
        W.inputs[c] = b.inputs[0]; W.inputs[N + c] = b.inputs[1]; W.inputs[2 * N + c] = b.inputs[2];
      } else {
        W.inputs[c] = (15 << 24) + (int)rng_below(b.lo, b.hi, ctr, 1u << 24);
        W.inputs[N + c] = (51 << 24) + (int)rng_below(b.lo, b.hi, ctr, 1u << 24);
        W.inputs[2 * N + c] = (85 << 24) + (int)rng_below(b.lo, b.hi, ctr, 1u << 24);
      }
      W.rng[c] = b.lo; W.rng[N + c] = b.hi; W.rng[2 * N + c] = ctr;
      if (W.rec_off) W.rec_off[c] = -1;         // offspring: counter streams
      break; }
    case 12 + AVGPU_NUM_LOGIC_TASKS: if (W.track_age) W.age[c] = 0; break;   // SetupOffspring (main/cPhenotype.cc:705)
    default:                                   // last_task_count = the parent's (:447)
      if (lane >= 12 && lane < 12 + AVGPU_NUM_LOGIC_TASKS)
        W.last_task[(int64_t)(lane - 12) * N + c] = b.ltask[(int64_t)(lane - 12) * b.lstride];
      break;
  }
}

// The same activation by ONE lane (k_activate: a lane per queued birth, so a
// launch of ~1k waves covers a 60k-birth update with all of its record loads
// in flight at once).  The genome moves in 16-byte quads; the bytes of the
// last quad past the genome are written as 0 (sites >= mem_size are never
// read before h-alloc fills them, and every export masks them).
// one 16-B quad k of an offspring's genome into the cell's tape: the sites
// past len cleared, the genotype key's words summed
__device__ __forceinline__ void child_quad(uint4 v, int k, int len, uint4* __restrict__ d4, uint64_t& gsum) {
  const int w = 4 * k;
  uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int keep = len - 4 * (w + j);     // sites of word w+j inside the genome
    if (keep <= 0) x[j] = 0u;
    else { if (keep < 4) x[j] &= (1u << (8 * keep)) - 1u; gsum += gk_word(x[j], w + j, len); }
  }
  d4[k] = make_uint4(x[0], x[1], x[2], x[3]);
}
// PRE: the genome's first PRE quads are already in registers (pre), loaded by
// the caller before it knew whether the record won its cell
template <int PRE = 0>
__device__ __forceinline__ void setup_child_lane(const DevWorld& W, int64_t c, const Child& b,
                                                 const uint8_t* __restrict__ src, const uint4* pre = nullptr) {
  const int64_t N = W.n;
  const int len = b.len;
  const uint4* __restrict__ s4 = reinterpret_cast<const uint4*>(src);
  uint4* __restrict__ d4 = reinterpret_cast<uint4*>(W.tape + c * TAPE_SLOT);
  uint64_t gsum = 0;
  const int nq = (len + 15) >> 4;
#pragma unroll
  for (int u = 0; u < PRE; u++)
    if (u < nq) child_quad(pre[u], u, len, d4, gsum);
  for (int k0 = PRE; k0 < nq; k0 += 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (k0 + u < nq) v[u] = s4[k0 + u];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (k0 + u >= nq) break;
      child_quad(v[u], k0 + u, len, d4, gsum);
    }
  }
  W.gkey[c] = gk_final(gsum, len);
  W.ctl[c] = CTL_ALIVE | CTL_FRESH | (b.hs << CTL_HS_SHIFT);
  W.mem_size[c] = len;
  int mx = 0;
  if (W.death_method > 0) { mx = W.age_limit; if (W.death_method == 2) mx *= len; if (mx < 1) mx = 1; }
  W.max_exec[c] = mx;
  W.birth_len[c] = len;
  if (W.track_age) W.age[c] = 0;               // SetupOffspring (main/cPhenotype.cc:705)
  W.merit[c] = b.merit;
  W.fitness[c] = b.fitness;
  W.credit[c] = 0.0;
  W.gest_time[c] = b.gest;
  W.generation[c] = b.gen;
  W.copied[c] = b.ccopied;
  W.executed[c] = b.exec;
  uint32_t ctr = b.ctr;
  // cEnvironment::SetupInputs random (main/cEnvironment.cc:1268-1271)
  W.inputs[c] = (15 << 24) + (int)rng_below(b.lo, b.hi, ctr, 1u << 24);
  W.inputs[N + c] = (51 << 24) + (int)rng_below(b.lo, b.hi, ctr, 1u << 24);
  W.inputs[2 * N + c] = (85 << 24) + (int)rng_below(b.lo, b.hi, ctr, 1u << 24);
  W.rng[c] = b.lo; W.rng[N + c] = b.hi; W.rng[2 * N + c] = ctr;
  if (W.rec_off) W.rec_off[c] = -1;             // offspring: counter streams
#pragma unroll
  for (int q = 0; q < AVGPU_NUM_LOGIC_TASKS; q++)   // last_task_count = the parent's (:447)
    W.last_task[(int64_t)q * N + c] = b.ltask[(int64_t)q * b.lstride];
}

// the phenotype record r hands its offspring
__device__ __forceinline__ Child child_of_record(const DevWorld& W, int64_t i) {
  Child b;
  const int4* row = reinterpret_cast<const int4*>(W.b_inh + i * BI_WORDS);
  const int4 q0 = row[0], q1 = row[1], q2 = row[2];       // 16-B loads of the record's row
  static_assert(BI_MERIT == 0 && BI_GEN == 4 && BI_RLO == 8 && BI_LTASK == 12, "b_inh row layout");
  b.len = W.b_len[i];
  b.merit = __hiloint2double(q0.y, q0.x); b.fitness = __hiloint2double(q0.w, q0.z);
  b.gen = q1.x; b.ccopied = q1.y; b.exec = q1.z; b.gest = q1.w;
  b.lo = (uint32_t)q2.x; b.hi = (uint32_t)q2.y; b.ctr = (uint32_t)q2.z;
  b.hs = 0x10000u - BI_TIME(q2.w);
  b.ltask = W.b_inh + i * BI_WORDS + BI_LTASK; b.lstride = 1;
  return b;
}

}  // namespace
