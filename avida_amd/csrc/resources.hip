// resources.hip -- environment resources around the interpreter (config 5):
//   k_res_step<true>     one cSpatialResCount step of every resource without
//                        CELL entries (one launch; a wave walks a 64-column
//                        window down, each flow computed once), fused: Source + Sink
//                        (main/cSpatialResCount.cc:341-394), FlowAll / FlowMatter
//                        (:323-338, main/cResourceCount.cc:40-110), StateAll
//                        (:307-314), double-buffered
//   k_res_spatial_rates  Source + Sink into res_delta  } resources with CELL
//   k_res_cell_rates     CellInflow + CellOutflow      } entries: then
//                        (:356-404), list order        } k_res_step<false>
//   k_res_global_begin   DoNonSpatialUpdates over one update   (main/cResourceCount.cc:757-827)
//   k_res_global_end     the update's consumption of global resources
//   k_res_pack / k_res_settle   strip tiles: edge rows out; summed consumption in
// Every per-cell sum is formed in the reference's order (the sequential loops
// of cSpatialResCount add into a cell's delta in increasing index of the cell
// doing the computing), so the device agrees bit for bit with the oracle's
// literal restatement of those loops (oracle/oracle.cc res_begin).
#include "device.h"

#include <cstdlib>

#pragma clang fp contract(off)

namespace {

// x + d for |d| <= 1 wrapped into [0, L): amod without the division
__device__ __forceinline__ int wrap1(int x, int L) {
  return x >= L ? x - L : (x < 0 ? x + L : x);
}

__device__ __forceinline__ int amod(int x, int y) {   // AvidaTools::Mod
  x %= y;
  return x < 0 ? x + y : x;
}
// how many i in [a, b] have Mod(i, L) == v (a box may wrap or exceed the world)
__device__ __forceinline__ int cover(int v, int a, int b, int L) {
  if (b < a) return 0;
  const int i0 = a + amod(v - a, L);
  return i0 > b ? 0 : 1 + (b - i0) / L;
}

// coordinates are global (a strip tile holds rows [row0, row0 + rows) of the
// WORLD_X x world_y grid; boxes and CELL ids refer to the global grid)
__global__ void k_res_spatial_rates(DevWorld W, int r) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W.n) return;
  const ResParam P = W.res_param[r];
  const int X = W.world_x, Y = W.world_y;
  const int x = (int)(c % X), y = W.row0 + (int)(c / X);
  double d = 0.0;
  const int nin = cover(y, P.in_y1, P.in_y2, Y) * cover(x, P.in_x1, P.in_x2, X);
  for (int k = 0; k < nin; k++) d = __dadd_rn(d, P.in_share);
  if (P.has_sink) {
    const int nout = cover(y, P.out_y1, P.out_y2, Y) * cover(x, P.out_x1, P.out_x2, X);
    const double a = W.res_amount[(int64_t)P.slot * W.n + c];
    const double dec = fmax(__dmul_rn(a, P.sink_frac), 0.0);
    for (int k = 0; k < nout; k++) d = __dadd_rn(d, -dec);
  }
  W.res_delta[c] = d;
}

__global__ void k_res_cell_rates(DevWorld W, int r) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ResParam P = W.res_param[r];
  const double* amt = W.res_amount + (int64_t)P.slot * W.n;
  const int64_t nglobal = (int64_t)W.world_x * W.world_y;
  for (int i = 0; i < W.n_cellres; i++) {
    const avgpu_cell_resource e = W.res_cells[i];
    const int64_t l = e.cell - W.cell0;
    if (e.resource == r && e.cell >= 0 && e.cell < nglobal && l >= 0 && l < W.n)
      W.res_delta[l] = __dadd_rn(W.res_delta[l], e.inflow);
  }
  for (int i = 0; i < W.n_cellres; i++) {
    const avgpu_cell_resource e = W.res_cells[i];
    const int64_t l = e.cell - W.cell0;
    if (e.resource == r && e.cell >= 0 && e.cell < nglobal && l >= 0 && l < W.n) {
      const double dec = fmax(__dmul_rn(amt[l], e.outflow), 0.0);
      W.res_delta[l] = __dadd_rn(W.res_delta[l], -dec);
    }
  }
}

// x / c correctly rounded for a constant c with r = RN(1 / c): y = RN(x r) is
// a faithful quotient, the residual x - c y is exact by FMA, and
// RN(y + r (x - c y)) = RN(x / c) (Markstein's correction) away from
// underflow and overflow -- tiny, huge and non-finite x take the full
// division (zero: x r, which keeps the sign).  3 FP64 operations instead of
// __ddiv_rn's scaled Newton sequence; tests/test_res_division.py checks the
// identity on 2e7 quotients per c (4e8 when it was written).
__device__ __forceinline__ double div_const(double x, double c, double r) {
  const double ax = fabs(x);
  const double y = __dmul_rn(x, r);
  if (!(ax >= 0x1p-900 && ax <= 0x1p+900) && ax != 0.0) return __ddiv_rn(x, c);
  const double e = __fma_rn(-c, y, x);
  return ax == 0.0 ? y : __fma_rn(e, r, y);                 // +-0 (equal amounts: a common flow): x r
}
constexpr double SQRT2 = 1.4142135623730951, R_SQRT2 = 1.0 / 1.4142135623730951, R_3 = 1.0 / 3.0;

// FlowMatter (main/cResourceCount.cc:40-110) from elem1 = a1 to elem2 = a2.
// Exact rewrites: x / 16 == x * 0.0625 and x / 2 == x * 0.5 (power-of-two
// divisors: the same real value, so the same rounding), and with zero gravity
// the reference's (-a2 * 0) / 3 is the signed zero (-a2 * 0) itself.
__device__ __forceinline__ double gravity_term(double a1, double a2, int dist, double g) {
  if (g == 0.0) return __dmul_rn(-a2, 0.0);
  if ((dist > 0 && g > 0.0) || (dist < 0 && g < 0.0)) return div_const(__dmul_rn(a1, fabs(g)), 3.0, R_3);
  return div_const(__dmul_rn(-a2, fabs(g)), 3.0, R_3);
}

// GRAV false: the launch's resources have no gravity (the terms are the
// signed zero -a2 * 0, gravity_term's own value for g == 0, without its tests)
template <bool GRAV = true>
__device__ __forceinline__ double flow_amt(const ResParam& P, double a1, double a2, int xdist, int ydist,
                                           bool diagonal) {
  const double diff = __dsub_rn(a1, a2);
  double xg = 0.0, xd = 0.0, yg = 0.0, yd = 0.0;
  if (xdist != 0) {
    xg = GRAV ? gravity_term(a1, a2, xdist, P.xgravity) : __dmul_rn(-a2, 0.0);
    xd = __dmul_rn(__dmul_rn(P.xdiffuse, diff), 0.0625);
  }
  if (ydist != 0) {
    yg = GRAV ? gravity_term(a1, a2, ydist, P.ygravity) : __dmul_rn(-a2, 0.0);
    yd = __dmul_rn(__dmul_rn(P.ydiffuse, diff), 0.0625);
  }
  const double num = __dadd_rn(__dadd_rn(__dadd_rn(xd, yd), xg), yg);
  const double q = diagonal ? __dmul_rn(num, 0.5) : num;        // / (|xdist| + |ydist|)
  return diagonal ? div_const(q, SQRT2, R_SQRT2) : q;           // / dist (sqrt(2.0) or 1)
}

// pointer k = 3..6 of cell (x, y): E, SE, S, SW (cSpatialResCount::SetPointers)
__device__ __forceinline__ bool res_ptr(int geometry, int X, int Y, int x, int y, int k, int& nx, int& ny) {
  const int dx = (k == 3 || k == 4) ? 1 : (k == 5 ? 0 : -1);
  const int dy = (k == 3) ? 0 : 1;
  if (geometry == AVGPU_RES_GRID) {
    if ((k == 3 || k == 4) && x == X - 1) return false;
    if (k == 6 && x == 0) return false;
    if (k != 3 && y == Y - 1) return false;
  }
  nx = wrap1(x + dx, X);
  ny = wrap1(y + dy, Y);
  return true;
}

// amount of global cell (gx, gy): this world's rows, else the edge row the
// tile above (gy = row0 - 1) or below sent
__device__ __forceinline__ double res_at(const DevWorld& W, const double* amt, int slot, int gx, int gy) {
  const int ly = gy - W.row0;
  if (ly >= 0 && ly < W.rows) return amt[(int64_t)ly * W.world_x + gx];
  const int up = wrap1(W.row0 - 1, W.world_y);
  return (gy == up ? W.rs_recv[0] : W.rs_recv[1])[(int64_t)slot * W.world_x + gx];
}

template <int I, int J>
__device__ __forceinline__ void cswap(int64_t (&key)[8], double (&val)[8]) {
  if (key[J] < key[I]) {
    const int64_t tk = key[I]; key[I] = key[J]; key[J] = tk;
    const double tv = val[I]; val[I] = val[J]; val[J] = tv;
  }
}

// the spatial resources one k_res_step launch steps: blockIdx.y = index into
// r[] (the resources own disjoint grids, so their steps are independent)
struct ResIds {
  int r[AVGPU_MAX_RESOURCES];
};

// Source + Sink of cell (x, y) (main/cSpatialResCount.cc:341-394): the rate
// the flows are added to
__device__ __forceinline__ double res_source_sink(const ResParam& P, double a_c, int x, int y, int X, int Y) {
  double d = 0.0;
  if (P.in_all) {
    d = __dadd_rn(d, P.in_share);
  } else {
    const int nin = cover(y, P.in_y1, P.in_y2, Y) * cover(x, P.in_x1, P.in_x2, X);
    for (int k = 0; k < nin; k++) d = __dadd_rn(d, P.in_share);
  }
  if (P.has_sink) {
    const double dec = fmax(__dmul_rn(a_c, P.sink_frac), 0.0);
    if (P.out_all) {
      d = __dadd_rn(d, -dec);
    } else {
      const int nout = cover(y, P.out_y1, P.out_y2, Y) * cover(x, P.out_x1, P.out_x2, X);
      for (int k = 0; k < nout; k++) d = __dadd_rn(d, -dec);
    }
  }
  return d;
}

// A world-edge cell's FlowAll terms onto its rate d: its own pointers' flows
// own[k - 3] and the flows in[k - 3] of the cells whose pointer k is c
// (k = 3..6: E, SE, S, SW), added in increasing (computing cell, k) order of
// global cell ids like the reference's loop over i (an 8-entry sorting
// network keeps the order in registers); a pointer the geometry lacks adds
// nothing (cSpatialResCount::SetPointers)
__device__ __forceinline__ double res_edge_sum(const ResParam& P, int X, int Y, int x, int y, const double (&own)[4],
                                               const double (&in)[4], double d) {
  const int64_t gc = (int64_t)y * X + x;
  int64_t key[8];
  double val[8];
#pragma unroll
  for (int k = 3; k <= 6; k++) {                     // own pointers: slots 0..3
    int nx, ny;
    const bool ok = res_ptr(P.geometry, X, Y, x, y, k, nx, ny);
    key[k - 3] = ok ? gc * 8 + k : INT64_MAX;
    val[k - 3] = ok ? -own[k - 3] : 0.0;
  }
#pragma unroll
  for (int k = 3; k <= 6; k++) {                     // cells whose pointer k is c: slots 4..7
    const int dx = (k == 3 || k == 4) ? 1 : (k == 5 ? 0 : -1), dy = (k == 3) ? 0 : 1;
    const int jx = wrap1(x - dx, X), jy = wrap1(y - dy, Y);
    int nx, ny;
    const bool ok = res_ptr(P.geometry, X, Y, jx, jy, k, nx, ny) && nx == x && ny == y;
    key[k + 1] = ok ? ((int64_t)jy * X + jx) * 8 + k : INT64_MAX;
    val[k + 1] = ok ? in[k - 3] : 0.0;
  }
  // Batcher odd-even merge sort of 8 (19 compare-exchanges)
  cswap<0, 1>(key, val); cswap<2, 3>(key, val); cswap<4, 5>(key, val); cswap<6, 7>(key, val);
  cswap<0, 2>(key, val); cswap<1, 3>(key, val); cswap<4, 6>(key, val); cswap<5, 7>(key, val);
  cswap<1, 2>(key, val); cswap<5, 6>(key, val);
  cswap<0, 4>(key, val); cswap<1, 5>(key, val); cswap<2, 6>(key, val); cswap<3, 7>(key, val);
  cswap<2, 4>(key, val); cswap<3, 5>(key, val);
  cswap<1, 2>(key, val); cswap<3, 4>(key, val); cswap<5, 6>(key, val);
#pragma unroll
  for (int a = 0; a < 8; a++)
    if (key[a] != INT64_MAX) d = __dadd_rn(d, val[a]);
  return d;
}

// a double from the neighbouring lane of the wave (DPP wave shifts: every
// lane of the wave active; the rim lanes receive 0)
__device__ __forceinline__ double from_lane_below(double v) {   // lane i <- lane i - 1
  return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true),
                          __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ double from_lane_above(double v) {   // lane i <- lane i + 1
  return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true),
                          __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true));
}

// where the amount of local row ly (-1 .. rows, wave-uniform) at column x
// lies: this world's rows, else the wrapped global row as res_at reads it
// (the world's own, or the edge row a strip's neighbour sent)
__device__ __forceinline__ const double* row_ptr(const DevWorld& W, const double* amt, int slot, int x, int ly) {
  const int gy = wrap1(W.row0 + ly, W.world_y), l = gy - W.row0;
  if (l >= 0 && l < W.rows) return amt + (int64_t)l * W.world_x + x;
  const int up = wrap1(W.row0 - 1, W.world_y);
  return (gy == up ? W.rs_recv[0] : W.rs_recv[1]) + (int64_t)slot * W.world_x + x;
}

constexpr int RES_ROWS = 8;    // rows a wave walks down (AVGPU_RES_ROWS: 8 / 16 / 32 = 67 / 76 / 104 us on configs[4])
constexpr int RES_COLS = 62;   // columns a wave writes: lanes 1..62 (lanes 0 and 63 its rim)

// One DoSpatialUpdates step of every resource without CELL entries (FUSED:
// Source + Sink computed here; else res_delta after k_res_spatial_rates +
// k_res_cell_rates, one resource a launch), double-buffered (res_amount ->
// res_amount_alt): the cell's rate, then FlowAll, then StateAll.
//
// A wave owns a 64-column x RES_ROWS-row window (lane l: column
// g * RES_COLS + l - 1 mod X) and walks it down a row at a time.  Each flow
// between two cells is computed ONCE, by the cell whose pointer it is (its
// E, SE, S, SW flows, cResourceCount.cc FlowMatter), and reaches the cell at
// the other end through a DPP lane shift (W: the left lane's E flow; NW /
// NE: the previous row's SE of the left lane and SW of the right lane; N: the
// lane's own previous S), so a cell reads one new amount per row and
// computes four flows instead of eight -- the same values, so the rates agree
// bit for bit with the reference's loop.  Interior cells add the eight terms
// in their fixed order (NW, N, NE, W computing cells, then c's own E, SE, S,
// SW); world-edge cells through res_edge_sum.  blockIdx.y = index into
// ids.r (the resources own disjoint grids).  (Round 5's thread-per-cell
// kernel computed every flow at both ends: 143 us per update on configs[4];
// this one 67 us, profiles/r06t_res_step_ab.txt.)
template <bool FUSED, bool GRAV>
__global__ __launch_bounds__(256) void k_res_step(DevWorld W, ResIds ids, int ngroups, int nwaves, int band) {
  // blocks are dealt to the 8 XCDs round robin: XCD k takes the k-th eighth
  // of the windows, so neighbouring windows share an L2
  unsigned bx = blockIdx.x;
  if ((gridDim.x & 7u) == 0u) bx = (bx & 7u) * (gridDim.x >> 3) + (bx >> 3);
  const int wid = __builtin_amdgcn_readfirstlane((int)(bx * 4 + (threadIdx.x >> 6)));   // wave-uniform
  if (wid >= nwaves) return;                          // whole waves
  const int lane = threadIdx.x & 63;
  const int X = W.world_x, Y = W.world_y;
  const int g = wid % ngroups, ly0 = (wid / ngroups) * band;
  const int ly1 = min(W.rows, ly0 + band);
  const int r = ids.r[blockIdx.y];
  const ResParam P = W.res_param[r];
  const double* amt = W.res_amount + (int64_t)P.slot * W.n;
  double* out = W.res_amount_alt + (int64_t)P.slot * W.n;
  const int xr = g * RES_COLS + lane - 1;
  const int x = ((xr % X) + X) % X;
  const bool writes = lane >= 1 && lane <= RES_COLS && xr < X;
  // no lane that writes sits on a world-edge column: the interior rows take
  // the fixed order without a per-lane test
  const bool wave_xin = __all((x >= 1 && x <= X - 2) || !writes);
  if (!P.flows) {
    if (writes)
      for (int ly = ly0; ly < ly1; ly++) {
        const int64_t c = (int64_t)ly * X + x;
        const double a_c = amt[c];
        const double d = FUSED ? res_source_sink(P, a_c, x, W.row0 + ly, X, Y) : W.res_delta[c];
        out[c] = __dadd_rn(a_c, d);
      }
    return;
  }
  // the flows of the row above the window onto its first row; rows ly + 1
  // and ly + 2 in registers, row ly + 3 loaded each iteration (clamped to
  // the row below the world: never used past the window).  Every load and
  // store of the loop is unconditional -- a lane that writes no cell stores
  // into res_delta's tail -- so the memory-counter waits stay exact (stores
  // count too on this generation) and a load is waited for two iterations
  // after it was issued.
  double* junk = W.res_delta + W.n + lane;
  // four row registers in fixed roles over a 4-row unrolled step, so a load
  // lands in its own register and no copy waits for it
  const double* ghost = row_ptr(W, amt, P.slot, x, W.rows);   // the row below the world
  const double* pa = amt + (int64_t)(ly0 + 3) * X + x;         // row ly + 3 while it is this world's
  double r0 = *row_ptr(W, amt, P.slot, x, ly0);
  double r1 = *row_ptr(W, amt, P.slot, x, ly0 + 1);
  double r2 = *row_ptr(W, amt, P.slot, x, min(ly0 + 2, W.rows));
  double r3;
  double f_n, f_nw, f_ne;
  {
    const double a_up = *row_ptr(W, amt, P.slot, x, ly0 - 1);
    f_n = flow_amt<GRAV>(P, a_up, r0, 0, 1, false);
    f_nw = from_lane_below(flow_amt<GRAV>(P, a_up, from_lane_above(r0), 1, 1, true));
    f_ne = from_lane_above(flow_amt<GRAV>(P, a_up, from_lane_below(r0), -1, 1, true));
  }
  double a_cr = from_lane_above(r0);
  // row ly: a_cur = its amounts, a_nx = row ly + 1's; loads row ly + 3 into ld
  auto row = [&](int ly, double a_cur, double a_nx, double& ld) {
    ld = *(ly + 3 < W.rows ? pa : ghost);
    pa += X;
    const int y = W.row0 + ly;
    const double a_nr = from_lane_above(a_nx), a_nl = from_lane_below(a_nx);
    const double f_e = flow_amt<GRAV>(P, a_cur, a_cr, 1, 0, false);
    const double f_se = flow_amt<GRAV>(P, a_cur, a_nr, 1, 1, true);
    const double f_s = flow_amt<GRAV>(P, a_cur, a_nx, 0, 1, false);
    const double f_sw = flow_amt<GRAV>(P, a_cur, a_nl, -1, 1, true);
    const double f_w = from_lane_below(f_e);
    const int64_t c = (int64_t)ly * X + x;
    double d = FUSED ? res_source_sink(P, a_cur, x, y, X, Y) : W.res_delta[c];
    if ((wave_xin && y >= 1 && y <= Y - 2) || (x >= 1 && x <= X - 2 && y >= 1 && y <= Y - 2)) {
      d = __dadd_rn(d, f_nw);
      d = __dadd_rn(d, f_n);
      d = __dadd_rn(d, f_ne);
      d = __dadd_rn(d, f_w);
      d = __dadd_rn(d, -f_e);
      d = __dadd_rn(d, -f_se);
      d = __dadd_rn(d, -f_s);
      d = __dadd_rn(d, -f_sw);
    } else {
      const double own[4] = {f_e, f_se, f_s, f_sw}, in[4] = {f_w, f_nw, f_n, f_ne};
      d = res_edge_sum(P, X, Y, x, y, own, in, d);
    }
    *(writes ? out + c : junk) = __dadd_rn(a_cur, d);
    f_nw = from_lane_below(f_se);
    f_n = f_s;
    f_ne = from_lane_above(f_sw);
    a_cr = a_nr;
  };
  for (int ly = ly0; ly < ly1; ly += 4) {
    row(ly, r0, r1, r3);
    if (ly + 1 >= ly1) break;
    row(ly + 1, r1, r2, r0);
    if (ly + 2 >= ly1) break;
    row(ly + 2, r2, r3, r1);
    if (ly + 3 >= ly1) break;
    row(ly + 3, r3, r0, r2);
  }
}

// one update of DoNonSpatialUpdates (main/cResourceCount.cc:814-827): 10000
// steps = 100 blocks of PRECALC_DISTANCE steps; update 0 is 9999 steps = 99
// blocks + precalc[99] (oracle/oracle.cc res_begin says why)
__global__ void k_res_global_begin(DevWorld W, int first) {
  const int r = threadIdx.x;
  if (r >= W.n_res || W.res_param[r].slot >= 0) return;
  const ResParam& P = W.res_param[r];
  double R = W.res_global[r];
  for (int k = 0; k < 99; k++) {
    R = __dmul_rn(R, P.decay100);
    R = __dadd_rn(R, P.inflow100);
  }
  R = __dmul_rn(R, first ? P.decay99 : P.decay100);
  R = __dadd_rn(R, first ? P.inflow99 : P.inflow100);
  W.res_global[r] = R;
}

// the update's consumption (fixed point, so the sum is order independent)
__global__ void k_res_global_end(DevWorld W) {
  const int r = threadIdx.x;
  if (r >= W.n_res || W.res_param[r].slot >= 0) return;
  const double used = (double)W.res_cons[r] / RES_FIX;
  W.res_global[r] = fmax(__dsub_rn(W.res_global[r], used), 0.0);
  W.res_cons[r] = 0ull;
}

// strip tiles: first and last row of every spatial resource for the neighbours
__global__ void k_res_pack(DevWorld W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int X = W.world_x;
  if (i >= (int64_t)W.n_spatial * X) return;
  const int slot = (int)(i / X), x = (int)(i % X);
  const double* amt = W.res_amount + (int64_t)slot * W.n;
  W.rs_send[0][i] = amt[x];
  W.rs_send[1][i] = amt[(int64_t)(W.rows - 1) * X + x];
}

// strip tiles: every tile subtracts the consumption summed over all tiles
__global__ void k_res_settle(DevWorld W, const unsigned long long* sum) {
  const int r = threadIdx.x;
  if (r >= W.n_res || W.res_param[r].slot >= 0) return;
  const double used = (double)sum[r] / RES_FIX;
  W.res_global[r] = fmax(__dsub_rn(W.res_global[r], used), 0.0);
  W.res_cons[r] = 0ull;
}

}  // namespace

static inline unsigned rblk(int64_t n) { return (unsigned)((n + 255) / 256); }

// k_res_step's windows: RES_COLS-column groups x RES_ROWS-row bands, four
// waves a block
static void launch_res_step(const DevWorld& W, hipStream_t s, const ResIds& ids, int nres, bool fused) {
  bool grav = false;
  for (int i = 0; i < nres; i++) grav |= W.res_grav_host[ids.r[i]] != 0;
  static const int band = [] {
    const char* e = getenv("AVGPU_RES_ROWS");
    const int v = e ? atoi(e) : RES_ROWS;
    return v >= 1 ? v : RES_ROWS;
  }();
  const int ngroups = (W.world_x + RES_COLS - 1) / RES_COLS;
  const int nwaves = ngroups * ((W.rows + band - 1) / band);
  const dim3 grid((unsigned)((nwaves + 3) / 4), (unsigned)nres);
  auto k = fused ? (grav ? k_res_step<true, true> : k_res_step<true, false>)
                 : (grav ? k_res_step<false, true> : k_res_step<false, false>);
  hipLaunchKernelGGL(k, grid, dim3(256), 0, s, W, ids, ngroups, nwaves, band);
}

void launch_resources_begin(const DevWorld& W, hipStream_t s) {
  if (W.n_res == 0) return;
  // spatial resources: one step of the reference's DoSpatialUpdates (each
  // resource owns its own grid, so the order across resources is free); none
  // in update 0.  Every resource without CELL entries steps in ONE launch
  // (blockIdx.y = resource); one with them goes through the rates kernels
  // (res_delta is shared scratch, so those run one resource at a time).  The
  // caller swaps res_amount / res_amount_alt afterwards (res_stepped).
  if (!W.res_first) {
    ResIds fused{};
    int nf = 0;
    for (int r = 0; r < W.n_res; r++) {
      if (!W.res_spatial_host[r]) continue;
      if (W.res_cells_host[r]) {
        ResIds one{};
        one.r[0] = r;
        hipLaunchKernelGGL(k_res_spatial_rates, dim3(rblk(W.n)), dim3(256), 0, s, W, r);
        hipLaunchKernelGGL(k_res_cell_rates, dim3(1), dim3(64), 0, s, W, r);
        launch_res_step(W, s, one, 1, false);
      } else {
        fused.r[nf++] = r;
      }
    }
    if (nf) launch_res_step(W, s, fused, nf, true);
  }
  hipLaunchKernelGGL(k_res_global_begin, dim3(1), dim3(64), 0, s, W, (int)W.res_first);
}

bool res_stepped(const DevWorld& W) { return W.n_spatial > 0 && !W.res_first; }

void launch_resources_end(const DevWorld& W, hipStream_t s) {
  if (W.n_res == 0) return;
  hipLaunchKernelGGL(k_res_global_end, dim3(1), dim3(64), 0, s, W);
}

void launch_resources_pack(const DevWorld& W, hipStream_t s) {
  if (W.n_spatial == 0 || !W.rs_send[0]) return;
  hipLaunchKernelGGL(k_res_pack, dim3(rblk((int64_t)W.n_spatial * W.world_x)), dim3(256), 0, s, W);
}

void launch_resources_settle(const DevWorld& W, hipStream_t s, const unsigned long long* sum) {
  hipLaunchKernelGGL(k_res_settle, dim3(1), dim3(64), 0, s, W, sum);
}
