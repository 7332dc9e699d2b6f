// resources.hip -- environment resources around the interpreter (config 5):
//   k_res_step<true>     one cSpatialResCount step of every resource without
//                        CELL entries (one launch), fused: Source + Sink
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
  if (ax == 0.0) return __dmul_rn(x, r);                    // +-0 (equal amounts: a common flow)
  if (!(ax >= 0x1p-900 && ax <= 0x1p+900)) return __ddiv_rn(x, c);
  const double y = __dmul_rn(x, r);
  const double e = __fma_rn(-c, y, x);
  return __fma_rn(e, r, y);
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

__device__ __forceinline__ double flow_amt(const ResParam& P, double a1, double a2, int xdist, int ydist,
                                           bool diagonal) {
  const double diff = __dsub_rn(a1, a2);
  double xg = 0.0, xd = 0.0, yg = 0.0, yd = 0.0;
  if (xdist != 0) {
    xg = gravity_term(a1, a2, xdist, P.xgravity);
    xd = __dmul_rn(__dmul_rn(P.xdiffuse, diff), 0.0625);
  }
  if (ydist != 0) {
    yg = gravity_term(a1, a2, ydist, P.ygravity);
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

// One DoSpatialUpdates step of resource r for cell c, double-buffered
// (res_amount -> res_amount_alt): the cell's rate is Source + Sink (FUSED; or
// res_delta after k_res_spatial_rates + k_res_cell_rates when r has CELL
// entries), then FlowAll -- -flow for its own pointers 3..6 and +flow from
// every cell whose pointer 3..6 is c, added in increasing (computing cell, k)
// order of global cell ids like the reference's loop over i (an 8-entry
// sorting network keeps the order in registers) -- then StateAll.
// the spatial resources one launch steps: blockIdx.y = index into r[]
// (the resources own disjoint grids, so their steps are independent)
struct ResIds {
  int r[AVGPU_MAX_RESOURCES];
};

// Source + Sink of cell (x, y) (main/cSpatialResCount.cc:341-394): the rate
// the flows are added to
__device__ __forceinline__ double res_source_sink(const ResParam& P, double a_c, int x, int y, int X, int Y) {
  double d = 0.0;
  const int nin = P.in_all ? 1 : cover(y, P.in_y1, P.in_y2, Y) * cover(x, P.in_x1, P.in_x2, X);
  for (int k = 0; k < nin; k++) d = __dadd_rn(d, P.in_share);
  if (P.has_sink) {
    const int nout = P.out_all ? 1 : cover(y, P.out_y1, P.out_y2, Y) * cover(x, P.out_x1, P.out_x2, X);
    const double dec = fmax(__dmul_rn(a_c, P.sink_frac), 0.0);
    for (int k = 0; k < nout; k++) d = __dadd_rn(d, -dec);
  }
  return d;
}

// FlowAll's terms of cell c = (x, y) onto its rate d, read from the amounts in
// memory: an interior cell's eight flows in their fixed order (NW, N, NE, W
// computing cells, then c's own E, SE, S, SW), a world-edge cell's through
// an 8-entry sorting network in increasing (computing cell, k) order of
// global cell ids like the reference's loop over i
__device__ __forceinline__ double res_flows(const DevWorld& W, const ResParam& P, const double* amt, int c, int x,
                                            int y, double a_c, double d) {
  const int X = W.world_x, Y = W.world_y;
  if (x >= 1 && x <= X - 2 && y >= 1 && y <= Y - 2) {
    const double a_nw = res_at(W, amt, P.slot, x - 1, y - 1), a_n = res_at(W, amt, P.slot, x, y - 1);
    const double a_ne = res_at(W, amt, P.slot, x + 1, y - 1), a_w = amt[c - 1];
    d = __dadd_rn(d, flow_amt(P, a_nw, a_c, 1, 1, true));
    d = __dadd_rn(d, flow_amt(P, a_n, a_c, 0, 1, false));
    d = __dadd_rn(d, flow_amt(P, a_ne, a_c, -1, 1, true));
    d = __dadd_rn(d, flow_amt(P, a_w, a_c, 1, 0, false));
    d = __dadd_rn(d, -flow_amt(P, a_c, amt[c + 1], 1, 0, false));
    d = __dadd_rn(d, -flow_amt(P, a_c, res_at(W, amt, P.slot, x + 1, y + 1), 1, 1, true));
    d = __dadd_rn(d, -flow_amt(P, a_c, res_at(W, amt, P.slot, x, y + 1), 0, 1, false));
    d = __dadd_rn(d, -flow_amt(P, a_c, res_at(W, amt, P.slot, x - 1, y + 1), -1, 1, true));
    return d;
  }
  const int64_t gc = (int64_t)y * X + x;
  int64_t key[8];
  double val[8];
#pragma unroll
  for (int k = 3; k <= 6; k++) {                     // own pointers: slots 0..3
    const int dx = (k == 3 || k == 4) ? 1 : (k == 5 ? 0 : -1), dy = (k == 3) ? 0 : 1;
    int nx, ny;
    const bool ok = res_ptr(P.geometry, X, Y, x, y, k, nx, ny);
    key[k - 3] = ok ? gc * 8 + k : INT64_MAX;
    val[k - 3] = ok ? -flow_amt(P, a_c, res_at(W, amt, P.slot, nx, ny), dx, dy, k == 4 || k == 6) : 0.0;
  }
#pragma unroll
  for (int k = 3; k <= 6; k++) {                     // cells whose pointer k is c: slots 4..7
    const int dx = (k == 3 || k == 4) ? 1 : (k == 5 ? 0 : -1), dy = (k == 3) ? 0 : 1;
    const int jx = wrap1(x - dx, X), jy = wrap1(y - dy, Y);
    int nx, ny;
    const bool ok = res_ptr(P.geometry, X, Y, jx, jy, k, nx, ny) && nx == x && ny == y;
    key[k + 1] = ok ? ((int64_t)jy * X + jx) * 8 + k : INT64_MAX;
    val[k + 1] = ok ? flow_amt(P, res_at(W, amt, P.slot, jx, jy), a_c, dx, dy, k == 4 || k == 6) : 0.0;
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

// One DoSpatialUpdates step of resource r for cell c, double-buffered
// (res_amount -> res_amount_alt): the cell's rate is Source + Sink (FUSED; or
// res_delta after k_res_spatial_rates + k_res_cell_rates when r has CELL
// entries), then FlowAll (res_flows), then StateAll.  Every resource without
// CELL entries steps in one launch (blockIdx.y).  (A tiled variant that staged
// a 64 x 8 tile and its rim in LDS and computed each flow once instead of at
// both ends ran at 306 against 138 us per update for the 9 resources of
// configs[4]: profiles/r04o_res_step_tiled.txt.)
template <bool FUSED>
__global__ void k_res_step(DevWorld W, ResIds ids) {
  // blocks are dealt to the 8 XCDs round robin: XCD k takes the k-th eighth
  // of the rows, so the rows above and below a block are in its own L2
  unsigned bx = blockIdx.x;
  if ((gridDim.x & 7u) == 0u) bx = (bx & 7u) * (gridDim.x >> 3) + (bx >> 3);
  const int c = (int)(bx * blockDim.x + threadIdx.x);   // n < 2^31 (avgpu_load_resources)
  if (c >= W.n) return;
  const int r = ids.r[blockIdx.y];
  const ResParam P = W.res_param[r];
  const int X = W.world_x;
  const double* amt = W.res_amount + (int64_t)P.slot * W.n;
  const int ly = (int)((unsigned)c / (unsigned)X), x = c - ly * X, y = W.row0 + ly;
  const double a_c = amt[c];
  double d = FUSED ? res_source_sink(P, a_c, x, y, X, W.world_y) : W.res_delta[c];
  if (P.flows) d = res_flows(W, P, amt, c, x, y, a_c, d);
  W.res_amount_alt[(int64_t)P.slot * W.n + c] = __dadd_rn(a_c, d);
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
        hipLaunchKernelGGL(k_res_step<false>, dim3(rblk(W.n)), dim3(256), 0, s, W, one);
      } else {
        fused.r[nf++] = r;
      }
    }
    if (nf) hipLaunchKernelGGL(k_res_step<true>, dim3(rblk(W.n), nf), dim3(256), 0, s, W, fused);
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
