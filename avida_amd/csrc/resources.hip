// resources.hip -- environment resources around the interpreter (config 5):
//   k_res_spatial_rates  cSpatialResCount::Source + Sink      (main/cSpatialResCount.cc:341-394)
//   k_res_cell_rates     CellInflow + CellOutflow              (:356-404), list order, one thread
//   k_res_flow           FlowAll / FlowMatter                  (:323-338, main/cResourceCount.cc:40-110)
//   k_res_state          StateAll                              (:307-314)
//   k_res_global_begin   DoNonSpatialUpdates over one update   (main/cResourceCount.cc:757-827)
//   k_res_global_end     the update's consumption of global resources
// Every per-cell sum is formed in the reference's order (the sequential loops
// of cSpatialResCount add into a cell's delta in increasing index of the cell
// doing the computing), so the device agrees bit for bit with the oracle's
// literal restatement of those loops (oracle/oracle.cc res_spatial_step).
#include "device.h"

#pragma clang fp contract(off)

namespace {

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

// FlowMatter (main/cResourceCount.cc:40-110) from elem1 = a1 to elem2 = a2
__device__ __forceinline__ double flow_amt(const ResParam& P, double a1, double a2, int xdist, int ydist,
                                           double dist) {
  const double diff = __dsub_rn(a1, a2);
  double xg = 0.0, xd = 0.0, yg = 0.0, yd = 0.0;
  if (xdist != 0) {
    if ((xdist > 0 && P.xgravity > 0.0) || (xdist < 0 && P.xgravity < 0.0))
      xg = __ddiv_rn(__dmul_rn(a1, fabs(P.xgravity)), 3.0);
    else
      xg = __ddiv_rn(__dmul_rn(-a2, fabs(P.xgravity)), 3.0);
    xd = __ddiv_rn(__dmul_rn(P.xdiffuse, diff), 16.0);
  }
  if (ydist != 0) {
    if ((ydist > 0 && P.ygravity > 0.0) || (ydist < 0 && P.ygravity < 0.0))
      yg = __ddiv_rn(__dmul_rn(a1, fabs(P.ygravity)), 3.0);
    else
      yg = __ddiv_rn(__dmul_rn(-a2, fabs(P.ygravity)), 3.0);
    yd = __ddiv_rn(__dmul_rn(P.ydiffuse, diff), 16.0);
  }
  const double num = __dadd_rn(__dadd_rn(__dadd_rn(xd, yd), xg), yg);
  const double den = __dadd_rn(fabs((double)xdist), fabs((double)ydist));
  return __ddiv_rn(__ddiv_rn(num, den), dist);
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
  nx = amod(x + dx, X);
  ny = amod(y + dy, Y);
  return true;
}

// amount of global cell (gx, gy): this world's rows, else the edge row the
// tile above (gy = row0 - 1) or below sent
__device__ __forceinline__ double res_at(const DevWorld& W, const double* amt, int slot, int gx, int gy) {
  const int ly = gy - W.row0;
  if (ly >= 0 && ly < W.rows) return amt[(int64_t)ly * W.world_x + gx];
  const int up = amod(W.row0 - 1, W.world_y);
  return (gy == up ? W.rs_recv[0] : W.rs_recv[1])[(int64_t)slot * W.world_x + gx];
}

// FlowAll: cell c's delta gets -flow for its own pointers 3..6 and +flow from
// every cell whose pointer 3..6 is c, added in increasing (computing cell, k)
// order (global cell ids) like the reference's loop over i
__global__ void k_res_flow(DevWorld W, int r) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W.n) return;
  const ResParam P = W.res_param[r];
  const int X = W.world_x, Y = W.world_y;
  const double* amt = W.res_amount + (int64_t)P.slot * W.n;
  const int x = (int)(c % X), y = W.row0 + (int)(c / X);
  const int64_t gc = (int64_t)y * X + x;
  const double a_c = amt[c];
  const double SQRT2 = 1.4142135623730951;   // sqrt(2.0)
  int64_t key[8];
  double val[8];
  int m = 0;
  for (int k = 3; k <= 6; k++) {                       // own pointers
    int nx, ny;
    if (!res_ptr(P.geometry, X, Y, x, y, k, nx, ny)) continue;
    const int xd = (k == 3 || k == 4) ? 1 : (k == 5 ? 0 : -1), yd = (k == 3) ? 0 : 1;
    key[m] = gc * 8 + k;
    val[m] = -flow_amt(P, a_c, res_at(W, amt, P.slot, nx, ny), xd, yd, (k == 4 || k == 6) ? SQRT2 : 1.0);
    m++;
  }
  for (int k = 3; k <= 6; k++) {                       // cells whose pointer k is c
    const int dx = (k == 3 || k == 4) ? 1 : (k == 5 ? 0 : -1), dy = (k == 3) ? 0 : 1;
    const int jx = amod(x - dx, X), jy = amod(y - dy, Y);
    int nx, ny;
    if (!res_ptr(P.geometry, X, Y, jx, jy, k, nx, ny) || nx != x || ny != y) continue;
    key[m] = ((int64_t)jy * X + jx) * 8 + k;
    val[m] = flow_amt(P, res_at(W, amt, P.slot, jx, jy), a_c, dx, dy, (k == 4 || k == 6) ? SQRT2 : 1.0);
    m++;
  }
  for (int a = 1; a < m; a++)                          // insertion sort by (cell, k)
    for (int b = a; b > 0 && key[b - 1] > key[b]; b--) {
      const int64_t tk = key[b]; key[b] = key[b - 1]; key[b - 1] = tk;
      const double tv = val[b]; val[b] = val[b - 1]; val[b - 1] = tv;
    }
  double d = W.res_delta[c];
  for (int a = 0; a < m; a++) d = __dadd_rn(d, val[a]);
  W.res_delta[c] = d;
}

__global__ void k_res_state(DevWorld W, int r) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= W.n) return;
  double* a = W.res_amount + (int64_t)W.res_param[r].slot * W.n + c;
  *a = __dadd_rn(*a, W.res_delta[c]);
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
  // spatial resources: one step of the reference's DoSpatialUpdates, in
  // resource order (each resource owns its own grid); none in update 0
  for (int r = 0; r < W.n_res && !W.res_first; r++) {
    if (!W.res_spatial_host[r]) continue;
    hipLaunchKernelGGL(k_res_spatial_rates, dim3(rblk(W.n)), dim3(256), 0, s, W, r);
    if (W.n_cellres) hipLaunchKernelGGL(k_res_cell_rates, dim3(1), dim3(64), 0, s, W, r);
    if (W.res_flows_host[r]) hipLaunchKernelGGL(k_res_flow, dim3(rblk(W.n)), dim3(256), 0, s, W, r);
    hipLaunchKernelGGL(k_res_state, dim3(rblk(W.n)), dim3(256), 0, s, W, r);
  }
  hipLaunchKernelGGL(k_res_global_begin, dim3(1), dim3(64), 0, s, W, (int)W.res_first);
}

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
