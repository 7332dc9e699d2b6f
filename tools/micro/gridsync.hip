// Microbenchmark (diagnostic): cost of a grid-wide barrier in a cooperative
// launch versus a kernel boundary, with a little global traffic per phase.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
#include <chrono>
namespace cg = cooperative_groups;

__global__ void k_phases(int* buf, int n, int phases) {
  cg::grid_group g = cg::this_grid();
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  for (int p = 0; p < phases; p++) {
    for (int i = tid; i < n; i += gridDim.x * blockDim.x) buf[i] += p;
    g.sync();
  }
}
__global__ void k_one(int* buf, int n, int p) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = tid; i < n; i += gridDim.x * blockDim.x) buf[i] += p;
}

int main() {
  const int n = 1 << 20, phases = 200;
  int* buf;
  hipMalloc(&buf, n * sizeof(int));
  hipMemset(buf, 0, n * sizeof(int));
  hipStream_t s;
  hipStreamCreate(&s);
  int dev = 0, ncu = 0, per = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_phases, 256, 0);
  printf("CUs %d, co-resident blocks/CU %d\n", ncu, per);
  for (int blocks : {256, 512, 1024, 2048}) {
    if (blocks > ncu * per) continue;
    int nn = n, ph = phases;
    void* args[] = {&buf, &nn, &ph};
    hipLaunchCooperativeKernel((void*)k_phases, dim3(blocks), dim3(256), args, 0, s);
    hipStreamSynchronize(s);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a, s);
    hipLaunchCooperativeKernel((void*)k_phases, dim3(blocks), dim3(256), args, 0, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    printf("cooperative %4d blocks: %.2f us per phase\n", blocks, 1000.f * ms / phases);
    hipEventRecord(a, s);
    for (int p = 0; p < phases; p++) hipLaunchKernelGGL(k_one, dim3(blocks), dim3(256), 0, s, buf, n, p);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("kernels     %4d blocks: %.2f us per launch\n", blocks, 1000.f * ms / phases);
  }
  hipError_t e = hipGetLastError();
  printf("status %s\n", hipGetErrorString(e));
  return 0;
}
