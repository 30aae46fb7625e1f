// Microbenchmark: cost of a kernel boundary (graph of empty kernels) vs a grid-wide
// barrier inside one cooperative kernel (flat counter vs per-XCD counters).
// Every spin has a bounded poll count: a broken barrier sets an error flag and
// the grid drains instead of hanging.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void empty_kernel(const int* ctl) {
  if (ctl[0] == 12345 && threadIdx.x == 0) printf("never\n");
}

constexpr unsigned kSpin = 1u << 22;

__device__ inline unsigned ld_acq(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT); }

// counters: [0] global arrivals, [32*g] group arrivals (g = 1..8), [32*9] error flag
__global__ void barrier_kernel(unsigned* c, int iters, int hier) {
  unsigned epoch = 0;
  const unsigned nb = gridDim.x;
  const int g = blockIdx.x & 7;
  const unsigned gsize = nb / 8 + ((blockIdx.x & 7) < (nb & 7) ? 1 : 0);
  for (int it = 0; it < iters; ++it) {
    __syncthreads();
    if (threadIdx.x == 0) {
      ++epoch;
      __atomic_thread_fence(__ATOMIC_RELEASE);
      if (!hier) {
        __hip_atomic_fetch_add(&c[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const unsigned a = __hip_atomic_fetch_add(&c[32 * (g + 1)], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
        if (a == epoch * gsize) __hip_atomic_fetch_add(&c[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      const unsigned want = hier ? epoch * 8 : epoch * nb;
      unsigned spins = 0;
      while (ld_acq(&c[0]) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpin) { c[32 * 9] = 1; break; }
      }
    }
    __syncthreads();
    if (c[32 * 9]) return;
  }
}

int main() {
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int* ctl; unsigned* cnt;
  CK(hipMalloc(&ctl, 64)); CK(hipMemset(ctl, 0, 64));
  CK(hipMalloc(&cnt, 4096)); 
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int per : {1, 2, 4}) {
    const int grid = cus * per;
    // graph of K empty kernels
    const int K = 96;
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, s, ctl);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    const int R = 10;
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / (R * K);
    printf("grid %5d: graph of empty kernels: %.2f us per kernel\n", grid, us);
    // cooperative barrier kernel
    for (int hier = 0; hier < 2; ++hier) {
      int maxb = 0;
      CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&maxb, barrier_kernel, 256, 0));
      if (maxb * cus < grid) { printf("grid %d not co-resident (max %d/CU)\n", grid, maxb); continue; }
      double best = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemsetAsync(cnt, 0, 4096, s));
        int iters = 200, h = hier;
        void* args[] = {&cnt, &iters, &h};
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipLaunchCooperativeKernel((void*)barrier_kernel, dim3(grid), dim3(256), args, 0, s));
        CK(hipStreamSynchronize(s));
        double bus = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count() / iters;
        unsigned err = 0;
        CK(hipMemcpy(&err, cnt + 32 * 9, 4, hipMemcpyDeviceToHost));
        if (err) { printf("barrier timeout (hier=%d)\n", hier); break; }
        best = std::min(best, bus);
      }
      printf("grid %5d: grid barrier (%s): %.2f us per barrier\n", grid, hier ? "per-XCD" : "flat", best);
    }
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }
  return 0;
}
