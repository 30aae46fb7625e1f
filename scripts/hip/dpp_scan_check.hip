// Checks the DPP inclusive wave scan used by the N-Queens finishing pass
// (queens_kernels.hpp) against a host prefix sum, for a few input patterns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void scan_kernel(const int* in, int* out, int* tot) {
  const int lane = threadIdx.x;
  const int c = in[blockIdx.x * 64 + lane];
  int x = c;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  out[blockIdx.x * 64 + lane] = x - c;
  if (lane == 0) tot[blockIdx.x] = __builtin_amdgcn_readlane(x, 63);
}

int main() {
  const int B = 8;
  std::vector<int> in(B * 64), out(B * 64), tot(B);
  for (int b = 0; b < B; ++b)
    for (int l = 0; l < 64; ++l) in[b * 64 + l] = b == 0 ? 1 : b == 1 ? l : (l * 7 + b * 3) % (b + 9);
  int *din, *dout, *dtot;
  if (hipMalloc(&din, in.size() * 4) || hipMalloc(&dout, out.size() * 4) || hipMalloc(&dtot, B * 4)) return 2;
  if (hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice)) return 2;
  hipLaunchKernelGGL(scan_kernel, dim3(B), dim3(64), 0, 0, din, dout, dtot);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  if (hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost)) return 2;
  if (hipMemcpy(tot.data(), dtot, B * 4, hipMemcpyDeviceToHost)) return 2;
  int bad = 0;
  for (int b = 0; b < B; ++b) {
    int acc = 0;
    for (int l = 0; l < 64; ++l) {
      if (out[b * 64 + l] != acc) ++bad;
      acc += in[b * 64 + l];
    }
    if (tot[b] != acc) ++bad;
  }
  std::printf("dpp scan check: %s (%d mismatches)\n", bad ? "FAILED" : "ok", bad);
  return bad ? 1 : 0;
}
