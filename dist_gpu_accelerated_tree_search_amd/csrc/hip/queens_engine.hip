// N-Queens device engine (traits + factory) and reference-style label evaluation.
#include <algorithm>
#include <cstdlib>

#include "queens_engine.hpp"
#include "queens_kernels.hpp"

namespace tts {

struct QueensTraits {
  using Node = QueensNode;
  using Args = dev::QueensArgs;
  using S = dev::QueensSmem;
  static constexpr int kParentsPerChunk = S::BP;
  static constexpr int kChildrenPerChunk = S::MAXCH;
  static constexpr int kMaxChildren = S::MAXCH / S::BP;
  static constexpr int kLocalSteps = 1;
  static constexpr int kLocalMin = 0;
  static constexpr int kMaxChunks = S::MAXCHUNKS;
  static void launch(const Args& a, int t, int grid, hipStream_t s) {
    hipLaunchKernelGGL(dev::queens_expand_kernel, dim3(grid), dim3(dev::kBlock), 0, s, a, t);
  }
  static void flatten(const dev::PoolArgs<Node>& pa, int b, int grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::pool_flatten_kernel<Node, S::MAXCH, S::MAXCHUNKS>), dim3(grid), dim3(dev::kBlock), 0, s,
                       pa, b);
  }
  static void finalize(const dev::PoolArgs<Node>& pa, int b, int slot, hipStream_t s) {
    hipLaunchKernelGGL((dev::pool_finalize_kernel<Node, S::MAXCHUNKS>), dim3(1), dim3(dev::kBlock), 0, s, pa, b, slot);
  }
  static int blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::queens_expand_kernel, dev::kBlock, 0) != hipSuccess)
      return 1;
    // 106 SGPRs allow 6 resident per CU; the grid takes 5 (N=17 47.1 -> 46.0 ms, 4 and 8
    // slower; profiles/r5/grid_ab.txt)
    return dev::resident_blocks(n, 5);
  }
};

static dev::QueensArgs queens_args(int N, int G) {
  if (N < 1 || N > 32) throw std::invalid_argument("N-Queens supports 1 <= N <= 32");
  if (G < 1) throw std::invalid_argument("g must be >= 1");
  dev::QueensArgs a{};
  a.N = N;
  a.G = G;
  a.full = N == 32 ? 0xffffffffu : ((1u << N) - 1u);
  // subtree finishing: parents with at most finish_k columns left (TTS_QUEENS_FINISH
  // overrides; 0 = level-by-level to the bottom). The wave-cooperative finishing is
  // fastest from 9 columns left (N=17: 6 / 7 / 8 / 9 / 10 / 11 / 12 columns 48 / 29 / 24 /
  // 21 / 25 / 37 / 138 ms; deeper subtrees overflow the LDS stacks into the register walk,
  // profiles/r6/queens/finish_depth_ab.txt)
  a.finish_k = 9;
  if (const char* f = std::getenv("TTS_QUEENS_FINISH")) a.finish_k = std::atoi(f);
  a.finish_k = std::max(0, std::min(a.finish_k, dev::kQueensFinishMax));
  return a;
}

std::unique_ptr<IEngine> make_queens_engine(int N, int G, const EngineConfig& cfg) {
  TTS_HIP_CHECK(hipSetDevice(cfg.device));
  return std::make_unique<DeviceEngine<QueensTraits>>(cfg, queens_args(N, G));
}

std::vector<uint8_t> queens_gpu_labels(int N, int G, const QueensNode* parents, size_t n, int device) {
  TTS_HIP_CHECK(hipSetDevice(device));
  dev::QueensArgs a = queens_args(N, G);
  std::vector<uint8_t> out(n * static_cast<size_t>(N), 0);
  if (n == 0) return out;
  QueensNode* dp = nullptr;
  uint8_t* dl = nullptr;
  TTS_HIP_CHECK(hipMalloc(&dp, n * sizeof(QueensNode)));
  TTS_HIP_CHECK(hipMalloc(&dl, out.size()));
  TTS_HIP_CHECK(hipMemcpy(dp, parents, n * sizeof(QueensNode), hipMemcpyHostToDevice));
  a.parents_in = dp;
  a.labels_out = dl;
  a.nparents = static_cast<int>(n);
  const int blocks = static_cast<int>((n + dev::kBlock - 1) / dev::kBlock);
  hipLaunchKernelGGL(dev::queens_labels_kernel, dim3(blocks), dim3(dev::kBlock), 0, 0, a);
  TTS_HIP_CHECK(hipGetLastError());
  TTS_HIP_CHECK(hipDeviceSynchronize());
  TTS_HIP_CHECK(hipMemcpy(out.data(), dl, out.size(), hipMemcpyDeviceToHost));
  (void)hipFree(dp);
  (void)hipFree(dl);
  return out;
}

}  // namespace tts
