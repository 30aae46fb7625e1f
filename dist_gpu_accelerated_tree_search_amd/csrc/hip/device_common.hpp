// Shared device helpers for the gfx950 (CDNA4) kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#define TTS_HIP_CHECK(expr)                                                                          \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess)                                                                            \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + __FILE__ + \
                               ":" + std::to_string(__LINE__) + " in " #expr);                      \
  } while (0)

namespace tts {
namespace dev {

using u64 = unsigned long long;

constexpr int kWave = 64;      // CDNA wavefront width
constexpr int kBlock = 256;    // 4 waves per workgroup for every search kernel

// 128-B padded scalars: a plain write-back of one never merges with another's
// line (the incumbent is the only word updated by device atomics).
struct alignas(128) CtlU64 {
  u64 v;
  u64 pad[15];
};
struct alignas(128) CtlI32 {
  int v;
  int pad[31];
};

// Resident workgroups per CU of a kBlock kernel: the occupancy API's count capped by
// what the SGPR file holds. A SIMD has 800 SGPRs and a wave takes ceil(sgpr / 16) * 16
// + 16 of them; the search kernels allocate 106 (the compiler's default without a
// waves-per-EU target), i.e. 6 waves per SIMD = 6 workgroups per CU, while the API
// reports one more (measured on MI355X: with 7 per CU in the grid, 256 workgroups
// started one workgroup lifetime late). Grids larger than the resident count only add
// that serialisation.
constexpr int kSgprResidentCap = 6;
inline int resident_blocks(int api_blocks_per_cu, int cap = kSgprResidentCap) {
  return api_blocks_per_cu < cap ? api_blocks_per_cu : cap;
}

// Workgroup exclusive scan of one int per thread (kBlock threads).
// `scratch` needs kBlock/kWave ints of LDS. Returns the exclusive prefix; *total
// receives the block sum. Contains __syncthreads().
__device__ inline int block_exclusive_scan(int v, int* scratch, int* total) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  int x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) scratch[wid] = x;
  __syncthreads();
  int wave_off = 0, sum = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const int s = scratch[w];
    wave_off += (w < wid) ? s : 0;
    sum += s;
  }
  *total = sum;
  __syncthreads();
  return wave_off + x - v;
}

__device__ inline u64 lanemask_lt() {
  const int lane = threadIdx.x & (kWave - 1);
  return lane == 0 ? 0ull : (~0ull >> (kWave - lane));
}

// Packed u16 pairs (v_pk_add_u16 / v_pk_max_u16 on ext_vector_type(2)): two
// independent 16-bit chains per VALU op where every value provably fits 16 bits.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ inline u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ inline uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

}  // namespace dev
}  // namespace tts
