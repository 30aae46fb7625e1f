// PFSP search node, shared bit-for-bit by the host pools and the device pools.
//
// Reference node (pfsp/lib/PFSP_node.h:15-20) is {int16 depth, int16 limit1,
// int16 prmu[MAX_JOBS=20]} = 44 B with a compile-time MAX_JOBS. Here:
//   * forward branching only, so limit1 == depth-1 is implicit (not stored);
//   * job ids are uint8 up to 255 jobs, uint16 for the 500-job class;
//   * the node is 16-byte aligned: 32 B for 20 jobs (one pair of dwordx4 per lane
//     on the GPU), 64 B for 50, 112 B for 100, 208 B for 200, 1008 B for 500;
//   * the job-count bucket NJ is a template parameter chosen at run time
//     (no MAX_JOBS edit + recompile as in ref pfsp/README.md:52).
// prmu[0..depth) is the scheduled prefix in order; prmu[depth..jobs) holds the
// unscheduled jobs in arbitrary order (only the set matters to every bound).
#pragma once

#include <cstddef>
#include <cstdint>
#include <type_traits>
#include <utility>

#ifndef TTS_HD
#if defined(__HIPCC__)
#define TTS_HD __host__ __device__
#else
#define TTS_HD
#endif
#endif

namespace tts {

template <int NJ>
struct alignas(16) PfspNode {
  static constexpr int kMaxJobs = NJ;
  using id_t = std::conditional_t<(NJ > 255), uint16_t, uint8_t>;
  id_t depth;
  id_t prmu[NJ];
};

static_assert(sizeof(PfspNode<20>) == 32, "20-job node must be 32 B");
static_assert(sizeof(PfspNode<50>) == 64, "50-job node must be 64 B");

template <int NJ>
TTS_HD inline void pfsp_init_root(PfspNode<NJ>& root, int jobs) {
  root.depth = 0;
  for (int i = 0; i < NJ; ++i) root.prmu[i] = static_cast<typename PfspNode<NJ>::id_t>(i < jobs ? i : 0);
}

// Child obtained by moving prmu[k] (k >= depth) to position depth.
template <int NJ>
TTS_HD inline PfspNode<NJ> pfsp_child(const PfspNode<NJ>& parent, int k) {
  PfspNode<NJ> c = parent;
  const int d = parent.depth;
  const auto t = c.prmu[d];
  c.prmu[d] = c.prmu[k];
  c.prmu[k] = t;
  c.depth = static_cast<typename PfspNode<NJ>::id_t>(d + 1);
  return c;
}

// Front-carrying node of the LB1 / LB1_d search on small instances (<= 32 jobs,
// machine bucket MB in {5, 10, 20}). LB1 only depends on the scheduled prefix through
// its per-machine completion times (front) and on the set of unscheduled jobs, so the
// node stores exactly that: a child costs O(M) from its parent instead of replaying
// the O(depth * M) prefix chain (ref schedule_front, c_bound_simple.c:52-69, which
// the reference repeats per child for LB1 and per parent for LB1_d). 32 B for up to
// 10 machines, 48 B for 20 (the permutation node is 32 B at 20 jobs).
//   depth       jobs scheduled
//   rest        bit j set: job j is not scheduled yet
//   front[m]    completion time of the prefix on machine m; at the root the minimum
//               heads (ref schedule_front with limit1 == -1)
// NJ (job bucket of the front layout): 20 keeps the unscheduled set in 32 bits, 50 in
// 64 (the set then starts at byte 8 and the fronts at byte 16).
template <int MB, int NJ = 20>
struct alignas(16) PfspFrontNode {
  static constexpr int kMachines = MB;
  static constexpr int kJobs = NJ;
  using Mask = std::conditional_t<(NJ <= 32), uint32_t, uint64_t>;
  uint8_t depth;
  uint8_t pad[sizeof(Mask) - 1];
  Mask rest;
  uint16_t front[MB];
};
static_assert(sizeof(PfspFrontNode<5>) == 32 && sizeof(PfspFrontNode<10>) == 32 && sizeof(PfspFrontNode<20>) == 48,
              "front node sizes");
static_assert(sizeof(PfspFrontNode<5, 50>) == 32 && sizeof(PfspFrontNode<10, 50>) == 48 &&
                  sizeof(PfspFrontNode<20, 50>) == 64,
              "50-job front node sizes");

// lowest set bit of a job set (32 or 64 bits)
TTS_HD inline int mask_ctz(uint32_t x) { return __builtin_ctz(x); }
TTS_HD inline int mask_ctz(uint64_t x) { return __builtin_ctzll(x); }

// Job-count buckets a run-time instance is dispatched to.
inline int pfsp_bucket(int jobs) {
  if (jobs <= 20) return 20;
  if (jobs <= 50) return 50;
  if (jobs <= 100) return 100;
  if (jobs <= 200) return 200;
  return 500;
}

// Calls f(std::integral_constant<int, NJ>{}) for the bucket of `jobs`.
template <class F>
decltype(auto) with_pfsp_bucket(int jobs, F&& f) {
  switch (pfsp_bucket(jobs)) {
    case 20: return f(std::integral_constant<int, 20>{});
    case 50: return f(std::integral_constant<int, 50>{});
    case 100: return f(std::integral_constant<int, 100>{});
    case 200: return f(std::integral_constant<int, 200>{});
    default: return f(std::integral_constant<int, 500>{});
  }
}

// N-Queens node (ref nqueens/lib/NQueens_node.h:13-17 stores the full board,
// 21 B). The tree only depends on which rows are used and which diagonals are
// attacked, so the node is three 32-bit masks + depth = 16 B.
struct alignas(16) QueensNode {
  uint32_t cols;   // rows already holding a queen (bit r)
  uint32_t diag;   // attacked "r - c" diagonal, shifted so the next column reads bit r
  uint32_t anti;   // attacked "r + c" diagonal, same convention
  uint32_t depth;  // number of queens placed (== column to fill next)
};
static_assert(sizeof(QueensNode) == 16, "queens node must be 16 B");

}  // namespace tts
