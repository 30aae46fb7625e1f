// LB1 / LB1_d search kernels on front-carrying nodes (core/pfsp_node.hpp
// PfspFrontNode, host twin core/pfsp_front.hpp) for gfx950 (CDNA4).
//
// The reference bounds a child from its permutation: LB1 recomputes the prefix's
// completion times per child, LB1_d once per parent (ref bounds_gpu.cu:12-248,
// c_bound_simple.c:52-244) — O(depth * M) dependent max-plus steps before the first
// child. Here a node carries its front (u16 per machine) and its unscheduled set (a
// 32-bit mask), so a parent costs two passes over its unscheduled jobs only:
//   1. remain + tail per machine: sum of the unscheduled jobs' p rows (independent
//      adds, one vectorised LDS row read per job),
//   2. per child (job j): the O(M) chain start_m = max(front'_{m-1}, front_m),
//      lb = max_m(start_m + remain_m + tail_m) — ref add_front_and_bound.
// A surviving child's front is the same chain from the parent's front (from 0 at the
// root, whose front holds the minimum heads), recomputed in the emit loop.
//
// Work mapping (one 256-thread workgroup = 4 wave64 per chunk of 256 parents, the node
// in 8 / 12 VGPRs, the p table staged once per workgroup in LDS with a padded row
// stride so a ds_read_b128 lane group spreads over the banks) and the three iteration
// shapes are the pool's (pool_device.hpp): one level per kernel, two-level chunks for
// narrow windows (level-1 children staged in LDS), and local depth-first steps on the
// chunk's own slot region when the pool holds a backlog. Prune, leaf counting
// (incumbent atomicMin), workgroup scan and compaction into the chunk's slot region
// follow ref generate_children (PFSP_lib.h:51-95) counting rules.
#pragma once

#include "../core/pfsp_node.hpp"
#include "pool_device.hpp"

namespace tts {
namespace dev {

template <int M, int NJ_ = 20>
struct FrontGeom {
  static constexpr int NJ = NJ_;                        // children per parent at most (job bucket 20 or 50)
  using Node = PfspFrontNode<M, NJ>;
  using Mask = typename Node::Mask;                     // unscheduled-job set: 32 or 64 bits
  static constexpr int MO = sizeof(Mask) / 4;           // first word of the set (1 or 2)
  static constexpr int FO = 2 * MO;                     // first word of the fronts (2 or 4)
  static constexpr int NW = sizeof(Node) / 4;           // node words in registers (8 or 12)
  static constexpr int VPN = sizeof(Node) / 16;         // 16-B vectors per node
  static constexpr int BP = 256;                        // parents per chunk: one per thread
  static constexpr int MAXCH = BP * NJ;                 // children per chunk (upper bound)
  static constexpr int LT = 8;                          // local DFS steps per chunk at most
  static constexpr int SLOT = 2 * MAXCH;                // chunk slot region = its private stack
  static constexpr int MAXCHUNKS = 2048;
  // multi-level chunks (front_multi_level): up to BPF_CP parents, spread over the grid
  // (pool_begin), expanded LMAX levels deep at most; a level's survivors past CAP go out
  // unexpanded, so the chunk's output stays within SLOT
  static constexpr int BPF = 12;     // default cap: two-level windows up to 12 x 2048 parents
  static constexpr int BPF_CP = 32;
  // nodes of one level kept in LDS (the rest go out): sized so that 7 workgroups of the
  // kernel fit a CU's 160 KB of LDS (the grid is 7 per CU; an 8th-of-LDS overshoot made
  // one workgroup per CU wait for another to finish)
  static constexpr int CAP = 96;
  static constexpr int LMAX = 4;
  static constexpr int WLMAX = 3;  // levels of a wide multi-level chunk (one thread per window parent first)
  // a level of at most CPMAX children is expanded child-parallel (one thread per child),
  // a wider one one thread per node (each runs its children in turn)
  static constexpr int CPMAX = 3 * 256;
  // resident workgroups (= waves per SIMD) the kernel is compiled for; the occupancy API
  // reports one more than fit at its SGPR count (the SGPR file, 800 per SIMD, holds
  // 800 / (ceil(sgpr / 16) * 16 + 16) waves), so the engine's grid uses this instead
  // (measured: a grid of 7 per CU with 6 resident made 256 workgroups start one workgroup
  // lifetime late, +1.3 us per wide iteration, +4 us per multi-level one)
  // (50-job nodes: 16 words for 20 machines, 12 for 10: 5 waves up to 10 machines)
  static constexpr int WAVES = NJ > 20 ? (M <= 5 ? 6 : M <= 10 ? 5 : 4) : (M <= 10 ? 6 : 4);
  // resident workgroups per CU the engine's grid is sized for: under the step priority one
  // below the register budget's 6 for 20-job, <= 10-machine instances (ta014 0.1840 ->
  // 0.1822 ms, 2/4/8-way shares -2..-4 %, ta008 3 engines +8 %; profiles/r5/grid_ab.txt)
  static constexpr int GRID_WGS = NJ > 20 ? WAVES : (M <= 10 ? 5 : 4);
  // probe records (tests): {job | kind << 8, lb, parent words, parent remain}
  static constexpr int DBGW = (2 + NW + (M + 1) / 2 + 3) / 4 * 4;
  static constexpr int HW = (M + 1) / 2;  // packed u16 pairs of a p row / a remain
  // u16 row stride of the LDS p table (as PfspConsts::MS): 16 B for M <= 8, else 48 B
  static constexpr int MS = M <= 8 ? 8 : 24;
  static constexpr int RV = (M + 7) / 8;                // 16-B vectors holding one row's M values
};

template <int M, int NJ = 20>
struct PfspFrontArgs {
  PoolArgs<PfspFrontNode<M, NJ>> pool;
  const uint16_t* ptab;  // job-major p, [jobs][MS], padded machines 0
  int jobs;
  int min_tails[M];      // padded machines: 0
  // bounds kernel only (tests): bounds of parent i's children at bounds_out[offsets[i] + rank of
  // the job among the parent's unscheduled jobs]
  const PfspFrontNode<M, NJ>* parents_in;
  const int* offsets;
  int* bounds_out;
  int nparents;
  int bpf;  // two-level chunks: at most this many parents (<= FrontGeom::BPF_CP)
  int cp_max;  // multi-level chunks: child-parallel levels up to this many children
  // element-wise probe of the search kernel (tests, null in production): every child
  // bound evaluated by any iteration shape appends a FrontGeom::DBGW-word record
  uint32_t* dbg_rec;
  unsigned* dbg_n;
  unsigned dbg_cap;
  // per-workgroup phase timeline (timing probe only, null in production): wall clock at
  // 16 stamps per workgroup (front_stamp)
  unsigned long long* dbg_blk;
};

// Timing probe stamp k of this workgroup (thread 0; a.dbg_blk is null in production).
// Stamp 0 also records where the workgroup runs (raw HW_ID: wave / SIMD / CU / SE fields,
// and the XCC id) in words 12 / 13; front_local puts its node counts in word 14.
template <class A>
__device__ inline void front_stamp(const A& a, int k) {
  if (a.dbg_blk && threadIdx.x == 0) {
    a.dbg_blk[blockIdx.x * 16 + k] = wall_clock64();
    if (k == 0) {
      a.dbg_blk[blockIdx.x * 16 + 12] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      a.dbg_blk[blockIdx.x * 16 + 13] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
  }
}

template <int M, int NJ = 20>
struct FrontSmem {
  using G = FrontGeom<M, NJ>;
  uint16_t ptab[G::NJ][G::MS];
  int scan[kBlock / kWave];
  // dynamic local DFS (front_dyn): the workgroup's protocol state, in LDS so the step's
  // registers stay those of front_local (kept in registers it spilled to scratch)
  struct {
    unsigned long long deadline;
    long long inner;  // nodes pushed in this iteration and expanded here
    unsigned long long idle_ticks;  // (probe) time spent waiting for a block
    int flags, dslot, best, claim, claim_n, idle, sweep, pad;
  } dyn;
  // multi-level chunks: two levels of nodes (ping-pong), each node with its remain
  // (unscheduled work per machine, packed u16 pairs), and the child offsets of the
  // level being expanded
  // (two CAP-node buffers, lvl[b * CAP + i]; a wide two-level chunk uses both as one
  // 2 * CAP-node level). Local DFS chunks use the same bytes for the nodes the next step
  // pops (front_local).
  union {
    struct {
      uint4 lvl[2 * G::CAP][G::VPN];
      uint32_t rlv[2 * G::CAP][G::HW];
      int coff[2 * G::CAP];
    };
    struct {
      uint4 stage[kBlock][G::VPN];
      uint32_t stage_r[kBlock][G::HW];  // their remains (packed u16 pairs)
    };
  };
  PoolSmem<G::MAXCHUNKS> pool;
};

template <int M, int NJ>
__device__ inline void front_row(const uint16_t* row, int (&pr)[M]) {
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
#pragma unroll
  for (int q = 0; q < FrontGeom<M, NJ>::RV; ++q) {
    const uint4 x = r4[q];
    const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int h = 0; h < 8; ++h)
      if (q * 8 + h < M) pr[q * 8 + h] = static_cast<int>((wv[h >> 1] >> ((h & 1) * 16)) & 0xffffu);
  }
}

template <int M, int NJ>
__device__ inline int front_of(const uint32_t (&w)[FrontGeom<M, NJ>::NW], int m) {
  return static_cast<int>((w[FrontGeom<M, NJ>::FO + (m >> 1)] >> ((m & 1) * 16)) & 0xffffu);
}

// The unscheduled-job set of the node held in w (word 1, or words 2-3 for 50 jobs).
template <int M, int NJ>
__device__ inline typename FrontGeom<M, NJ>::Mask front_mask(const uint32_t (&w)[FrontGeom<M, NJ>::NW]) {
  if constexpr (FrontGeom<M, NJ>::MO == 1)
    return w[1];
  else
    return static_cast<u64>(w[2]) | (static_cast<u64>(w[3]) << 32);
}
__device__ inline int mask_pop(uint32_t x) { return __popc(x); }
__device__ inline int mask_pop(uint64_t x) { return __popcll(x); }

template <int M, int NJ>
__device__ inline void front_load(const PfspFrontNode<M, NJ>* src, uint32_t (&w)[FrontGeom<M, NJ>::NW]) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int q = 0; q < FrontGeom<M, NJ>::VPN; ++q) {
    const uint4 x = s[q];
    w[4 * q] = x.x;
    w[4 * q + 1] = x.y;
    w[4 * q + 2] = x.z;
    w[4 * q + 3] = x.w;
  }
}

template <int M, int NJ>
__device__ inline void front_store(uint4* dst, const uint32_t (&c)[FrontGeom<M, NJ>::NW]) {
#pragma unroll
  for (int q = 0; q < FrontGeom<M, NJ>::VPN; ++q) dst[q] = make_uint4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
}

// Probe record of one evaluated child (tests; a.dbg_rec is null in production): the
// parent's words, its remain (packed u16 pairs, tails excluded), the job, the iteration
// shape (kind) and the bound. The host recomputes every field (pfsp_front_probe).
enum FrontDbgKind { kDbgOne = 0, kDbgCp = 1, kDbgTp = 2, kDbgLocal = 3, kDbgSplit = 4, kDbgDyn = 5 };
template <int M, int NJ>
__device__ inline void front_dbg(const PfspFrontArgs<M, NJ>& a, int kind, const uint32_t (&w)[FrontGeom<M, NJ>::NW],
                                 const uint32_t (&rp)[FrontGeom<M, NJ>::HW], int j, int lb) {
  using G = FrontGeom<M, NJ>;
  const unsigned i = atomicAdd(a.dbg_n, 1u);
  if (i >= a.dbg_cap) return;
  uint32_t* r = a.dbg_rec + static_cast<size_t>(i) * G::DBGW;
  r[0] = static_cast<uint32_t>(j) | (static_cast<uint32_t>(kind) << 8);
  r[1] = static_cast<uint32_t>(lb);
#pragma unroll
  for (int k = 0; k < G::NW; ++k) r[2 + k] = w[k];
#pragma unroll
  for (int h = 0; h < G::HW; ++h) r[2 + G::NW + h] = rp[h];
}

// Packed u16 pairs: two children's chains per VALU op (v_pk_max_u16 / v_pk_add_u16; the
// p rows of the pair interleaved by one v_perm_b32 per machine). Every value of the chain
// stays below 65536: the instance's processing times sum below it (pfsp_front_ok) and a
// bound never exceeds a schedule's makespan.

// Bounds of the children appending the jobs of `rest` to a parent whose front / remain +
// tail are fb[m] / rb[m] (each value in both halves): emit(j, lb) per job, ascending,
// two jobs per pass (ref add_front_and_bound, c_bound_simple.c:219-244).
template <int M, int NJ, class Emit>
__device__ inline void front_bounds_x2(const FrontSmem<M, NJ>& sm, const uint32_t (&fb)[M], const uint32_t (&rb)[M],
                                       typename FrontGeom<M, NJ>::Mask rest, Emit emit) {
  constexpr int HW = FrontGeom<M, NJ>::HW;
  // 20 machines: one child per pass (same-box A/B on ta021 LB1_d: packed pairs 9.82 s,
  // one child 9.31 s; on ta014's 10 machines the pairs win, 0.2245 -> 0.2209 ms:
  // profiles/r4/packed_bounds_ab.txt)
  if constexpr (M > 10) {
    for (auto x = rest; x; x &= x - 1) {
      const int j = mask_ctz(x);
      int pr[M];
      front_row<M, NJ>(sm.ptab[j], pr);
      int lb = static_cast<int>(fb[0] & 0xffffu) + static_cast<int>(rb[0] & 0xffffu);
      int tt = static_cast<int>(fb[0] & 0xffffu) + pr[0];
#pragma unroll
      for (int m = 1; m < M; ++m) {
        const int sv = max(tt, static_cast<int>(fb[m] & 0xffffu));
        lb = max(lb, sv + static_cast<int>(rb[m] & 0xffffu));
        tt = sv + pr[m];
      }
      emit(j, lb);
    }
    return;
  }
  for (auto x = rest; x;) {
    const int j1 = mask_ctz(x);
    x &= x - 1;
    const bool two = x != 0;
    const int j2 = two ? mask_ctz(x) : j1;
    x &= x - 1;
    const uint32_t* r1 = reinterpret_cast<const uint32_t*>(sm.ptab[j1]);
    const uint32_t* r2 = reinterpret_cast<const uint32_t*>(sm.ptab[j2]);
    uint32_t a[HW], b[HW];
#pragma unroll
    for (int h = 0; h < HW; ++h) {
      a[h] = r1[h];
      b[h] = r2[h];
    }
    u16x2 lb = as_u16x2(fb[0]) + as_u16x2(rb[0]);
    u16x2 tt = as_u16x2(fb[0]) + as_u16x2(__builtin_amdgcn_perm(b[0], a[0], 0x05040100u));
#pragma unroll
    for (int m = 1; m < M; ++m) {
      const u16x2 pm = as_u16x2(__builtin_amdgcn_perm(b[m >> 1], a[m >> 1], (m & 1) ? 0x07060302u : 0x05040100u));
      const u16x2 sv = __builtin_elementwise_max(tt, as_u16x2(fb[m]));
      lb = __builtin_elementwise_max(lb, sv + as_u16x2(rb[m]));
      tt = sv + pm;
    }
    const uint32_t l = as_u32(lb);
    emit(j1, static_cast<int>(l & 0xffffu));
    if (two) emit(j2, static_cast<int>(l >> 16));
  }
}

// fb / rb of a parent: its front (words of w) and its packed remain rp plus the tails
template <int M, int NJ>
__device__ inline void front_broadcast(const PfspFrontArgs<M, NJ>& a, const uint32_t (&w)[FrontGeom<M, NJ>::NW],
                                       const uint32_t (&rp)[FrontGeom<M, NJ>::HW], uint32_t (&fb)[M], uint32_t (&rb)[M]) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    fb[m] = static_cast<uint32_t>(front_of<M, NJ>(w, m)) * 0x10001u;
    rb[m] = (((rp[m >> 1] >> ((m & 1) * 16)) & 0xffffu) + static_cast<uint32_t>(a.min_tails[m])) * 0x10001u;
  }
}

// The packed remain of the node in w: the sum of its unscheduled jobs' p rows.
template <int M, int NJ>
__device__ inline void front_remain(const FrontSmem<M, NJ>& sm, const uint32_t (&w)[FrontGeom<M, NJ>::NW],
                                    uint32_t (&r2)[FrontGeom<M, NJ>::HW]) {
  constexpr int HW = FrontGeom<M, NJ>::HW;
#pragma unroll
  for (int h = 0; h < HW; ++h) r2[h] = 0;
  if constexpr (M <= 10) {
    // 4 jobs per pass, every row read issued before the first add: one LDS latency per
    // pass instead of one per job (the rolled loop waited on each row in turn; ta014
    // headline -0.9 % same box, profiles/r6/remain_ab.txt). 20 machines keep the rolled
    // loop (its registers are the kernel's budget).
    constexpr int U = 4;
    for (auto x = front_mask<M, NJ>(w); x;) {
      int j[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ok[u] = x != 0;
        j[u] = ok[u] ? mask_ctz(x) : 0;
        x &= x - 1;
      }
      uint32_t rw[U][HW];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[j[u]]);
#pragma unroll
        for (int h = 0; h < HW; ++h) rw[u][h] = row[h];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int h = 0; h < HW; ++h) r2[h] += ok[u] ? rw[u][h] : 0u;
    }
  } else {
    for (auto x = front_mask<M, NJ>(w); x; x &= x - 1) {
      const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[mask_ctz(x)]);
#pragma unroll
      for (int h = 0; h < HW; ++h) r2[h] += row[h];
    }
  }
}

// Bounds of every child of the parent held in w: emit(j, lb) for each unscheduled job j.
// (the parent's packed remain rp given)
template <int M, int NJ, class Emit>
__device__ inline void front_parent_r(const PfspFrontArgs<M, NJ>& a, const FrontSmem<M, NJ>& sm,
                                      const uint32_t (&w)[FrontGeom<M, NJ>::NW], const uint32_t (&rp)[FrontGeom<M, NJ>::HW],
                                      Emit emit, int kind) {
  uint32_t fb[M], rb[M];
  front_broadcast<M, NJ>(a, w, rp, fb, rb);
  front_bounds_x2<M, NJ>(sm, fb, rb, front_mask<M, NJ>(w), [&](int j, int lb) {
    if (a.dbg_rec) front_dbg<M, NJ>(a, kind, w, rp, j, lb);
    emit(j, lb);
  });
}

template <int M, int NJ, class Emit>
__device__ inline void front_parent(const PfspFrontArgs<M, NJ>& a, const FrontSmem<M, NJ>& sm,
                                    const uint32_t (&w)[FrontGeom<M, NJ>::NW], Emit emit, int kind = kDbgOne) {
  uint32_t rp[FrontGeom<M, NJ>::HW], fb[M], rb[M];
  front_remain<M, NJ>(sm, w, rp);
  front_broadcast<M, NJ>(a, w, rp, fb, rb);
  front_bounds_x2<M, NJ>(sm, fb, rb, front_mask<M, NJ>(w), [&](int j, int lb) {
    if (a.dbg_rec) front_dbg<M, NJ>(a, kind, w, rp, j, lb);
    emit(j, lb);
  });
}

// Child of the parent in w that appends job j: depth + 1, j removed from the set, and
// its front (the chain from the parent's front; from 0 at the root).
template <int M, int NJ>
__device__ inline void front_child(const FrontSmem<M, NJ>& sm, const uint32_t (&w)[FrontGeom<M, NJ>::NW], int j,
                                   uint32_t (&c)[FrontGeom<M, NJ>::NW]) {
  constexpr int NW = FrontGeom<M, NJ>::NW;
  const int d = static_cast<int>(w[0] & 0xffu);
  const bool root = d == 0;
  int pr[M];
  front_row<M, NJ>(sm.ptab[j], pr);
  constexpr int FO = FrontGeom<M, NJ>::FO;
  c[0] = static_cast<uint32_t>(d + 1);
#pragma unroll
  for (int i = 1; i < NW; ++i) c[i] = 0;
  const auto rest = front_mask<M, NJ>(w) & ~(static_cast<typename FrontGeom<M, NJ>::Mask>(1) << j);
  c[FrontGeom<M, NJ>::MO] = static_cast<uint32_t>(rest);
  if constexpr (FrontGeom<M, NJ>::MO == 2) c[3] = static_cast<uint32_t>(static_cast<u64>(rest) >> 32);
  int ft = (root ? 0 : front_of<M, NJ>(w, 0)) + pr[0];
  c[FO] = static_cast<uint32_t>(ft);
#pragma unroll
  for (int m = 1; m < M; ++m) {
    ft = max(ft, root ? 0 : front_of<M, NJ>(w, m)) + pr[m];
    c[FO + (m >> 1)] |= static_cast<uint32_t>(ft) << ((m & 1) * 16);
  }
}

// (store(i, child words, job) for the i-th surviving child of w)
template <int M, int NJ, class Store>
__device__ inline void front_emit_to(const FrontSmem<M, NJ>& sm, const uint32_t (&w)[FrontGeom<M, NJ>::NW],
                                     typename FrontGeom<M, NJ>::Mask surv,
                                     Store store) {
  for (int i = 0; surv; ++i) {
    const int j = mask_ctz(surv);
    surv &= surv - 1;
    uint32_t c[FrontGeom<M, NJ>::NW];
    front_child<M, NJ>(sm, w, j, c);
    store(i, c, j);
  }
}

template <int M, int NJ>
__device__ inline void front_emit(const FrontSmem<M, NJ>& sm, const uint32_t (&w)[FrontGeom<M, NJ>::NW],
                                  typename FrontGeom<M, NJ>::Mask surv,
                                  uint4* dst) {
  while (surv) {
    const int j = mask_ctz(surv);
    surv &= surv - 1;
    uint32_t c[FrontGeom<M, NJ>::NW];
    front_child<M, NJ>(sm, w, j, c);
    front_store<M, NJ>(dst, c);
    dst += FrontGeom<M, NJ>::VPN;
  }
}

// Position of the k-th (0-based) set bit of x, k < popcount(x): a 5-step binary
// search on popcounts of the low halves (no loop over the bits).
__device__ inline int kth_bit(uint32_t x, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 16; w; w >>= 1) {
    const uint32_t lo = x & ((1u << w) - 1u);
    const int c = __popc(lo);
    const bool up = k >= c;
    k = up ? k - c : k;
    x = up ? (x >> w) : lo;
    pos += up ? w : 0;
  }
  return pos;
}
// (64-bit sets: the low word first)
__device__ inline int kth_bit(uint64_t x, int k) {
  const uint32_t lo = static_cast<uint32_t>(x);
  const int c = __popc(lo);
  return k < c ? kth_bit(lo, k) : 32 + kth_bit(static_cast<uint32_t>(x >> 32), k - c);
}

// Child-parallel expansion of n nodes staged in LDS (src[i], with their remain
// rem[i]): ONE THREAD PER CHILD instead of one per parent. In a narrow level a
// thread-per-parent expansion runs its parent's ~20 children one after the other while
// most lanes idle; here child c finds its parent (binary search on the child offsets)
// and its job (k-th unscheduled bit), then bounds itself from the parent's front and
// remain (no pass over the parent's rows: remains are carried, a child's is its
// parent's minus its own row). Leaves lower the incumbent and are counted in nleaf;
// survivors are compacted (block scan) and handed to store(index, child words, child
// remain). Returns the survivor count. Every thread calls it (block-wide scans).
// Children of the n staged nodes: their offsets into sm.coff, the total returned.
template <int M, int NJ>
__device__ inline int front_child_offsets(FrontSmem<M, NJ>& sm, const uint4 (*src)[FrontGeom<M, NJ>::VPN], int n) {
  int T = 0;
  int k = 0;
  if (static_cast<int>(threadIdx.x) < n) {
    const uint4 h = src[threadIdx.x][0];  // the set: word 1 (20 jobs) or words 2-3 (50 jobs)
    k = FrontGeom<M, NJ>::MO == 1 ? __popc(h.y) : __popc(h.z) + __popc(h.w);
  }
  const int off = block_exclusive_scan(k, sm.scan, &T);
  if (static_cast<int>(threadIdx.x) < n) sm.coff[threadIdx.x] = off;
  __syncthreads();
  return T;
}

// Children a level keeps: all of them, except in a rank split's level (keep(node, job)).
struct FrontKeepAll {
  __device__ bool operator()(int, int) const { return true; }
};

// (T children, offsets in sm.coff: front_child_offsets)
template <int M, int NJ, class Store, class Keep = FrontKeepAll>
__device__ inline int front_expand_cp(const PfspFrontArgs<M, NJ>& a, FrontSmem<M, NJ>& sm, const uint4 (*src)[FrontGeom<M, NJ>::VPN],
                                      const uint32_t (*rem)[FrontGeom<M, NJ>::HW], int n, int T, int best, int& nleaf,
                                      Store store, Keep keep = {}, int kind = kDbgCp) {
  using G = FrontGeom<M, NJ>;
  constexpr int HW = G::HW;
  const int tid = threadIdx.x;
  int nout = 0;
  for (int cb = 0; cb < T; cb += kBlock) {
    const int c = cb + tid;
    bool surv = false;
    int j = 0;
    uint32_t w[G::NW], cr[HW];
#pragma unroll
    for (int i = 0; i < G::NW; ++i) w[i] = 0;
#pragma unroll
    for (int h = 0; h < HW; ++h) cr[h] = 0;
    if (c < T) {
      int lo = 0, hi = n - 1;  // last node whose children start at or before c
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sm.coff[mid] <= c)
          lo = mid;
        else
          hi = mid - 1;
      }
#pragma unroll
      for (int q = 0; q < G::VPN; ++q) {
        const uint4 x = src[lo][q];
        w[4 * q] = x.x;
        w[4 * q + 1] = x.y;
        w[4 * q + 2] = x.z;
        w[4 * q + 3] = x.w;
      }
      j = kth_bit(front_mask<M, NJ>(w), c - sm.coff[lo]);
      const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[j]);
      uint32_t pw[HW], rp[HW];
#pragma unroll
      for (int h = 0; h < HW; ++h) {
        pw[h] = row[h];
        rp[h] = rem[lo][h];
        cr[h] = rp[h] - pw[h];  // the child's remain (packed halves never borrow: row <= remain)
      }
      auto pm = [&](int m) { return static_cast<int>((pw[m >> 1] >> ((m & 1) * 16)) & 0xffffu); };
      auto rm = [&](int m) { return static_cast<int>((rp[m >> 1] >> ((m & 1) * 16)) & 0xffffu) + a.min_tails[m]; };
      const int f0 = front_of<M, NJ>(w, 0);
      int lb = f0 + rm(0);
      int tt = f0 + pm(0);
#pragma unroll
      for (int m = 1; m < M; ++m) {
        const int sv = max(tt, front_of<M, NJ>(w, m));
        lb = max(lb, sv + rm(m));
        tt = sv + pm(m);
      }
      if (a.dbg_rec) front_dbg<M, NJ>(a, kind, w, rp, j, lb);
      const bool kp = keep(lo, j);
      if (static_cast<int>(w[0] & 0xffu) + 1 == a.jobs) {
        nleaf += kp;
        if (lb < best) atomicMin(&a.pool.ctl->best.v, lb);
      } else {
        surv = kp && lb < best;
      }
    }
    int tot = 0;
    const int idx = nout + block_exclusive_scan(surv ? 1 : 0, sm.scan, &tot);
    if (surv) {
      uint32_t cw[G::NW];
      front_child<M, NJ>(sm, w, j, cw);
      store(idx, cw, cr);
    }
    nout += tot;
  }
  return nout;
}

// Thread-per-node expansion of n <= kBlock nodes staged in LDS with their carried
// remains: thread i bounds all children of node i in turn (the chain of front_parent,
// without its pass over the unscheduled rows), then the survivors are compacted (block
// scan) and handed to store(index, child words, child remain). Wider levels take this
// path: fewer instructions per child than front_expand_cp (no parent search, one node
// load per parent), and the serial loop is short once most lanes hold a node.
// (the node and its packed remain in registers; w = 0 for a thread without a node)
template <int M, int NJ, class Store, class Keep = FrontKeepAll>
__device__ inline int front_expand_tp_regs(const PfspFrontArgs<M, NJ>& a, FrontSmem<M, NJ>& sm,
                                           const uint32_t (&w)[FrontGeom<M, NJ>::NW], const uint32_t (&rp)[FrontGeom<M, NJ>::HW],
                                           int best, int& nleaf, Store store, int kind = kDbgTp, Keep keep = {}) {
  using G = FrontGeom<M, NJ>;
  constexpr int HW = G::HW;
  typename G::Mask surv = 0;
  int nsurv = 0;
  const bool leaf = static_cast<int>(w[0] & 0xffu) + 1 == a.jobs;
  {
    uint32_t fb[M], rb[M];
    front_broadcast<M, NJ>(a, w, rp, fb, rb);
    front_bounds_x2<M, NJ>(sm, fb, rb, front_mask<M, NJ>(w), [&](int j, int lb) {
      if (a.dbg_rec) front_dbg<M, NJ>(a, kind, w, rp, j, lb);
      const bool kp = keep(static_cast<int>(threadIdx.x), j);
      if (leaf) {
        nleaf += kp;
        if (lb < best) atomicMin(&a.pool.ctl->best.v, lb);
      } else if (kp && lb < best) {
        ++nsurv;
        surv |= static_cast<typename G::Mask>(1) << j;
      }
    });
  }
  int tot = 0;
  int idx = block_exclusive_scan(nsurv, sm.scan, &tot);
  while (surv) {
    const int j = mask_ctz(surv);
    surv &= surv - 1;
    uint32_t cw[G::NW], cr[HW];
    front_child<M, NJ>(sm, w, j, cw);
    const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[j]);
#pragma unroll
    for (int h = 0; h < HW; ++h) cr[h] = rp[h] - row[h];
    store(idx++, cw, cr);
  }
  return tot;
}

template <int M, int NJ, class Store, class Keep = FrontKeepAll>
__device__ inline int front_expand_tp(const PfspFrontArgs<M, NJ>& a, FrontSmem<M, NJ>& sm,
                                      const uint4 (*src)[FrontGeom<M, NJ>::VPN], const uint32_t (*rem)[FrontGeom<M, NJ>::HW],
                                      int n, int best, int& nleaf, Store store, Keep keep = {}, int kind = kDbgTp) {
  using G = FrontGeom<M, NJ>;
  constexpr int HW = G::HW;
  const int tid = threadIdx.x;
  uint32_t w[G::NW], rp[HW];
#pragma unroll
  for (int i = 0; i < G::NW; ++i) w[i] = 0;
#pragma unroll
  for (int h = 0; h < HW; ++h) rp[h] = 0;
  if (tid < n) {
#pragma unroll
    for (int q = 0; q < G::VPN; ++q) {
      const uint4 x = src[tid][q];
      w[4 * q] = x.x;
      w[4 * q + 1] = x.y;
      w[4 * q + 2] = x.z;
      w[4 * q + 3] = x.w;
    }
#pragma unroll
    for (int h = 0; h < HW; ++h) rp[h] = rem[tid][h];
  }
  return front_expand_tp_regs<M, NJ>(a, sm, w, rp, best, nleaf, store, kind, keep);
}

// Multi-level chunk (fused iterations): the chunk's v.bp parents go to LDS with their
// remains, then up to v.levels tree levels are expanded in place — each level's
// survivors become the next level's nodes in the other LDS buffer (at most CAP of them;
// the rest go out unexpanded, first in the slot region), and the last level's survivors
// go out. A level of at most a.cp_max children is expanded child-parallel (passes of
// kBlock children), a wider one thread-per-node. Counts: nodes staged and expanded here are pushed-and-expanded tree
// nodes (high half of the leaf word); everything that goes out is the chunk's output.
// One dependent kernel covers up to 4 tree levels of a narrow window (ref: one kernel
// per level, pfsp_multigpu_cuda.c:221-332).
template <int M, int NJ>
__device__ inline void front_multi_level(const PfspFrontArgs<M, NJ>& a, FrontSmem<M, NJ>& sm, const IterView& v, int t,
                                         int best) {
  using G = FrontGeom<M, NJ>;
  using Node = PfspFrontNode<M, NJ>;
  static_assert(G::BPF_CP * (G::NJ - 1) + (G::LMAX - 1) * G::CAP * (G::NJ - 1) <= G::SLOT,
                "chunk output must fit its slot region");
  static_assert(kBlock * (G::NJ - 1) + (G::WLMAX - 1) * G::CAP * (G::NJ - 1) <= G::SLOT,
                "wide chunk output must fit its slot region");
  static_assert(2 * G::CAP <= kBlock && G::BPF_CP <= G::CAP, "one thread per staged node");
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  // wide chunks (more parents than a staged level holds): the first level runs one
  // thread per window parent straight from the pool, its survivors go to LDS
  const bool wide = v.bp > G::BPF_CP;
  const int L = min(v.levels, wide ? G::WLMAX : G::LMAX);
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    const u64 g0 = static_cast<u64>(ch) * v.bp;
    const int n0 = static_cast<int>(min(static_cast<u64>(v.bp), v.B - g0));
    int nleaf = 0, inner = 0, o = 0, n = n0, cur = 0, lev0 = 0;
    uint4* const out = reinterpret_cast<uint4*>(bout + static_cast<size_t>(ch) * G::SLOT);
    const bool first = ch == static_cast<int>(blockIdx.x);
    // wave priority falls with the level, as in front_local (ta014 -1.3 %,
    // profiles/r5/fuse_prio_ab.txt); later chunks of a workgroup go last
    if (first) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(0);
    if (wide) {
      uint32_t w[G::NW], r2[G::HW];
#pragma unroll
      for (int i = 0; i < G::NW; ++i) w[i] = 0;
      if (tid < n0) front_load<M, NJ>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, g0 + tid, sm.pool), w);
      front_remain<M, NJ>(sm, w, r2);
      const bool last = L == 1;
      // the first LDS level: both buffers when it is also the last one expanded (two
      // levels), else buffer 1 (buffer 0 then takes the level after it)
      const int cap1 = L == 2 ? 2 * G::CAP : G::CAP;
      const int base1 = L == 2 ? 0 : G::CAP;
      const int nn = front_expand_tp_regs<M, NJ>(
          a, sm, w, r2, best, nleaf,
          [&](int i, const uint32_t (&c)[G::NW], const uint32_t (&r)[G::HW]) {
            if (!last && i < cap1) {
              front_store<M, NJ>(&sm.lvl[base1 + i][0], c);
#pragma unroll
              for (int h = 0; h < G::HW; ++h) sm.rlv[base1 + i][h] = r[h];
            } else {
              front_store<M, NJ>(out + (last ? i : i - cap1) * G::VPN, c);
            }
          },
          kDbgOne);
      __syncthreads();
      o = last ? nn : max(0, nn - cap1);
      n = last ? 0 : min(nn, cap1);
      inner = n;
      cur = L == 2 ? 0 : 1;
      lev0 = 1;
      if (first) front_stamp(a, 4);
    } else {
      if (tid < n0) {
        // the parent's remain: one pass over its unscheduled rows (packed u16 pairs; sums
        // < 65536, pfsp_front_ok), by the thread that stages it
        uint32_t w[G::NW], r2[G::HW];
        front_load<M, NJ>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, g0 + tid, sm.pool), w);
        front_store<M, NJ>(&sm.lvl[tid][0], w);
        front_remain<M, NJ>(sm, w, r2);
#pragma unroll
        for (int h = 0; h < G::HW; ++h) sm.rlv[tid][h] = r2[h];
      }
      __syncthreads();
    }
    if (first) front_stamp(a, 3);
    for (int lev = lev0; lev < L && n > 0; ++lev) {
      if (first) {
        if (lev == 0) __builtin_amdgcn_s_setprio(2);
        else if (lev == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      const bool last = lev == L - 1;
      const int nx = cur ^ 1;
      auto store = [&](int i, const uint32_t (&c)[G::NW], const uint32_t (&r)[G::HW]) {
        if (!last && i < G::CAP) {
          front_store<M, NJ>(&sm.lvl[nx * G::CAP + i][0], c);
#pragma unroll
          for (int h = 0; h < G::HW; ++h) sm.rlv[nx * G::CAP + i][h] = r[h];
        } else {
          front_store<M, NJ>(out + (o + (last ? i : i - G::CAP)) * G::VPN, c);
        }
      };
      const uint4(*src)[G::VPN] = sm.lvl + cur * G::CAP;
      const uint32_t(*rsrc)[G::HW] = sm.rlv + cur * G::CAP;
      const int T = front_child_offsets<M, NJ>(sm, src, n);
      // the first level of a rank split's iteration keeps this rank's children only
      // (split_keep of the parent's window position and the job, as the one-level split)
      const bool split_lev = v.split && lev == 0;
      const u64 gbase = g0;
      auto keep = [&](int p, int j) { return !split_lev || split_keep(v, gbase + static_cast<u64>(p), j); };
      const int nn = T > a.cp_max
                         ? front_expand_tp<M, NJ>(a, sm, src, rsrc, n, best, nleaf, store, keep, split_lev ? kDbgSplit : kDbgTp)
                         : front_expand_cp<M, NJ>(a, sm, src, rsrc, n, T, best, nleaf, store, keep,
                                              split_lev ? kDbgSplit : kDbgCp);
      __syncthreads();  // the next level is visible; this level's buffer is free
      o += last ? nn : max(0, nn - G::CAP);
      n = last ? 0 : min(nn, G::CAP);
      inner += n;
      cur = nx;
      if (first) front_stamp(a, 4 + lev);
    }
    int leaves = 0;
    (void)block_exclusive_scan(nleaf, sm.scan, &leaves);
    if (tid == 0) {
      cnt_out[ch] = o;
      lcnt_out[ch] = leaves | (inner << 16);
    }
    __syncthreads();  // sm.lvl / sm.coff are rewritten by the next chunk
    if (first) front_stamp(a, 8);
  }
  front_stamp(a, 15);
}

// Local DFS chunk loop (v.local): chunk ch takes v.bp window parents, then keeps
// popping up to kBlock nodes from the top of its own slot region (a private stack,
// written by this workgroup only) and pushing their survivors there, for up to
// v.steps steps or until the stack is empty. The stack left is the chunk's output
// (cnt); nodes pushed and expanded in between are explored tree nodes (high half of
// the leaf word). Pops read slots [top - n, top) and pushes write from top - n on:
// every pop is in registers before the scan's barrier that precedes the first push.
template <int M, int NJ>
__device__ inline void front_local(const PfspFrontArgs<M, NJ>& a, FrontSmem<M, NJ>& sm, const IterView& v, int t, int best) {
  using G = FrontGeom<M, NJ>;
  using Node = PfspFrontNode<M, NJ>;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    Node* const stk = bout + static_cast<size_t>(ch) * G::SLOT;
    // nst: how many of the nodes on top of the stack are held in sm.stage (the previous
    // step's last children, exactly the ones this step pops) instead of the slot region
    int top = 0, pushed = 0, nleaf = 0, nst = 0;
    for (int s = 0; s < v.steps; ++s) {
      // Wave priority falls with the step: workgroups behind in steps issue first. A CU
      // otherwise issues its oldest waves first, so late-dispatched workgroups trailed
      // (exit vs dispatch rank in the CU r = 0.93) and each CU's tail ran with few waves
      // on a latency-bound loop. ta014 window exits max/mean 1.50 -> 1.20, headline
      // 0.2182 -> 0.2021 ms, ta021 one engine 16.3 -> 14.1 s; a stack-size priority
      // gained nothing (profiles/r5/prio_ab.txt)
      // (4 levels spread over the steps)
      const int lvl = min(3, ((v.steps - 1 - s) * 4) / v.steps);
      if (lvl == 3) __builtin_amdgcn_s_setprio(3);
      else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
      else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      uint32_t w[G::NW], rp[G::HW];
      bool have_r = false;  // rp carried with a staged node
#pragma unroll
      for (int i = 0; i < G::NW; ++i) w[i] = 0;
      if (s == 0) {
        const u64 gi = v.stride ? static_cast<u64>(ch) + static_cast<u64>(tid) * static_cast<u64>(v.nchunks)
                                       : static_cast<u64>(ch) * v.bp + tid;
        if (tid < v.bp && gi < v.B) front_load<M, NJ>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, gi, sm.pool), w);
      } else {
        if (top == 0) break;  // uniform
        const int npop = min(top, kBlock);
        if (tid < npop) {
          const int k = tid - (npop - nst);
          if (k >= 0) {
#pragma unroll
            for (int q = 0; q < G::VPN; ++q) {
              const uint4 x = sm.stage[k][q];
              w[4 * q] = x.x;
              w[4 * q + 1] = x.y;
              w[4 * q + 2] = x.z;
              w[4 * q + 3] = x.w;
            }
#pragma unroll
            for (int h = 0; h < G::HW; ++h) rp[h] = sm.stage_r[k][h];
            have_r = true;
          } else {
            front_load<M, NJ>(stk + (top - npop + tid), w);
          }
        }
        top -= npop;
      }
      typename G::Mask surv = 0;
      int nsurv = 0;
      const bool leaf = static_cast<int>(w[0] & 0xffu) + 1 == a.jobs;
      if (!have_r) front_remain<M, NJ>(sm, w, rp);
      front_parent_r<M, NJ>(
          a, sm, w, rp,
          [&](int j, int lb) {
            if (leaf) {
              ++nleaf;
              if (lb < best) atomicMin(&pa.ctl->best.v, lb);
            } else if (lb < best) {
              ++nsurv;
              surv |= static_cast<typename G::Mask>(1) << j;
            }
          },
          kDbgLocal);
      int tot = 0;
      const int off = block_exclusive_scan(nsurv, sm.scan, &tot);
      // will another step run? then the children it pops (the last min(top, kBlock)
      // pushed) stay in LDS and skip the slot region's store / load round trip
      const int tnew = top + tot;
      const bool more = s + 1 < v.steps && tnew > 0 && tnew + kBlock * G::NJ <= G::SLOT;
      nst = more ? min(tot, min(tnew, kBlock)) : 0;
      const int lo = tot - nst;
      uint4* const dst = reinterpret_cast<uint4*>(stk + top);
      // (the scan's barrier: every thread holds its popped node in registers by now)
      front_emit_to<M, NJ>(sm, w, surv, [&](int i, const uint32_t (&c)[G::NW], int j) {
        const int o = off + i;
        if (o >= lo) {
          front_store<M, NJ>(&sm.stage[o - lo][0], c);
          const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[j]);
#pragma unroll
          for (int h = 0; h < G::HW; ++h) sm.stage_r[o - lo][h] = rp[h] - row[h];  // the child's remain
        } else {
          front_store<M, NJ>(dst + o * G::VPN, c);
        }
      });
      top = tnew;
      pushed += tot;
      // pushes visible to the next step's pops (workgroup scope), and room left for
      // one more full step
      __syncthreads();
      if (ch == static_cast<int>(blockIdx.x) && s < 4) front_stamp(a, 4 + s);
      if (!more) break;
    }
    int leaves = 0;
    (void)block_exclusive_scan(nleaf, sm.scan, &leaves);
    if (tid == 0) {
      cnt_out[ch] = top;
      lcnt_out[ch] = leaves | ((pushed - top) << 16);
      if (a.dbg_blk && ch == static_cast<int>(blockIdx.x))
        a.dbg_blk[blockIdx.x * 16 + 14] = static_cast<unsigned long long>(pushed - top) |
                                          (static_cast<unsigned long long>(top) << 32);
    }
  }
}

// ---- dynamic local DFS (v.dyn): work moves between the workgroups of one XCD ----
//
// front_local with no step count: every workgroup keeps expanding the top of its own
// stack until the iteration's time budget (pa.dyn_ticks of the 100 MHz wall clock) is
// spent, publishing one pop (<= kBlock nodes) into a free queue slot of its XCD's
// partition when partition workgroups wait for more blocks than are full (or when its
// stack nears the slot region's end), and claiming a full slot when its stack runs dry
// (ref steal-half between GPU threads, pfsp_multigpu_cuda.c:343-431, here between the
// workgroups of one kernel). Why: per-workgroup exits of a fixed-step local iteration
// follow the dispatch order inside each CU (corr 0.95, per-CU max exits within 10 %:
// profiles/r5/lb_probe.txt), so the loss is not one slow workgroup but the ~10 us every
// dependent kernel costs and the half-empty first steps of each new window
// (profiles/r5/ilog_ta014.txt: 9 kernels, four of them local). One dynamic iteration
// carries the tree until the budget ends or no partition workgroup has work.
//
// Every word and payload byte that crosses workgroups is an 8-B agent-scope atomic
// access (sc1: L1 bypassed) on lines of the partition's own L2 — the partition is the
// XCC id read from the hardware, never a dispatch-order assumption. Counts go to the
// xacc lines (64-bit); the last workgroup out writes the queue chunks' counts.
__device__ inline int dyn_ld(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline unsigned dyn_ldu(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline int dyn_add(int* p, int x) {
  return __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Slot hand-offs follow the memory model, not the hardware's in-order behaviour: the
// publishing store (full / free) is a release by the workgroup's thread 0 after the
// barrier that ends every wave's payload accesses, the claiming CAS an acquire before the
// barrier that starts the claimer's payload reads (barrier + agent-scope release /
// acquire are cumulative).
__device__ inline void dyn_stu_rel(unsigned* p, unsigned x) {
  __hip_atomic_store(p, x, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline bool dyn_cas(unsigned* p, unsigned expect, unsigned want) {
  return __hip_atomic_compare_exchange_strong(p, &expect, want, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}

template <int M, int NJ>
__device__ inline void dyn_node_store(PfspFrontNode<M, NJ>* dst, const uint32_t (&w)[FrontGeom<M, NJ>::NW]) {
  u64* d = reinterpret_cast<u64*>(dst);
#pragma unroll
  for (int k = 0; k < FrontGeom<M, NJ>::NW / 2; ++k)
    __hip_atomic_store(d + k, static_cast<u64>(w[2 * k]) | (static_cast<u64>(w[2 * k + 1]) << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
template <int M, int NJ>
__device__ inline void dyn_node_load(PfspFrontNode<M, NJ>* src, uint32_t (&w)[FrontGeom<M, NJ>::NW]) {
  u64* s = reinterpret_cast<u64*>(src);
#pragma unroll
  for (int k = 0; k < FrontGeom<M, NJ>::NW / 2; ++k) {
    const u64 x = __hip_atomic_load(s + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w[2 * k] = static_cast<uint32_t>(x);
    w[2 * k + 1] = static_cast<uint32_t>(x >> 32);
  }
}

// Wave 0: find a slot of the partition in state `want` (0 free / 2 full, low 2 bits)
// and move it to `to` (1 writing / 3 reading, keeping the count bits). Lanes scan 64
// states at a time; the pick rotates with the workgroup so claimers spread. Returns
// slot | n << 16, or -1.
__device__ inline int dyn_take(DynCtl* dc, int qbase, int qx, unsigned want, unsigned to) {
  const int lane = static_cast<int>(threadIdx.x) & (kWave - 1);
  const int r = static_cast<int>(blockIdx.x) & (kWave - 1);
  for (int k0 = 0; k0 < qx; k0 += kWave) {
    const bool in = k0 + lane < qx;
    const unsigned sv = in ? dyn_ldu(&dc->st[qbase + k0 + lane]) : 1u;
    u64 hit = __ballot(in && (sv & 3u) == want);
    while (hit) {
      const u64 rot = r ? ((hit >> r) | (hit << (kWave - r))) : hit;
      const int pick = (__builtin_ctzll(rot) + r) & (kWave - 1);
      bool ok = false;
      if (lane == pick) ok = dyn_cas(&dc->st[qbase + k0 + pick], sv, (sv & ~3u) | to);
      ok = __shfl(static_cast<int>(ok), pick, kWave) != 0;
      const unsigned n = static_cast<unsigned>(__shfl(static_cast<int>(sv), pick, kWave)) >> 8;
      if (ok) return (k0 + pick) | static_cast<int>(n << 16);
      hit &= ~(1ull << pick);
    }
  }
  return -1;
}

// Copy n nodes src[0..n) -> dst[0..n) within this workgroup's view (plain loads / stores:
// both in regions this workgroup alone writes), one node per thread and pass.
// (rare paths of front_dyn, kept out of line: inlined, their temporaries pushed the
// step's registers into scratch)
// mode 0: plain -> plain (this workgroup's own regions); 1: plain -> 8-B agent stores
// (publish); 2: 8-B agent loads -> plain (claim)
template <int M, int NJ>
__device__ __attribute__((noinline)) void dyn_copy(const PfspFrontNode<M, NJ>* src, PfspFrontNode<M, NJ>* dst, int n,
                                                   int mode) {
  for (int i = static_cast<int>(threadIdx.x); i < n; i += kBlock) {
    uint32_t x[FrontGeom<M, NJ>::NW];
    if (mode == 2)
      dyn_node_load<M, NJ>(const_cast<PfspFrontNode<M, NJ>*>(src + i), x);
    else
      front_load<M, NJ>(src + i, x);
    if (mode == 1)
      dyn_node_store<M, NJ>(dst + i, x);
    else
      front_store<M, NJ>(reinterpret_cast<uint4*>(dst + i), x);
  }
}
template <int M, int NJ>
__device__ inline void dyn_copy_own(const PfspFrontNode<M, NJ>* src, PfspFrontNode<M, NJ>* dst, int n) {
  dyn_copy<M, NJ>(src, dst, n, 0);
}

// A stack of at least this many nodes gives its bottom half to a waiting workgroup of its
// partition. Splitting small frontiers (64) balanced the per-CU work (p90/p10 1.35) but
// slowed every budget (ta014 headline 0.354 / 0.504 ms at 40 / 300 us against 0.238 / 0.332
// with 512): the thieves' steps are short and each step costs its full latency
// (profiles/r5/dyn_eager_ab.txt)
constexpr int kDynMinDonate = 512;

// Wave 0 of a workgroup whose stack ran dry: claim a full slot of the partition, polling
// until one is published, the deadline passes, or no partition workgroup has work and
// no slot is full (returns slot | n << 16, or -1).
__device__ __attribute__((noinline)) int dyn_claim_spin(DynCtl* dc, int qbase, int qx, DynCtl::Part* part,
                                                        unsigned long long deadline) {
  for (int spin = 0; spin < (1 << 20); ++spin) {
    const int r = dyn_take(dc, qbase, qx, 2u, 3u);
    if (r >= 0) return r;
    int stop = 0;
    if ((threadIdx.x & (kWave - 1)) == 0)
      stop = wall_clock64() >= deadline || (dyn_ld(&part->busy) == 0 && dyn_ld(&part->avail) == 0);
    if (__shfl(stop, 0, kWave)) return -1;
    __builtin_amdgcn_s_sleep(16);
  }
  return -1;
}

template <int M, int NJ>
__device__ inline void front_dyn(const PfspFrontArgs<M, NJ>& a, FrontSmem<M, NJ>& sm, const IterView& v, int t, int best0) {
  using G = FrontGeom<M, NJ>;
  using Node = PfspFrontNode<M, NJ>;
  constexpr int NW = G::NW;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  const int ch = static_cast<int>(blockIdx.x);  // v.nchunks == gridDim.x: chunk ch is workgroup ch's stack
  Node* const stk = pa.buf[(t & 1) ^ 1] + static_cast<size_t>(ch) * G::SLOT;
  // partition state (wave 0 only): the XCD's queue slots and counters
  auto qslot = [&](int q) {
    const int xcc = static_cast<int>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) & 7;  // HW_REG_XCC_ID
    return xcc * (v.qn / 8) + q;
  };
  auto part = [&]() -> DynCtl::Part& {
    return pa.dyn[t % 3].part[static_cast<int>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) & 7];
  };
  // slot q of the partition: the output chunk region nchunks + the slot's queue index
  auto region = [&](int q) { return pa.buf[(t & 1) ^ 1] + static_cast<size_t>(v.nchunks + qslot(q)) * G::SLOT; };
  if (tid == 0) {
    sm.dyn.deadline = wall_clock64() + static_cast<u64>(pa.dyn_ticks);  // the budget runs from this start
    sm.dyn.inner = 0;
    sm.dyn.claim = -1;
    sm.dyn.idle = 0;
    sm.dyn.pad = 0;  // (probe: steps | donations << 10 | claims << 20)
    sm.dyn.idle_ticks = 0;
    dyn_add(&part().busy, 1);
  }
  // the stack is stk[base, top): pushes and pops at the top, donations take the bottom
  // (the oldest, shallowest nodes: the largest subtrees, ref steal-half from the pool's
  // bottom, pfsp_multigpu_cuda.c:369-372); the top nst nodes are held in LDS
  int base = 0, top = 0, nst = 0, best = best0, nleaf = 0;
  for (int s = 0;; ++s) {
    uint32_t w[NW], rp[G::HW];
    bool have_r = false;
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = 0;
    if (s == 0) {
      const u64 gi = static_cast<u64>(ch) + static_cast<u64>(tid) * static_cast<u64>(v.nchunks);
      if (tid < v.bp && gi < v.B) front_load<M, NJ>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, gi, sm.pool), w);
    } else {
      const int npop = min(top - base, kBlock);
      if (tid < npop) {
        const int k = tid - (npop - nst);
        if (k >= 0) {
#pragma unroll
          for (int q = 0; q < G::VPN; ++q) {
            const uint4 x = sm.stage[k][q];
            w[4 * q] = x.x;
            w[4 * q + 1] = x.y;
            w[4 * q + 2] = x.z;
            w[4 * q + 3] = x.w;
          }
#pragma unroll
          for (int h = 0; h < G::HW; ++h) rp[h] = sm.stage_r[k][h];
          have_r = true;
        } else {
          front_load<M, NJ>(stk + (top - npop + tid), w);
        }
      }
      top -= npop;
      if (tid == 0) sm.dyn.inner += npop;
    }
    // the partition's demand and the incumbent, requested now and read after the step
    // (their round trips overlap the step instead of following it)
    u64 q_ha = 0;  // hungry | avail << 32
    if (tid == 0) q_ha = __hip_atomic_load(reinterpret_cast<u64*>(&part().hungry), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    typename G::Mask surv = 0;
    int nsurv = 0;
    const bool leaf = static_cast<int>(w[0] & 0xffu) + 1 == a.jobs;
    if (!have_r) front_remain<M, NJ>(sm, w, rp);
    front_parent_r<M, NJ>(
        a, sm, w, rp,
        [&](int j, int lb) {
          if (leaf) {
            ++nleaf;
            if (lb < best) atomicMin(&pa.ctl->best.v, lb);
          } else if (lb < best) {
            ++nsurv;
            surv |= static_cast<typename G::Mask>(1) << j;
          }
        },
        kDbgDyn);
    int tot = 0;
    const int off = block_exclusive_scan(nsurv, sm.scan, &tot);
    const int tnew = top + tot;
    nst = min(tot, min(tnew - base, kBlock));  // the next pop stays in LDS
    const int lo = tot - nst;
    uint4* const dst = reinterpret_cast<uint4*>(stk + top);
    front_emit_to<M, NJ>(sm, w, surv, [&](int i, const uint32_t (&c)[NW], int j) {
      const int o = off + i;
      if (o >= lo) {
        front_store<M, NJ>(&sm.stage[o - lo][0], c);
        const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[j]);
#pragma unroll
        for (int h = 0; h < G::HW; ++h) sm.stage_r[o - lo][h] = rp[h] - row[h];
      } else {
        front_store<M, NJ>(dst + o * G::VPN, c);
      }
    });
    top = tnew;
    // wave 0 decides what follows: stop at the deadline; publish the bottom half of the
    // stack (up to a slot region's worth below the LDS-held top) when partition
    // workgroups wait for more blocks than are full, or when the stack nears its end
    if (tid < kWave) {
      int flags = 0, dslot = -1;
      if (tid == 0 && wall_clock64() >= sm.dyn.deadline) flags = 1;
      flags = __shfl(flags, 0, kWave);
      if (!flags && top - base >= kDynMinDonate) {
        const int q_h = static_cast<int>(static_cast<uint32_t>(q_ha)), q_a = static_cast<int>(q_ha >> 32);
        const int want = __shfl(tid == 0 ? static_cast<int>(q_h > q_a || top + kBlock * (G::NJ - 1) > G::SLOT) : 0, 0,
                                kWave);
        if (want) {
          const int r = dyn_take(pa.dyn + t % 3, qslot(0), v.qn / 8, 0u, 1u);
          dslot = r < 0 ? -1 : (r & 0xffff);
        }
      }
      if (tid == 0) {
        sm.dyn.flags = flags;
        sm.dyn.dslot = dslot;
        // the incumbent, every 8th step (other workgroups' leaves lower it: -u 0)
        sm.dyn.best = (s & 7) == 7 ? __hip_atomic_load(&pa.ctl->best.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : best;
      }
    }
    __syncthreads();  // pushes visible to the next pops; decisions in sm.dyn
    if (s < 4) front_stamp(a, 4 + s);
    best = min(best, sm.dyn.best);
    const int dslot = sm.dyn.dslot;
    if (dslot >= 0) {
      // the bottom half; when the LDS-held top reaches into it, the stage goes to the
      // stack first (its place in the region is free: pops and pushes at the top)
      const int n = min((top - base) / 2, G::SLOT);
      if (base + n > top - nst) {
        if (tid < nst) {
          uint32_t x[NW];
#pragma unroll
          for (int q = 0; q < G::VPN; ++q) {
            const uint4 y = sm.stage[tid][q];
            x[4 * q] = y.x;
            x[4 * q + 1] = y.y;
            x[4 * q + 2] = y.z;
            x[4 * q + 3] = y.w;
          }
          front_store<M, NJ>(reinterpret_cast<uint4*>(stk + (top - nst + tid)), x);
        }
        nst = 0;
        __syncthreads();
      }
      dyn_copy<M, NJ>(stk + base, region(dslot), n, 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its payload is complete
      __syncthreads();
      if (tid == 0) {
        dyn_stu_rel(&pa.dyn[t % 3].st[qslot(dslot)], 2u | (static_cast<unsigned>(n) << 8));
        dyn_add(&part().avail, 1);
        sm.dyn.pad += 1 << 10;
      }
      base += n;
    }
    if (tid == 0) sm.dyn.pad += 1;
    if (sm.dyn.flags) break;
    if (top + kBlock * (G::NJ - 1) > G::SLOT) {
      // a full pop could overflow the region: move the stack down to its start
      if (base == 0) break;
      const int n = top - nst - base;  // (the LDS-held top moves with top)
      for (int c = 0; c < n; c += base) {
        dyn_copy_own<M, NJ>(stk + base + c, stk + c, min(base, n - c));
        __syncthreads();
      }
      top -= base;
      base = 0;
      if (top + kBlock * (G::NJ - 1) > G::SLOT) break;
    }
    if (top == base) {
      // stack dry: claim a published block of the partition (wave 0; the others wait)
      if (tid < kWave) {
        const u64 t_idle = wall_clock64();
        if (tid == 0 && !sm.dyn.idle) {
          dyn_add(&part().busy, -1);
          dyn_add(&part().hungry, 1);
          sm.dyn.idle = 1;
        }
        const int r = dyn_claim_spin(pa.dyn + t % 3, qslot(0), v.qn / 8, &part(), sm.dyn.deadline);
        if (tid == 0 && r >= 0) {
          dyn_add(&part().busy, 1);
          dyn_add(&part().hungry, -1);
          dyn_add(&part().avail, -1);
          sm.dyn.idle = 0;
          sm.dyn.pad += 1 << 20;
        }
        if (tid == 0) {
          sm.dyn.claim = r;
          sm.dyn.idle_ticks += wall_clock64() - t_idle;
        }
      }
      __syncthreads();
      const int r = sm.dyn.claim;
      if (r < 0) break;
      // the block becomes this workgroup's stack
      const int q = r & 0xffff, n = r >> 16;
      dyn_copy<M, NJ>(region(q), stk, n, 2);
      __syncthreads();  // the block is read (and the copy visible to the next pops)
      if (tid == 0) dyn_stu_rel(&pa.dyn[t % 3].st[qslot(q)], 0u);
      base = 0;
      top = n;
      nst = 0;
    }
  }
  // the nodes staged for a next step are the top of the stack; then the stack moves to
  // the start of the region (the chunk's output)
  if (tid < nst) {
    uint32_t x[NW];
#pragma unroll
    for (int q = 0; q < G::VPN; ++q) {
      const uint4 y = sm.stage[tid][q];
      x[4 * q] = y.x;
      x[4 * q + 1] = y.y;
      x[4 * q + 2] = y.z;
      x[4 * q + 3] = y.w;
    }
    front_store<M, NJ>(reinterpret_cast<uint4*>(stk + (top - nst + tid)), x);
  }
  __syncthreads();
  if (base > 0) {
    const int n = top - base;
    for (int c = 0; c < n; c += base) {
      dyn_copy_own<M, NJ>(stk + base + c, stk + c, min(base, n - c));
      __syncthreads();
    }
  }
  int leaves = 0;
  (void)block_exclusive_scan(nleaf, sm.scan, &leaves);
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  if (tid == 0) {
    dyn_add(sm.dyn.idle ? &part().hungry : &part().busy, -1);
    cnt_out[ch] = top - base;
    lcnt_out[ch] = 0;
    auto& x = pa.ctl->xacc[ch & 7];
    const long long inner = sm.dyn.inner;
    if (inner) __hip_atomic_fetch_add(&x.tree, static_cast<u64>(inner), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (leaves) __hip_atomic_fetch_add(&x.sol, static_cast<u64>(leaves), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.dbg_blk) {
      a.dbg_blk[blockIdx.x * 16 + 14] = static_cast<unsigned long long>(inner) |
                                        (static_cast<unsigned long long>(top - base) << 32);
      a.dbg_blk[blockIdx.x * 16 + 9] = static_cast<unsigned long long>(static_cast<unsigned>(sm.dyn.pad));
      a.dbg_blk[blockIdx.x * 16 + 10] = sm.dyn.idle_ticks;
    }
    // the last workgroup out (every slot state final) writes the queue chunks' counts
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DynCtl* const dc = pa.dyn + t % 3;
    const int g = ch & 7;
    const int gs = (static_cast<int>(gridDim.x) - g + 7) / 8;
    int sweep = 0;
    if (dyn_add(&dc->fin[g].n, 1) == gs - 1)
      sweep = dyn_add(&dc->fin[8].n, 1) == min(8, static_cast<int>(gridDim.x)) - 1;
    sm.dyn.sweep = sweep;
  }
  __syncthreads();
  if (sm.dyn.sweep) {
    DynCtl* const dc = pa.dyn + t % 3;
    for (int q = tid; q < v.qn; q += kBlock) {
      const unsigned sv = dyn_ldu(&dc->st[q]);
      cnt_out[v.nchunks + q] = (sv & 3u) == 2u ? static_cast<int>(sv >> 8) : 0;
      lcnt_out[v.nchunks + q] = 0;
    }
  }
}

// One B&B iteration on the device-resident pool (pool_device.hpp); t in [0, 6): state
// slot t % 3, buffer parity t % 2.
//
// Occupancy: the iterations are latency-bound (the per-child chain, LDS row reads), so
// the register budget is capped for more resident waves: 6 per SIMD up to 10 machines,
// 4 for 20 (f, remain and a p row stay in registers without scratch); the engine's grid
// holds FrontGeom::GRID_WGS workgroups per CU (5 of the 6 up to 10 machines). (Compiled for 7 — 94 SGPRs, 72 spilled to VGPR
// lanes — the headline was 3 % slower than at 6.)
template <int M, int NJ = 20>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FrontGeom<M, NJ>::WAVES)))
void pfsp_front_kernel(PfspFrontArgs<M, NJ> a, int t) {
  using G = FrontGeom<M, NJ>;
  using Node = PfspFrontNode<M, NJ>;
  __shared__ FrontSmem<M, NJ> sm;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  front_stamp(a, 0);
  // p table loads issued together with pool_begin's (one memory round trip)
  constexpr int PTN = (G::NJ * G::MS + kBlock - 1) / kBlock;
  uint16_t ptv[PTN];
#pragma unroll
  for (int i = 0; i < PTN; ++i) {
    const int x = tid + i * kBlock;
    ptv[i] = x < a.jobs * G::MS ? a.ptab[x] : 0;
  }
  const IterView v =
      pool_begin<Node, G::MAXCHUNKS>(pa, t, G::BP, sm.pool, a.bpf, G::LT, G::NJ * (G::NJ - 1), G::LMAX, true);
  front_stamp(a, 1);
  if (v.B == 0 || v.overflow) return;
  {
    uint16_t* pt = &sm.ptab[0][0];
#pragma unroll
    for (int i = 0; i < PTN; ++i)
      if (tid + i * kBlock < G::NJ * G::MS) pt[tid + i * kBlock] = ptv[i];
  }
  const int best = prune_best(pa, v);
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  pool_spill_leftovers<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, sm.pool);
  __syncthreads();
  front_stamp(a, 2);
  if (v.dyn) {
    front_dyn<M, NJ>(a, sm, v, t, best);
    front_stamp(a, 15);
    return;
  }
  if (v.local) {
    front_local<M, NJ>(a, sm, v, t, best);
    front_stamp(a, 15);
    return;
  }
  if (v.fused) {
    front_multi_level<M, NJ>(a, sm, v, t, best);
    return;
  }
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    const u64 gi = static_cast<u64>(ch) * G::BP + tid;
    uint32_t w[G::NW];
#pragma unroll
    for (int i = 0; i < G::NW; ++i) w[i] = 0;
    if (gi < v.B) front_load<M, NJ>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, gi, sm.pool), w);
    const bool first = ch == static_cast<int>(blockIdx.x);
    const bool leaf = static_cast<int>(w[0] & 0xffu) + 1 == a.jobs;
    // children this rank keeps (all of them outside the split iteration)
    using Mask = typename G::Mask;
    Mask kmask = ~Mask(0);
    if (v.split) {
      kmask = 0;
      for (Mask x = front_mask<M, NJ>(w); x; x &= x - 1) {
        const int j = mask_ctz(x);
        kmask |= split_keep(v, gi, j) ? (Mask(1) << j) : Mask(0);
      }
    }
    Mask surv = 0;
    int nsurv = 0, nleaf = 0;
    front_parent<M, NJ>(
        a, sm, w,
        [&](int j, int lb) {
          const bool keep = (kmask >> j) & Mask(1);
          if (leaf) {
            nleaf += keep;
            if (lb < best) atomicMin(&pa.ctl->best.v, lb);
          } else if (keep && lb < best) {
            ++nsurv;
            surv |= static_cast<typename G::Mask>(1) << j;
          }
        },
        v.split ? kDbgSplit : kDbgOne);
    if (first) front_stamp(a, 4);
    // one scan for both counts: survivors (<= 256 x 19) in bits 0-12, leaves (<= 256)
    // in bits 13-21
    int tot = 0;
    const int off = block_exclusive_scan(nsurv | (nleaf << 13), sm.scan, &tot) & 0x1fff;
    if (tid == 0) {
      cnt_out[ch] = tot & 0x1fff;
      lcnt_out[ch] = (tot >> 13) & 0x1ff;
    }
    if (first) front_stamp(a, 5);
    front_emit<M, NJ>(sm, w, surv, reinterpret_cast<uint4*>(bout + static_cast<size_t>(ch) * G::SLOT + off));
    if (first) front_stamp(a, 6);
  }
  front_stamp(a, 15);
}

// Reference-style evaluation for the tests (ref evaluate_gpu, PFSP_gpu_lib.cu:129-152):
// bounds of every child of every parent, in ascending job order per parent.
template <int M, int NJ = 20>
__global__ __launch_bounds__(kBlock) void pfsp_front_bounds_kernel(PfspFrontArgs<M, NJ> a) {
  using G = FrontGeom<M, NJ>;
  __shared__ FrontSmem<M, NJ> sm;
  uint16_t* pt = &sm.ptab[0][0];
  for (int i = threadIdx.x; i < a.jobs * G::MS; i += kBlock) pt[i] = a.ptab[i];
  __syncthreads();
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < a.nparents; i += gridDim.x * kBlock) {
    uint32_t w[G::NW];
    front_load<M, NJ>(a.parents_in + i, w);
    using Mask = typename G::Mask;
    const Mask rest = front_mask<M, NJ>(w);
    int* out = a.bounds_out + a.offsets[i];
    front_parent<M, NJ>(a, sm, w, [&](int j, int lb) { out[mask_pop(rest & ((Mask(1) << j) - Mask(1)))] = lb; });
  }
}

}  // namespace dev
}  // namespace tts
