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

template <int M>
struct FrontGeom {
  using Node = PfspFrontNode<M>;
  static constexpr int NJ = 20;                         // at most 20 children per parent (20-job bucket)
  static constexpr int NW = sizeof(Node) / 4;           // node words in registers (8 or 12)
  static constexpr int VPN = sizeof(Node) / 16;         // 16-B vectors per node
  static constexpr int BP = 256;                        // parents per chunk: one per thread
  static constexpr int MAXCH = BP * NJ;                 // children per chunk (upper bound)
  static constexpr int LT = 8;                          // local DFS steps per chunk at most
  static constexpr int SLOT = 2 * MAXCH;                // chunk slot region = its private stack
  static constexpr int MAXCHUNKS = 2048;
  // two-level chunks (front_two_level_cp): up to BPF_CP parents, spread over the grid
  // (pool_begin); level-1 survivors past kBlock go out unexpanded, so the chunk's output
  // stays within SLOT
  static constexpr int BPF = 12;     // default cap: two-level windows up to 12 x 2048 parents
  static constexpr int BPF_CP = 32;
  static constexpr int MID = M > 10 ? 96 : 128;  // level-1 survivors expanded in place (the rest go out)
  static constexpr int HW = (M + 1) / 2;  // packed u16 pairs of a p row / a remain
  // u16 row stride of the LDS p table (as PfspConsts::MS): 16 B for M <= 8, else 48 B
  static constexpr int MS = M <= 8 ? 8 : 24;
  static constexpr int RV = (M + 7) / 8;                // 16-B vectors holding one row's M values
};

template <int M>
struct PfspFrontArgs {
  PoolArgs<PfspFrontNode<M>> pool;
  const uint16_t* ptab;  // job-major p, [jobs][MS], padded machines 0
  int jobs;
  int min_tails[M];      // padded machines: 0
  // bounds kernel only (tests): bounds of parent i's children at bounds_out[offsets[i] + rank of
  // the job among the parent's unscheduled jobs]
  const PfspFrontNode<M>* parents_in;
  const int* offsets;
  int* bounds_out;
  int nparents;
  int bpf;  // two-level chunks: at most this many parents (<= FrontGeom::BPF_CP)
};

template <int M>
struct FrontSmem {
  using G = FrontGeom<M>;
  uint16_t ptab[G::NJ][G::MS];
  int scan[kBlock / kWave];
  // two-level chunks (child-parallel expansion): the chunk's parents and the level-1
  // survivors expanded in place, each with its remain (unscheduled work per machine,
  // packed u16 pairs), and the child offsets of the nodes being expanded
  uint4 par[G::BPF_CP][G::VPN];
  uint32_t rpar[G::BPF_CP][G::HW];
  uint4 mid[G::MID][G::VPN];
  uint32_t rmid[G::MID][G::HW];
  int coff[G::MID];
  PoolSmem<G::MAXCHUNKS> pool;
};

template <int M>
__device__ inline void front_row(const uint16_t* row, int (&pr)[M]) {
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
#pragma unroll
  for (int q = 0; q < FrontGeom<M>::RV; ++q) {
    const uint4 x = r4[q];
    const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int h = 0; h < 8; ++h)
      if (q * 8 + h < M) pr[q * 8 + h] = static_cast<int>((wv[h >> 1] >> ((h & 1) * 16)) & 0xffffu);
  }
}

template <int M>
__device__ inline int front_of(const uint32_t (&w)[FrontGeom<M>::NW], int m) {
  return static_cast<int>((w[2 + (m >> 1)] >> ((m & 1) * 16)) & 0xffffu);
}

template <int M>
__device__ inline void front_load(const PfspFrontNode<M>* src, uint32_t (&w)[FrontGeom<M>::NW]) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int q = 0; q < FrontGeom<M>::VPN; ++q) {
    const uint4 x = s[q];
    w[4 * q] = x.x;
    w[4 * q + 1] = x.y;
    w[4 * q + 2] = x.z;
    w[4 * q + 3] = x.w;
  }
}

template <int M>
__device__ inline void front_store(uint4* dst, const uint32_t (&c)[FrontGeom<M>::NW]) {
#pragma unroll
  for (int q = 0; q < FrontGeom<M>::VPN; ++q) dst[q] = make_uint4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
}

// Bounds of every child of the parent held in w: emit(j, lb) for each unscheduled job j.
template <int M, class Emit>
__device__ inline void front_parent(const PfspFrontArgs<M>& a, const FrontSmem<M>& sm,
                                    const uint32_t (&w)[FrontGeom<M>::NW], Emit emit) {
  const uint32_t rest = w[1];
  int f[M], r[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    f[m] = front_of<M>(w, m);
    r[m] = a.min_tails[m];
  }
  for (uint32_t x = rest; x; x &= x - 1) {
    int pr[M];
    front_row<M>(sm.ptab[__builtin_ctz(x)], pr);
#pragma unroll
    for (int m = 0; m < M; ++m) r[m] += pr[m];
  }
  for (uint32_t x = rest; x; x &= x - 1) {
    const int j = __builtin_ctz(x);
    int pr[M];
    front_row<M>(sm.ptab[j], pr);
    int lb = f[0] + r[0];
    int tt = f[0] + pr[0];
#pragma unroll
    for (int m = 1; m < M; ++m) {
      const int sv = max(tt, f[m]);
      lb = max(lb, sv + r[m]);
      tt = sv + pr[m];
    }
    emit(j, lb);
  }
}

// Child of the parent in w that appends job j: depth + 1, j removed from the set, and
// its front (the chain from the parent's front; from 0 at the root).
template <int M>
__device__ inline void front_child(const FrontSmem<M>& sm, const uint32_t (&w)[FrontGeom<M>::NW], int j,
                                   uint32_t (&c)[FrontGeom<M>::NW]) {
  constexpr int NW = FrontGeom<M>::NW;
  const int d = static_cast<int>(w[0] & 0xffu);
  const bool root = d == 0;
  int pr[M];
  front_row<M>(sm.ptab[j], pr);
  c[0] = static_cast<uint32_t>(d + 1);
  c[1] = w[1] & ~(1u << j);
#pragma unroll
  for (int i = 2; i < NW; ++i) c[i] = 0;
  int ft = (root ? 0 : front_of<M>(w, 0)) + pr[0];
  c[2] = static_cast<uint32_t>(ft);
#pragma unroll
  for (int m = 1; m < M; ++m) {
    ft = max(ft, root ? 0 : front_of<M>(w, m)) + pr[m];
    c[2 + (m >> 1)] |= static_cast<uint32_t>(ft) << ((m & 1) * 16);
  }
}

template <int M>
__device__ inline void front_emit(const FrontSmem<M>& sm, const uint32_t (&w)[FrontGeom<M>::NW], uint32_t surv,
                                  uint4* dst) {
  while (surv) {
    const int j = __builtin_ctz(surv);
    surv &= surv - 1;
    uint32_t c[FrontGeom<M>::NW];
    front_child<M>(sm, w, j, c);
    front_store<M>(dst, c);
    dst += FrontGeom<M>::VPN;
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

// Child-parallel expansion of n nodes staged in LDS (src[i], with their remain
// rem[i]): ONE THREAD PER CHILD instead of one per parent. In a narrow window a
// thread-per-parent expansion runs its parent's ~20 children one after the other while
// most lanes idle; here child c finds its parent (binary search on the child offsets)
// and its job (k-th unscheduled bit), then bounds itself from the parent's front and
// remain (no pass over the parent's rows: remains are carried, a child's is its
// parent's minus its own row). Leaves lower the incumbent and are counted in nleaf;
// survivors are compacted (block scan) and handed to store(index, child words, child
// remain). Returns the survivor count. Every thread calls it (block-wide scans).
template <int M, class Store>
__device__ inline int front_expand_cp(const PfspFrontArgs<M>& a, FrontSmem<M>& sm, const uint4 (*src)[FrontGeom<M>::VPN],
                                      const uint32_t (*rem)[FrontGeom<M>::HW], int n, int best, int& nleaf, Store store) {
  using G = FrontGeom<M>;
  constexpr int HW = G::HW;
  const int tid = threadIdx.x;
  int T = 0;
  const int off = block_exclusive_scan(tid < n ? __popc(src[tid][0].y) : 0, sm.scan, &T);
  if (tid < n) sm.coff[tid] = off;
  __syncthreads();
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
      j = kth_bit(w[1], c - sm.coff[lo]);
      const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[j]);
      uint32_t pw[HW];
#pragma unroll
      for (int h = 0; h < HW; ++h) {
        pw[h] = row[h];
        cr[h] = rem[lo][h] - pw[h];  // the child's remain (packed halves never borrow: row <= remain)
      }
      auto pm = [&](int m) { return static_cast<int>((pw[m >> 1] >> ((m & 1) * 16)) & 0xffffu); };
      auto rm = [&](int m) { return static_cast<int>((rem[lo][m >> 1] >> ((m & 1) * 16)) & 0xffffu) + a.min_tails[m]; };
      const int f0 = front_of<M>(w, 0);
      int lb = f0 + rm(0);
      int tt = f0 + pm(0);
#pragma unroll
      for (int m = 1; m < M; ++m) {
        const int sv = max(tt, front_of<M>(w, m));
        lb = max(lb, sv + rm(m));
        tt = sv + pm(m);
      }
      if (static_cast<int>(w[0] & 0xffu) + 1 == a.jobs) {
        ++nleaf;
        if (lb < best) atomicMin(&a.pool.ctl->best.v, lb);
      } else {
        surv = lb < best;
      }
    }
    int tot = 0;
    const int idx = nout + block_exclusive_scan(surv ? 1 : 0, sm.scan, &tot);
    if (surv) {
      uint32_t cw[G::NW];
      front_child<M>(sm, w, j, cw);
      store(idx, cw, cr);
    }
    nout += tot;
  }
  return nout;
}

// Two-level chunk, child-parallel (default): the chunk's v.bp parents go to LDS, their
// children are expanded one per thread into sm.mid, then the survivors' children one
// per thread into the chunk's slot region. Same counts as front_two_level: level-1
// survivors expanded here are pushed-and-expanded tree nodes (high half of the leaf
// word); level-1 survivors beyond sm.mid's kBlock nodes go out unexpanded (first in the
// slot region) with the level-2 survivors as the chunk's output.
template <int M>
__device__ inline void front_two_level_cp(const PfspFrontArgs<M>& a, FrontSmem<M>& sm, const IterView& v, int t,
                                          int best) {
  using G = FrontGeom<M>;
  using Node = PfspFrontNode<M>;
  static_assert(G::BPF_CP * (G::NJ - 1) + G::MID * (G::NJ - 1) <= G::SLOT, "chunk output must fit its slot region");
  static_assert(G::MID <= kBlock && G::BPF_CP <= kBlock, "one thread per staged node");
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    const u64 g0 = static_cast<u64>(ch) * v.bp;
    const int n0 = static_cast<int>(min(static_cast<u64>(v.bp), v.B - g0));
    if (tid < n0) {
      // the parent's remain: one pass over its unscheduled rows (packed u16 pairs; sums
      // < 65536, pfsp_front_ok), by the thread that stages it
      uint32_t w[G::NW];
      front_load<M>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, g0 + tid, sm.pool), w);
      front_store<M>(&sm.par[tid][0], w);
      uint32_t r2[G::HW];
#pragma unroll
      for (int h = 0; h < G::HW; ++h) r2[h] = 0;
      for (uint32_t x = w[1]; x; x &= x - 1) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(sm.ptab[__builtin_ctz(x)]);
#pragma unroll
        for (int h = 0; h < G::HW; ++h) r2[h] += row[h];
      }
#pragma unroll
      for (int h = 0; h < G::HW; ++h) sm.rpar[tid][h] = r2[h];
    }
    __syncthreads();
    int nleaf = 0;
    uint4* const out = reinterpret_cast<uint4*>(bout + static_cast<size_t>(ch) * G::SLOT);
    const int n1 = front_expand_cp<M>(a, sm, sm.par, sm.rpar, n0, best, nleaf,
                                      [&](int i, const uint32_t (&c)[G::NW], const uint32_t (&r)[G::HW]) {
                                        if (i < G::MID) {
                                          front_store<M>(&sm.mid[i][0], c);
#pragma unroll
                                          for (int h = 0; h < G::HW; ++h) sm.rmid[i][h] = r[h];
                                        } else {
                                          front_store<M>(out + (i - G::MID) * G::VPN, c);  // out unexpanded
                                        }
                                      });
    __syncthreads();  // level-1 survivors visible
    const int n1e = min(n1, G::MID), ovf = n1 - n1e;
    const int n2 = front_expand_cp<M>(a, sm, sm.mid, sm.rmid, n1e, best, nleaf,
                                      [&](int i, const uint32_t (&c)[G::NW], const uint32_t (&)[G::HW]) {
                                        front_store<M>(out + (ovf + i) * G::VPN, c);
                                      });
    int leaves = 0;
    (void)block_exclusive_scan(nleaf, sm.scan, &leaves);
    if (tid == 0) {
      cnt_out[ch] = ovf + n2;
      lcnt_out[ch] = leaves | (n1e << 16);
    }
    __syncthreads();  // sm.par / sm.mid / sm.coff are rewritten by the next chunk
  }
}

// Local DFS chunk loop (v.local): chunk ch takes v.bp window parents, then keeps
// popping up to kBlock nodes from the top of its own slot region (a private stack,
// written by this workgroup only) and pushing their survivors there, for up to
// v.steps steps or until the stack is empty. The stack left is the chunk's output
// (cnt); nodes pushed and expanded in between are explored tree nodes (high half of
// the leaf word). Pops read slots [top - n, top) and pushes write from top - n on:
// every pop is in registers before the scan's barrier that precedes the first push.
template <int M>
__device__ inline void front_local(const PfspFrontArgs<M>& a, FrontSmem<M>& sm, const IterView& v, int t, int best) {
  using G = FrontGeom<M>;
  using Node = PfspFrontNode<M>;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    Node* const stk = bout + static_cast<size_t>(ch) * G::SLOT;
    int top = 0, pushed = 0, nleaf = 0;
    for (int s = 0; s < v.steps; ++s) {
      uint32_t w[G::NW];
#pragma unroll
      for (int i = 0; i < G::NW; ++i) w[i] = 0;
      if (s == 0) {
        const u64 gi = static_cast<u64>(ch) * v.bp + tid;
        if (tid < v.bp && gi < v.B) front_load<M>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, gi, sm.pool), w);
      } else {
        if (top == 0) break;  // uniform
        const int npop = min(top, kBlock);
        if (tid < npop) front_load<M>(stk + (top - npop + tid), w);
        top -= npop;
      }
      uint32_t surv = 0;
      int nsurv = 0;
      const bool leaf = static_cast<int>(w[0] & 0xffu) + 1 == a.jobs;
      front_parent<M>(a, sm, w, [&](int j, int lb) {
        if (leaf) {
          ++nleaf;
          if (lb < best) atomicMin(&pa.ctl->best.v, lb);
        } else if (lb < best) {
          ++nsurv;
          surv |= 1u << j;
        }
      });
      int tot = 0;
      const int off = block_exclusive_scan(nsurv, sm.scan, &tot);
      front_emit<M>(sm, w, surv, reinterpret_cast<uint4*>(stk + top + off));
      top += tot;
      pushed += tot;
      // pushes visible to the next step's pops (workgroup scope), and room left for
      // one more full step
      __syncthreads();
      if (top + kBlock * G::NJ > G::SLOT || top > v.cap) break;
    }
    int leaves = 0;
    (void)block_exclusive_scan(nleaf, sm.scan, &leaves);
    if (tid == 0) {
      cnt_out[ch] = top;
      lcnt_out[ch] = leaves | ((pushed - top) << 16);
    }
  }
}

// One B&B iteration on the device-resident pool (pool_device.hpp); t in [0, 6): state
// slot t % 3, buffer parity t % 2.
//
// Occupancy: the iterations are latency-bound (the per-child chain, LDS row reads), so
// the register budget is capped for more resident waves: 6 per SIMD up to 10 machines,
// 4 for 20 (f, remain and a p row stay in registers without scratch).
// (8 waves per SIMD for M <= 10, SGPRs spilled to VGPR lanes, measured: ta014 +2 %,
// ta008 -4 %; not kept, profiles/r3/probes/front_w8_ab.txt)
template <int M>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(M <= 10 ? 6 : 4)))
void pfsp_front_kernel(PfspFrontArgs<M> a, int t) {
  using G = FrontGeom<M>;
  using Node = PfspFrontNode<M>;
  __shared__ FrontSmem<M> sm;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  // p table loads issued together with pool_begin's (one memory round trip)
  constexpr int PTN = (G::NJ * G::MS + kBlock - 1) / kBlock;
  uint16_t ptv[PTN];
#pragma unroll
  for (int i = 0; i < PTN; ++i) {
    const int x = tid + i * kBlock;
    ptv[i] = x < a.jobs * G::MS ? a.ptab[x] : 0;
  }
  const IterView v = pool_begin<Node, G::MAXCHUNKS>(pa, t, G::BP, sm.pool, a.bpf, G::LT, G::NJ * (G::NJ - 1));
  if (v.B == 0 || v.overflow) return;
  {
    uint16_t* pt = &sm.ptab[0][0];
#pragma unroll
    for (int i = 0; i < PTN; ++i)
      if (tid + i * kBlock < G::NJ * G::MS) pt[tid + i * kBlock] = ptv[i];
  }
  const int best = __hip_atomic_load(&pa.ctl->best.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  pool_spill_leftovers<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, sm.pool);
  __syncthreads();
  if (v.local) {
    front_local<M>(a, sm, v, t, best);
    return;
  }
  if (v.fused) {
    front_two_level_cp<M>(a, sm, v, t, best);
    return;
  }
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    const u64 gi = static_cast<u64>(ch) * G::BP + tid;
    uint32_t w[G::NW];
#pragma unroll
    for (int i = 0; i < G::NW; ++i) w[i] = 0;
    if (gi < v.B) front_load<M>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, gi, sm.pool), w);
    const bool leaf = static_cast<int>(w[0] & 0xffu) + 1 == a.jobs;
    // children this rank keeps (all of them outside the split iteration)
    uint32_t kmask = ~0u;
    if (v.split) {
      kmask = 0;
      for (uint32_t x = w[1]; x; x &= x - 1) {
        const int j = __builtin_ctz(x);
        kmask |= split_keep(v, gi, j) ? (1u << j) : 0u;
      }
    }
    uint32_t surv = 0;
    int nsurv = 0, nleaf = 0;
    front_parent<M>(a, sm, w, [&](int j, int lb) {
      const bool keep = (kmask >> j) & 1u;
      if (leaf) {
        nleaf += keep;
        if (lb < best) atomicMin(&pa.ctl->best.v, lb);
      } else if (keep && lb < best) {
        ++nsurv;
        surv |= 1u << j;
      }
    });
    // one scan for both counts: survivors (<= 256 x 19) in bits 0-12, leaves (<= 256)
    // in bits 13-21
    int tot = 0;
    const int off = block_exclusive_scan(nsurv | (nleaf << 13), sm.scan, &tot) & 0x1fff;
    if (tid == 0) {
      cnt_out[ch] = tot & 0x1fff;
      lcnt_out[ch] = (tot >> 13) & 0x1ff;
    }
    front_emit<M>(sm, w, surv, reinterpret_cast<uint4*>(bout + static_cast<size_t>(ch) * G::SLOT + off));
  }
}

// Reference-style evaluation for the tests (ref evaluate_gpu, PFSP_gpu_lib.cu:129-152):
// bounds of every child of every parent, in ascending job order per parent.
template <int M>
__global__ __launch_bounds__(kBlock) void pfsp_front_bounds_kernel(PfspFrontArgs<M> a) {
  using G = FrontGeom<M>;
  __shared__ FrontSmem<M> sm;
  uint16_t* pt = &sm.ptab[0][0];
  for (int i = threadIdx.x; i < a.jobs * G::MS; i += kBlock) pt[i] = a.ptab[i];
  __syncthreads();
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < a.nparents; i += gridDim.x * kBlock) {
    uint32_t w[G::NW];
    front_load<M>(a.parents_in + i, w);
    const uint32_t rest = w[1];
    int* out = a.bounds_out + a.offsets[i];
    front_parent<M>(a, sm, w, [&](int j, int lb) { out[__popc(rest & ((1u << j) - 1u))] = lb; });
  }
}

}  // namespace dev
}  // namespace tts
