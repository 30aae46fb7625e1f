// PFSP search kernels for gfx950 (CDNA4).
//
// What the reference does (ref pfsp/lib/PFSP_gpu_lib.cu:43-152, bounds_gpu.cu):
// one thread per child (LB1/LB2) or per parent (LB1_d), each copying the 44-B node
// and 20-int arrays into scratch (176-256 B/lane spilled on gfx950), no LDS, a
// synchronous bounds round trip to the host, and child generation on the CPU.
//
// What happens here, per 256-thread workgroup and per chunk of BP parents:
//   Phase A  thread-per-parent: parent nodes -> LDS; the parent's schedule prefix is
//            replayed once (front[M] = completion times, remain[M] = unscheduled
//            work) from the LDS-staged job-major p table; both packed u16|u16 into
//            one LDS row per parent. Child counts are scanned across the workgroup
//            and a child->parent map is written to LDS.
//   Phase B  thread-per-child: LB1 (== LB1_d) costs O(M) per child from
//            the parent's LDS row. LB2 walks each machine pair's Johnson order with
//            wave-uniform records (one LDS broadcast per step) and a per-lane
//            scheduled-set bitmask, exiting a lane as soon as lb > best (ref
//            c_bound_johnson.c:211-237, same pair order => same prune decisions).
//   Phase C  (expand kernel) prune + stream compaction: one 64-bit ballot per wave
//            into an LDS bitmap, a popcount scan, then each survivor writes its
//            child node into the chunk's own slot region of the device pool and
//            the chunk publishes its survivor / leaf counts (pool_device.hpp: no
//            device atomics). Leaves lower the incumbent (atomicMin), exactly the
//            counting rules of ref PFSP_lib.h:51-95 (generate_children).
// Nothing returns to the host per iteration.
#pragma once

#include <climits>

#include "../core/pfsp_node.hpp"
#include "pool_device.hpp"

namespace tts {
namespace dev {

// Parents per chunk: LB1's per-child cost is O(M) so a chunk holds 256 parents;
// LB2's is O(M^2 N / 2): chunks shrink with the number of machine pairs so an
// iteration spreads over as many workgroups as the chip holds.
template <int NJ, int LBK = 1, int M = 20>
struct PfspGeom {
  static constexpr int BP1 = NJ <= 50 ? 256 : (NJ <= 100 ? 128 : (NJ <= 200 ? 64 : 32));
  // LB2: parallelism comes from (child, machine pair) tasks, so a chunk only needs
  // enough children to feed a workgroup; small chunks spread an iteration over
  // many workgroups and keep the per-chunk LDS (child fronts) small.
  static constexpr int NM = NJ * M;
  static constexpr int BP2 = NM <= 100 ? 64 :(NM <= 200 ? 16 : (NM <= 1000 ? 8 : 2));
  static constexpr int BP = LBK >= 2 ? BP2 : BP1;  // LBK 5 = LB2 with packed two-child walks
  // 50-job LB2 (NM 500..1000): 8-parent chunks, half as many per iteration (same
  // 16K-parent window, half the per-chunk barriers; the smaller chunk-count prefix
  // pays for the larger child arrays in LDS)
  static constexpr int MAXCHUNKS = LBK >= 2 ? (NM > 400 && NM <= 1000 ? 2048 : 4096) : 2048;
  static constexpr int MAXCH = BP * NJ;                  // children per chunk (upper bound)
  // local DFS steps per chunk and iteration (the LB1 register path only) and the
  // chunk's slot region in the children buffers = its private stack. Two chunks'
  // worth of children: a chunk keeps stepping while one more full expansion fits,
  // and the ring's worst-case growth per iteration (engine pick_graph) only doubles.
  static constexpr int LT = (LBK < 2 && sizeof(PfspNode<NJ>) == 32) ? 8 : 1;
  static constexpr int SLOT = MAXCH * (LT > 1 ? 2 : 1);
  static constexpr int NWORDS = (MAXCH + 63) / 64;       // survivor bitmap words
  static constexpr int NW = (NJ + 63) / 64;              // 64-bit words of a job set
  using map_t = std::conditional_t<(BP <= 256), uint8_t, uint16_t>;
  static_assert(NWORDS <= kBlock, "survivor bitmap scan assumes <= 256 words");
};

template <int M>
struct PfspConsts {
  static constexpr int P = M * (M - 1) / 2;
  // u16 row stride of the LDS p table: 16 B for M <= 8, else 48 B. A 48-B stride
  // (12 dwords) sends the 16 rows a ds_read_b128 lane group touches to 16
  // different bank quads; a 32-B stride would put rows j and j+8 on the same banks.
  static constexpr int MS = M <= 8 ? 8 : ((M + 7) & ~7) == 16 ? 24 : ((M + 7) & ~7);
  static constexpr int RV = (M + 7) / 8;   // 16-B vectors holding one row's M values
};

// Kernel arguments (by value -> kernarg segment -> SGPRs for the uniform tables).
template <int NJ, int M>
struct PfspArgs {
  PoolArgs<PfspNode<NJ>> pool;  // device-resident pool (pool_device.hpp)
  const uint16_t* ptab;    // job-major p, [jobs][MS]
  const uint2* recs;       // LB2 Johnson records, [P][jobs]: {job | p0<<16, p1 | lag<<16}
  const uint2* pinfo;      // LB2 pairs in evaluation order: {m0 | m1<<8 | recs pair<<16, tail0 | tail1<<16}
  const int* offsets;      // bounds kernel only: exclusive prefix of child counts
  int* bounds_out;         // bounds kernel only
  const PfspNode<NJ>* parents_in;  // bounds kernel only
  int jobs;
  int npairs;              // machine pairs of the instance (<= P: machines padded up to M, see pfsp_fill_args)
  int nparents;            // bounds kernel only
  int best_in;             // bounds kernel only
  int min_heads[M];
  int min_tails[M];
  int sum_all[M];
  uint8_t pm0[PfspConsts<M>::P];
  uint8_t pm1[PfspConsts<M>::P];
  // LB2 expand knob (after the tables so the LB1 kernels' argument layout is unchanged)
  int lb2_rounds;          // B2 in rounds of pairs, re-compacting the children still below best
  // element-wise probe of the expand kernels (tests): bound of every child of window
  // parent i at dbg_lb[dbg_off[i] + (k - depth)] (LB2: exact below best, else >= best;
  // LB1 / LB1_d: exact)
  int* dbg_lb;
  const int* dbg_off;
  // LB2 records again, padded per pair to rs4 16-B vectors (two records each, zero
  // records after the last job: a zero record is a no-op step, see lb2_walk_pipe) for
  // the software-pipelined walk; lb2_pipe selects it (default on)
  const uint4* recs4;
  int rs4;
  int lb2_pipe;
  // LB2 chunk ch takes window parents ch, ch + nchunks, ch + 2 nchunks, ... instead of
  // BP consecutive ones: consecutive pool nodes are siblings with similar work, so
  // consecutive chunks ranged from 0 to ~4x the mean active children and the slowest
  // workgroup took twice the mean (ta056 windows, scripts/lb2_kernel_bench.py)
  int lb2_stride;
  // phase timers of the LB2 expand kernel (probe only): shader clocks summed over the
  // workgroups for phases A, B1, B2, B3+C, the chunk count, the largest and the summed
  // per-workgroup totals, and the workgroups that had a chunk
  unsigned long long* dbg_time;
  // per-workgroup timeline (probe only): wall clock (s_memrealtime) at entry, after
  // the iteration prologue, and at exit, 3 values per workgroup
  unsigned long long* dbg_blk;
};

template <int NJ, int M, int LBK>
struct PfspSmem {
  using G = PfspGeom<NJ, LBK, M>;
  using C = PfspConsts<M>;
  static constexpr bool kRecsInLds = (LBK == 2) && (C::P * NJ * 8 <= 32 * 1024);
  PfspNode<NJ> node[G::BP];
  uint32_t fr[G::BP][M];                          // front | remain << 16
  uint16_t ptab[NJ][C::MS];
  int off[G::BP];
  typename G::map_t map[G::MAXCH];
  u64 bits[G::NWORDS + kBlock / kWave];
  int wpre[kBlock];
  int scan[kBlock / kWave];
  int red[kBlock / kWave];
  u64 pmask[LBK == 2 ? G::BP : 1][G::NW];         // scheduled set (LB2)
  uint16_t cf[LBK == 2 ? kBlock : 1][M];          // child front (LB2)
  uint2 recs[kRecsInLds ? C::P * NJ : 1];
  PoolSmem<G::MAXCHUNKS> pool;
};

// ---------------------------------------------------------------------------
// Phase A: stage `nvalid` parents (fetched through `src(i)`) and their prefixes.
// Returns the number of children of the chunk.
template <int NJ, int M, int LBK, class Smem, class Src>
__device__ inline int pfsp_phase_a(const PfspArgs<NJ, M>& a, Smem& sm, int nvalid, Src src) {
  using G = PfspGeom<NJ, LBK, M>;
  using Node = PfspNode<NJ>;
  constexpr int VPN = sizeof(Node) / 16;
  const int tid = threadIdx.x;
  // coalesced node copy: VPN 16-byte vectors per node
  for (int v = tid; v < nvalid * VPN; v += kBlock) {
    const int i = v / VPN, w = v - i * VPN;
    reinterpret_cast<uint4*>(&sm.node[i])[w] = reinterpret_cast<const uint4*>(src(i))[w];
  }
  __syncthreads();
  int nchild = 0;
  if (tid < nvalid) {
    const Node& nd = sm.node[tid];
    const int d = nd.depth;
    int f[M], r[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      f[m] = (d == 0) ? a.min_heads[m] : 0;
      r[m] = a.sum_all[m];
    }
    u64 msk[G::NW];
#pragma unroll
    for (int w = 0; w < G::NW; ++w) msk[w] = 0;
    for (int i = 0; i < d; ++i) {
      const int job = nd.prmu[i];
      const uint16_t* row = sm.ptab[job];
      int pr[M];
#pragma unroll
      for (int m = 0; m < M; ++m) pr[m] = row[m];
      f[0] += pr[0];
      r[0] -= pr[0];
#pragma unroll
      for (int m = 1; m < M; ++m) {
        f[m] = max(f[m - 1], f[m]) + pr[m];
        r[m] -= pr[m];
      }
      if constexpr (LBK == 2) {
#pragma unroll
        for (int w = 0; w < G::NW; ++w)
          if ((job >> 6) == w) msk[w] |= 1ull << (job & 63);
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) sm.fr[tid][m] = static_cast<uint32_t>(f[m]) | (static_cast<uint32_t>(r[m]) << 16);
    if constexpr (LBK == 2) {
#pragma unroll
      for (int w = 0; w < G::NW; ++w) sm.pmask[tid][w] = msk[w];
    }
    nchild = a.jobs - d;
  }
  int total = 0;
  const int off = block_exclusive_scan(nchild, sm.scan, &total);
  if (tid < nvalid) {
    sm.off[tid] = off;
    for (int j = 0; j < nchild; ++j) sm.map[off + j] = static_cast<typename G::map_t>(tid);
  }
  __syncthreads();
  return total;
}

// Phase A of the LB2 expand kernel, machine-parallel. The prefix replay
// f[i][m] = max(f[i-1][m], f[i][m-1]) + p[job_i][m] is a 2-D recurrence: lane m of a
// parent's M-lane group computes column m one step behind lane m - 1 (anti-diagonal
// wavefront, the left neighbour's value comes in by a DPP lane shift), so a parent at
// depth d costs d + M - 1 steps instead of d * M dependent steps on one lane (the
// serial replay was ~18 % of the kernel's clocks on ta056 windows, 8 lanes of 256
// busy). Several parents per wave (64 / M), all waves.
template <int NJ, int M, class Smem, class Src>
__device__ inline int pfsp_phase_a_wf(const PfspArgs<NJ, M>& a, Smem& sm, int nvalid, Src src) {
  using G = PfspGeom<NJ, 2, M>;
  using Node = PfspNode<NJ>;
  constexpr int VPN = sizeof(Node) / 16;
  constexpr int PW = kWave / M;                 // parent groups per wave
  constexpr int PB = PW * (kBlock / kWave);     // parents per pass
  static_assert(PW >= 1, "one parent group per wave at least");
  const int tid = threadIdx.x;
  for (int v = tid; v < nvalid * VPN; v += kBlock) {
    const int i = v / VPN, w = v - i * VPN;
    reinterpret_cast<uint4*>(&sm.node[i])[w] = reinterpret_cast<const uint4*>(src(i))[w];
  }
  for (int i = tid; i < nvalid * G::NW; i += kBlock) (&sm.pmask[0][0])[i] = 0;
  __syncthreads();
  const int lane = tid & (kWave - 1), wave = tid >> 6;
  const int gl = lane / M, m = lane - gl * M;
  for (int base = 0; base < nvalid; base += PB) {
    const int p = base + wave * PW + gl;
    const bool own = gl < PW && p < nvalid;
    const int d = own ? static_cast<int>(sm.node[own ? p : 0].depth) : 0;
    int steps = own ? d + m : 0;  // lane m's last step is d - 1 + m
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) steps = max(steps, __shfl_xor(steps, o, kWave));
    int f = 0, r = own ? a.sum_all[m] : 0;
    for (int s0 = 0; s0 < steps; s0 += 8) {
      // the next 8 p values of this lane's column, read together (two dependent LDS
      // reads each: job, then p), then 8 wavefront steps
      int pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = s0 + u - m;
        pv[u] = (own && i >= 0 && i < d) ? static_cast<int>(sm.ptab[sm.node[p].prmu[i]][m]) : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        // left neighbour's column value by DPP wave_shr:1 (a VALU move; a shuffle
        // through the LDS crossbar would put its latency on every step)
        const int left = __builtin_amdgcn_update_dpp(0, f, 0x138, 0xf, 0xf, false);
        const int i = s0 + u - m;
        if (own && i >= 0 && i < d) {
          f = max(f, m > 0 ? left : 0) + pv[u];
          r -= pv[u];
        }
      }
    }
    if (own) {
      if (d == 0) f = a.min_heads[m];
      sm.fr[p][m] = static_cast<uint32_t>(f) | (static_cast<uint32_t>(r) << 16);
      for (int i = m; i < d; i += M) {
        const int job = sm.node[p].prmu[i];
        atomicOr(&sm.pmask[p][job >> 6], 1ull << (job & 63));
      }
    }
  }
  const int nchild = tid < nvalid ? a.jobs - static_cast<int>(sm.node[tid].depth) : 0;
  int total = 0;
  const int off = block_exclusive_scan(nchild, sm.scan, &total);
  if (tid < nvalid) sm.off[tid] = off;
  __syncthreads();
  for (int c = tid; c < total; c += kBlock) {
    int lo = 0, hi = nvalid - 1;  // last parent with off <= c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sm.off[mid] <= c)
        lo = mid;
      else
        hi = mid - 1;
    }
    sm.map[c] = static_cast<typename G::map_t>(lo);
  }
  __syncthreads();
  return total;
}

template <int NW>
__device__ inline bool job_in(const u64 (&msk)[NW], int job) {
  if constexpr (NW == 1) {
    return (msk[0] >> job) & 1ull;
  } else {
    u64 word = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) word = ((job >> 6) == w) ? msk[w] : word;
    return (word >> (job & 63)) & 1ull;
  }
}

// Where phase B reads the LB2 records from: LDS when they fit (staged once per
// workgroup), otherwise global memory (uniform addresses -> broadcast / L2 hits).
template <int NJ, int M, int LBK>
struct SmemRecs {
  __device__ static const uint2* get(const PfspArgs<NJ, M>& a, PfspSmem<NJ, M, LBK>& sm) {
    if constexpr (PfspSmem<NJ, M, LBK>::kRecsInLds)
      return sm.recs;
    else
      return a.recs;
  }
};

// Phase B: bound of child c of the staged chunk. Sets p (chunk parent), k (prmu
// position moved to the front), job.
template <int NJ, int M, int LBK>
__device__ inline int pfsp_child_bound(const PfspArgs<NJ, M>& a, PfspSmem<NJ, M, LBK>& sm, int c, int best, int& p,
                                       int& k, int& job) {
  using G = PfspGeom<NJ, LBK, M>;
  using C = PfspConsts<M>;
  p = sm.map[c];
  const int d = sm.node[p].depth;
  k = d + (c - sm.off[p]);
  job = sm.node[p].prmu[k];
  const uint16_t* row = sm.ptab[job];
  const uint32_t* fr = sm.fr[p];
  if constexpr (LBK != 2) {
    // LB1 / LB1_d: max over machines of child front + child remain + min tail.
    const int f0 = fr[0] & 0xffff, r0 = fr[0] >> 16;
    int lb = f0 + r0 + a.min_tails[0];
    int t = f0 + row[0];
#pragma unroll
    for (int m = 1; m < M; ++m) {
      const int fm = fr[m] & 0xffff, rm = fr[m] >> 16;
      const int s = max(t, fm);
      lb = max(lb, s + rm + a.min_tails[m]);
      t = s + row[m];
    }
    return lb;
  } else {
    // LB2: child front, then the Johnson walk of every machine pair.
    uint16_t* cf = sm.cf[threadIdx.x];
    {
      int t = (fr[0] & 0xffff) + row[0];
      cf[0] = static_cast<uint16_t>(t);
#pragma unroll
      for (int m = 1; m < M; ++m) {
        t = max(t, static_cast<int>(fr[m] & 0xffff)) + row[m];
        cf[m] = static_cast<uint16_t>(t);
      }
    }
    u64 msk[G::NW];
#pragma unroll
    for (int w = 0; w < G::NW; ++w) msk[w] = sm.pmask[p][w] | (((job >> 6) == w) ? (1ull << (job & 63)) : 0ull);
    const uint2* recs = SmemRecs<NJ, M, LBK>::get(a, sm);
    const int N = a.jobs;
    int lb = 0;
    for (int q = 0; q < a.npairs; ++q) {
      const int ma0 = a.pm0[q], ma1 = a.pm1[q];
      int t0 = cf[ma0], t1 = cf[ma1];
      const uint2* rq = recs + q * N;
#pragma unroll 4
      for (int r = 0; r < N; ++r) {
        const uint2 rc = rq[r];
        const int jb = rc.x & 0xffff;
        const int p0 = rc.x >> 16, p1 = rc.y & 0xffff, lag = rc.y >> 16;
        const int n0 = t0 + p0;
        const int n1 = max(t1, n0 + lag) + p1;
        const bool sched = job_in<G::NW>(msk, jb);
        t0 = sched ? t0 : n0;
        t1 = sched ? t1 : n1;
      }
      lb = max(lb, max(t1 + a.min_tails[ma1], t0 + a.min_tails[ma0]));
      if (lb > best) break;
    }
    return lb;
  }
}

template <int NJ, int M, int LBK>
__device__ inline void pfsp_stage_tables(const PfspArgs<NJ, M>& a, PfspSmem<NJ, M, LBK>& sm) {
  using C = PfspConsts<M>;
  const int tid = threadIdx.x;
  const int nrow = a.jobs * C::MS;
  uint16_t* pt = &sm.ptab[0][0];
  for (int i = tid; i < nrow; i += kBlock) pt[i] = a.ptab[i];
  if constexpr (PfspSmem<NJ, M, LBK>::kRecsInLds) {
    const int nrec = a.npairs * a.jobs;
    for (int i = tid; i < nrec; i += kBlock) sm.recs[i] = a.recs[i];
  }
  __syncthreads();
}

// Write one id (element e = 1 + position, element 0 = depth) into a node held as
// 32-bit words in registers; every word is touched with a select so the node
// never spills to scratch.
template <int NJ, int NWD>
__device__ inline void node_set(uint32_t (&w)[NWD], int e, uint32_t v) {
  using id_t = typename PfspNode<NJ>::id_t;
  constexpr int per = 4 / sizeof(id_t);
  constexpr uint32_t mask = sizeof(id_t) == 1 ? 0xffu : 0xffffu;
  const int wi = e / per;
  const int sh = (e % per) * 8 * sizeof(id_t);
#pragma unroll
  for (int i = 0; i < NWD; ++i) w[i] = (i == wi) ? ((w[i] & ~(mask << sh)) | (v << sh)) : w[i];
}

// ---------------------------------------------------------------------------
// LB1 / LB1_d: thread-per-parent. The parent's front and remain live in registers
// (M is a template constant, loops fully unrolled); each child costs O(M) with
// one vectorised LDS read of its job's p row — no child->parent map, no per-child
// gathers of parent rows, no bitmap. The i-th child's bound is handed to `emit`.
template <int NJ, int M>
struct PfspSmemLB1 {
  using G = PfspGeom<NJ, 1>;
  using C = PfspConsts<M>;
  PfspNode<NJ> node[G::BP];
  uint16_t ptab[NJ][C::MS];
  int scan[kBlock / kWave];
  int red[kBlock / kWave];
  PoolSmem<G::MAXCHUNKS> pool;
};

template <int M>
__device__ inline void load_prow(const uint16_t* row, int (&pr)[M]) {
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
#pragma unroll
  for (int q = 0; q < PfspConsts<M>::RV; ++q) {
    const uint4 x = r4[q];
    const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int h = 0; h < 8; ++h)
      if (q * 8 + h < M) pr[q * 8 + h] = static_cast<int>((wv[h >> 1] >> ((h & 1) * 16)) & 0xffffu);
  }
}

template <int NJ, int M, class Smem, class Emit>
__device__ inline void pfsp_lb1_parent(const PfspArgs<NJ, M>& a, Smem& sm, int p, Emit emit) {
  const PfspNode<NJ>& nd = sm.node[p];
  const int d = nd.depth;
  int f[M], r[M];  // r: unscheduled work + min tail, folded in once per parent
#pragma unroll
  for (int m = 0; m < M; ++m) {
    f[m] = (d == 0) ? a.min_heads[m] : 0;
    r[m] = a.sum_all[m] + a.min_tails[m];
  }
  for (int i = 0; i < d; ++i) {
    int pr[M];
    load_prow<M>(sm.ptab[nd.prmu[i]], pr);
    f[0] += pr[0];
    r[0] -= pr[0];
#pragma unroll
    for (int m = 1; m < M; ++m) {
      f[m] = max(f[m - 1], f[m]) + pr[m];
      r[m] -= pr[m];
    }
  }
  for (int k = d; k < a.jobs; ++k) {
    const int job = nd.prmu[k];
    int pr[M];
    load_prow<M>(sm.ptab[job], pr);
    // child front on machine m = s + p[m]; parent remain still holds p[m][job]:
    // max over m of (child front + child remain + min tail)  (ref c_bound_simple.c:219-244)
    int lb = f[0] + r[0];
    int t = f[0] + pr[0];
#pragma unroll
    for (int m = 1; m < M; ++m) {
      const int s = max(t, f[m]);
      lb = max(lb, s + r[m]);
      t = s + pr[m];
    }
    emit(k - d, k, lb);
  }
}

// ---------------------------------------------------------------------------
// One B&B iteration on the device-resident pool (pool_device.hpp). `t` in [0, 6):
// state slot t%3, buffer parity t%2.
template <int NJ, int M>
__device__ inline void pfsp_expand_lb1(const PfspArgs<NJ, M>& a, int t);

template <int NJ, int M, bool PK = false>
__device__ inline void pfsp_expand_lb2(const PfspArgs<NJ, M>& a, int t);

// Occupancy: the LB1 kernels are latency-bound (profiles/r1/r1o), so the register
// budget is capped for more resident waves (6 per SIMD for M <= 10: 80 VGPRs, no
// spills); LB2 is bounded by its LDS footprint instead (4 workgroups per CU for
// 50 x 20), and the packed-walk kernel (LBK 5) is held to the 128 VGPRs of 4 waves
// per SIMD (its unrolled walk would otherwise take 130).
// (Variants measured slower and removed in round 3, numbers in profiles/r2/lb2_variants.md
// and profiles/r1/r1af: every record packed in LDS, prefix/suffix walks per (parent,
// pair), wave-uniform pair walks, a dynamic chunk queue.)
template <int NJ, int M, int LBK>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(LBK == 5 ? 4 : LBK >= 2 ? 1 : (M <= 10 ? 6 : 4))))
void pfsp_expand_kernel(PfspArgs<NJ, M> a, int t) {
  if constexpr (LBK == 2)
    pfsp_expand_lb2<NJ, M>(a, t);
  else if constexpr (LBK == 5)
    pfsp_expand_lb2<NJ, M, true>(a, t);  // two children per lane, packed u16 walks
  else
    pfsp_expand_lb1<NJ, M>(a, t);  // permutation nodes (20-job instances use pfsp_front_kernels.hpp)
}

// ---------------------------------------------------------------------------
// LB2 expand. The reference evaluates one child per thread and walks the P machine
// pairs one after the other (ref bounds_gpu.cu:252-316): O(P*N) dependent steps per
// lane and, with few children per iteration, a handful of waves on a 256-CU chip.
// Here the work unit is one (child, machine pair) Johnson walk:
//   B1  thread-per-child: child front, LB1 of the child from the parent prefix
//       (O(M)), leaves, and the LB1 filter — LB2 >= LB1 pointwise,
//       so a child with LB1 >= best is pruned by LB2 as well: only the others enter
//       the active list (fronts machine-major in LDS, scheduled-set bitmask).
//   B2  pair-major task loop over (pair q, active child): consecutive lanes share
//       q, so each Johnson record read is an LDS broadcast; per-pair results are
//       folded with an LDS atomicMax. A task whose child already exceeds `best`
//       is skipped (the reference's early exit, c_bound_johnson.c:231-234: only
//       the lb < best decision matters, and it is unchanged).
//   B3  survivors (LB2 < best) -> ballot bitmap -> compaction as in every kernel.
template <int NJ, int M>
struct PfspSmemLB2 {
  using G = PfspGeom<NJ, 2, M>;
  using C = PfspConsts<M>;
  // records in LDS when they fit 32 KB (20 x 20: 30 KB); otherwise (50 x 20: 76 KB)
  // they are read from L2 (packing the leading pairs to 4 B in LDS measured no gain,
  // profiles/r1/r1ag; all of them in LDS halved the occupancy, profiles/r2/lb2_variants.md)
  static constexpr bool kRecsInLds = C::P * NJ * 8 <= 32 * 1024;
  PfspNode<NJ> node[G::BP];
  uint32_t fr[G::BP][M];                  // parent front | remain << 16
  u64 pmask[G::BP][G::NW];                // parent scheduled set
  int off[G::BP];
  typename G::map_t map[G::MAXCH];
  uint16_t ptab[NJ][C::MS];
  uint16_t cf[M][G::MAXCH];               // active child fronts, machine-major
  u64 cm[G::MAXCH][G::NW];                // active child scheduled sets
  int lbv[G::MAXCH];                      // active child LB2 (max over pairs)
  int16_t act[G::MAXCH];                  // child -> active slot, -1 if decided in B1
  int16_t alist[G::MAXCH];                // B2 rounds: active slots still below best
  uint8_t aparent[G::MAXCH];              // active slot -> chunk parent
  uint8_t ajob[G::MAXCH];                 // active slot -> its job
  u64 bits[G::NWORDS + kBlock / kWave];
  int wpre[kBlock];
  int scan[kBlock / kWave];
  int red[kBlock / kWave];
  uint2 pinfo[C::P];
  uint2 recs[kRecsInLds ? C::P * NJ : 1];
  PoolSmem<G::MAXCHUNKS> pool;
};

// Records read with scalar loads (constant address space: the tables are written
// once, before the engine's first launch) when every active lane walks the same pair.
using kconst_u64 = const __attribute__((address_space(4))) unsigned long long;  // {x, y} of a uint2

// One Johnson walk (ref c_bound_johnson.c:190-209) of machine pair `pi` from child
// fronts (t0, t1) over the jobs not in `msk`. Records come from `recs` (LDS or L2),
// or with scalar loads when every lane of the wave walks the same pair (uniform_ref).
template <int NJ, int M, class S>
__device__ inline void lb2_johnson_walk(const uint2* recs, uint2 pi, int N, const u64 (&msk)[PfspGeom<NJ, 2, M>::NW],
                                        int& t0, int& t1, int uniform_ref = -1) {
  using G = PfspGeom<NJ, 2, M>;
  if constexpr (!S::kRecsInLds) {
    // every active lane of the wave walks the same pair: the records are wave-uniform,
    // read with scalar loads (constant address space, scalar cache) into SGPRs instead
    // of one vector load per step (the tables are written before the first launch)
    if (uniform_ref >= 0) {
      kconst_u64* const rq = (kconst_u64*)(uintptr_t)recs + uniform_ref * N;
#pragma unroll 8
      for (int r = 0; r < N; ++r) {
        const u64 rw = rq[r];
        const uint32_t rx = static_cast<uint32_t>(rw), ry = static_cast<uint32_t>(rw >> 32);
        const int n0 = t0 + static_cast<int>(rx >> 16);
        const int n1 = max(t1, n0 + static_cast<int>(ry >> 16)) + static_cast<int>(ry & 0xffff);
        const bool sched = job_in<G::NW>(msk, static_cast<int>(rx & 0xffff));
        t0 = sched ? t0 : n0;
        t1 = sched ? t1 : n1;
      }
      return;
    }
  }
  const uint2* rq = recs + static_cast<int>(pi.x >> 16) * N;
#pragma unroll 4
  for (int r = 0; r < N; ++r) {
    const uint2 rc = rq[r];
    const int n0 = t0 + static_cast<int>(rc.x >> 16);
    const int n1 = max(t1, n0 + static_cast<int>(rc.y >> 16)) + static_cast<int>(rc.y & 0xffff);
    const bool sched = job_in<G::NW>(msk, static_cast<int>(rc.x & 0xffff));
    t0 = sched ? t0 : n0;
    t1 = sched ? t1 : n1;
  }
}

// Johnson step on one record {x = job | p0 << 16, y = p1 | lag << 16}.
template <int NW>
__device__ inline void lb2_step(uint32_t x, uint32_t y, const u64 (&msk)[NW], int& t0, int& t1) {
  const int n0 = t0 + static_cast<int>(x >> 16);
  const int n1 = max(t1, n0 + static_cast<int>(y >> 16)) + static_cast<int>(y & 0xffff);
  const bool sched = job_in<NW>(msk, static_cast<int>(x & 0xffff));
  t0 = sched ? t0 : n0;
  t1 = sched ? t1 : n1;
}

// The Johnson walk with its record loads software-pipelined: the walk runs in
// double groups of 8 records (four 16-B loads); group A's records for the next
// double group are requested right after A is consumed, B's after B, so each load
// has a whole group of steps (plus the other waves' issue) to land instead of
// stalling the step that needs it (the plain loop waits on every load: L1/L2
// latency per four steps). The table is padded per pair with zero records up to one
// double group past the walk; a zero record is a no-op step (n0 = t0 and, as a
// front on the later machine never trails the earlier one, n1 = max(t1, t0) = t1).
template <int NW>
__device__ inline void lb2_walk_pipe(const uint4* rq, int ndouble, const u64 (&msk)[NW], int& t0, int& t1) {
  uint4 a0 = rq[0], a1 = rq[1], b0 = rq[2], b1 = rq[3];
  for (int g = 0; g < ndouble; ++g) {
    lb2_step<NW>(a0.x, a0.y, msk, t0, t1);
    lb2_step<NW>(a0.z, a0.w, msk, t0, t1);
    lb2_step<NW>(a1.x, a1.y, msk, t0, t1);
    lb2_step<NW>(a1.z, a1.w, msk, t0, t1);
    a0 = rq[4 * g + 4];
    a1 = rq[4 * g + 5];
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch here (the scheduler sinks it to its use)
    lb2_step<NW>(b0.x, b0.y, msk, t0, t1);
    lb2_step<NW>(b0.z, b0.w, msk, t0, t1);
    lb2_step<NW>(b1.x, b1.y, msk, t0, t1);
    lb2_step<NW>(b1.z, b1.w, msk, t0, t1);
    b0 = rq[4 * g + 6];
    b1 = rq[4 * g + 7];
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Two children per lane (kernel LBK 5): both walk the same machine pair, so one
// record load serves two Johnson steps and the max-plus arithmetic runs on packed u16
// halves (v_pk_add_u16 / v_pk_max_u16, the record fields broadcast by op_sel); each
// half skips the jobs of its own child's scheduled set (bit field insert on a
// per-half keep mask). Exact as long as every value of the walk fits 16 bits: a walk
// value is a path length through the p matrix (host check lb2_pk_ok: (jobs + machines
// - 1) x max p < 65536: 500 x 20 with p <= 99 gives 51,381). Job sets of two words
// (100-job instances) pick the word of the record's job by a select per child; wider
// ones (200 / 500 jobs) read it from LDS (lb2_step2_lds).
// (u16x2 helpers: device_common.hpp)

template <int NW>
__device__ inline void lb2_step2(uint32_t x, uint32_t y, const u64 (&mav)[NW], const u64 (&mbv)[NW], uint32_t& t0,
                                 uint32_t& t1) {
  const u16x2 p0 = static_cast<u16x2>(static_cast<unsigned short>(x >> 16));
  const u16x2 lag = static_cast<u16x2>(static_cast<unsigned short>(y >> 16));
  const u16x2 p1 = static_cast<u16x2>(static_cast<unsigned short>(y & 0xffff));
  const u16x2 n0 = as_u16x2(t0) + p0;
  const u16x2 n1 = __builtin_elementwise_max(as_u16x2(t1), n0 + lag) + p1;
  const uint32_t job = x & 63u;
  u64 ma = mav[0], mb = mbv[0];
  if constexpr (NW > 1) {
    const uint32_t wj = (x & 0xffffu) >> 6;
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      ma = wj == static_cast<uint32_t>(w) ? mav[w] : ma;
      mb = wj == static_cast<uint32_t>(w) ? mbv[w] : mb;
    }
  }
  // all ones where the half's child skips the job: v_lshrrev_b64 + v_bfe_i32 per child
  // (spelled with the intrinsics: the plain (m >> job) & 1 becomes a mask-and-compare
  // sequence twice as long), halves merged by one v_perm_b32
  const int ka = __builtin_amdgcn_sbfe(static_cast<int>(static_cast<uint32_t>(ma >> job)), 0, 1);
  const int kb = __builtin_amdgcn_sbfe(static_cast<int>(static_cast<uint32_t>(mb >> job)), 0, 1);
  const uint32_t keep = __builtin_amdgcn_perm(static_cast<uint32_t>(kb), static_cast<uint32_t>(ka), 0x05040100u);
  t0 = (t0 & keep) | (as_u32(n0) & ~keep);
  t1 = (t1 & keep) | (as_u32(n1) & ~keep);
}

template <int NW>
__device__ inline void lb2_walk_pipe2(const uint4* rq, int ndouble, const u64 (&ma)[NW], const u64 (&mb)[NW],
                                      uint32_t& t0, uint32_t& t1) {
  uint4 a0 = rq[0], a1 = rq[1], b0 = rq[2], b1 = rq[3];
  for (int g = 0; g < ndouble; ++g) {
    lb2_step2<NW>(a0.x, a0.y, ma, mb, t0, t1);
    lb2_step2<NW>(a0.z, a0.w, ma, mb, t0, t1);
    lb2_step2<NW>(a1.x, a1.y, ma, mb, t0, t1);
    lb2_step2<NW>(a1.z, a1.w, ma, mb, t0, t1);
    a0 = rq[4 * g + 4];
    a1 = rq[4 * g + 5];
    __builtin_amdgcn_sched_barrier(0);
    lb2_step2<NW>(b0.x, b0.y, ma, mb, t0, t1);
    lb2_step2<NW>(b0.z, b0.w, ma, mb, t0, t1);
    lb2_step2<NW>(b1.x, b1.y, ma, mb, t0, t1);
    lb2_step2<NW>(b1.z, b1.w, ma, mb, t0, t1);
    b0 = rq[4 * g + 6];
    b1 = rq[4 * g + 7];
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Job sets of more than two words (200 / 500-job instances): the word of the record's
// job is read from the children's LDS rows (one ds_read_b64 per child and step, issued
// with the record group, independent of the walk's dependence chain) instead of
// selecting it among NW words held in registers (2 (NW - 1) 64-bit selects per child).
__device__ inline void lb2_step2_lds(uint32_t x, uint32_t y, const u64* ma, const u64* mb, uint32_t& t0,
                                     uint32_t& t1) {
  const u16x2 p0 = static_cast<u16x2>(static_cast<unsigned short>(x >> 16));
  const u16x2 lag = static_cast<u16x2>(static_cast<unsigned short>(y >> 16));
  const u16x2 p1 = static_cast<u16x2>(static_cast<unsigned short>(y & 0xffff));
  const u16x2 n0 = as_u16x2(t0) + p0;
  const u16x2 n1 = __builtin_elementwise_max(as_u16x2(t1), n0 + lag) + p1;
  const uint32_t job = x & 63u, wj = (x & 0xffffu) >> 6;
  const int ka = __builtin_amdgcn_sbfe(static_cast<int>(static_cast<uint32_t>(ma[wj] >> job)), 0, 1);
  const int kb = __builtin_amdgcn_sbfe(static_cast<int>(static_cast<uint32_t>(mb[wj] >> job)), 0, 1);
  const uint32_t keep = __builtin_amdgcn_perm(static_cast<uint32_t>(kb), static_cast<uint32_t>(ka), 0x05040100u);
  t0 = (t0 & keep) | (as_u32(n0) & ~keep);
  t1 = (t1 & keep) | (as_u32(n1) & ~keep);
}

__device__ inline void lb2_walk_pipe2_lds(const uint4* rq, int ndouble, const u64* ma, const u64* mb, uint32_t& t0,
                                          uint32_t& t1) {
  uint4 a0 = rq[0], a1 = rq[1], b0 = rq[2], b1 = rq[3];
  for (int g = 0; g < ndouble; ++g) {
    lb2_step2_lds(a0.x, a0.y, ma, mb, t0, t1);
    lb2_step2_lds(a0.z, a0.w, ma, mb, t0, t1);
    lb2_step2_lds(a1.x, a1.y, ma, mb, t0, t1);
    lb2_step2_lds(a1.z, a1.w, ma, mb, t0, t1);
    a0 = rq[4 * g + 4];
    a1 = rq[4 * g + 5];
    __builtin_amdgcn_sched_barrier(0);
    lb2_step2_lds(b0.x, b0.y, ma, mb, t0, t1);
    lb2_step2_lds(b0.z, b0.w, ma, mb, t0, t1);
    lb2_step2_lds(b1.x, b1.y, ma, mb, t0, t1);
    lb2_step2_lds(b1.z, b1.w, ma, mb, t0, t1);
    b0 = rq[4 * g + 6];
    b1 = rq[4 * g + 7];
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int NJ, int M, bool PK>
__device__ inline void pfsp_expand_lb2(const PfspArgs<NJ, M>& a, int t) {
  using G = PfspGeom<NJ, 2, M>;
  using C = PfspConsts<M>;
  using S = PfspSmemLB2<NJ, M>;
  using Node = PfspNode<NJ>;
  constexpr int VPN = sizeof(Node) / 16;
  constexpr int NWD = sizeof(Node) / 4;
  const int P = a.npairs;
  __shared__ S sm;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  const unsigned long long t_entry = a.dbg_blk ? wall_clock64() : 0;
  const IterView v = pool_begin<Node, G::MAXCHUNKS>(pa, t, G::BP, sm.pool);
  if (v.B == 0 || v.overflow) return;
  const int best = prune_best(pa, v);
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  pool_spill_leftovers<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, sm.pool);
  {  // tables -> LDS (visible after phase A's first barrier)
    uint16_t* pt = &sm.ptab[0][0];
    for (int i = tid; i < a.jobs * C::MS; i += kBlock) pt[i] = a.ptab[i];
    for (int i = tid; i < P; i += kBlock) sm.pinfo[i] = a.pinfo[i];
    if constexpr (S::kRecsInLds)
      for (int i = tid; i < P * a.jobs; i += kBlock) sm.recs[i] = a.recs[i];
  }
  const uint2* recs = S::kRecsInLds ? sm.recs : a.recs;
  const int N = a.jobs;
  const bool pipe = !S::kRecsInLds && a.lb2_pipe;
  const int ndouble = (N + 7) >> 3;
  unsigned long long tm[4] = {0, 0, 0, 0}, tc = 0;
  const bool timed = a.dbg_time != nullptr;
  const bool stride = a.lb2_stride != 0;
  int nchunks_done = 0;
  const unsigned long long t_pro = a.dbg_blk ? wall_clock64() : 0;
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    ++nchunks_done;
    if (timed) tc = clock64();
    // window parents of this chunk: ch + i * nchunks (strided) or ch * BP + i
    const u64 first = stride ? static_cast<u64>(ch) : static_cast<u64>(ch) * G::BP;
    const u64 step = stride ? static_cast<u64>(v.nchunks) : 1ull;
    const int nvalid = stride ? static_cast<int>((v.B - first + step - 1) / step)
                              : static_cast<int>(min(static_cast<u64>(G::BP), v.B - first));
    auto gidx = [&](int i) -> u64 { return first + static_cast<u64>(i) * step; };
    auto src = [&](int i) -> const Node* {
      return pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, gidx(i), sm.pool);
    };
    // machine-parallel prefix replay from 10 machines; with 5 the serial replay is
    // only 5 steps per prefix job and the wavefront's shuffles cost more (ta010 LB2
    // 4.2 -> 5.7 ms)
    int total;
    if constexpr (M >= 10)
      total = pfsp_phase_a_wf<NJ, M>(a, sm, nvalid, src);
    else
      total = pfsp_phase_a<NJ, M, 2>(a, sm, nvalid, src);
    if (timed) {
      const unsigned long long c = clock64();
      tm[0] += c - tc;
      tc = c;
    }
    // ---- B1: child fronts, LB1 filter, leaves, active list ----
    int my_leaves = 0, nact = 0;
    for (int cb = 0; cb < total; cb += kBlock) {
      const int c = cb + tid;
      int active = 0, job = 0, p = 0;
      int f[M];
      if (c < total) {
        p = sm.map[c];
        const int d = sm.node[p].depth;
        const int k = d + (c - sm.off[p]);
        job = sm.node[p].prmu[k];
        int pr[M];
        load_prow<M>(sm.ptab[job], pr);
        const uint32_t* fr = sm.fr[p];
        // LB1 of the child (ref c_bound_simple.c:219-244) and its front
        int lb1 = static_cast<int>(fr[0] & 0xffff) + static_cast<int>(fr[0] >> 16) + a.min_tails[0];
        int tt = static_cast<int>(fr[0] & 0xffff) + pr[0];
        f[0] = tt;
#pragma unroll
        for (int m = 1; m < M; ++m) {
          const int sv = max(tt, static_cast<int>(fr[m] & 0xffff));
          lb1 = max(lb1, sv + static_cast<int>(fr[m] >> 16) + a.min_tails[m]);
          tt = sv + pr[m];
          f[m] = tt;
        }
        const bool keep = split_keep(v, gidx(p), k);
        if (d + 1 == N) {
          // a leaf's LB2 is its makespan bound max_m(front + tail) == LB1
          my_leaves += keep;
          if (lb1 < best) atomicMin(&pa.ctl->best.v, lb1);
        } else {
          active = (keep && lb1 < best) ? 1 : 0;
        }
        if (a.dbg_lb && !active) a.dbg_lb[a.dbg_off[gidx(p)] + (k - d)] = lb1;
      }
      int cnt = 0;
      const int slot = nact + block_exclusive_scan(active, sm.scan, &cnt);
      if (c < total) {
        sm.act[c] = static_cast<int16_t>(active ? slot : -1);
      }
      if (active) {
#pragma unroll
        for (int m = 0; m < M; ++m) sm.cf[m][slot] = static_cast<uint16_t>(f[m]);
#pragma unroll
        for (int w = 0; w < G::NW; ++w)
          sm.cm[slot][w] = sm.pmask[p][w] | (((job >> 6) == w) ? (1ull << (job & 63)) : 0ull);
        sm.lbv[slot] = 0;
        sm.aparent[slot] = static_cast<uint8_t>(p);
        sm.ajob[slot] = static_cast<uint8_t>(job);
      }
      nact += cnt;
    }
    __syncthreads();
    if (timed) {
      const unsigned long long c = clock64();
      tm[1] += c - tc;
      tc = c;
    }
    // ---- B2: (pair, child) Johnson walks, pair-major ----
    if (nact > 0 && a.lb2_rounds) {
      // Rounds of 8, 16, 32, ... pairs (learned early-exit order: the first pairs
      // prune most children). Between rounds the children whose LB2 already exceeds
      // best are dropped from the task list, so a wave's lanes no longer idle on
      // skipped tasks; a round's tasks are dense (pair-major, consecutive lanes
      // share the pair's records).
      constexpr int PER = (G::MAXCH + kBlock - 1) / kBlock;
      for (int i = tid; i < nact; i += kBlock) sm.alist[i] = static_cast<int16_t>(i);
      __syncthreads();
      int na = nact, q0 = 0, R = 8;
      while (q0 < P && na > 0) {
        const int nq = min(P - q0, R);
        if constexpr (PK) {
          // tasks (pair, child pair): children alist[2k], alist[2k + 1] share a lane
          const int nk = (na + 1) >> 1;
          int qq = tid / nk, kk = tid - (tid / nk) * nk;
          const int dq = kBlock / nk, dk = kBlock - dq * nk;
          while (qq < nq) {
            const int ca = sm.alist[2 * kk];
            const int cb = 2 * kk + 1 < na ? sm.alist[2 * kk + 1] : -1;
            const bool la = sm.lbv[ca] < best, lbb = cb >= 0 && sm.lbv[cb] < best;
            if (la || lbb) {
              const uint2 pi = sm.pinfo[q0 + qq];
              const int m0 = pi.x & 0xff, m1 = (pi.x >> 8) & 0xff;
              const int cbb = cb >= 0 ? cb : ca;
              uint32_t t0 = static_cast<uint32_t>(sm.cf[m0][ca]) | (static_cast<uint32_t>(sm.cf[m0][cbb]) << 16);
              uint32_t t1 = static_cast<uint32_t>(sm.cf[m1][ca]) | (static_cast<uint32_t>(sm.cf[m1][cbb]) << 16);
              if constexpr (G::NW > 2) {
                // (a lone child walks in both halves; the second half's result is unused)
                lb2_walk_pipe2_lds(a.recs4 + static_cast<int>(pi.x >> 16) * a.rs4, ndouble, sm.cm[ca],
                                   sm.cm[cbb], t0, t1);
              } else {
                u64 ma[G::NW], mb[G::NW];
#pragma unroll
                for (int w = 0; w < G::NW; ++w) {
                  ma[w] = sm.cm[ca][w];
                  mb[w] = cb >= 0 ? sm.cm[cbb][w] : ~0ull;
                }
                lb2_walk_pipe2(a.recs4 + static_cast<int>(pi.x >> 16) * a.rs4, ndouble, ma, mb, t0, t1);
              }
              const int tl0 = static_cast<int>(pi.y & 0xffff), tl1 = static_cast<int>(pi.y >> 16);
              if (la)
                atomicMax(&sm.lbv[ca], max(static_cast<int>(t1 & 0xffff) + tl1, static_cast<int>(t0 & 0xffff) + tl0));
              if (lbb) atomicMax(&sm.lbv[cb], max(static_cast<int>(t1 >> 16) + tl1, static_cast<int>(t0 >> 16) + tl0));
            }
            kk += dk;
            qq += dq;
            if (kk >= nk) {
              kk -= nk;
              ++qq;
            }
          }
        } else {
        int qq = tid / na, ii = tid - (tid / na) * na;
        const int dq = kBlock / na, di = kBlock - dq * na;
        while (qq < nq) {
          const int ai = sm.alist[ii];
          // wave-uniform pair among the lanes still in the loop?
          const int qf = __builtin_amdgcn_readfirstlane(qq);
          const int uref = __ballot(qq != qf) == 0
                               ? __builtin_amdgcn_readfirstlane(static_cast<int>(sm.pinfo[q0 + qf].x >> 16))
                               : -1;
          if (sm.lbv[ai] < best) {
            const uint2 pi = sm.pinfo[q0 + qq];
            int t0 = sm.cf[pi.x & 0xff][ai], t1 = sm.cf[(pi.x >> 8) & 0xff][ai];
            u64 msk[G::NW];
#pragma unroll
            for (int w = 0; w < G::NW; ++w) msk[w] = sm.cm[ai][w];
            if (pipe && uref < 0)
              lb2_walk_pipe<G::NW>(a.recs4 + static_cast<int>(pi.x >> 16) * a.rs4, ndouble, msk, t0, t1);
            else
              lb2_johnson_walk<NJ, M, S>(recs, pi, N, msk, t0, t1, uref);
            atomicMax(&sm.lbv[ai], max(t1 + static_cast<int>(pi.y >> 16), t0 + static_cast<int>(pi.y & 0xffff)));
          }
          ii += di;
          qq += dq;
          if (ii >= na) {
            ii -= na;
            ++qq;
          }
        }
        }
        q0 += nq;
        R *= 2;
        __syncthreads();  // the round's LB2 maxima are final
        if (q0 >= P) break;
        int ent[PER];
        bool kp[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const int i = k * kBlock + tid;
          ent[k] = i < na ? sm.alist[i] : -1;
          kp[k] = ent[k] >= 0 && sm.lbv[ent[k]] < best;
        }
        int nn = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {  // the scan's first barrier orders the reads above before the writes
          int c = 0;
          const int pos = nn + block_exclusive_scan(kp[k] ? 1 : 0, sm.scan, &c);
          if (kp[k]) sm.alist[pos] = static_cast<int16_t>(ent[k]);
          nn += c;
        }
        __syncthreads();
        na = nn;
      }
    } else if (nact > 0) {
      int q = tid / nact, ai = tid - (tid / nact) * nact;
      const int dq = kBlock / nact, da = kBlock - dq * nact;
      while (q < P) {
        const int qf = __builtin_amdgcn_readfirstlane(q);
        const int uref =
            __ballot(q != qf) == 0 ? __builtin_amdgcn_readfirstlane(static_cast<int>(sm.pinfo[qf].x >> 16)) : -1;
        if (sm.lbv[ai] < best) {
          const uint2 pi = sm.pinfo[q];
          int t0 = sm.cf[pi.x & 0xff][ai], t1 = sm.cf[(pi.x >> 8) & 0xff][ai];
          u64 msk[G::NW];
#pragma unroll
          for (int w = 0; w < G::NW; ++w) msk[w] = sm.cm[ai][w];
          lb2_johnson_walk<NJ, M, S>(recs, pi, N, msk, t0, t1, uref);
          atomicMax(&sm.lbv[ai], max(t1 + static_cast<int>(pi.y >> 16), t0 + static_cast<int>(pi.y & 0xffff)));
        }
        ai += da;
        q += dq;
        if (ai >= nact) {
          ai -= nact;
          ++q;
        }
      }
    }
    __syncthreads();
    if (timed) {
      const unsigned long long c = clock64();
      tm[2] += c - tc;
      tc = c;
    }
    // ---- B3: survivor bitmap ----
    for (int cb = 0; cb < total; cb += kBlock) {
      const int c = cb + tid;
      bool survive = false;
      if (c < total) {
        const int s = sm.act[c];
        survive = s >= 0 && sm.lbv[s] < best;
        if (a.dbg_lb && s >= 0) {
          const int p = sm.map[c];
          a.dbg_lb[a.dbg_off[gidx(p)] + (c - sm.off[p])] = sm.lbv[s];
        }
      }
      const u64 bal = __ballot(survive);
      if ((tid & (kWave - 1)) == 0) sm.bits[c >> 6] = bal;
    }
    __syncthreads();
    // ---- C: compaction into this chunk's slot region + published counts ----
    const int nwords = (total + 63) >> 6;
    int nsurv = 0, nleaves = 0;
    const int wp = block_exclusive_scan(tid < nwords ? __popcll(sm.bits[tid]) : 0, sm.scan, &nsurv);
    (void)block_exclusive_scan(my_leaves, sm.red, &nleaves);
    sm.wpre[tid] = wp;
    if (tid == 0) {
      cnt_out[ch] = nsurv;
      lcnt_out[ch] = nleaves;
    }
    __syncthreads();
    Node* const dst_chunk = bout + static_cast<size_t>(ch) * G::SLOT;
    for (int c = tid; c < total; c += kBlock) {
      const u64 word = sm.bits[c >> 6];
      if (!((word >> (c & 63)) & 1ull)) continue;
      const int rank = sm.wpre[c >> 6] + __popcll(word & ((1ull << (c & 63)) - 1ull));
      const int p = sm.map[c];
      const int d = sm.node[p].depth;
      const int k = d + (c - sm.off[p]);
      uint32_t w[NWD];
#pragma unroll
      for (int i = 0; i < NWD; ++i) w[i] = reinterpret_cast<const uint32_t*>(&sm.node[p])[i];
      const uint32_t jd = sm.node[p].prmu[d], jk = sm.node[p].prmu[k];
      node_set<NJ>(w, 0, static_cast<uint32_t>(d + 1));
      node_set<NJ>(w, 1 + d, jk);
      node_set<NJ>(w, 1 + k, jd);
      uint4* dst = reinterpret_cast<uint4*>(dst_chunk + rank);
#pragma unroll
      for (int q = 0; q < VPN; ++q) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    __syncthreads();
    if (timed) tm[3] += clock64() - tc;
  }
  if (timed && tid == 0) {
    const unsigned long long tot = tm[0] + tm[1] + tm[2] + tm[3];
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&a.dbg_time[i], tm[i]);
    atomicAdd(&a.dbg_time[4], static_cast<unsigned long long>(nchunks_done));
    atomicMax(&a.dbg_time[5], tot);
    atomicAdd(&a.dbg_time[6], tot);
    if (nchunks_done) atomicAdd(&a.dbg_time[7], 1ull);
  }
  if (a.dbg_blk && tid == 0) {
    a.dbg_blk[3 * blockIdx.x] = t_entry;
    a.dbg_blk[3 * blockIdx.x + 1] = t_pro;
    a.dbg_blk[3 * blockIdx.x + 2] = wall_clock64();
  }
}

// LB1 / LB1_d expand: per chunk, thread p owns parent p end to end.
template <int NJ, int M>
__device__ inline void pfsp_expand_lb1(const PfspArgs<NJ, M>& a, int t) {
  using G = PfspGeom<NJ, 1>;
  using Node = PfspNode<NJ>;
  using id_t = typename Node::id_t;
  constexpr int VPN = sizeof(Node) / 16;
  constexpr int NWD = sizeof(Node) / 4;
  constexpr int SW = (NJ + 63) / 64;  // survivor mask words
  __shared__ PfspSmemLB1<NJ, M> sm;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  const IterView v = pool_begin<Node, G::MAXCHUNKS>(pa, t, G::BP, sm.pool);
  if (v.B == 0 || v.overflow) return;
  const int best = prune_best(pa, v);
  Node* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  pool_spill_leftovers<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, sm.pool);
  {
    constexpr int MS = PfspConsts<M>::MS;
    uint16_t* pt = &sm.ptab[0][0];
    for (int i = tid; i < a.jobs * MS; i += kBlock) pt[i] = a.ptab[i];
  }
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    const u64 first = static_cast<u64>(ch) * G::BP;
    const int nvalid = static_cast<int>(min(static_cast<u64>(G::BP), v.B - first));
    for (int x = tid; x < nvalid * VPN; x += kBlock) {
      const int i = x / VPN, w = x - i * VPN;
      reinterpret_cast<uint4*>(&sm.node[i])[w] =
          reinterpret_cast<const uint4*>(pool_parent<Node, G::SLOT, G::MAXCHUNKS>(pa, v, t, first + i, sm.pool))[w];
    }
    __syncthreads();
    u64 surv[SW];
#pragma unroll
    for (int q = 0; q < SW; ++q) surv[q] = 0;
    int nsurv = 0, nleaf = 0;
    if (tid < nvalid) {
      const bool leaf = sm.node[tid].depth + 1 == a.jobs;
      pfsp_lb1_parent<NJ, M>(a, sm, tid, [&](int j, int k, int lb) {
        if (a.dbg_lb) a.dbg_lb[a.dbg_off[first + tid] + j] = lb;  // element-wise probe (tests)
        const bool keep = split_keep(v, first + tid, k);
        if (leaf) {
          nleaf += keep;
          if (lb < best) atomicMin(&pa.ctl->best.v, lb);
        } else if (keep && lb < best) {
          ++nsurv;
#pragma unroll
          for (int q = 0; q < SW; ++q)
            if ((j >> 6) == q) surv[q] |= 1ull << (j & 63);
        }
      });
    }
    int total = 0, leaves = 0;
    const int off = block_exclusive_scan(nsurv, sm.scan, &total);
    (void)block_exclusive_scan(nleaf, sm.red, &leaves);
    if (tid == 0) {
      cnt_out[ch] = total;
      lcnt_out[ch] = leaves;
    }
    if (nsurv) {
      const Node& nd = sm.node[tid];
      const int d = nd.depth;
      uint32_t w[NWD];
#pragma unroll
      for (int i = 0; i < NWD; ++i) w[i] = reinterpret_cast<const uint32_t*>(&nd)[i];
      const uint32_t jd = nd.prmu[d];
      node_set<NJ>(w, 0, static_cast<uint32_t>(d + 1));
      Node* dst = bout + static_cast<size_t>(ch) * G::SLOT + off;
#pragma unroll
      for (int q = 0; q < SW; ++q) {
        u64 m = surv[q];
        while (m) {
          const int j = q * 64 + __ffsll(static_cast<long long>(m)) - 1;
          m &= m - 1;
          const int k = d + j;
          uint32_t c[NWD];
#pragma unroll
          for (int i = 0; i < NWD; ++i) c[i] = w[i];
          node_set<NJ>(c, 1 + d, static_cast<uint32_t>(nd.prmu[k]));
          node_set<NJ>(c, 1 + k, jd);
          uint4* o = reinterpret_cast<uint4*>(dst);
#pragma unroll
          for (int qq = 0; qq < VPN; ++qq) o[qq] = make_uint4(c[4 * qq], c[4 * qq + 1], c[4 * qq + 2], c[4 * qq + 3]);
          ++dst;
        }
      }
    }
    __syncthreads();
  }
  (void)sizeof(id_t);
}

// Reference-style evaluation (ref evaluate_gpu, PFSP_gpu_lib.cu:129-152): bounds of
// every child of `nparents` parents, bounds_out[offsets[i] + (k - depth_i)].
template <int NJ, int M, int LBK>
__global__ __launch_bounds__(kBlock) void pfsp_bounds_kernel(PfspArgs<NJ, M> a) {
  using G = PfspGeom<NJ, LBK, M>;
  using Node = PfspNode<NJ>;
  const int tid = threadIdx.x;
  if constexpr (LBK != 2) {
    constexpr int VPN = sizeof(Node) / 16;
    __shared__ PfspSmemLB1<NJ, M> sm;
    constexpr int MS = PfspConsts<M>::MS;
    uint16_t* pt = &sm.ptab[0][0];
    for (int i = tid; i < a.jobs * MS; i += kBlock) pt[i] = a.ptab[i];
    const int nchunks = (a.nparents + G::BP - 1) / G::BP;
    for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
      const int first = ch * G::BP;
      const int nvalid = min(G::BP, a.nparents - first);
      __syncthreads();
      for (int x = tid; x < nvalid * VPN; x += kBlock) {
        const int i = x / VPN, w = x - i * VPN;
        reinterpret_cast<uint4*>(&sm.node[i])[w] = reinterpret_cast<const uint4*>(a.parents_in + first + i)[w];
      }
      __syncthreads();
      if (tid < nvalid) {
        int* out = a.bounds_out + a.offsets[first + tid];
        pfsp_lb1_parent<NJ, M>(a, sm, tid, [&](int j, int, int lb) { out[j] = lb; });
      }
    }
  } else {
    __shared__ PfspSmem<NJ, M, LBK> sm;
    pfsp_stage_tables(a, sm);
    const int nchunks = (a.nparents + G::BP - 1) / G::BP;
    for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
      const int first = ch * G::BP;
      const int nvalid = min(G::BP, a.nparents - first);
      const int total =
          pfsp_phase_a<NJ, M, LBK>(a, sm, nvalid, [&](int i) -> const Node* { return a.parents_in + first + i; });
      for (int c = tid; c < total; c += kBlock) {
        int p, k, job;
        const int lb = pfsp_child_bound(a, sm, c, a.best_in, p, k, job);
        a.bounds_out[a.offsets[first + p] + (k - sm.node[p].depth)] = lb;
      }
      __syncthreads();
    }
  }
}

}  // namespace dev
}  // namespace tts
