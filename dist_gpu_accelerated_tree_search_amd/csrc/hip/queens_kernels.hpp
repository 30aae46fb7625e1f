// N-Queens backtracking kernel for gfx950.
//
// Reference (ref nqueens/nqueens_gpu_cuda.cu:143-171): one thread per (parent,
// column) label, re-reading the 21-B board per thread and scanning `depth` queens
// G times; labels go back to the host which builds the children.
//
// Here the node is three 32-bit attack masks (16 B, csrc/core/pfsp_node.hpp), so
// the safety test of all children is one AND; the kernel is pool-bandwidth bound.
// Per 256-thread workgroup and chunk of 256 parents:
//   Phase A  thread-per-parent: one 16-B load, free-row mask (G-times repeated test
//            kept as real work for -g), child counts scanned across the workgroup,
//            child->parent map in LDS, leaves (depth == N) counted as solutions.
//   Phase B  thread-per-child: the r-th free row of its parent via a 5-step popcount
//            search, then consecutive threads store consecutive 16-B children:
//            fully coalesced writes into the chunk's slot region of the device
//            pool (pool_device.hpp, no device atomics).
#pragma once

#include <climits>

#include "../core/pfsp_node.hpp"
#include "pool_device.hpp"

namespace tts {
namespace dev {

struct QueensArgs {
  PoolArgs<QueensNode> pool;
  int N;
  int G;
  uint32_t full;
  int finish_k;  // parents with at most this many columns left are explored to the end by their thread (0: off)
  // labels kernel only (reference-style evaluation, tests)
  const QueensNode* parents_in;
  uint8_t* labels_out;
  int nparents;
};

constexpr int kQueensFinishMax = 12;  // columns left at most in a finished subtree

// Nodes per wave in the LDS stack of the wave-cooperative subtree finishing (3 masks each).
// 448 keeps 5 workgroups per CU with the 2048-chunk window (4 with 4096 chunks) (N=17 finishing from 7 columns left:
// 768 / 448 / 320 / 256 / 192 nodes 37 / 32 / 34 / 32 / 37 ms; from 9 columns: 448 / 640
// nodes 21 / 22 ms; profiles/r6/queens/)
#ifndef TTS_QSTACK
#define TTS_QSTACK 448
#endif
constexpr int kQStack = TTS_QSTACK;

struct QueensSmem {
  static constexpr int BP = kBlock;
  static constexpr int MAXCH = BP * 32;
// (2048 chunks = a 2^19-parent window: the 8 KB of chunk prefix it saves give a fifth
// workgroup per CU, N=17 21 -> 20 ms)
#ifndef TTS_QMAXCHUNKS
#define TTS_QMAXCHUNKS 2048
#endif
  static constexpr int MAXCHUNKS = TTS_QMAXCHUNKS;
  // the level-by-level arrays of the chunk loop and the finishing stacks (after the
  // loop's last barrier) share their LDS
  union {
    struct {
      QueensNode node[BP];
      uint32_t avail[BP];
      int off[BP];
      uint8_t map[MAXCH];
    };
    uint32_t st[kBlock / kWave][3][kQStack];  // per wave: cols, diag, anti
  };
  int scan[kBlock / kWave];
  int red[kBlock / kWave];
  u64 fin[kBlock / kWave][2];
  PoolSmem<MAXCHUNKS> pool;
};

// Free rows of the next column. -g > 1 keeps the reference's artificial-work cost
// model (ref nqueens_c.c:80-96, nqueens_gpu_cuda.cu:143-171): every candidate row is
// tested G times against the `depth` placed queens, G * depth dependent compares per
// candidate. The mask node names no per-queen rows, so each compare step re-tests the
// candidate against the attack masks in a dependent chain the compiler cannot fold
// (same count and dependency as the reference's scan, same result as the one AND).
__device__ inline uint32_t queens_free_rows(const QueensNode& nd, uint32_t full, int G) {
  const uint32_t avail = ~(nd.cols | nd.diag | nd.anti) & full;
  if (G <= 1) return avail;
  const uint32_t att = nd.diag | nd.anti;
  const int depth = static_cast<int>(nd.depth);
  uint32_t ok = avail, cand = ~nd.cols & full;
  while (cand) {
    const uint32_t bit = cand & (0u - cand);
    cand ^= bit;
    uint32_t hit = 0;
    for (int g = 0; g < G; ++g)
      for (int i = 0; i < depth; ++i) {
        hit |= att & bit;
        asm volatile("" : "+v"(hit));
      }
    ok &= ~hit;
  }
  return ok;
}

// Subtree finishing. Near the bottom of the tree a node's whole subtree is small and
// generating it level by level through the device pool costs two 16-B global accesses per
// node; instead the parent's thread walks it depth-first with every level's masks in
// registers (template recursion = nested loops, no indexed stack) and counts with the
// pool's rules: every safe child is a pushed node (tree), a child in the last column is
// a complete board (sol) — the same tree as level-by-level expansion, -g work included.
// A flat loop with the levels' untried rows in LDS (every lane advancing on its own,
// no union of the lanes' trees) was measured 2x slower on N = 16 / 17
// (profiles/r2/queens/README.md): the register walk's passes are cheap enough that
// its divergence costs less than the flat loop's LDS round trips and branches.
template <int L>
__device__ inline void queens_dfs(uint32_t cols, uint32_t diag, uint32_t anti, int depth, const QueensArgs& a,
                                  u64& tree, u64& sol) {
  const QueensNode nd{cols, diag, anti, static_cast<uint32_t>(depth)};
  uint32_t av = queens_free_rows(nd, a.full, a.G);
  if (depth + 1 == a.N) {
    const int c = __popc(av);
    tree += static_cast<u64>(c);
    sol += static_cast<u64>(c);
    return;
  }
  if constexpr (L + 1 < kQueensFinishMax) {
    tree += static_cast<u64>(__popc(av));
    while (av) {
      const uint32_t bit = av & (0u - av);
      av ^= bit;
      queens_dfs<L + 1>(cols | bit, (diag | bit) << 1, (anti | bit) >> 1, depth + 1, a, tree, sol);
    }
  }
}

// Wave-cooperative subtree finishing. The wave's finishing parents go on an LDS stack
// (three mask arrays per wave, kQStack nodes); each pass pops up to 64 nodes from the top,
// one per lane, counts their safe children with the pool's rules (tree; sol in the last
// column) and pushes the children of nodes above the last column back on top, at offsets
// from a ballot prefix sum. Every lane bounds a node in every pass: no lane idles while
// another walks a longer subtree, which is what the register walk above pays for (a wave
// executes the union of its lanes' walks). A node whose children would not fit the stack
// is walked in registers by its lane (queens_dfs, same counts).
__device__ inline void queens_finish_wave(uint32_t (*st)[kQStack], int sp, const QueensArgs& a, u64& tree,
                                          u64& sol) {
  const int lane = static_cast<int>(threadIdx.x) & (kWave - 1);
  uint32_t t32 = 0, s32 = 0;
  while (sp > 0) {
    const int n = min(sp, kWave);
    const int base = sp - n;
    uint32_t cols = 0, diag = 0, anti = 0, av = 0;
    int depth = 0;
    if (lane < n) {
      cols = st[0][base + lane];
      diag = st[1][base + lane];
      anti = st[2][base + lane];
      depth = __popc(cols);
      av = queens_free_rows(QueensNode{cols, diag, anti, static_cast<uint32_t>(depth)}, a.full, a.G);
    }
    const int c = __popc(av);
    const bool last = depth + 1 == a.N;
    // (counting the next-to-last column's boards in the parent's lane instead of pushing
    // it measured slower: N=17 21 -> 25 ms, profiles/r6/queens/finish_depth_ab.txt)
    int cpush = last ? 0 : c;
    // exclusive wave prefix of the pushed counts: a stacked node has at most
    // kQueensFinishMax columns left, so at most 15 children (four ballots)
    static_assert(kQueensFinishMax < 16, "pushed counts must fit four bits");
    int off = 0, total = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u64 bal = __ballot((cpush >> k) & 1);
      off += static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u)))
             << k;
      total += __popcll(bal) << k;
    }
    const int room = kQStack - base;
    bool walk = false;
    if (total > room) {
      // the lanes from the first one whose children do not fit walk their nodes in registers
      const bool fits = cpush == 0 || off + cpush <= room;
      const u64 nf = __ballot(!fits);
      total = __builtin_amdgcn_readlane(off, static_cast<int>(__builtin_ctzll(nf)));
      walk = !fits;
    }
    if (walk) {
      queens_dfs<0>(cols, diag, anti, depth, a, tree, sol);
      cpush = 0;
    } else {
      t32 += static_cast<uint32_t>(c);
      if (last) s32 += static_cast<uint32_t>(c);
    }
    uint32_t m = cpush ? av : 0u;
    int p = base + off;
    while (m) {
      const uint32_t bit = m & (0u - m);
      m ^= bit;
      st[0][p] = cols | bit;
      st[1][p] = (diag | bit) << 1;
      st[2][p] = (anti | bit) >> 1;
      ++p;
    }
    __builtin_amdgcn_wave_barrier();
    sp = base + total;
  }
  tree += t32;
  sol += s32;
}

// Position of the r-th (0-based) set bit of x (r < popcount(x)).
__device__ inline int nth_set_bit(uint32_t x, int r) {
  int pos = 0;
#pragma unroll
  for (int w = 16; w > 0; w >>= 1) {
    const int c = __popc(x & ((1u << w) - 1u));
    if (r >= c) {
      r -= c;
      x >>= w;
      pos += w;
    }
  }
  return pos;
}

__global__ __launch_bounds__(kBlock) void queens_expand_kernel(QueensArgs a, int t) {
  using S = QueensSmem;
  __shared__ QueensSmem sm;
  const int tid = threadIdx.x;
  const auto& pa = a.pool;
  const IterView v = pool_begin<QueensNode, S::MAXCHUNKS>(pa, t, S::BP, sm.pool);
  if (v.B == 0 || v.overflow) return;
  QueensNode* const bout = pa.buf[(t & 1) ^ 1];
  int* const cnt_out = pa.cnt[(t & 1) ^ 1];
  int* const lcnt_out = pa.lcnt[(t & 1) ^ 1];
  pool_spill_leftovers<QueensNode, S::MAXCH, S::MAXCHUNKS>(pa, v, t, sm.pool);

  // finishing (not while the pool is replicated across ranks: the split must see it)
  const int fin_from = (a.finish_k > 0 && !v.armed) ? a.N - a.finish_k : INT_MAX;
  u64 ftree = 0, fsol = 0;
  for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
    const u64 gi = static_cast<u64>(ch) * S::BP + tid;
    int nchild = 0, leaf = 0;
    if (gi < v.B) {
      const QueensNode nd = *pool_parent<QueensNode, S::MAXCH, S::MAXCHUNKS>(pa, v, t, gi, sm.pool);
      sm.node[tid] = nd;
      if (static_cast<int>(nd.depth) == a.N) {
        // a leaf parent of the split iteration is replicated on every rank: rank 0 counts it
        leaf = (!v.split || v.srank == 0) ? 1 : 0;
      } else if (static_cast<int>(nd.depth) >= fin_from) {
        // finished after the chunk loop, outside its barriers (no child, no leaf here)
      } else {
        uint32_t av = queens_free_rows(nd, a.full, a.G);
        if (v.split) {
          uint32_t keep = 0;
          for (int r = 0; r < 32; ++r) keep |= split_keep(v, gi, r) ? (1u << r) : 0u;
          av &= keep;
        }
        sm.avail[tid] = av;
        nchild = __popc(av);
      }
    }
    int total = 0, leaves = 0;
    const int off = block_exclusive_scan(nchild, sm.scan, &total);
    (void)block_exclusive_scan(leaf, sm.red, &leaves);
    sm.off[tid] = off;
    for (int j = 0; j < nchild; ++j) sm.map[off + j] = static_cast<uint8_t>(tid);
    if (tid == 0) {
      cnt_out[ch] = total;
      lcnt_out[ch] = leaves;
    }
    __syncthreads();
    QueensNode* const dst = bout + static_cast<size_t>(ch) * S::MAXCH;
    for (int c = tid; c < total; c += kBlock) {
      const int p = sm.map[c];
      const QueensNode nd = sm.node[p];
      const uint32_t bit = 1u << nth_set_bit(sm.avail[p], c - sm.off[p]);
      dst[c] = QueensNode{nd.cols | bit, (nd.diag | bit) << 1, (nd.anti | bit) >> 1, nd.depth + 1};
    }
    __syncthreads();
  }
  if (fin_from != INT_MAX) {
    // the subtrees of this workgroup's finishing parents (read again from the window):
    // no barrier between them, so a wave with a deep subtree holds up no other wave
    // wave priority falls with the chunks a workgroup has finished: the CU's late-dispatched
    // workgroups catch up instead of trailing (N=17 170 -> 174 G nodes/s,
    // profiles/r5/queens_prio_ab.txt; the same age-priority effect as front_local's)
    int k = 0;
#ifndef TTS_QUEENS_REGWALK_AB
    uint32_t (*const st)[kQStack] = sm.st[tid / kWave];
#endif
    for (int ch = blockIdx.x; ch < v.nchunks; ch += gridDim.x) {
      if (k == 0) __builtin_amdgcn_s_setprio(3);
      else if (k == 1) __builtin_amdgcn_s_setprio(2);
      else if (k == 2) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      ++k;
      const u64 gi = static_cast<u64>(ch) * S::BP + tid;
      QueensNode nd{0, 0, 0, 0};
      bool fin = false;
      if (gi < v.B) {
        nd = *pool_parent<QueensNode, S::MAXCH, S::MAXCHUNKS>(pa, v, t, gi, sm.pool);
        const int d = static_cast<int>(nd.depth);
        fin = d < a.N && d >= fin_from;
      }
#ifdef TTS_QUEENS_REGWALK_AB  // (A/B builds only: the per-lane register walk)
      if (fin) queens_dfs<0>(nd.cols, nd.diag, nd.anti, static_cast<int>(nd.depth), a, ftree, fsol);
#else
      // this wave's finishing parents start its stack (at most 64 <= kQStack)
      const u64 bal = __ballot(fin);
      if (fin) {
        const int pos = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u)));
        st[0][pos] = nd.cols;
        st[1][pos] = nd.diag;
        st[2][pos] = nd.anti;
      }
      __builtin_amdgcn_wave_barrier();
      queens_finish_wave(st, __popcll(bal), a, ftree, fsol);
#endif
    }
    // one pair of 64-bit adds per workgroup, on the line of its 8th of the grid
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      ftree += __shfl_xor(ftree, o, kWave);
      fsol += __shfl_xor(fsol, o, kWave);
    }
    if ((tid & (kWave - 1)) == 0) {
      sm.fin[tid / kWave][0] = ftree;
      sm.fin[tid / kWave][1] = fsol;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < kBlock / kWave; ++w) {
        ftree += sm.fin[w][0];
        fsol += sm.fin[w][1];
      }
      if (ftree | fsol) {
        auto& x = pa.ctl->xacc[blockIdx.x & 7];
        __hip_atomic_fetch_add(&x.tree, ftree, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&x.sol, fsol, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Reference-style labels (ref evaluate_gpu): labels[i*N + k] = 1 iff row k is a
// safe, unused row for parent i. (The reference labels board positions; with the
// mask node the label index is the row itself.)
__global__ __launch_bounds__(kBlock) void queens_labels_kernel(QueensArgs a) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.nparents) return;
  const QueensNode nd = a.parents_in[i];
  const uint32_t av = static_cast<int>(nd.depth) == a.N ? 0u : queens_free_rows(nd, a.full, a.G);
  for (int k = 0; k < a.N; ++k) a.labels_out[static_cast<size_t>(i) * a.N + k] = (av >> k) & 1u;
}

}  // namespace dev
}  // namespace tts
