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
//            fully coalesced writes into the device pool after ONE device atomic
//            per chunk reserved the slots.
#pragma once

#include "../core/pfsp_node.hpp"
#include "device_common.hpp"

namespace tts {
namespace dev {

struct QueensArgs {
  QueensNode* stack;
  QueensNode* buf[2];
  PoolCtl* ctl;
  u64 cap_mask;
  int N;
  int G;
  int max_parents;
  uint32_t full;
  // labels kernel only (reference-style evaluation, tests)
  const QueensNode* parents_in;
  uint8_t* labels_out;
  int nparents;
};

struct QueensSmem {
  static constexpr int BP = kBlock;
  static constexpr int MAXCH = BP * 32;
  QueensNode node[BP];
  uint32_t avail[BP];
  int off[BP];
  uint8_t map[MAXCH];
  int scan[kBlock / kWave];
  u64 base;
};

__device__ inline uint32_t queens_free_rows(const QueensNode& nd, uint32_t full, int G) {
  uint32_t avail = ~(nd.cols | nd.diag | nd.anti) & full;
  for (int g = 1; g < G; ++g) {  // -g: repeat the safety test (artificial work)
    uint32_t again = ~(nd.cols | nd.diag | nd.anti) & full;
    asm volatile("" : "+v"(again));
    avail &= again;
  }
  return avail;
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
  __shared__ QueensSmem sm;
  const int tid = threadIdx.x;
  const int s_in = t % 3, s_out = (t + 1) % 3, s_zero = (t + 2) % 3;
  QueensNode* const bin = a.buf[t & 1];
  QueensNode* const bout = a.buf[(t & 1) ^ 1];
  PoolCtl* ctl = a.ctl;

  const u64 S = ctl->stack[s_in].v;
  const u64 Cn = ctl->buf[s_in].v;
  const u64 bot = ctl->bot;
  const u64 B = min(S + Cn, static_cast<u64>(a.max_parents));
  const u64 nb = min(B, Cn);
  const u64 ns = B - nb;
  const u64 L = Cn - nb;
  const u64 Snew = S - ns + L;
  const bool overflow = Snew > a.cap_mask + 1;
  if (blockIdx.x == 0 && tid == 0) {
    ctl->stack[s_out].v = overflow ? S : Snew;
    ctl->stack[s_zero].v = 0;
    ctl->buf[s_zero].v = 0;
    if (B > 0) {
      ctl->parents += B;
      ctl->iters += 1;
    }
    if (overflow) ctl->overflow = 1;
  }
  if (B == 0 || overflow) return;

  for (u64 i = static_cast<u64>(blockIdx.x) * kBlock + tid; i < L; i += static_cast<u64>(gridDim.x) * kBlock)
    a.stack[(bot + S + i) & a.cap_mask] = bin[i];

  const u64 nchunks = (B + QueensSmem::BP - 1) / QueensSmem::BP;
  u64 my_sol = 0;
  for (u64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const u64 gi = ch * QueensSmem::BP + tid;
    int nchild = 0;
    if (gi < B) {
      const QueensNode nd = gi < nb ? bin[Cn - nb + gi] : a.stack[(bot + S - ns + (gi - nb)) & a.cap_mask];
      sm.node[tid] = nd;
      if (static_cast<int>(nd.depth) == a.N) {
        ++my_sol;
      } else {
        const uint32_t av = queens_free_rows(nd, a.full, a.G);
        sm.avail[tid] = av;
        nchild = __popc(av);
      }
    }
    int total = 0;
    const int off = block_exclusive_scan(nchild, sm.scan, &total);
    sm.off[tid] = off;
    for (int j = 0; j < nchild; ++j) sm.map[off + j] = static_cast<uint8_t>(tid);
    if (tid == 0) {
      sm.base = total ? atomicAdd(&ctl->buf[s_out].v, static_cast<u64>(total)) : 0;
      if (total) atomicAdd(&ctl->tree.v, static_cast<u64>(total));
    }
    __syncthreads();
    const u64 base = sm.base;
    for (int c = tid; c < total; c += kBlock) {
      const int p = sm.map[c];
      const QueensNode nd = sm.node[p];
      const uint32_t bit = 1u << nth_set_bit(sm.avail[p], c - sm.off[p]);
      bout[base + c] = QueensNode{nd.cols | bit, (nd.diag | bit) << 1, (nd.anti | bit) >> 1, nd.depth + 1};
    }
    __syncthreads();
  }
  u64 s = my_sol;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
  if ((tid & (kWave - 1)) == 0 && s) atomicAdd(&ctl->sol.v, s);
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
