// Device-resident pool shared by every search kernel — atomic-free.
//
// Layout (per GPU):
//   ring    the stack, ring[(bot + i) & mask] for i < stack size (HBM, 2^k nodes)
//   bufs    two children buffers (ping-pong). Iteration t expands up to
//           max_parents parents in chunks of BP; chunk c writes its surviving
//           children to buf[(t+1)%2][c * MAXCH ...] and their count to cnt[c]
//           (leaves it evaluated to lcnt[c]). No device atomics: the next
//           iteration rebuilds the exclusive prefix of cnt[] in LDS (every
//           workgroup, a few KB of L2 reads) and addresses child i of the
//           buffer through a binary search of that prefix.
//   ctl     per-iteration scalars in 3 rotating slots (t%3 read, (t+1)%3
//           written by workgroup 0), counters, incumbent.
// Iteration t: parents = the top of [ring ++ buffer] (buffer first: DFS), the
// buffer's unexpanded part is appended to the ring, children -> other buffer.
// Nothing goes back to the host per iteration and no two workgroups ever touch
// the same word, except the incumbent (atomicMin, leaves only).
//
// Why not one atomic slot counter per chunk: measured on MI355X, 1024 returning
// atomicAdds on one word per iteration serialise at ~88/us (~12 us per
// iteration, profiles/r1/r1_baseline); the prefix costs ~1 us of LDS work.
#pragma once

#include <cstddef>

#include "device_common.hpp"

namespace tts {
namespace dev {

struct PoolCtl {
  // Rotating per-iteration state, one 128-B line per slot so an iteration's
  // inputs arrive in one load: iteration t reads slot t%3, workgroup 0 writes
  // slot (t+1)%3.
  struct alignas(128) Slot {
    u64 stack;  // ring occupancy at the start of iteration t
    int nch;    // chunks written by iteration t-1 into buffer t%2
    int sdone;  // armed rank split already done (see split_world)
    // -u 0 dive: parent-window cap of iteration t (0: none). A solve that starts without
    // an incumbent expands at most this many parents per iteration — the top of the
    // stack, so the search dives depth-first to its first leaves (ref pfsp_c.c:55-63,
    // DFS from +inf) — and the cap widens by 2^dive_shift per iteration once a leaf set
    // the incumbent, back to the full window
    unsigned cap;
    unsigned cpad;  // the incumbent iteration t-1 saw (dive: widen when it stops improving)
  };
  Slot slot[3];
  // plain counters, updated by workgroup 0 (or the host between launches)
  u64 tree;         // pushed children (explored tree), lags one iteration
  u64 sol;          // evaluated leaves (explored solutions), lags one iteration
  u64 parents;      // parents expanded (diagnostics)
  u64 iters;        // iterations that had work (diagnostics)
  u64 bot;          // ring base
  u64 pend_children;  // children in the latest buffer (finalize kernel)
  u64 pend_leaves;    // leaves counted by the latest iteration (finalize kernel)
  u64 pend_internal;  // children pushed and expanded inside the latest (two-level) iteration
  u64 seq;            // finalize kernels run so far; published LAST to the host mirror
  int overflow;       // 1: ring too small, 2: pool outgrew the window before a pending split
  // In-graph rank split (multi-rank solves): every rank starts from the same nodes
  // and runs identical iterations until the first one whose window holds at least
  // split_min parents (and the whole pool); that iteration keeps only the children
  // whose (parent, position) hash falls on split_rank (split_keep), and ranks != 0
  // drop the replicated counts gathered so far. Same line as `bot`.
  int split_world;    // <= 1: no split armed
  int split_rank;
  int dive_shift;     // -u 0 dive: log2 of the cap's growth per iteration after the first leaf
  u64 split_min;
  // Pruning threshold of replicated iterations (prune_best): the incumbent the solve began
  // with (or the warm_split passes start from)
  int best0;
  int pad0;
  // nodes pushed and leaves counted inside subtrees a thread explored to the end (N-Queens
  // finishing: 64-bit counts, one accumulator line per 8th of the grid; the host folds them)
  struct alignas(128) XAcc {
    u64 tree, sol;
    u64 pad[14];
  } xacc[8];
  CtlI32 best;      // incumbent (atomicMin by leaves)
};

// Dynamic local DFS iterations (kernels that implement them, front_dyn): one iteration's
// control, in 3 rotating sets — iteration t uses set t % 3 and zeroes set (t + 1) % 3 for
// the next one (the slot rotation of PoolCtl; kernels of one stream never overlap).
// Work moves between the workgroups of ONE XCD (partition = the XCC id read from the
// hardware, so the L2 every hand-off goes through is shared by construction): a workgroup
// whose stack holds more than it needs publishes one pop (<= kBlock nodes) into a free
// slot of its partition; a workgroup whose stack ran dry claims a full slot. Slots are
// chunk regions past the workgroups' own ([grid, grid + qn) of the output buffer), so a
// block nobody claimed is simply an output chunk (its count written by the last
// workgroup to leave).
constexpr int kDynQMax = 1024;
struct DynCtl {
  struct alignas(128) Part {
    int hungry;  // workgroups of the partition waiting for a block
    int avail;   // full slots (hungry and avail: one 8-B load)
    int busy;    // workgroups of the partition with work (a stack or a claimed block)
    int pad[29];
  } part[8];
  struct alignas(128) Fin {
    int n;
    int pad[31];
  } fin[9];  // workgroups gone per blockIdx % 8 group; [8]: groups gone
  // slot state: 0 free, 1 being written, 2 | n << 8 full (n nodes), 3 | n << 8 being read
  unsigned st[kDynQMax];
};

template <class Node>
struct PoolArgs {
  Node* ring;
  Node* buf[2];
  int* cnt[2];
  int* lcnt[2];
  PoolCtl* ctl;
  PoolCtl* mirror;  // host-mapped pinned copy written by the finalize kernel
  u64 cap_mask;
  int max_parents;
  int max_chunks;
  int fuse_max;     // two-level iterations for windows of at most this many parents (0: off)
  int local_steps;  // > 1: local DFS iterations of up to this many steps per chunk (kernels that have them)
  int local_min;    // wide local DFS when the pool holds at least this many parents (0: 4 grid windows)
  int local_stride;    // local DFS chunks take strided window parents (ch, ch + nchunks, ...)
  int local_wide_steps;  // > 0: steps of a strided local window of at least 160 parents per workgroup
  // multi-level iterations (kernels with LMAX > 2): a fused window of at most deep_per[0]
  // parents per workgroup is expanded 3 levels deep, of at most deep_per[1] 4 levels deep
  // (capped by deep_levels); 2 levels otherwise
  int deep_levels;
  int deep_per[2];
  // wide multi-level iterations: a window of more than a narrow chunk's parents per
  // workgroup but at most one per thread is expanded this many levels deep (< 2: off)
  int wide_levels;
  // 1: prune with ctl->best0, not the live incumbent (warm_split passes, identical on every rank)
  int prune_fixed;
  // dynamic local DFS (front kernel): 3 DynCtl sets (null: off), the time budget of
  // one iteration in wall-clock ticks (100 MHz) and the queue slots (a multiple of 8)
  DynCtl* dyn;
  int dyn_ticks;
  int dyn_q;
  // iteration log (probe builds: -DTTS_ILOG_BUILD, scripts/build_variant.py; env TTS_ILOG):
  // word 0 counts records, record r
  // at 8 + 8 r holds {wall clock at pool_begin, S, C, B, shape word, tree so far, t, 0}
  u64* ilog;
};

// Shape word of an iteration log record: chunks | bp << 20 | steps << 36 | flags << 44
// (bit 0 local, 1 stride, 2 fused, 3 split, 4 armed, 5 overflow; levels << 48).
__device__ inline void ilog_record(u64* ilog, u64 clk, u64 S, u64 C, u64 B, int nchunks, int bp, int steps,
                                   int flags, int levels, u64 tree, int t) {
  const u64 r = ilog[0];
  if (r >= 4095) return;
  u64* x = ilog + 8 + 8 * r;
  x[0] = clk;
  x[1] = S;
  x[2] = C;
  x[3] = B;
  x[4] = static_cast<u64>(nchunks) | (static_cast<u64>(bp) << 20) | (static_cast<u64>(steps & 0xff) << 36) |
         (static_cast<u64>(flags & 0xff) << 44) | (static_cast<u64>(levels & 0xf) << 48);
  x[5] = tree;
  x[6] = static_cast<u64>(t);
  ilog[0] = r + 1;
}

// Per-chunk leaf word: leaves in the low 16 bits; the high 16 bits count the
// children a two-level iteration pushed and expanded itself (explored tree).
__device__ inline int lcnt_leaves(int x) { return x & 0xffff; }
__device__ inline int lcnt_inner(int x) { return static_cast<int>(static_cast<uint32_t>(x) >> 16); }

template <int MAXCHUNKS>
struct PoolSmem {
  int pre[MAXCHUNKS + 1];
  int scan[kBlock / kWave];
  int red[kBlock / kWave];
  u64 red64[kBlock / kWave][6];
};

// Exclusive prefix of cnt[0..n) into pre[0..n] (pre[n] = total) by one workgroup.
// Every count is loaded in one memory round trip (R predicated loads per thread,
// unrolled, coalesced, staged in LDS), then each thread scans a contiguous run from
// LDS: a loop of dependent global loads here cost ~3 round trips per kernel start
// (s_waitcnt after every load pair in the ISA).
template <int MAXCHUNKS>
__device__ inline int build_prefix(const int* cnt, int n, PoolSmem<MAXCHUNKS>& ps) {
  constexpr int R = (MAXCHUNKS + kBlock - 1) / kBlock;
  const int tid = static_cast<int>(threadIdx.x);
  int x[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = tid + k * kBlock;
    x[k] = i < n ? cnt[i] : 0;
  }
#pragma unroll
  for (int k = 0; k < R; ++k)
    if (tid + k * kBlock < n) ps.pre[tid + k * kBlock] = x[k];
  __syncthreads();
  const int per = (n + kBlock - 1) / kBlock;
  const int lo = min(n, tid * per);
  const int hi = min(n, lo + per);
  int s = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    x[k] = lo + k < hi ? ps.pre[lo + k] : 0;
    s += x[k];
  }
  int total = 0;
  int run = block_exclusive_scan(s, ps.scan, &total);  // (its barrier: every run read)
#pragma unroll
  for (int k = 0; k < R; ++k)
    if (lo + k < hi) {
      ps.pre[lo + k] = run;
      run += x[k];
    }
  if (threadIdx.x == 0) ps.pre[n] = total;
  __syncthreads();
  return total;
}

// Sums over the per-chunk leaf words lcnt[0..n) (leaves, inner nodes) by one workgroup:
// all loads in one round trip.
template <int MAXCHUNKS>
__device__ inline void sum_leaf_words(const int* lcnt, int n, int& lf, int& in) {
  constexpr int R = (MAXCHUNKS + kBlock - 1) / kBlock;
  int x[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = static_cast<int>(threadIdx.x) + k * kBlock;
    x[k] = i < n ? lcnt[i] : 0;
  }
  lf = in = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    lf += lcnt_leaves(x[k]);
    in += lcnt_inner(x[k]);
  }
}

// Chunk holding buffered child li: the largest c < n with pre[c] <= li.
__device__ inline int find_chunk(const int* pre, int n, int li) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= li)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

struct IterView {
  u64 S, C, B, nb, ns, L, Snew, bot;
  int nch_in, nchunks;
  bool overflow;
  bool split;         // this iteration splits the (replicated) pool between ranks
  bool fused;         // multi-level iteration: chunks of BPF parents, `levels` tree levels deep
  int levels;         // fused iterations: tree levels expanded per chunk (2..LMAX)
  bool local;         // local DFS iteration: each chunk steps on its own stack
  bool stride;        // local DFS: chunk ch takes window parents ch, ch + nchunks, ... (pa.local_stride)
  int bp;             // window parents per chunk
  int steps;          // local DFS: steps per chunk at most
  int srank, sworld;
  bool armed;         // a rank split is pending: the pool is replicated on every rank
  bool dyn;           // dynamic local DFS (front_dyn): chunk ch = workgroup ch, queue chunks after them
  int qn;             // dynamic: queue slots (output chunks [nchunks, nchunks + qn))
};

// Zero the DynCtl set the next iteration uses (workgroup 0, every launch of a kernel that
// has dynamic iterations; busy starts at 0 and counts workgroups in as they start).
__device__ inline void dyn_zero_next(DynCtl* dyn, int t) {
  if (!dyn || blockIdx.x != 0) return;
  uint32_t* d = reinterpret_cast<uint32_t*>(dyn + (t + 1) % 3);
  for (int i = threadIdx.x; i < static_cast<int>(sizeof(DynCtl) / 4); i += kBlock) d[i] = 0;
}

// Does this rank keep child position k of window parent gi? (always, outside the
// split iteration). The owner is a hash of (gi, k) (splitmix64 finalizer): a plain
// (gi * 1024 + k) % world would hand every child position k to one rank when
// world divides 1024, and sibling subtrees are strongly correlated in size.
__device__ inline bool split_keep(const IterView& v, u64 gi, int k) {
  if (!v.split) return true;
  u64 x = gi * 1024ull + static_cast<u64>(k) + 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  x ^= x >> 31;
  return (x % static_cast<u64>(v.sworld)) == static_cast<u64>(v.srank);
}

// Everything an iteration needs to know, identical in every workgroup; workgroup
// 0 also publishes the next slot and folds the previous iteration's counts.
template <class Node, int MAXCHUNKS>
//
// Two-level iterations (BPF > 0, kernels that implement them): a window of at most
// pa.fuse_max parents, outside a pending rank split, is expanded two tree levels
// deep in chunks of BPF parents — one dependent kernel instead of two where an
// iteration is latency-bound (few parents), same chunk slot layout.
//
// Local DFS iterations (LT > 1 and pa.local_steps > 1): the window is dealt out over
// the grid (chunks of at most BP parents) and each workgroup keeps expanding the top
// of its chunk's own slot region — a private stack in L2 — for up to local_steps
// levels; what is left on the stack is the chunk's output. Several tree levels per
// dependent kernel, and the next iteration re-deals the stacks over the grid.
__device__ inline IterView pool_begin(const PoolArgs<Node>& pa, int t, int BP, PoolSmem<MAXCHUNKS>& ps,
                                      int BPF = 0, int LT = 1, int GROW2 = 0, int LMAX = 2, bool DYN = false) {
  const int s_in = t % 3, s_out = (t + 1) % 3;
  const int b_in = t & 1;
  PoolCtl* ctl = pa.ctl;
  // The slot and the control line are loaded together (one round trip). The
  // per-chunk counts are read once nch is known: reading the whole window's
  // counts speculatively in the same round trip made ta014 slower (0.32 -> 0.39
  // ms, profiles/r1/r1q: cold count lines), though ta008 gained 4 %.
  IterView v;
  v.S = ctl->slot[s_in].stack;
  v.nch_in = ctl->slot[s_in].nch;
  const int done_in = ctl->slot[s_in].sdone;
  const unsigned cap_in = ctl->slot[s_in].cap;
  v.bot = ctl->bot;
  v.sworld = ctl->split_world;
  v.srank = ctl->split_rank;
  const u64 split_min = ctl->split_min;
  if (v.S == 0 && v.nch_in == 0) {
    // empty pool (the tail of a replay that outlived its tree): hand the slot on
    // and leave — no table staging, no scans, no counter traffic
    v.C = v.B = v.nb = v.ns = v.L = v.Snew = v.bot = 0;
    v.nchunks = 0;
    v.overflow = v.split = v.fused = v.local = v.armed = v.stride = v.dyn = false;
    v.qn = 0;
    v.levels = 1;
    if (DYN) dyn_zero_next(pa.dyn, t);
    v.bp = BP;
    v.steps = 0;
    v.srank = v.sworld = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      ctl->slot[s_out].stack = 0;
      ctl->slot[s_out].nch = 0;
      ctl->slot[s_out].sdone = done_in;
      ctl->slot[s_out].cap = cap_in;
      ctl->slot[s_out].cpad = ctl->slot[s_in].cpad;
#ifdef TTS_ILOG_BUILD  // (probe builds only: its live values made the front kernel spill)
      if (pa.ilog) ilog_record(pa.ilog, wall_clock64(), 0, 0, 0, 0, 0, 0, 0, 0, ctl->tree, t);
#endif
    }
    return v;
  }
  // uniform by construction: readfirstlane keeps the window arithmetic in SGPRs
  v.C = static_cast<u64>(__builtin_amdgcn_readfirstlane(build_prefix(pa.cnt[b_in], v.nch_in, ps)));
  v.B = min(v.S + v.C, static_cast<u64>(pa.max_parents));
  // the dive cap never applies while a rank split is pending (the split iteration needs
  // the whole replicated pool in its window)
  if (cap_in != 0 && !(v.sworld > 1 && !done_in)) v.B = min(v.B, static_cast<u64>(cap_in));
  const bool armed = v.sworld > 1 && !done_in && v.B > 0;
  v.armed = armed;
  // Local DFS when the pool holds a backlog of pa.local_min parents (default: four
  // grid-filling windows of BP-parent chunks), never while the pool is replicated
  // (the split must see every level). Below that, breadth (one level per kernel,
  // every chunk short) keeps the grid busier than chunks that step for different
  // lengths. A local window is one chunk per workgroup, at most BP parents each: a
  // workgroup's steps are not queued behind another chunk's. (A narrow-window variant
  // for the ramp-up and the tail measured slower and was removed: profiles/r2/.)
  const u64 full = static_cast<u64>(gridDim.x) * BP;
  const u64 lmin = pa.local_min > 0 ? static_cast<u64>(pa.local_min) : 4 * full;
  // (an explicit pa.local_min may be below one grid window: wide BFS levels of a small
  // tree then also take a few local steps per dependent kernel)
  v.local = LT > 1 && pa.local_steps > 1 && !armed && v.S + v.C >= (pa.local_min > 0 ? lmin : max(lmin, full));
  v.steps = pa.local_steps;
  // strided local windows below a backlog of four grid windows (a tree's wide levels); on a
  // backlog (ta021 LB1_d: millions of pooled nodes) contiguous dealing was faster
  v.stride = v.local && pa.local_stride && v.S + v.C < 4 * full;
  // wide strided windows (a tree's widest levels, full 256-node pops) take fewer steps: a
  // step more there mostly lengthens the slowest workgroup (ta014 one rank: 3 steps 0.215
  // vs 4 steps 0.219 ms; under the step priority 3 / 4 / 5 steps 0.206 / 0.210 / 0.215 ms,
  // profiles/r5/steps_ab.txt)
  if (v.stride && pa.local_wide_steps > 0 && min(v.B, full) >= 160ull * gridDim.x) v.steps = pa.local_wide_steps;
  // dynamic local DFS: every workgroup owns its chunk (the window dealt strided over the
  // grid) and steps until the time budget, sharing work through the queue slots
  v.dyn = DYN && v.local && pa.dyn != nullptr && pa.dyn_ticks > 0 && pa.dyn_q > 0 &&
          static_cast<int>(gridDim.x) + pa.dyn_q <= pa.max_chunks;
  v.qn = v.dyn ? pa.dyn_q : 0;
  if (v.dyn) v.stride = true;
  if (DYN) dyn_zero_next(pa.dyn, t);
  if (v.local) v.B = min(v.B, full);
  v.nb = min(v.B, v.C);
  v.ns = v.B - v.nb;
  v.L = v.C - v.nb;
  v.Snew = v.S - v.ns + v.L;
  v.overflow = v.Snew > pa.cap_mask + 1;
  // a pending split needs the whole (replicated) pool inside the window
  const bool bad_split = armed && v.B < v.S + v.C;
  v.split = armed && !bad_split && v.B >= split_min;
  // Two-level iterations also run while a rank split is armed (the replicated prefix
  // of a multi-rank solve), but never as the split iteration itself, and only while
  // two levels of growth (at most GROW2 grandchildren per parent) cannot carry the
  // pool past the parent window before the split.
  const bool fuse_armed = armed && !(v.B >= split_min) &&
                          v.B * static_cast<u64>(max(GROW2, 1)) <= static_cast<u64>(pa.max_parents) && GROW2 > 0;
  // (the split iteration itself is fused too when the kernel passes LMAX > 2: its first
  // level keeps this rank's children, the second expands them)
  const bool fuse_split = v.split && LMAX > 2 && GROW2 > 0;
  v.fused = !v.local && BPF > 0 && (!armed || fuse_armed || fuse_split) &&
            v.B <= static_cast<u64>(min(pa.fuse_max, BPF * pa.max_chunks));
  int bp = BP;
  v.levels = v.fused ? 2 : 1;
  if (v.fused) {
    // up to BPF parents per two-level chunk, fewer when the window is narrower than the
    // grid: more workgroups share a narrow window (each with fewer serial passes). While
    // a split is armed the pool order must not depend on the grid (every rank deals the
    // same frontier by position): the window is then spread over a fixed 1024 chunks
    // instead of the grid (chunk order, not workgroup order, lays out the output). Never
    // more chunks than the count / slot arrays hold (max_chunks; the grid is within it).
    const u64 spread = min(armed ? 1024ull : static_cast<u64>(gridDim.x), static_cast<u64>(pa.max_chunks));
    const u64 per = (v.B + spread - 1) / spread;
    bp = static_cast<int>(min(static_cast<u64>(BPF), max(per, 1ull)));
    // narrower windows go deeper: 3 or 4 levels per dependent kernel while a chunk's
    // levels stay in LDS (never while armed: the split must see the replicated levels)
    const int lmax = min(LMAX, pa.deep_levels);
    if (!armed && lmax >= 3 && per <= static_cast<u64>(pa.deep_per[0])) v.levels = 3;
    if (!armed && lmax >= 4 && per <= static_cast<u64>(pa.deep_per[1])) v.levels = 4;
  } else if (LMAX > 2 && !v.local && !armed && pa.wide_levels >= 2 && v.B <= static_cast<u64>(pa.fuse_max) &&
             (v.B + gridDim.x - 1) / gridDim.x <= static_cast<u64>(BP)) {
    // wide multi-level: every workgroup takes one chunk of up to one parent per thread
    // (the kernel's first level runs from the pool, the next ones from LDS)
    v.fused = true;
    bp = static_cast<int>(max((v.B + gridDim.x - 1) / gridDim.x, 1ull));
    v.levels = min(pa.wide_levels, LMAX);
  }
  if (v.local) {
    // spread a window smaller than the grid over every workgroup
    const u64 per = (v.B + gridDim.x - 1) / gridDim.x;
    bp = static_cast<int>(min(static_cast<u64>(BP), max(per, 1ull)));
  }
  v.bp = bp;
  v.nchunks = v.dyn ? static_cast<int>(gridDim.x) : static_cast<int>((v.B + bp - 1) / bp);
  const bool overflow = v.overflow;
  v.overflow = overflow || bad_split;
  if (blockIdx.x == 0) {
    // leaves evaluated by the previous iteration
    int lf = 0, in = 0;
    sum_leaf_words<MAXCHUNKS>(pa.lcnt[b_in], v.nch_in, lf, in);
    int lf_total = 0, in_total = 0;
    (void)block_exclusive_scan(lf, ps.red, &lf_total);
    (void)block_exclusive_scan(in, ps.scan, &in_total);
    if (threadIdx.x == 0) {
      ctl->slot[s_out].stack = v.overflow ? v.S : v.Snew;
      ctl->slot[s_out].nch = v.overflow ? 0 : v.nchunks + v.qn;
      ctl->slot[s_out].sdone = (done_in || v.split) ? 1 : 0;
      {
        // the dive cap holds until a leaf set the incumbent, then widens geometrically
        // (dive_shift bit 8: hold the cap while the incumbent still improves, like a DFS
        // that keeps finding better leaves; widen once an iteration brought no improvement)
        unsigned cap = cap_in;
        const unsigned b = static_cast<unsigned>(__hip_atomic_load(&ctl->best.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const unsigned prev = ctl->slot[s_in].cpad;
        if (cap != 0 && b != 0x7fffffffu && !((ctl->dive_shift & 0x100) && b < prev)) {
          const u64 w = static_cast<u64>(cap) << max(0, min(ctl->dive_shift & 0xff, 16));
          cap = w >= static_cast<u64>(pa.max_parents) ? 0u : static_cast<unsigned>(w);
        }
        ctl->slot[s_out].cap = cap;
        ctl->slot[s_out].cpad = b;
      }
      if (v.split && v.srank != 0) {
        // everything counted so far was explored identically by every rank: rank 0 keeps it
        ctl->tree = 0;
        ctl->sol = 0;
      } else {
        ctl->tree += v.C + static_cast<u64>(in_total);
        ctl->sol += static_cast<u64>(lf_total);
      }
      if (v.B > 0) {
        ctl->parents += v.B;
        ctl->iters += 1;
      }
      if (overflow) ctl->overflow = 1;
      else if (bad_split) ctl->overflow = 2;
#ifdef TTS_ILOG_BUILD
      if (pa.ilog)
        ilog_record(pa.ilog, wall_clock64(), v.S, v.C, v.B, v.nchunks, v.bp, v.local ? v.steps : 0,
                    (v.local ? 1 : 0) | (v.stride ? 2 : 0) | (v.fused ? 4 : 0) | (v.split ? 8 : 0) |
                        (v.armed ? 16 : 0) | (v.overflow ? 32 : 0) | (v.dyn ? 64 : 0),
                    v.levels, ctl->tree, t);
#endif
    }
  }
  return v;
}

// The incumbent an iteration prunes with. While a rank split is pending (or in the
// warm_split passes: pa.prune_fixed) every rank must expand the replicated iterations identically, and the live
// incumbent is not a rank-independent value there: a leaf found by one workgroup lowers it
// for the workgroups that start later in the same kernel, and an incumbent received from a
// peer between replays reaches the ranks at different iterations. Those iterations prune
// with the incumbent the solve began with; leaves still lower ctl->best, which every
// iteration after the split uses.
template <class Node>
__device__ inline int prune_best(const PoolArgs<Node>& pa, const IterView& v) {
  // (the switch is uniform and known without a load: a kernel argument and the window view)
#ifndef TTS_PRUNE_LIVE_AB  // (A/B builds only, scripts/build_variant.py: the live incumbent everywhere)
  if (v.armed || pa.prune_fixed) return pa.ctl->best0;
#endif
  return __hip_atomic_load(&pa.ctl->best.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (An XCD-aware chunk order — XCD x of the 8 taking a contiguous range of chunks, so a
// slice of the pool is re-read through the L2 that wrote it — measured 1-5 % slower on
// ta014 / ta008 / ta021: profiles/r3/probes/xcd_chunk_order_ab.txt. Chunk ch runs on
// workgroup ch, dealt round-robin over the XCDs.)

// Address of logical element i of the pool window read by this iteration:
// buffer children first (top of the DFS stack), then the ring top.
template <class Node, int MAXCH, int MAXCHUNKS>
__device__ inline const Node* pool_parent(const PoolArgs<Node>& pa, const IterView& v, int t, u64 gi,
                                          const PoolSmem<MAXCHUNKS>& ps) {
  if (gi < v.nb) {
    const int li = static_cast<int>(v.C - v.nb + gi);
    const int c = find_chunk(ps.pre, v.nch_in, li);
    return pa.buf[t & 1] + static_cast<size_t>(c) * MAXCH + (li - ps.pre[c]);
  }
  return pa.ring + ((v.bot + v.S - v.ns + (gi - v.nb)) & pa.cap_mask);
}

// Buffered children not expanded this iteration go to the ring top.
template <class Node, int MAXCH, int MAXCHUNKS>
__device__ inline void pool_spill_leftovers(const PoolArgs<Node>& pa, const IterView& v, int t,
                                            const PoolSmem<MAXCHUNKS>& ps) {
  constexpr int VPN = sizeof(Node) / 16;
  const Node* bin = pa.buf[t & 1];
  for (u64 x = static_cast<u64>(blockIdx.x) * kBlock + threadIdx.x; x < v.L * VPN;
       x += static_cast<u64>(gridDim.x) * kBlock) {
    const int li = static_cast<int>(x / VPN);
    const int w = static_cast<int>(x - static_cast<u64>(li) * VPN);
    const int c = find_chunk(ps.pre, v.nch_in, li);
    const Node* src = bin + static_cast<size_t>(c) * MAXCH + (li - ps.pre[c]);
    Node* dst = pa.ring + ((v.bot + v.S + li) & pa.cap_mask);
    reinterpret_cast<uint4*>(dst)[w] = reinterpret_cast<const uint4*>(src)[w];
  }
}

// Host-requested: move the whole buffer (slot 0 / buffer 0, i.e. between graph
// replays) onto the ring top. The host then folds the counts into ctl.
// (b: the buffer the latest iteration wrote; graphs end at phase 0 or 3, slot 0 either way)
template <class Node, int MAXCH, int MAXCHUNKS>
__global__ __launch_bounds__(kBlock) void pool_flatten_kernel(PoolArgs<Node> pa, int b) {
  __shared__ PoolSmem<MAXCHUNKS> ps;
  IterView v;
  v.S = pa.ctl->slot[0].stack;
  v.bot = pa.ctl->bot;
  v.nch_in = pa.ctl->slot[0].nch;
  v.C = static_cast<u64>(build_prefix(pa.cnt[b], v.nch_in, ps));
  v.nb = 0;
  v.L = v.C;
  pool_spill_leftovers<Node, MAXCH, MAXCHUNKS>(pa, v, b, ps);
}

// Start of a solve (DeviceEngine::begin): the control block and the first nodes are
// read straight from host-mapped pinned memory — one kernel instead of two copies
// (each a blit dispatch plus its API call) ahead of the first graph replay. The nodes
// go to ring[0..n) (begin() resets the ring base).
template <class Node>
__device__ inline void pool_load_body(const uint32_t* __restrict__ src_ctl, PoolCtl* dctl,
                                      const uint4* __restrict__ src_nodes, Node* ring, u64 n) {
  constexpr int VPN = sizeof(Node) / 16;
  constexpr int W = static_cast<int>(sizeof(PoolCtl) / 4);
  const u64 stride = static_cast<u64>(gridDim.x) * kBlock;
  const u64 tid = static_cast<u64>(blockIdx.x) * kBlock + threadIdx.x;
  uint32_t* d = reinterpret_cast<uint32_t*>(dctl);
  for (u64 i = tid; i < static_cast<u64>(W); i += stride) d[i] = src_ctl[i];
  uint4* dn = reinterpret_cast<uint4*>(ring);
  for (u64 x = tid; x < n * VPN; x += stride) dn[x] = src_nodes[x];
}
template <class Node>
__global__ __launch_bounds__(kBlock) void pool_load_kernel(const uint32_t* __restrict__ src_ctl, PoolCtl* dctl,
                                                           const uint4* __restrict__ src_nodes, Node* ring, u64 n) {
  pool_load_body<Node>(src_ctl, dctl, src_nodes, ring, n);
}

// The same load with the node count read from the staged control block (slot 0's
// stack): a kernel node of a captured graph (the learned first replay starts with it,
// so a solve is one graph launch; DeviceEngine::begin defers its load to that graph).
template <class Node>
__global__ __launch_bounds__(kBlock) void pool_load_staged_kernel(const uint32_t* __restrict__ src_ctl, PoolCtl* dctl,
                                                                  const uint4* __restrict__ src_nodes, Node* ring) {
  const u64 n = reinterpret_cast<const PoolCtl*>(src_ctl)->slot[0].stack;  // uniform: one scalar load per wave
  pool_load_body<Node>(src_ctl, dctl, src_nodes, ring, n);
}

// Rank share of a replicated pool: out[t] = ring[bot + rank + t*world], t < keep
// (a strided pick gives every rank a sample of every subtree of the frontier).
template <class Node>
__global__ __launch_bounds__(kBlock) void pool_gather_strided_kernel(const Node* __restrict__ ring, u64 cap_mask,
                                                                     u64 bot, u64 keep, int rank, int world,
                                                                     Node* __restrict__ out) {
  constexpr int VPN = sizeof(Node) / 16;
  for (u64 x = static_cast<u64>(blockIdx.x) * kBlock + threadIdx.x; x < keep * VPN;
       x += static_cast<u64>(gridDim.x) * kBlock) {
    const u64 t = x / VPN;
    const int w = static_cast<int>(x - t * VPN);
    const Node* src = ring + ((bot + static_cast<u64>(rank) + t * static_cast<u64>(world)) & cap_mask);
    reinterpret_cast<uint4*>(out + t)[w] = reinterpret_cast<const uint4*>(src)[w];
  }
}

// Progress measure: sum over the ring nodes of w[depth] (the share of the search
// space a node at that depth stands for), one double atomic per workgroup.
template <class Node>
__global__ __launch_bounds__(kBlock) void pool_weight_kernel(const Node* __restrict__ ring, u64 cap_mask, u64 bot,
                                                            u64 n, const double* __restrict__ w, int nw,
                                                            double* __restrict__ out) {
  __shared__ double part[kBlock / kWave];
  double acc = 0;
  for (u64 i = static_cast<u64>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += static_cast<u64>(gridDim.x) * kBlock) {
    const int d = static_cast<int>(ring[(bot + i) & cap_mask].depth);
    acc += w[d < nw ? d : nw - 1];
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) part[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int i = 0; i < kBlock / kWave; ++i) s += part[i];
    atomicAdd(out, s);
  }
}

// Last node of every graph: counts of the latest buffer for the host.
// The control block is published to host-mapped memory with system-scope stores,
// the sequence number last (release): the host polls that word instead of
// waiting for the graph's completion signal (engine.hpp wait_oldest).
// (b: the buffer the graph's last iteration wrote, s: the slot the next iteration would
// read. Graphs of 3k iterations end at phase 0 or 3: slot 0. A learned first replay of
// any length ends at slot s = K % 3; its slot is moved to slot 0, so the next replay
// starts at phase 0 or 3 — the one whose buffer parity is b — engine.hpp launch_graph)
template <class Node, int MAXCHUNKS>
__global__ __launch_bounds__(kBlock) void pool_finalize_kernel(PoolArgs<Node> pa, int b, int s) {
  __shared__ PoolSmem<MAXCHUNKS> ps;
  const int n = pa.ctl->slot[s].nch;
  if (s != 0 && threadIdx.x == 0) pa.ctl->slot[0] = pa.ctl->slot[s];
  const u64 seq = pa.ctl->seq + 1;
  int c = 0, l = 0, in = 0;
  {
    constexpr int R = (MAXCHUNKS + kBlock - 1) / kBlock;
    int xc[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = static_cast<int>(threadIdx.x) + k * kBlock;
      xc[k] = i < n ? pa.cnt[b][i] : 0;
    }
    sum_leaf_words<MAXCHUNKS>(pa.lcnt[b], n, l, in);
#pragma unroll
    for (int k = 0; k < R; ++k) c += xc[k];
  }
  int ct = 0, lt = 0, it = 0;
  (void)block_exclusive_scan(c, ps.scan, &ct);
  (void)block_exclusive_scan(l, ps.red, &lt);
  (void)block_exclusive_scan(in, ps.scan, &it);
  if (threadIdx.x == 0) {
    pa.ctl->pend_children = static_cast<u64>(ct);
    pa.ctl->pend_leaves = static_cast<u64>(lt);
    pa.ctl->pend_internal = static_cast<u64>(it);
    pa.ctl->seq = seq;
  }
  // publish the whole control block to host-mapped memory: the host reads it
  // without a device-to-host copy
  static_assert(sizeof(PoolCtl) % 4 == 0, "ctl must be dword-sized");
  constexpr int kPc = static_cast<int>(offsetof(PoolCtl, pend_children) / 4);
  constexpr int kPl = static_cast<int>(offsetof(PoolCtl, pend_leaves) / 4);
  constexpr int kPi = static_cast<int>(offsetof(PoolCtl, pend_internal) / 4);
  constexpr int kSeq = static_cast<int>(offsetof(PoolCtl, seq) / 4);
  constexpr int kSlotW = static_cast<int>(sizeof(PoolCtl::Slot) / 4);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(pa.ctl);
  uint32_t* dst = reinterpret_cast<uint32_t*>(pa.mirror);
  for (int i = threadIdx.x; i < static_cast<int>(sizeof(PoolCtl) / 4); i += kBlock) {
    if (i == kSeq || i == kSeq + 1) continue;
    uint32_t x = src[(s != 0 && i < kSlotW) ? i + s * kSlotW : i];
    if (i == kPc) x = static_cast<uint32_t>(ct);
    if (i == kPc + 1) x = 0;
    if (i == kPl) x = static_cast<uint32_t>(lt);
    if (i == kPl + 1) x = 0;
    if (i == kPi) x = static_cast<uint32_t>(it);
    if (i == kPi + 1) x = 0;
    __hip_atomic_store(dst + i, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&pa.mirror->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace dev
}  // namespace tts
