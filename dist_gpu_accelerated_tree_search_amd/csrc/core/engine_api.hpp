// Engine contract shared by the GPU engine (csrc/hip/engine.hpp) and the CPU engine
// (csrc/core/cpu_engine.hpp), so the Python runtime and the distributed protocol
// (parallel/) drive either one through the same calls.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

namespace tts {

// Called by run() between two graph replays (nothing in flight) with the current
// pool size and the engine's incumbent; returning true ends run() early. The hook
// may lower `best` (a peer found a better solution): the engine adopts it before
// its next replay. The distributed runtime uses it to publish its pool size and
// incumbent on the node-wide board, to pull the node-wide incumbent (ref
// checkBest around every batch, pfsp_multigpu_cuda.c:30-50,307-312) and to answer
// a peer's early round request (core/dist_rounds.hpp).
using ProgressHook = std::function<bool(size_t pool, int& best)>;

struct EngineConfig {
  int device = 0;
  size_t max_parents = size_t(1) << 18;  // parents expanded per iteration (reference -M)
  size_t ring_bytes = size_t(16) << 30;  // device ring capacity in bytes (rounded down to 2^k nodes)
  int iters_small = 6;                   // iterations per small graph (multiple of 6)
  int iters_large = 48;                  // iterations per large graph (multiple of 6)
  int iters_first = 18;                  // first replay after begin(): covers a 20-job tree in one graph
  int fuse_max = 1 << 30;                // two-level iterations for windows up to this many parents (0: off)
  // local DFS steps per chunk and iteration (<= 1: off; capped per kernel). 6 under the
  // step priority (ta014 0.205 -> 0.198 ms, 5 / 7 / 8 slower; ta021 3 engines 10.1 -> 9.6 s;
  // profiles/r5/steps_ab.txt)
  int local_steps = 6;
  // local DFS iterations once the pool holds this many parents (-1: the kernel's default,
  // Traits::kLocalMin; 0: four grid-filling windows)
  int local_min = -1;
  // (measured on ta014, one MI355X: 3 / 4-level narrow chunks and 2 / 3-level wide ones
  // were 1-2 % / 2-19 % slower than two levels — the extra in-workgroup levels run
  // serially behind one another at ~6 us each, what a new iteration kernel also costs)
  // fused iterations: at most this many tree levels (kernels that have them); 3 under the
  // wave priority (ta014 0.188 -> 0.1855 ms, 4 slower; profiles/r5/ab2.txt)
  int deep_levels = 3;
  int deep_per3 = 8;                     // ... 3 levels when a workgroup takes at most this many parents
  int deep_per4 = 2;                     // ... 4 levels when a workgroup takes at most this many parents
  // dynamic local DFS iterations (front kernel): time budget of one iteration in us
  // (0: fixed-step local iterations)
  int dyn_us = 0;
  int wide_levels = 1;                   // wide windows (<= one parent per thread): levels per iteration (< 2: off)
  // -u 0 dive (pool_device.hpp Slot::cap): a solve begun without an incumbent expands at
  // most this many parents per iteration until its first leaf, then the cap grows by
  // 2^dive_shift per iteration (0: off — N-Queens, which has no incumbent)
  int dive_window = 0;
  int dive_shift = 2;
  bool use_graphs = true;
  uintptr_t external_stream = 0;         // run on this stream when non-zero
};

struct EngineStats {
  unsigned long long tree = 0, sol = 0, parents = 0, iters = 0;
  int best = 0;
  unsigned long long launches = 0, syncs = 0, spilled = 0, refilled = 0, exports = 0, imports = 0;
  // overlapped rounds: run() calls that returned with a replay in flight, and exports
  // copied from under a running replay
  unsigned long long left_inflight = 0, overlapped_exports = 0;
  size_t pinned_bytes = 0;  // pinned host spill blocks held
  double t_run = 0, t_memcpy = 0, t_malloc = 0;
  size_t device_nodes = 0, host_nodes = 0, capacity = 0;
  // share of tree / sol explored by the CPU worker of a hybrid rank engine
  // (core/hybrid_engine.hpp); 0 for plain engines
  unsigned long long cpu_tree = 0, cpu_sol = 0;
};

// Device staging buffers for GPU -> GPU transfers (implemented by the HIP side,
// csrc/hip/host_support.hpp HipStaging).
class DeviceStaging {
 public:
  virtual ~DeviceStaging() = default;
  virtual void* alloc(int device, size_t bytes) = 0;
  virtual void release(int device, void* p) = 0;
  // events for stream ordering between engines (IEngine::record_event / wait_event);
  // 0 where there is no device
  virtual uintptr_t make_event(int device) { (void)device; return 0; }
  virtual void free_event(int device, uintptr_t ev) { (void)device; (void)ev; }
};

// Type-erased interface used by the Python bindings and the native CLIs.
class IEngine {
 public:
  virtual ~IEngine() = default;
  virtual size_t node_bytes() const = 0;
  virtual void push_host(const void* nodes, size_t n) = 0;
  virtual size_t pop_host(void* out, size_t max_n) = 0;
  // Work-sharing transfers through a device staging buffer, stream-ordered without
  // host synchronisation (GPU engines): export_device enqueues the copy of the
  // oldest nodes into `dst` and makes the transfer stream (transfer_stream())
  // wait for it; import_device makes the compute stream wait for the transfer
  // stream, then appends the nodes. A send/recv enqueued on the transfer stream
  // between the two is therefore ordered on both sides. fence() waits on the host
  // for everything enqueued so far (used before a host-side handoff).
  virtual size_t export_device(void* dst, size_t max_n) = 0;
  virtual void import_device(const void* src, size_t n) = 0;
  virtual uintptr_t transfer_stream() const { return 0; }
  virtual void fence() {}
  // Ordering between engines without host waits (GPU engines; no-ops elsewhere):
  // record_event marks everything enqueued so far on the compute stream, wait_event
  // makes the compute stream wait for an event recorded by another engine (possibly
  // on another device). Events come from DeviceStaging::make_event.
  virtual void record_event(uintptr_t ev) { (void)ev; }
  virtual void wait_event(uintptr_t ev) { (void)ev; }
  virtual void set_progress_hook(ProgressHook hook) { (void)hook; }
  // Overlapped rounds (core/dist_rounds.hpp; ref pfsp_dist_multigpu_cuda.c:283,364-469,
  // where the comm thread's collectives run while the GPU threads keep searching).
  // With overlap on, run() may return with one replay still in flight when the pool
  // holds several parent windows, so the round's all-gather, plan and transfers run
  // while the GPU works. The *_known calls answer from the last completed replay
  // without waiting (a pool with work in flight reports at least one node);
  // offer_best applies a lower incumbent at the next replay; export_device may copy
  // the pool bottom while the replay runs. Engines without in-flight work (CPU,
  // multi/hybrid wrappers) keep the plain calls.
  virtual void set_overlap(bool on) { (void)on; }
  virtual bool in_flight() { return false; }
  virtual size_t size_known() { return size(); }
  // ... and what export_device can take right now without waiting for work in flight
  // (the round plan's cap on this rank as a donor)
  virtual size_t size_exportable() { return size_known(); }
  virtual int best_known() { return best(); }
  virtual bool split_pending_known() { return split_pending(); }
  virtual void offer_best(int b) {
    if (b < best()) set_best(b);
  }
  // Explored tree as of the last completed replay, without waiting (diagnostics from
  // the progress hook; 0 where unknown)
  virtual unsigned long long tree_known() { return 0; }
  // Sum over the pool of w[depth] (clamped to the last entry): with w[d] the share
  // of the search space below a node of depth d, 1 - pool_weight is the explored
  // fraction of the space (the B&B progress measure of tools/progress estimates).
  virtual double pool_weight(const std::vector<double>& w) { (void)w; return 0; }
  // Device timeline of graph replays and pool copies (GPU engines; evidence that the
  // pinned spill/refill overlaps the search): set_trace(true) starts a fresh record,
  // trace() returns {kind, start ms, end ms} triples relative to the first record,
  // kind 0 = graph replay (compute stream), 1 = spill D2H, 2 = refill H2D (transfer
  // stream). Timing events around each launch; off by default.
  virtual void set_trace(bool on) { (void)on; }
  virtual std::vector<double> trace() { return {}; }
  virtual size_t size() = 0;
  // Replays expand graphs until the pool is empty, `max_launches` graphs were
  // launched (<0: unlimited), `max_seconds` elapsed (<=0: unlimited), or the pool
  // dropped below `stop_below` nodes. Returns the number of graph launches.
  virtual long run(long max_launches, double max_seconds, size_t stop_below) = 0;
  // Fresh start (counters reset, incumbent set) from `n` nodes, without running.
  virtual void begin(const void* nodes, size_t n, int best) = 0;
  // One complete solve from `n` nodes with incumbent `best` (begin + run + stats).
  virtual EngineStats solve_from(const void* nodes, size_t n, int best) = 0;
  // Deterministic redundant warm start of a multi-rank solve: every rank has
  // begun from the same nodes with the same configuration; `passes` x 6
  // expansion steps with a parent window of `window` grow a wide frontier, then
  // the rank keeps the pool elements i with i % world == rank (bottom first).
  // Counters of the redundant phase are kept by rank 0 only, so the sum over
  // ranks is the explored tree. Returns the pool size kept.
  virtual size_t warm_split(int rank, int world, size_t window, int passes) = 0;
  // Arm an in-search rank split for the next begin(): every rank begins from the
  // same nodes; the search runs identically on all ranks until the pool holds at
  // least `min_parents` nodes, then each rank keeps a disjoint 1/world share of
  // the next expansion (interleaved per parent) and ranks != 0 drop the counts of
  // the replicated part. No host round trip and no collective is involved; if the
  // tree dies out before the split point, rank 0 alone reports it.
  virtual void set_split(int rank, int world, size_t min_parents) = 0;
  // An armed split has not happened yet (the pool is still replicated).
  virtual bool split_pending() = 0;
  virtual void set_best(int b) = 0;
  virtual int best() = 0;
  virtual void reset_counters() = 0;
  virtual EngineStats stats() = 0;
  virtual void synchronize() = 0;
  virtual uintptr_t stream() const = 0;
  virtual int device() const = 0;
};

}  // namespace tts
