// Host orchestration of one GPU's device-resident B&B pool.
//
// Replaces the reference's per-batch host loop (ref pfsp_multigpu_cuda.c:221-332:
// popBackBulk -> build nodeIndex/sumOffSets on the CPU -> 3 synchronous H2D copies
// -> kernel -> cudaDeviceSynchronize -> D2H bounds -> generate_children on the CPU
// -> pushBackBulk) with:
//   * a ring-buffer stack + ping-pong children buffers in HBM (sized for 288 GB),
//   * K fused expand iterations captured once into a hipGraph and replayed; the
//     iteration count, parent window and pool sizes live in device memory
//     (PoolCtl), so the host only reads a 1-KB control block between replays,
//   * a pinned host extension of the ring bottom (host_spill.hpp): spills and
//     refills are asynchronous DMA on a second (transfer) stream that overlap the
//     graph replays; the ring span a copy touches stays reserved until its event
//     completes, and refills are issued ahead of need (below 4 windows),
//   * bottom export/import for work sharing between GPUs (steal the shallowest,
//     largest subtrees): stream-ordered with events against the transfer stream,
//     on which the caller enqueues the RCCL send/recv (parallel/comm.py), so no
//     side waits on the host.
#pragma once

#include <algorithm>
#include <array>
#include <map>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <thread>
#include <type_traits>
#include <mutex>
#include <vector>

#include "../core/engine_api.hpp"
#include "device_resource.hpp"
#include "host_spill.hpp"
#include "pool_device.hpp"

namespace tts {

// Traits with dynamic local DFS iterations (pool_device.hpp DynCtl) set kDyn = true.
template <class T, class = void>
struct traits_dyn : std::false_type {};
template <class T>
struct traits_dyn<T, std::void_t<decltype(T::kDyn)>> : std::bool_constant<T::kDyn> {};

// Traits contract:
//   using Node; using Args (with a `PoolArgs<Node> pool` member);
//   static constexpr int kParentsPerChunk, kChildrenPerChunk, kMaxChunks;
//   static void launch(const Args&, int t, int grid, hipStream_t);
//   static void flatten(const dev::PoolArgs<Node>&, int grid, hipStream_t);
//   static void finalize(const dev::PoolArgs<Node>&, hipStream_t);
//   static int blocks_per_cu();
template <class Traits>
class DeviceEngine final : public IEngine, public DeviceResource {
 public:
  using Node = typename Traits::Node;
  using Args = typename Traits::Args;

  DeviceEngine(const EngineConfig& cfg, const Args& problem_args)
      : cfg_(cfg), args_(problem_args), spill_(spill_block_nodes(cfg)) {
    if (cfg_.iters_small % 6 || cfg_.iters_large % 6 || cfg_.iters_small <= 0 || cfg_.iters_large <= 0)
      throw std::invalid_argument("iterations per graph must be positive multiples of 6");
    if (cfg_.max_parents == 0) throw std::invalid_argument("max_parents must be > 0");
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    const auto t0 = std::chrono::steady_clock::now();
    int cus = 0;
    TTS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg_.device));
    cus_ = cus;
    int per_cu = std::max(1, Traits::blocks_per_cu());
    if (const char* g = std::getenv("TTS_BLOCKS_PER_CU")) per_cu = std::max(1, std::atoi(g));  // tuning
    const size_t resident = static_cast<size_t>(cus) * per_cu;
    // the parent window is a whole number of chunks, at most kMaxChunks of them (capping
    // it at one chunk per resident workgroup measured no gain: profiles/r3/probes/window*)
    const size_t bp = Traits::kParentsPerChunk;
    max_chunks_ = std::min<size_t>((cfg_.max_parents + bp - 1) / bp, Traits::kMaxChunks);
    cfg_.max_parents = max_chunks_ * bp;
    buf_nodes_ = max_chunks_ * static_cast<size_t>(Traits::kChildrenPerChunk);
    size_t cap = 1;
    while (cap * 2 * sizeof(Node) <= cfg_.ring_bytes) cap *= 2;
    while (cap < buf_nodes_ * 8) cap *= 2;
    cap_ = cap;
    TTS_HIP_CHECK(hipMalloc(&d_ring_, cap_ * sizeof(Node)));
    for (int b = 0; b < 2; ++b) {
      TTS_HIP_CHECK(hipMalloc(&d_buf_[b], buf_nodes_ * sizeof(Node)));
      TTS_HIP_CHECK(hipMalloc(&d_cnt_[b], max_chunks_ * sizeof(int)));
      TTS_HIP_CHECK(hipMalloc(&d_lcnt_[b], max_chunks_ * sizeof(int)));
    }
    TTS_HIP_CHECK(hipMalloc(&d_ctl_, sizeof(dev::PoolCtl)));
    TTS_HIP_CHECK(hipHostMalloc(&h_ctl_, sizeof(dev::PoolCtl), hipHostMallocDefault));
    // control-block upload, followed by a pinned staging area for begin()'s nodes (a
    // pageable source would make the node copy synchronous and staged by the runtime)
    TTS_HIP_CHECK(hipHostMalloc(&h_up_, kUpBytes + kStageNodes * sizeof(Node), hipHostMallocDefault));
    // begin()'s staging, read by the load kernel through its device mapping
    TTS_HIP_CHECK(hipHostMalloc(&h_begin_, kUpBytes + kStageNodes * sizeof(Node),
                                hipHostMallocMapped | hipHostMallocCoherent));
    TTS_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_begin_), h_begin_, 0));
    for (int m = 0; m < 2; ++m) {
      TTS_HIP_CHECK(
          hipHostMalloc(&h_mirror_[m], sizeof(dev::PoolCtl), hipHostMallocMapped | hipHostMallocCoherent));
      TTS_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_mirror_[m]), h_mirror_[m], 0));
      TTS_HIP_CHECK(hipEventCreateWithFlags(&graph_done_[m], hipEventDisableTiming));
    }
    TTS_HIP_CHECK(hipEventCreateWithFlags(&up_done_, hipEventDisableTiming));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&ev_comp_, hipEventDisableTiming));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&ev_xfer_, hipEventDisableTiming));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&ev_ahead_, hipEventDisableTiming));
#ifdef TTS_EAGER_XFER_AB  // (A/B builds only: the transfer stream created with the engine)
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&xfer_, hipStreamNonBlocking));
#endif
    std::memset(h_ctl_, 0, sizeof(dev::PoolCtl));
    h_ctl_->best.v = 0x7fffffff;
    h_ctl_->dive_shift = cfg_.dive_shift;
    if (cfg_.external_stream) {
      stream_ = reinterpret_cast<hipStream_t>(cfg_.external_stream);
    } else {
      TTS_HIP_CHECK(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking));
      stream_ = own_stream_;
    }
    auto& pa = args_.pool;
    pa.ring = d_ring_;
    for (int b = 0; b < 2; ++b) {
      pa.buf[b] = d_buf_[b];
      pa.cnt[b] = d_cnt_[b];
      pa.lcnt[b] = d_lcnt_[b];
    }
    pa.ctl = d_ctl_;
    pa.mirror = d_mirror_[0];
    pa.cap_mask = cap_ - 1;
    pa.max_parents = static_cast<int>(cfg_.max_parents);
    pa.max_chunks = static_cast<int>(max_chunks_);
    // two-level iterations (kernels that implement them) for windows up to this many
    // parents; TTS_FUSE_MAX overrides (0 = off) for A/B runs
    pa.fuse_max = cfg_.fuse_max;
    if (const char* f = std::getenv("TTS_FUSE_MAX")) pa.fuse_max = std::max(0, std::atoi(f));
    pa.local_steps = std::min(cfg_.local_steps, Traits::kLocalSteps);
    if (const char* f = std::getenv("TTS_LOCAL_STEPS")) pa.local_steps = std::min(std::max(0, std::atoi(f)), Traits::kLocalSteps);
    // multi-level fused iterations (kernels with LMAX > 2): 3 levels up to deep_per[0]
    // parents per workgroup, 4 up to deep_per[1]; TTS_DEEP_LEVELS / _P3 / _P4 for A/B runs
    pa.deep_levels = cfg_.deep_levels;
    pa.deep_per[0] = cfg_.deep_per3;
    pa.deep_per[1] = cfg_.deep_per4;
    if (const char* f = std::getenv("TTS_DEEP_LEVELS")) pa.deep_levels = std::max(2, std::atoi(f));
    if (const char* f = std::getenv("TTS_DEEP_P3")) pa.deep_per[0] = std::max(0, std::atoi(f));
    if (const char* f = std::getenv("TTS_DEEP_P4")) pa.deep_per[1] = std::max(0, std::atoi(f));
    pa.wide_levels = cfg_.wide_levels;
    if (const char* f = std::getenv("TTS_WIDE_LEVELS")) pa.wide_levels = std::atoi(f);
    pa.prune_fixed = 0;
    grid_ = static_cast<int>(std::max<size_t>(1, std::min<size_t>(max_chunks_, resident)));
    // the kernel's local DFS threshold only with a parent window of at least a resident
    // grid of chunks: a narrower window cannot take in what a local iteration leaves (up to
    // a slot region per workgroup), and a 4-rank ta008 solve on 2^14-parent windows lost
    // its balance that way (tests/test_gpu_distributed.py skewed start)
    pa.local_min = cfg_.local_min >= 0 ? cfg_.local_min
                   : (cfg_.max_parents >= resident * Traits::kParentsPerChunk ? Traits::kLocalMin : 0);
    if (const char* f = std::getenv("TTS_LOCAL_MIN")) pa.local_min = std::max(0, std::atoi(f));
    // local DFS windows dealt strided (chunk ch takes window parents ch, ch + nchunks, ...)
    // below a backlog (pool_begin): consecutive window nodes are one previous chunk's stack,
    // siblings with alike survivor counts, so contiguous dealing handed some workgroups all
    // the heavy subtrees (per-workgroup exit times track the first step's at r = 0.97;
    // ta014 0.2305 -> 0.2182 ms, rank shares -5..-9 %; profiles/r4/local_stride_ab.txt)
    pa.local_stride = 1;
    if (const char* f = std::getenv("TTS_LOCAL_STRIDE")) pa.local_stride = std::atoi(f);
    pa.local_wide_steps = 3;
    if (const char* f = std::getenv("TTS_LOCAL_WIDE_STEPS")) pa.local_wide_steps = std::atoi(f);
    // dynamic local DFS iterations (kernels that have them, Traits::kDyn): 3 control
    // sets, a time budget per iteration (cfg dyn_us, TTS_DYN_US; 0 = fixed-step local
    // iterations) and the queue slots left after one chunk per resident workgroup
    pa.dyn = nullptr;
    pa.dyn_ticks = 0;
    pa.dyn_q = 0;
    if constexpr (traits_dyn<Traits>::value) {
      int us = cfg_.dyn_us;
      if (const char* f = std::getenv("TTS_DYN_US")) us = std::max(0, std::atoi(f));
      const int q = static_cast<int>(std::min<size_t>(dev::kDynQMax, max_chunks_ - std::min(max_chunks_, resident))) / 8 * 8;
      if (us > 0 && q >= 8) {
        int rate_khz = 0;
        TTS_HIP_CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, cfg_.device));
        TTS_HIP_CHECK(hipMalloc(&pa.dyn, 3 * sizeof(dev::DynCtl)));
        TTS_HIP_CHECK(hipMemset(pa.dyn, 0, 3 * sizeof(dev::DynCtl)));
        owned_.push_back(pa.dyn);
        pa.dyn_ticks = static_cast<int>(std::min<long long>(1ll << 30, static_cast<long long>(us) * std::max(1, rate_khz) / 1000));
        pa.dyn_q = q;
        if (const char* f = std::getenv("TTS_DYN_Q")) pa.dyn_q = std::max(8, std::min(q, std::atoi(f) / 8 * 8));
      }
    }
    // iteration log (probes): TTS_ILOG=<file> records every iteration's window and shape
    // (pool_device.hpp ilog_record), appended to the file when the engine is released
    pa.ilog = nullptr;
    if (const char* f = std::getenv("TTS_ILOG")) {
      ilog_path_ = f;
      TTS_HIP_CHECK(hipMalloc(&pa.ilog, kIlogWords * sizeof(dev::u64)));
      TTS_HIP_CHECK(hipMemset(pa.ilog, 0, kIlogWords * sizeof(dev::u64)));
      owned_.push_back(pa.ilog);
    }
    upload_ctl();
    // Pipelined replays: queue the next graph while one runs when the last known
    // pool spans a whole parent window (spec_min_). Queuing it earlier
    // (TTS_SPECULATE=1) was measured slower on ta014: an empty iteration still
    // costs ~4.5 us and two queued graphs are still ~13 us apart
    // (profiles/r1/r1f).
    {
      const char* e = std::getenv("TTS_SPECULATE");
      spec_min_ = (e && e[0] == '1') ? 1 : cfg_.max_parents;
      const char* p = std::getenv("TTS_POLL");
      poll_ = !(p && p[0] == '0');
    }
    // graphs of 6, 12, 24, ... iterations up to iters_large; run() picks one from
    // the pool size and the worst-case ring growth
    // (and the first replay's length, when it is not one of them)
    if (const char* f = std::getenv("TTS_ITERS_FIRST")) cfg_.iters_first = std::max(6, std::atoi(f) / 6 * 6);
    for (int k = cfg_.iters_small; k <= cfg_.iters_large; k *= 2) ks_.push_back(k);
    if (cfg_.iters_first % 6 == 0 && cfg_.iters_first < cfg_.iters_large &&
        std::find(ks_.begin(), ks_.end(), cfg_.iters_first) == ks_.end()) {
      ks_.push_back(cfg_.iters_first);
      std::sort(ks_.begin(), ks_.end());
    }
    if (cfg_.use_graphs)
      for (int ph = 0; ph < 2; ++ph)
        for (int k : ks_)
          for (int m = 0; m < 2; ++m) graphs_[ph][m].push_back(capture(k, m, 3 * ph));
    if (const char* f = std::getenv("TTS_LEARN_FIRST")) learn_first_ = std::atoi(f) != 0;
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
    stats_.t_malloc = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  ~DeviceEngine() override { release(); }

  // Every device / pinned resource of the engine (DeviceResource: also from the
  // module's atexit hook, before runtime teardown). Idempotent.
  void release() override {
    if (released_) return;
    released_ = true;
    (void)hipSetDevice(cfg_.device);
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (xfer_) (void)hipStreamSynchronize(xfer_);
    trace_clear();
    if (!ilog_path_.empty() && args_.pool.ilog) {
      std::vector<dev::u64> log(kIlogWords);
      if (hipMemcpy(log.data(), args_.pool.ilog, kIlogWords * sizeof(dev::u64), hipMemcpyDeviceToHost) == hipSuccess)
        if (FILE* fp = std::fopen(ilog_path_.c_str(), "ab")) {
          const dev::u64 n = std::min<dev::u64>(log[0], 4095);
          std::fwrite(log.data() + 8, sizeof(dev::u64), 8 * n, fp);
          std::fclose(fp);
        }
    }
    spill_.free_all();
    for (auto& gp : graphs_)
      for (auto& gs : gp)
        for (auto g : gs) (void)hipGraphExecDestroy(g);
    for (auto& kv : first_graphs_)
      for (auto g : kv.second) (void)hipGraphExecDestroy(g);
    for (void* p : owned_) (void)hipFree(p);
    (void)hipFree(d_ring_);
    for (int b = 0; b < 2; ++b) {
      (void)hipFree(d_buf_[b]);
      (void)hipFree(d_cnt_[b]);
      (void)hipFree(d_lcnt_[b]);
    }
    (void)hipFree(d_ctl_);
    (void)hipHostFree(h_ctl_);
    (void)hipHostFree(h_up_);
    (void)hipHostFree(h_begin_);
    for (int m = 0; m < 2; ++m) {
      (void)hipHostFree(h_mirror_[m]);
      (void)hipEventDestroy(graph_done_[m]);
    }
    (void)hipEventDestroy(up_done_);
    (void)hipEventDestroy(ev_comp_);
    (void)hipEventDestroy(ev_xfer_);
    (void)hipEventDestroy(ev_ahead_);
    if (xfer_) (void)hipStreamDestroy(xfer_);
    if (own_stream_) (void)hipStreamDestroy(own_stream_);
    graphs_[0][0].clear();
    graphs_[0][1].clear();
    graphs_[1][0].clear();
    graphs_[1][1].clear();
    first_graphs_.clear();
    owned_.clear();
    xfer_ = own_stream_ = stream_ = nullptr;
  }

  size_t node_bytes() const override { return sizeof(Node); }
  uintptr_t stream() const override { return reinterpret_cast<uintptr_t>(stream_); }
  uintptr_t transfer_stream() const override { return reinterpret_cast<uintptr_t>(xs()); }
  // The transfer stream is created on first use: HIP maps a process's streams onto its
  // hardware queues (GPU_MAX_HW_QUEUES, 4) in creation order, so engines that never
  // transfer (one GPU) leave the queues to the compute streams of the other engines
  // (once: the round loop may ask for it from another thread than the engine's)
  hipStream_t xs() const {
    std::call_once(xfer_once_, [this] {
      if (xfer_) return;
      TTS_HIP_CHECK(hipSetDevice(cfg_.device));
      TTS_HIP_CHECK(hipStreamCreateWithFlags(&xfer_, hipStreamNonBlocking));
    });
    return xfer_;
  }
  void set_progress_hook(ProgressHook hook) override { hook_ = std::move(hook); }
  void set_trace(bool on) override {
    trace_clear();
    trace_ = on;
  }
  std::vector<double> trace() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    flush_load();
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
    if (xfer_) TTS_HIP_CHECK(hipStreamSynchronize(xfer_));
    std::vector<double> out;
    if (trace_rec_.empty()) return out;
    const hipEvent_t ref = trace_rec_.front().a;
    for (const auto& r : trace_rec_) {
      float a = 0, b = 0;
      TTS_HIP_CHECK(hipEventElapsedTime(&a, ref, r.a));
      TTS_HIP_CHECK(hipEventElapsedTime(&b, ref, r.b));
      out.push_back(r.kind);
      out.push_back(a);
      out.push_back(b);
    }
    return out;
  }
  void record_event(uintptr_t ev) override {
    if (!ev) return;
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    flush_load();
    TTS_HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), stream_));
  }
  void wait_event(uintptr_t ev) override {
    if (!ev) return;
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    TTS_HIP_CHECK(hipStreamWaitEvent(stream_, reinterpret_cast<hipEvent_t>(ev), 0));
  }
  void fence() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    flush_load();
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
    if (xfer_) TTS_HIP_CHECK(hipStreamSynchronize(xfer_));
  }
  int device() const override { return cfg_.device; }
  int grid() const { return grid_; }
  size_t max_parents() const { return cfg_.max_parents; }
  // Device allocations (instance tables) released with the engine.
  void adopt(void* device_ptr) { owned_.push_back(device_ptr); }

  void push_host(const void* nodes, size_t n) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    if (n == 0) return;
    settle();
    normalize();
    const Node* src = static_cast<const Node*>(nodes);
    // keep at least half the ring free for in-flight growth; the rest waits in the
    // pinned spill (it joins the pool's bottom, DeviceEngine::run refills it)
    const size_t used = dev_stack() + reserved_;
    const size_t room = cap_ / 2 > used ? cap_ / 2 - used : 0;
    const size_t to_dev = std::min(n, room);
    if (to_dev < n) spill_.push_host(src + to_dev, n - to_dev);
    ring_write_top(src, to_dev, hipMemcpyHostToDevice);
    upload_ctl();
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
  }

  // Oldest nodes first: the pinned spill, then the ring bottom.
  size_t pop_host(void* out, size_t max_n) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    settle();
    normalize();
    Node* dst = static_cast<Node*>(out);
    size_t got = spill_.pop_oldest(dst, max_n);
    const size_t from_dev = std::min(max_n - got, dev_stack());
    ring_read_bottom(dst + got, from_dev, hipMemcpyDeviceToHost);
    got += from_dev;
    upload_ctl();
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
    return got;
  }

  // Stream-ordered (engine_api.hpp): no host wait unless spilled nodes must come back first.
  size_t export_device(void* dst, size_t max_n) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    if (overlap_ && !inflight_.empty() && max_n > 0 && export_ahead(static_cast<Node*>(dst), max_n)) return max_n;
    settle();
    normalize();
    while (dev_stack() < max_n && !spill_.empty()) {
      if (!start_refill(max_n - dev_stack())) break;
      finish_refill();
    }
    const size_t n = std::min(max_n, dev_stack());
    if (n == 0) return 0;
    // the staging buffer may still be read by the previous send on the transfer stream
    order(xs(), stream_);
    ring_read_bottom(static_cast<Node*>(dst), n, hipMemcpyDeviceToDevice);
    upload_ctl();
    order(stream_, xs());  // the send waits for the copy
    ++stats_.exports;
    return n;
  }

  void import_device(const void* src, size_t n) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    if (n == 0) return;
    settle();
    normalize();
    if (dev_stack() + reserved_ + n > cap_ / 2) {
      // make room on the device: the ring bottom goes to the pinned spill
      spill_bottom(dev_stack() + reserved_ + n - cap_ / 2);
    }
    order(xs(), stream_);  // the receive has landed
    ring_write_top(static_cast<const Node*>(src), n, hipMemcpyDeviceToDevice);
    upload_ctl();
    order(stream_, xs());  // the next receive into the buffer waits for this copy
    ++stats_.imports;
  }

  size_t size() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    sync_ctl();
    commit_export();
    return dev_total() + spill_.size() + refill_n_;
  }

  // ---- overlapped rounds (engine_api.hpp) ----
  void set_overlap(bool on) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    overlap_ = on;
    if (!on) {
      sync_ctl();
      commit_export();
      apply_pending_best();
    }
  }
  bool in_flight() override { return !inflight_.empty(); }
  // With a replay in flight: what can be exported from under it (export_ahead) — the
  // ring part the running replays cannot reach — so a plan built on this size never
  // asks for more than the pool can give without waiting; at least 1 (the replay is work).
  // With a replay in flight: the pool as of the last completed replay (plus the host
  // spill), the size the round's needy / donor / termination decisions use (at least 1:
  // the replay is work), and separately what can be exported from under the running
  // replays without waiting (export_ahead), the cap on what the plan asks of this rank.
  size_t size_known() override {
    if (inflight_.empty()) return size();
    const size_t held = dev_total() + spill_.size() + refill_n_;
    return std::max<size_t>(held > export_pending_ ? held - export_pending_ : 0, 1);
  }
  size_t size_exportable() override {
    if (inflight_.empty()) return size();
    return exportable_ahead();
  }
  int best_known() override { return std::min(h_ctl_->best.v, pending_best_); }
  unsigned long long tree_known() override {
    unsigned long long t = h_ctl_->tree + h_ctl_->pend_children + h_ctl_->pend_internal;
    for (const auto& x : h_ctl_->xacc) t += x.tree;
    return t;
  }
  bool split_pending_known() override {
    if (inflight_.empty()) return split_pending();
    return h_ctl_->split_world > 1 && !h_ctl_->slot[0].sdone;
  }
  void offer_best(int b) override {
    if (!inflight_.empty()) {
      pending_best_ = std::min(pending_best_, b);
      return;
    }
    if (b < best()) set_best(b);
  }

  double pool_weight(const std::vector<double>& w) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    if (w.empty()) return 0;
    settle();
    normalize();
    upload_ctl();
    double* dw = nullptr;
    TTS_HIP_CHECK(hipMalloc(&dw, (w.size() + 1) * sizeof(double)));
    TTS_HIP_CHECK(hipMemcpyAsync(dw, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice, stream_));
    TTS_HIP_CHECK(hipMemsetAsync(dw + w.size(), 0, sizeof(double), stream_));
    const size_t n = dev_stack();
    if (n) {
      const int blocks = static_cast<int>(std::min<size_t>((n + dev::kBlock - 1) / dev::kBlock, 4096));
      hipLaunchKernelGGL(dev::pool_weight_kernel<Node>, dim3(blocks), dim3(dev::kBlock), 0, stream_, d_ring_,
                         static_cast<dev::u64>(cap_ - 1), static_cast<dev::u64>(h_ctl_->bot), static_cast<dev::u64>(n),
                         dw, static_cast<int>(w.size()), dw + w.size());
      TTS_HIP_CHECK(hipGetLastError());
    }
    double dev_sum = 0;
    TTS_HIP_CHECK(hipMemcpyAsync(&dev_sum, dw + w.size(), sizeof(double), hipMemcpyDeviceToHost, stream_));
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
    (void)hipFree(dw);
    std::vector<Node> host;
    spill_.snapshot(host);
    double host_sum = 0;
    for (const Node& x : host) host_sum += w[std::min<size_t>(static_cast<size_t>(x.depth), w.size() - 1)];
    return dev_sum + host_sum;
  }

  long run(long max_launches, double max_seconds, size_t stop_below) override {
    if (released_) throw std::runtime_error("engine closed");
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    const auto t0 = std::chrono::steady_clock::now();
    auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    long launches = 0;
    bool hook_stopped = false;
    sync_ctl();  // a replay the previous (overlapped) run left in flight
    for (;;) {
      // ---- nothing in flight on the compute stream: the host shadow is the device state ----
      check_overflow();
      commit_spill_ahead();
      commit_export();
      apply_pending_best();
      poll_transfers();
      size_t total = dev_total();
      const size_t all = total + spill_.size() + refill_n_;
      if (all == 0) {
        // the tree is done: the next solve's first replay gets this solve's iteration
        // count, so it ends without empty iterations (ta014: 2 empty launches of ~5 us
        // each when rounded up to whole phases). Exact only when two solves in a row took
        // the same count (a count that varies — rank shares, -u 0 — keeps the fewer
        // whole-phase lengths, each a graph captured on first use); dynamic iterations
        // keep whole phases: their control sets rotate with the slot (dyn_zero_next)
        const dev::u64 it = h_ctl_->iters;
        const bool stable = static_cast<int>(it) == last_iters_;
        last_iters_ = static_cast<int>(it);
#ifdef TTS_LEARN_ROUND  // A/B builds: whole phases
        const bool exact = false;
#else
        const bool exact = args_.pool.dyn == nullptr;
#endif
        learned_k_ = (it >= 1 && it <= 48) ? static_cast<int>(exact && stable ? it : (it + 2) / 3 * 3) : 0;
        break;
      }
      if (all < stop_below) break;
      if (max_launches >= 0 && launches >= max_launches) break;
      if ((max_seconds > 0 && elapsed() >= max_seconds) || hook_stopped) {
        // overlapped rounds: the slice is over, but a pool of several windows keeps the
        // GPU busy with one more replay while the caller's round runs
        if (leave_one(total)) ++launches;
        break;
      }
      if (hook_) {
        int b = h_ctl_->best.v;
        const bool stop = hook_(all, b);
        if (b < h_ctl_->best.v) {  // a peer's better incumbent: prune with it from the next replay on
          h_ctl_->best.v = b;
          upload_ctl();
        }
        if (stop) {
          if (leave_one(total)) ++launches;
          break;
        }
      }
      // refill ahead of need from the pinned spill, one pinned block at a time, while
      // the device still holds work for the next replays to overlap the copy with
      const size_t low = std::max(4 * cfg_.max_parents, spill_.block_nodes() / 2);
      if (refill_n_ == 0 && !spill_.empty() && total < low) {
        normalize();
        start_refill(std::max(4 * cfg_.max_parents, spill_.block_nodes()));
        upload_ctl();
        total = dev_total();
      }
      if (total == 0) {  // the pool is all on the host: wait for a copy to land
        if (refill_n_)
          finish_refill();
        else if (!resv_.empty())
          TTS_HIP_CHECK(hipEventSynchronize(resv_.front().first));
        else
          throw std::runtime_error("pinned spill: no room on the device ring for a refill");
        continue;
      }
      int gi = pick_graph(total, 0);
      // right after begin(): as many iterations as the previous solve took, when known
      const int kf = (fresh_ && learn_first_ && learned_k_ > 0 &&
                      total + reserved_ + static_cast<size_t>(learned_k_ + 1) * buf_nodes_ <= cap_)
                         ? learned_k_
                         : 0;
      if (gi < 0) {
        if (!resv_.empty()) {  // ring span still being copied out: wait for the oldest copy
          TTS_HIP_CHECK(hipEventSynchronize(resv_.front().first));
          continue;
        }
        if (refill_n_) {
          finish_refill();
          continue;
        }
        normalize();
        spill_bottom(dev_stack() / 2 + 1);
        upload_ctl();
        continue;
      }
      launch_graph(gi, kf);
      ++launches;
      start_spill_ahead();
      // ---- pipelined replays: while one graph runs, queue the next one if the
      // last known pool spans at least one parent window and the worst-case
      // growth of both fits; then read the older graph's mirror. Hides the host
      // sync + launch gap between replays. ----
      size_t known = total;
      size_t inflight_growth = static_cast<size_t>((kf ? kf : ks_[gi]) + 1) * buf_nodes_;
      bool hook_stop = false, leaving = false;
      while (!inflight_.empty()) {
        const bool budget_ok = !hook_stop && (max_launches < 0 || launches < max_launches) &&
                               (max_seconds <= 0 || elapsed() < max_seconds);
        // overlapped rounds: the slice ends with the last pipelined replay still running
        // (only a replay short enough that half of the pool stays exportable from under
        // it, as leave_one's: a long one would hide a donor's pool from the plan)
        if (overlap_ && !budget_ok && inflight_.size() == 1 && (max_launches < 0 || launches < max_launches) &&
            leave_ok(known) &&
            static_cast<size_t>(inflight_k_.front()) <= std::max<size_t>(6, known / 2 / cfg_.max_parents)) {
          leaving = true;
          ++stats_.left_inflight;
          break;
        }
        if (inflight_.size() == 1 && budget_ok && known >= spec_min_) {
          const int g2 = pick_graph(known, inflight_growth);
          if (g2 >= 0) {
            launch_graph(g2);
            ++launches;
            inflight_growth += static_cast<size_t>(ks_[g2] + 1) * buf_nodes_;
          }
        }
        wait_oldest();
        check_overflow();
        known = dev_total();
        inflight_growth = inflight_.empty() ? 0 : static_cast<size_t>(inflight_k_.front() + 1) * buf_nodes_;
        // a long pipelined stretch still answers the hook (live pool size for siblings
        // and peers, stop requests); a better incumbent from it is applied once nothing
        // is in flight, at the top of the outer loop
        if (hook_ && !inflight_.empty() && !hook_stop) {
          int b = h_ctl_->best.v;
          hook_stop = hook_(known + spill_.size() + refill_n_, b);
          if (b < pending_best_) pending_best_ = b;
        }
      }
      if (leaving) break;  // pending_best_ is applied after the replay (apply_pending_best)
      apply_pending_best();
      hook_stopped = hook_stop;
    }
    stats_.t_run += elapsed();
    return launches;
  }

  // Fused start of a solve: fresh counters and incumbent, `n` nodes loaded at the
  // ring base, one asynchronous control upload (no stream synchronisation).
  void begin(const void* nodes, size_t n, int best) override {
    if (released_) throw std::runtime_error("engine closed");
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    settle();
    normalize();
    // an armed split applies to this solve only
    h_ctl_->split_world = arm_world_ > 1 ? arm_world_ : 0;
    h_ctl_->split_rank = arm_rank_;
    h_ctl_->split_min = arm_min_;
    for (int i = 0; i < 3; ++i) h_ctl_->slot[i].sdone = 0;
    // -u 0 (no incumbent yet): dive to the first leaves through a narrow window
    h_ctl_->slot[0].cap = (best == 0x7fffffff && cfg_.dive_window > 0) ? static_cast<unsigned>(cfg_.dive_window) : 0u;
    h_ctl_->slot[0].cpad = 0x7fffffffu;
    // replicated iterations (a pending split) prune with this incumbent (pool_device.hpp prune_best)
    h_ctl_->best0 = best;
    const bool armed = arm_world_ > 1;
    arm_world_ = 0;
    if (armed && n > cfg_.max_parents)
      throw std::invalid_argument("set_split: begin() with more nodes than the parent window");
    if (dev_total() != 0 || !spill_.empty() || reserved_ || n > cap_ / 2) {
      reset_counters();
      set_best(best);
      push_host(nodes, n);
      fresh_ = true;
      return;
    }
    h_ctl_->tree = h_ctl_->sol = h_ctl_->parents = h_ctl_->iters = 0;
    for (auto& x : h_ctl_->xacc) x.tree = x.sol = 0;
    h_ctl_->best.v = best;
    h_ctl_->bot = 0;
    h_ctl_->slot[0].stack = 0;
    h_ctl_->slot[0].nch = 0;
    h_ctl_->pend_children = h_ctl_->pend_leaves = h_ctl_->pend_internal = 0;
    h_ctl_->overflow = 0;
    if (n <= kStageNodes) {
      // one load kernel reads the control block and the nodes from mapped pinned memory
      if (loader_pending_) TTS_HIP_CHECK(hipStreamSynchronize(stream_));  // it still reads the staging area
      h_ctl_->slot[0].stack = n;
      std::memcpy(h_begin_, h_ctl_, sizeof(dev::PoolCtl));
      Node* stage = reinterpret_cast<Node*>(reinterpret_cast<char*>(h_begin_) + kUpBytes);
      std::memcpy(stage, nodes, n * sizeof(Node));
      // deferred: the learned first replay starts with the load (one graph launch per
      // solve); any other device operation launches it first (flush_load)
      load_n_ = n;
      load_deferred_ = true;
      loader_pending_ = true;
      if (!defer_load_) flush_load();
    } else {
      ring_write_top(static_cast<const Node*>(nodes), n, hipMemcpyHostToDevice);
      upload_ctl();  // records up_done_ after both copies
    }
    fresh_ = true;
  }

  EngineStats solve_from(const void* nodes, size_t n, int best) override {
    begin(nodes, n, best);
    run(-1, 0.0, 0);
    return stats();
  }

  size_t warm_split(int rank, int world, size_t window, int passes) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("bad rank/world");
    const auto t0 = std::chrono::steady_clock::now();
    settle();
    // 6-iteration passes with a narrower parent window (plain launches: the
    // window is a kernel argument); identical on every rank
    const size_t win = std::max<size_t>(1, std::min(window, cfg_.max_parents));
    // the passes must be identical on every rank: no -u 0 dive cap in them (a dive reaches
    // leaves, and an incumbent lowered in the middle of an iteration prunes differently
    // from rank to rank); the rank's own search dives from its share afterwards
    const unsigned dive_cap = h_ctl_->slot[0].cap;
    h_ctl_->slot[0].cap = 0;
    h_ctl_->best0 = h_ctl_->best.v;  // and prune every pass with the incumbent they start from
    if (phase_) normalize();  // the passes below start from phase 0
    upload_ctl();
    for (int p = 0; p < passes; ++p) {
      if (h_ctl_->overflow) throw std::runtime_error("device pool overflow (ring too small)");
      const size_t total = dev_total();
      if (total == 0 || total + 7 * buf_nodes_ > cap_) break;
      auto a = args_;
      a.pool.max_parents = static_cast<int>(win);
      a.pool.prune_fixed = 1;
      a.pool.max_chunks = static_cast<int>((win + Traits::kParentsPerChunk - 1) / Traits::kParentsPerChunk);
      const int m = next_mirror_;
      next_mirror_ ^= 1;
      for (int i = 0; i < 6; ++i) Traits::launch(a, i, grid_, stream_);
      a.pool.mirror = d_mirror_[m];
      Traits::finalize(a.pool, 0, 0, stream_);
      TTS_HIP_CHECK(hipGetLastError());
      TTS_HIP_CHECK(hipEventRecord(graph_done_[m], stream_));
      push_inflight(m, 6);
      ++stats_.launches;
      sync_ctl();
    }
    if (h_ctl_->overflow) throw std::runtime_error("device pool overflow (ring too small)");
    normalize();
    h_ctl_->slot[0].cap = h_ctl_->best.v == 0x7fffffff ? dive_cap : 0u;
    if (world == 1) upload_ctl();
    if (world > 1) {
      // strided share of the device part, then of the host spill
      const size_t n = dev_stack();
      const size_t keep = n > static_cast<size_t>(rank) ? (n - rank + world - 1) / world : 0;
      if (keep) {
        Node* tmp = d_buf_[1];
        if (keep > buf_nodes_) TTS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&tmp), keep * sizeof(Node)));
        const int vpn = static_cast<int>(sizeof(Node) / 16);
        const int blocks = static_cast<int>(std::min<size_t>((keep * vpn + dev::kBlock - 1) / dev::kBlock, 4096));
        hipLaunchKernelGGL(dev::pool_gather_strided_kernel<Node>, dim3(blocks), dim3(dev::kBlock), 0, stream_, d_ring_,
                           static_cast<dev::u64>(cap_ - 1), static_cast<dev::u64>(h_ctl_->bot), static_cast<dev::u64>(keep), rank,
                           world, tmp);
        TTS_HIP_CHECK(hipGetLastError());
        TTS_HIP_CHECK(hipMemcpyAsync(d_ring_, tmp, keep * sizeof(Node), hipMemcpyDeviceToDevice, stream_));
        if (tmp != d_buf_[1]) {
          TTS_HIP_CHECK(hipStreamSynchronize(stream_));
          TTS_HIP_CHECK(hipFree(tmp));
        }
      }
      h_ctl_->bot = 0;
      h_ctl_->slot[0].stack = keep;
      if (!spill_.empty()) spill_.keep_strided(rank, world);
      if (rank != 0) h_ctl_->tree = h_ctl_->sol = h_ctl_->parents = h_ctl_->iters = 0;
      upload_ctl();
    }
    stats_.t_run += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fresh_ = true;  // the rank's own search starts now: one long first replay
    return dev_total() + spill_.size();
  }

  void set_split(int rank, int world, size_t min_parents) override {
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("set_split: bad rank/world");
    arm_world_ = world;
    arm_rank_ = rank;
    // the pool must pass through [min, window] before it can outgrow the window:
    // one iteration multiplies it by at most the children per parent
    const size_t per = std::max<size_t>(1, static_cast<size_t>(Traits::kMaxChildren));
    arm_min_ = std::max<size_t>(1, std::min(min_parents, cfg_.max_parents / per));
  }
  bool split_pending() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    sync_ctl();
    return h_ctl_->split_world > 1 && !h_ctl_->slot[0].sdone;
  }

  void set_best(int b) override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    sync_ctl();
    h_ctl_->best.v = b;
    upload_ctl();
  }
  int best() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    sync_ctl();
    return h_ctl_->best.v;
  }
  void reset_counters() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    sync_ctl();
    normalize();
    h_ctl_->tree = h_ctl_->sol = 0;
    h_ctl_->parents = h_ctl_->iters = 0;
    upload_ctl();
  }
  EngineStats stats() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    sync_ctl();
    EngineStats s = stats_;
    s.tree = h_ctl_->tree + h_ctl_->pend_children + h_ctl_->pend_internal;
    s.sol = h_ctl_->sol + h_ctl_->pend_leaves;
    for (const auto& x : h_ctl_->xacc) {
      s.tree += x.tree;
      s.sol += x.sol;
    }
    if (h_ctl_->split_world > 1 && !h_ctl_->slot[0].sdone && h_ctl_->split_rank != 0 && dev_total() == 0 &&
        spill_.empty() && refill_n_ == 0)
      s.tree = s.sol = 0;  // the tree died out before the split: every rank explored all of it
    s.parents = h_ctl_->parents;
    s.iters = h_ctl_->iters;
    s.best = h_ctl_->best.v;
    s.device_nodes = dev_total();
    s.host_nodes = spill_.size() + refill_n_;
    s.capacity = cap_;
    s.pinned_bytes = spill_.pinned_bytes();
    return s;
  }
  void synchronize() override {
    TTS_HIP_CHECK(hipSetDevice(cfg_.device));
    flush_load();
    TTS_HIP_CHECK(hipStreamSynchronize(stream_));
  }

 private:
  // Overlapped rounds: may a replay run on while the caller does its round? The pool
  // must hold enough that the replay cannot run dry (and its donors can export from
  // under it), and no rank split may be pending (the split replays every level).
  bool leave_ok(size_t total) const {
    return overlap_ && total >= 2 * cfg_.max_parents && !(h_ctl_->split_world > 1 && !h_ctl_->slot[0].sdone);
  }
  // Nothing in flight: launch one replay and leave it running (returns true if launched).
  bool leave_one(size_t total) {
    if (!leave_ok(total) || !inflight_.empty()) return false;
    // a replay short enough that half of the pool stays exportable from under it
    // (exportable_ahead): a donor still looks like one to the round's plan (a 4-rank
    // skewed start lost its balance behind 48-iteration replays)
    const size_t kmax = std::max<size_t>(6, total / 2 / cfg_.max_parents);
    const int gi = pick_graph(total, 0, kmax);
    if (gi < 0) return false;
    launch_graph(gi);
    start_spill_ahead();
    ++stats_.left_inflight;
    return true;
  }
  // Export from under running replays: the replays in flight pop at most their
  // iterations x window parents from the top, so the oldest nodes above that (plus one
  // window of margin) are read by no replay; they were written by completed ones. The
  // copy runs on the transfer stream now; the nodes leave the host shadow's stack when
  // the replays have completed (commit_export).
  size_t exportable_ahead() const {
    if (ahead_n_ || refill_n_ || !resv_.empty()) return 0;
    size_t k = 0;
    for (int x : inflight_k_) k += static_cast<size_t>(x);
    const size_t safe = (k + 1) * cfg_.max_parents;
    const size_t stack = dev_stack() - export_pending_;
    return stack > safe ? stack - safe : 0;
  }
  bool export_ahead(Node* dst, size_t n) {
    if (exportable_ahead() < n) return false;
    const size_t start = (h_ctl_->bot + export_pending_) & (cap_ - 1);
    const size_t first = std::min(n, cap_ - start);
    TTS_HIP_CHECK(hipMemcpyAsync(dst, d_ring_ + start, first * sizeof(Node), hipMemcpyDeviceToDevice, xs()));
    if (first < n)
      TTS_HIP_CHECK(hipMemcpyAsync(dst + first, d_ring_, (n - first) * sizeof(Node), hipMemcpyDeviceToDevice, xs()));
    export_pending_ += n;
    // the ring span is handed back to the compute stream only after this copy
    // (commit_export makes the stream wait for it: a replay that wraps around the ring
    // must not overwrite nodes still being copied out behind a slow transfer queue)
    TTS_HIP_CHECK(hipEventRecord(ev_ahead_, xs()));
    ahead_copy_ = true;
    ++stats_.exports;
    ++stats_.overlapped_exports;
    return true;
  }
  void commit_export() {
    if (!export_pending_ || !inflight_.empty()) return;
    if (ahead_copy_) {
      TTS_HIP_CHECK(hipStreamWaitEvent(stream_, ev_ahead_, 0));
      ahead_copy_ = false;
    }
    h_ctl_->bot = (h_ctl_->bot + export_pending_) & (cap_ - 1);
    h_ctl_->slot[0].stack -= export_pending_;
    export_pending_ = 0;
    upload_ctl();
  }
  void apply_pending_best() {
    if (pending_best_ < h_ctl_->best.v && inflight_.empty()) {
      h_ctl_->best.v = pending_best_;
      upload_ctl();
    }
    if (inflight_.empty()) pending_best_ = 0x7fffffff;
  }

  void check_overflow() {
    if (h_ctl_->overflow == 2)
      throw std::runtime_error("pool outgrew the parent window before the armed rank split (set_split)");
    if (h_ctl_->overflow) throw std::runtime_error("device pool overflow (ring too small)");
  }
  size_t dev_stack() const { return static_cast<size_t>(h_ctl_->slot[0].stack); }
  size_t dev_buf() const { return static_cast<size_t>(h_ctl_->pend_children); }
  size_t dev_total() const { return dev_stack() + dev_buf(); }

  // Bring the host shadow up to date. After a graph replay the finalize kernel has
  // already published the control block to host-mapped memory: one stream
  // synchronisation, no copy. Otherwise the shadow is current by construction
  // (every host edit is uploaded from it).
  void sync_ctl() {
    while (!inflight_.empty()) wait_oldest();
    commit_export();
    apply_pending_best();
  }
  // The finalize kernel publishes the mirror's sequence word last (release, system
  // scope): spinning on it returns as soon as the block is in host memory, without
  // the completion-signal round trip of hipEventSynchronize. The event is still
  // queried now and then so a failed graph raises instead of spinning forever.
  void wait_oldest() {
    const auto t0 = std::chrono::steady_clock::now();
    const int m = inflight_.front();
    const dev::u64 want = inflight_seq_.front();
    inflight_.pop_front();
    inflight_k_.pop_front();
    inflight_seq_.pop_front();
    if (poll_) {
      const dev::u64* seq = &h_mirror_[m]->seq;
      unsigned spins = 0;
      while (__atomic_load_n(seq, __ATOMIC_ACQUIRE) < want) {
        __builtin_ia32_pause();
        // back off after ~50 us of spinning: yield the core now and then, so several
        // engines per GPU plus CPU workers on a full host do not starve each other
        // (sched_yield returns at once when no other thread wants the core)
        if (spins > 4096 && (spins & 63) == 0) std::this_thread::yield();
        if ((++spins & 1023) == 0) {
          const hipError_t q = hipEventQuery(graph_done_[m]);
          if (q == hipSuccess) {
            if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) < want)
              throw std::runtime_error("graph completed without publishing its control block");
          } else if (q != hipErrorNotReady) {
            TTS_HIP_CHECK(q);
          }
        }
      }
    } else {
      TTS_HIP_CHECK(hipEventSynchronize(graph_done_[m]));
    }
    std::memcpy(h_ctl_, h_mirror_[m], sizeof(dev::PoolCtl));
    loader_pending_ = false;  // everything enqueued before that graph has completed
    ++stats_.syncs;
    stats_.t_memcpy += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  // Largest graph whose worst-case ring growth (plus `extra` already in flight)
  // fits, no longer than the pool size suggests: 6 iterations while ramping up or
  // draining, more when the pool holds several parent windows.
  int pick_graph(size_t total, size_t extra, size_t kmax = SIZE_MAX) const {
    // right after begin(): one long replay (iters_first) — a graph boundary costs
    // ~50 us of host sync + relaunch, an empty iteration ~4.5 us (profiles/r1/r1f)
    size_t want = fresh_ ? std::max<size_t>(6, static_cast<size_t>(cfg_.iters_first)) : 6;
    while (want < static_cast<size_t>(cfg_.iters_large) && total >= (want / 6) * 2 * cfg_.max_parents &&
           want * 2 <= kmax)
      want *= 2;
    for (int i = static_cast<int>(ks_.size()) - 1; i >= 0; --i) {
      if (static_cast<size_t>(ks_[i]) > want && i > 0) continue;
      if (total + extra + reserved_ + static_cast<size_t>(ks_[i] + 1) * buf_nodes_ <= cap_) return i;
    }
    return -1;
  }
  // Asynchronous upload of the host shadow (through its own pinned staging copy,
  // so the shadow can be edited again immediately).
  void upload_ctl() {
    flush_load();
    TTS_HIP_CHECK(hipEventSynchronize(up_done_));
    std::memcpy(h_up_, h_ctl_, sizeof(dev::PoolCtl));
    TTS_HIP_CHECK(hipMemcpyAsync(d_ctl_, h_up_, sizeof(dev::PoolCtl), hipMemcpyHostToDevice, stream_));
    TTS_HIP_CHECK(hipEventRecord(up_done_, stream_));
  }

  // Host shadow must be current (sync_ctl); between graph replays slot 0 is active
  // and the latest children are in buffer phase_ & 1 (graphs of 3k iterations).
  void normalize() {
    flush_load();
    // subtrees finished inside iterations (N-Queens)
    for (auto& x : h_ctl_->xacc) {
      h_ctl_->tree += x.tree;
      h_ctl_->sol += x.sol;
      x.tree = x.sol = 0;
    }
    const size_t c = dev_buf();
    if (c == 0) {
      phase_ = 0;
      h_ctl_->slot[0].nch = 0;
      h_ctl_->sol += h_ctl_->pend_leaves;
      h_ctl_->tree += h_ctl_->pend_internal;
      h_ctl_->pend_leaves = h_ctl_->pend_internal = 0;
      return;
    }
    if (dev_stack() + c > cap_) throw std::runtime_error("device ring capacity exceeded");
    // the flatten kernel reads the device ctl, which equals the host shadow here
    Traits::flatten(args_.pool, phase_ & 1, grid_, stream_);
    TTS_HIP_CHECK(hipGetLastError());
    h_ctl_->slot[0].stack += c;
    h_ctl_->tree += c + h_ctl_->pend_internal;
    h_ctl_->sol += h_ctl_->pend_leaves;
    h_ctl_->slot[0].nch = 0;
    h_ctl_->pend_children = h_ctl_->pend_leaves = h_ctl_->pend_internal = 0;
    phase_ = 0;  // no buffered children: the next iteration may read either buffer
  }

  void ring_write_top(const Node* src, size_t n, hipMemcpyKind kind) {
    if (n == 0) return;
    if (dev_stack() + n > cap_) throw std::runtime_error("device ring capacity exceeded");
    const size_t start = (h_ctl_->bot + dev_stack()) & (cap_ - 1);
    const size_t first = std::min(n, cap_ - start);
    TTS_HIP_CHECK(hipMemcpyAsync(d_ring_ + start, src, first * sizeof(Node), kind, stream_));
    if (first < n) TTS_HIP_CHECK(hipMemcpyAsync(d_ring_, src + first, (n - first) * sizeof(Node), kind, stream_));
    h_ctl_->slot[0].stack += n;
  }

  void ring_read_bottom(Node* dst, size_t n, hipMemcpyKind kind) {
    if (n == 0) return;
    const size_t start = h_ctl_->bot & (cap_ - 1);
    const size_t first = std::min(n, cap_ - start);
    TTS_HIP_CHECK(hipMemcpyAsync(dst, d_ring_ + start, first * sizeof(Node), kind, stream_));
    if (first < n) TTS_HIP_CHECK(hipMemcpyAsync(dst + first, d_ring_, (n - first) * sizeof(Node), kind, stream_));
    if (kind != hipMemcpyDeviceToDevice) TTS_HIP_CHECK(hipStreamSynchronize(stream_));
    h_ctl_->bot = (h_ctl_->bot + n) & (cap_ - 1);
    h_ctl_->slot[0].stack -= n;
  }

  // Pinned spill blocks: 1/16 of the ring, between 64K nodes and 256 MB.
  static size_t spill_block_nodes(const EngineConfig& c) {
    const size_t by_ring = c.ring_bytes / 16 / sizeof(Node);
    const size_t cap = (size_t(256) << 20) / sizeof(Node);
    return std::max<size_t>(size_t(1) << 16, std::min(by_ring, cap));
  }
  // `after` waits for everything enqueued on `before` so far (no host wait).
  void order(hipStream_t before, hipStream_t after) {
    hipEvent_t ev = before == stream_ ? ev_comp_ : ev_xfer_;
    TTS_HIP_CHECK(hipEventRecord(ev, before));
    TTS_HIP_CHECK(hipStreamWaitEvent(after, ev, 0));
  }
  // Host shadow current and every asynchronous spill copy folded in.
  void settle() {
    flush_load();
    sync_ctl();
    commit_export();
    apply_pending_best();
    commit_spill_ahead();
    if (refill_n_) finish_refill();
    poll_transfers();
  }
  // Release the ring span of spill copies that have completed; fold a completed
  // refill (host shadow current, i.e. nothing in flight on the compute stream).
  void poll_transfers() {
    while (!resv_.empty()) {
      const hipError_t q = hipEventQuery(resv_.front().first);
      if (q == hipErrorNotReady) break;
      TTS_HIP_CHECK(q);
      reserved_ -= resv_.front().second;
      resv_.pop_front();
    }
    if (refill_n_) {
      const hipError_t q = hipEventQuery(refill_ev_);
      if (q == hipSuccess)
        fold_refill();
      else if (q != hipErrorNotReady)
        TTS_HIP_CHECK(q);
    }
  }
  // Asynchronous D2H of the n oldest ring nodes into the pinned spill, on the
  // transfer stream; the ring span stays reserved until the copy has completed.
  void spill_bottom(size_t n) {
    flush_load();
    n = std::min(n, dev_stack());
    if (n == 0) return;
    order(stream_, xs());  // the nodes were written by earlier replays
    const size_t start = h_ctl_->bot & (cap_ - 1);
    const size_t first = std::min(n, cap_ - start);
    auto reserve = [&](hipEvent_t ev, size_t k) {
      resv_.emplace_back(ev, k);
      reserved_ += k;
    };
    const hipEvent_t tr = trace_ ? trace_mark(xs()) : nullptr;
    spill_.push_from_device(d_ring_ + start, first, xs(), reserve);
    if (first < n) spill_.push_from_device(d_ring_, n - first, xs(), reserve);
    if (tr) trace_rec_.push_back({1, tr, trace_mark(xs())});
    h_ctl_->bot = (h_ctl_->bot + n) & (cap_ - 1);
    h_ctl_->slot[0].stack -= n;
    stats_.spilled += n;
  }
  // Spill ahead, overlapped with the replays. Past 3/4 of the ring, right after a graph
  // launch, the oldest nodes above half the ring start their D2H on the transfer
  // stream. The running graphs cannot touch them: a graph consumes at most its
  // iterations x window parents from the top, and two graphs in flight take far
  // less than the half ring kept (the ring holds >= 16 windows of children per
  // window parent), so the copy reads nodes no replay reads or writes. They leave
  // the stack (and stay reserved until the copy is done) once the replays have
  // completed (commit_spill_ahead, nothing in flight).
  void start_spill_ahead() {
    if (ahead_n_ || !resv_.empty() || dev_stack() <= cap_ / 4 * 3) return;
    const size_t keep = std::max(cap_ / 2, 2 * static_cast<size_t>(ks_.back() + 1) * cfg_.max_parents);
    if (dev_stack() <= keep) return;
    const size_t n = dev_stack() - keep;
    const size_t start = h_ctl_->bot & (cap_ - 1);
    const size_t first = std::min(n, cap_ - start);
    auto reserve = [&](hipEvent_t ev, size_t k) { ahead_.emplace_back(ev, k); };
    const hipEvent_t tr = trace_ ? trace_mark(xs()) : nullptr;
    spill_.push_from_device(d_ring_ + start, first, xs(), reserve);
    if (first < n) spill_.push_from_device(d_ring_, n - first, xs(), reserve);
    if (tr) trace_rec_.push_back({1, tr, trace_mark(xs())});
    ahead_n_ = n;
  }
  void commit_spill_ahead() {
    if (!ahead_n_) return;
    h_ctl_->bot = (h_ctl_->bot + ahead_n_) & (cap_ - 1);
    h_ctl_->slot[0].stack -= ahead_n_;
    for (auto& r : ahead_) {
      resv_.push_back(r);
      reserved_ += r.second;
    }
    ahead_.clear();
    stats_.spilled += ahead_n_;
    ahead_n_ = 0;
    upload_ctl();
  }

  // Asynchronous H2D of up to `want` of the newest spilled nodes under the ring
  // bottom (one pinned block at most), on the transfer stream. The nodes join the
  // pool when the copy has completed (fold_refill). Returns false without room.
  bool start_refill(size_t want) {
    if (refill_n_ || spill_.empty() || want == 0) return false;
    flush_load();
    // like push_host: the device part stays within half the ring, and the smallest
    // graph must still fit afterwards (else refills and spills would alternate)
    const size_t used = dev_total() + reserved_;
    const size_t growth = static_cast<size_t>(ks_.front() + 1) * buf_nodes_;
    const size_t limit = std::min(cap_ / 2, cap_ > growth ? cap_ - growth : 0);
    if (used >= limit) return false;
    const size_t b0 = h_ctl_->bot & (cap_ - 1);
    // one pinned block at most, contiguous under the ring bottom
    const size_t k = std::min({want, spill_.top_count(), limit - used, b0 ? b0 : cap_});
    if (k == 0) return false;
    Node* dst = d_ring_ + ((b0 + cap_ - k) & (cap_ - 1));
    const hipEvent_t tr = trace_ ? trace_mark(xs()) : nullptr;
    if (spill_.pop_to_device(dst, k, xs(), &refill_ev_) != k) throw std::logic_error("pinned spill: short refill");
    if (tr) trace_rec_.push_back({2, tr, trace_mark(xs())});
    refill_n_ = k;
    reserved_ += k;
    return true;
  }
  void finish_refill() {
    if (!refill_n_) return;
    TTS_HIP_CHECK(hipEventSynchronize(refill_ev_));
    fold_refill();
  }
  void fold_refill() {
    TTS_HIP_CHECK(hipStreamWaitEvent(stream_, refill_ev_, 0));
    h_ctl_->bot = (h_ctl_->bot + cap_ - refill_n_) & (cap_ - 1);
    h_ctl_->slot[0].stack += refill_n_;
    reserved_ -= refill_n_;
    stats_.refilled += refill_n_;
    refill_n_ = 0;
    upload_ctl();
  }

  // Graphs hold 3k iterations (learned first replays any count, their finalize moving the
  // last slot to slot 0), so a replay starts and ends at phase 0 or 3 (iteration t
  // reads slot t % 3 — slot 0 at both — and buffer t & 1): phase_ is the next
  // iteration's t, and every graph exists for both start phases. K < 0: the learned
  // first-replay graph of -K iterations (learn_first_).
  void launch_graph(int gi, int K = 0) {
    const int m = next_mirror_;
    next_mirror_ ^= 1;
    const int k = K > 0 ? K : ks_[gi];
    const bool with_load = load_deferred_ && K > 0 && cfg_.use_graphs;
    if (!with_load) flush_load();
    const hipEvent_t tr = trace_ ? trace_mark(stream_) : nullptr;
    if (cfg_.use_graphs) {
      hipGraphExec_t g = K > 0 ? first_graph(K, with_load)[m] : graphs_[phase_ / 3][m][gi];
      load_deferred_ = false;
      if (tr) TTS_HIP_CHECK(hipEventRecord(tr, stream_));  // after a first-use capture's sync
      TTS_HIP_CHECK(hipGraphLaunch(g, stream_));
    } else {
      for (int i = 0; i < k; ++i) Traits::launch(args_, (phase_ + i) % 6, grid_, stream_);
      auto pa = args_.pool;
      pa.mirror = d_mirror_[m];
      Traits::finalize(pa, ((phase_ + k) % 6) & 1, (phase_ + k) % 3, stream_);
      TTS_HIP_CHECK(hipGetLastError());
    }
    TTS_HIP_CHECK(hipEventRecord(graph_done_[m], stream_));
    if (tr) trace_rec_.push_back({0, tr, trace_mark(stream_)});
    push_inflight(m, k);
    phase_ = (phase_ + k) % 6;
    // (a learned replay of k != 3j iterations: its finalize moved slot k % 3 to slot 0)
    if (phase_ % 3) phase_ = (phase_ & 1) ? 3 : 0;
    ++stats_.launches;
    fresh_ = false;
  }
  // The learned first replay (phase 0, both mirrors), captured on first use; with_load:
  // the graph starts with begin()'s deferred load (pool_load_staged_kernel).
  const std::array<hipGraphExec_t, 2>& first_graph(int K, bool with_load) {
    const int key = with_load ? -K : K;
    auto it = first_graphs_.find(key);
    if (it == first_graphs_.end()) {
      TTS_HIP_CHECK(hipStreamSynchronize(stream_));
      std::array<hipGraphExec_t, 2> g{capture(K, 0, 0, with_load), capture(K, 1, 0, with_load)};
      it = first_graphs_.emplace(key, g).first;
    }
    return it->second;
  }
  // begin()'s load kernel, unless a graph replay already started with it
  void launch_load(hipStream_t s, bool staged) {
    const int blocks = static_cast<int>(
        std::min<size_t>(64, (std::max<size_t>(load_n_, kStageNodes * !!staged) * (sizeof(Node) / 16) + dev::kBlock - 1) /
                                     dev::kBlock + 1));
    const uint32_t* sc = reinterpret_cast<const uint32_t*>(d_begin_);
    const uint4* sn = reinterpret_cast<const uint4*>(reinterpret_cast<char*>(d_begin_) + kUpBytes);
    if (staged)
      hipLaunchKernelGGL(dev::pool_load_staged_kernel<Node>, dim3(blocks), dim3(dev::kBlock), 0, s, sc, d_ctl_, sn,
                         d_ring_);
    else
      hipLaunchKernelGGL(dev::pool_load_kernel<Node>, dim3(blocks), dim3(dev::kBlock), 0, s, sc, d_ctl_, sn, d_ring_,
                         static_cast<dev::u64>(load_n_));
    TTS_HIP_CHECK(hipGetLastError());
  }
  void flush_load() {
    if (!load_deferred_) return;
    load_deferred_ = false;
    launch_load(stream_, false);
  }
  void push_inflight(int m, int k) {
    inflight_.push_back(m);
    inflight_k_.push_back(k);  // iterations of the replay
    inflight_seq_.push_back(++launched_seq_);
  }

  hipGraphExec_t capture(int K, int mirror, int phase, bool with_load = false) {
    hipStream_t cs;
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t g;
    TTS_HIP_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    if (with_load) launch_load(cs, true);
    for (int i = 0; i < K; ++i) Traits::launch(args_, (phase + i) % 6, grid_, cs);
    auto pa = args_.pool;
    pa.mirror = d_mirror_[mirror];
    Traits::finalize(pa, ((phase + K) % 6) & 1, (phase + K) % 3, cs);
    TTS_HIP_CHECK(hipStreamEndCapture(cs, &g));
    hipGraphExec_t exec;
    TTS_HIP_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    TTS_HIP_CHECK(hipGraphDestroy(g));
    TTS_HIP_CHECK(hipStreamDestroy(cs));
    return exec;
  }

  EngineConfig cfg_;
  Args args_;
  size_t cap_ = 0, buf_nodes_ = 0, max_chunks_ = 0, spec_min_ = 1;
  int grid_ = 1, cus_ = 0;
  Node* d_ring_ = nullptr;
  Node* d_buf_[2] = {nullptr, nullptr};
  int* d_cnt_[2] = {nullptr, nullptr};
  int* d_lcnt_[2] = {nullptr, nullptr};
  dev::PoolCtl* d_ctl_ = nullptr;
  dev::PoolCtl* h_ctl_ = nullptr;
  dev::PoolCtl* h_up_ = nullptr;  // + staging for up to kStageNodes nodes at kUpBytes
  dev::PoolCtl* h_begin_ = nullptr;  // begin()'s mapped staging (control block + nodes), read by pool_load_kernel
  dev::PoolCtl* d_begin_ = nullptr;  // ... its device address
  bool loader_pending_ = false;      // a load kernel may still read h_begin_
  bool load_deferred_ = false;       // begin()'s load not launched yet (see launch_graph / flush_load)
  bool defer_load_ = [] {            // TTS_DEFER_LOAD=0: launch it in begin() (A/B runs)
    const char* f = std::getenv("TTS_DEFER_LOAD");
    return !(f && f[0] == '0');
  }();
  size_t load_n_ = 0;
  static constexpr size_t kUpBytes = (sizeof(dev::PoolCtl) + 255) & ~size_t(255);
  static constexpr size_t kStageNodes = 4096;
  dev::PoolCtl* h_mirror_[2] = {nullptr, nullptr};
  dev::PoolCtl* d_mirror_[2] = {nullptr, nullptr};
  hipEvent_t graph_done_[2] = {nullptr, nullptr};
  hipEvent_t up_done_ = nullptr;
  hipEvent_t ev_comp_ = nullptr, ev_xfer_ = nullptr;  // stream ordering (order())
  mutable std::once_flag xfer_once_;
  mutable hipStream_t xfer_ = nullptr;                 // spills, refills, work-sharing sends/receives (xs())
  // replay / copy timeline (set_trace): timing events, freed by trace_clear
  struct TraceRec {
    int kind;
    hipEvent_t a, b;
  };
  std::vector<TraceRec> trace_rec_;
  bool trace_ = false;
  hipEvent_t trace_mark(hipStream_t s) {
    hipEvent_t e = nullptr;
    TTS_HIP_CHECK(hipEventCreate(&e));
    TTS_HIP_CHECK(hipEventRecord(e, s));
    return e;
  }
  void trace_clear() {
    if (!trace_rec_.empty()) {
      (void)hipStreamSynchronize(stream_);
      if (xfer_) (void)hipStreamSynchronize(xfer_);
    }
    for (auto& r : trace_rec_) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
    trace_rec_.clear();
  }
  std::deque<std::pair<hipEvent_t, size_t>> resv_;     // spill copies in flight (ring span reserved)
  size_t reserved_ = 0;                                // ring nodes reserved by copies in flight
  size_t refill_n_ = 0;                                // nodes of the refill in flight
  size_t ahead_n_ = 0;                                 // spill-ahead copy in flight, not yet committed
  std::deque<std::pair<hipEvent_t, size_t>> ahead_;
  hipEvent_t refill_ev_ = nullptr;
  ProgressHook hook_;
  bool released_ = false;          // release(): nothing left to free
  int pending_best_ = 0x7fffffff;  // incumbent handed in by the hook while graphs were in flight
  bool overlap_ = false;           // overlapped rounds (set_overlap)
  size_t export_pending_ = 0;      // exported from under running replays, not yet off the shadow
  int next_mirror_ = 0;
  std::deque<int> inflight_, inflight_k_;
  std::deque<dev::u64> inflight_seq_;
  dev::u64 launched_seq_ = 0;  // finalize kernels enqueued (== device ctl->seq when idle)
  bool poll_ = true;           // spin on the mirror's sequence word (TTS_POLL=0: event sync)
  bool fresh_ = false;         // no graph launched since begin()
  int arm_world_ = 0, arm_rank_ = 0;  // split armed for the next begin() (set_split)
  size_t arm_min_ = 1;
  hipStream_t stream_ = nullptr, own_stream_ = nullptr;
  std::vector<int> ks_;
  std::vector<hipGraphExec_t> graphs_[2][2];  // [start phase 0 / 3][mirror][graph]
  std::map<int, std::array<hipGraphExec_t, 2>> first_graphs_;  // learned first replays by length
  int phase_ = 0;         // t of the next iteration: 0 or 3
  bool learn_first_ = true;  // first replay after begin() = the previous solve's iterations (TTS_LEARN_FIRST=0: off)
  int learned_k_ = 0;     // ... (0: unknown)
  int last_iters_ = -1;   // the previous finished solve's iteration count
  std::vector<void*> owned_;
  hipEvent_t ev_ahead_ = nullptr;  // after the latest export_ahead copy (transfer stream)
  bool ahead_copy_ = false;
  static constexpr size_t kIlogWords = 8 + 8 * 4095;
  std::string ilog_path_;
  PinnedSpill<Node> spill_;
  EngineStats stats_;
};

}  // namespace tts
