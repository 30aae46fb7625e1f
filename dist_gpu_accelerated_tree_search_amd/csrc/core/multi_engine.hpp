// Several engines on ONE device, one stream and one host thread each, as one engine.
//
// Measured on MI355X (profiles/r3/concurrency_probe.txt): one engine leaves the GPU
// partly idle on large trees — every iteration is one kernel whose last workgroups
// drain alone before the next dependent iteration can start — while two engines
// sharing the device fill each other's tails: ta021 LB1_d 15.5 s with one engine,
// 9.9 s with two, 9.1 s with three; ta056 LB2 0.116 -> 0.169 G nodes/s with two. A
// wider parent window helps less (ta021 +14 % from 2^18 to 2^19 parents, capped by
// the chunk count). This composite runs K such sub-engines concurrently inside one
// rank, so one process per GPU gets the same overlap:
//   * run(): a time slice in which every sub-engine runs its own graph replays on its
//     own host thread (threads parked between slices); a sub-engine that runs dry
//     while another holds at least a parent window ends the slice for all of them at
//     their next replay boundary;
//   * between slices, dry sub-engines receive half of the largest pool (device to
//     device through a staging buffer on the same GPU: export_device, fence,
//     import_device), like the runner's steal-half but without leaving the device;
//   * the incumbent is exchanged through one atomic after every replay;
//   * towards the round loop it is one engine: sizes, counters and the incumbent are
//     summed / minimised, node transfers with other ranks go through sub-engine 0's
//     transfer stream (exports gather from the largest pools first).
// Nodes only move while no sub-engine's host thread is running, so the sub-engines need
// no locks.
//
// Overlapped rounds (set_overlap, ref pfsp_dist_multigpu_cuda.c:364-469 against
// :471-575: the comm thread's collectives run while every GPU thread keeps searching):
// each sub-engine ends a slice with its last graph replay still running on the device
// (DeviceEngine::leave_one), so towards the round loop the composite is "in flight"
// while K replays run: sizes / incumbent / split state are answered from the last
// completed replays (the *_known calls, summed or minimised), exports take from under
// the running replays (size_exportable), and nothing here waits for the device until
// the next slice starts.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <memory>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <thread>
#include <vector>

#include "engine_api.hpp"

namespace tts {

struct MultiConfig {
  size_t needy_below = 1;   // a sub-engine below this many nodes takes work between slices
  size_t donor_min = 2;     // a donor holds at least this many
  size_t cap = 1 << 22;     // at most this many nodes per hand-over
  // > 0: every begin() splits the solve between the sub-engines in the graph (each
  // begins from the same nodes; sub-engine k keeps share k of K once the replicated
  // pool holds split_min * K parents, combined with a rank split as share rank * K + k
  // of world * K), so K concurrent streams expand disjoint subtrees from the start
  size_t split_min = 0;
};

class MultiEngine final : public IEngine {
 public:
  // staging: device buffers for same-device hand-overs (null: host buffers, CPU
  // sub-engines in tests), owned by the engine. The sub-engines stay owned by the caller.
  MultiEngine(std::vector<IEngine*> subs, std::unique_ptr<DeviceStaging> staging, const MultiConfig& cfg)
      : e_(std::move(subs)), own_staging_(std::move(staging)), cfg_(cfg), sizes_(e_.size()) {
    staging_ = own_staging_.get();
    if (e_.empty()) throw std::invalid_argument("MultiEngine: no sub-engine");
    for (auto* x : e_) {
      if (!x) throw std::invalid_argument("MultiEngine: null sub-engine");
      if (x->node_bytes() != e_[0]->node_bytes() || x->device() != e_[0]->device())
        throw std::invalid_argument("MultiEngine: sub-engines must share the node layout and the device");
    }
    const int K = static_cast<int>(e_.size());
    for (int i = 1; i < K; ++i) th_.emplace_back([this, i] { worker(i); });
  }
  ~MultiEngine() override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
      cv_.notify_all();
    }
    for (auto& t : th_) t.join();
    if (buf_ && staging_) staging_->release(e_[0]->device(), buf_);
  }
  MultiEngine(const MultiEngine&) = delete;
  MultiEngine& operator=(const MultiEngine&) = delete;

  int count() const { return static_cast<int>(e_.size()); }
  size_t node_bytes() const override { return e_[0]->node_bytes(); }
  uintptr_t transfer_stream() const override { return e_[0]->transfer_stream(); }
  uintptr_t stream() const override { return e_[0]->stream(); }
  int device() const override { return e_[0]->device(); }
  void fence() override {
    for (auto* x : e_) x->fence();
  }
  // exports from other sub-engines are fenced (export_device), imports go to sub-engine 0
  void record_event(uintptr_t ev) override { e_[0]->record_event(ev); }
  void wait_event(uintptr_t ev) override {
    for (auto* x : e_) x->wait_event(ev);
  }
  void synchronize() override {
    for (auto* x : e_) x->synchronize();
  }
  void set_progress_hook(ProgressHook hook) override { hook_ = std::move(hook); }

  size_t size() override {
    size_t s = 0;
    for (auto* x : e_) s += x->size();
    return s;
  }
  // ---- overlapped rounds (engine_api.hpp) ----
  void set_overlap(bool on) override {
    overlap_ = on;
    for (auto* x : e_) x->set_overlap(on);
  }
  bool in_flight() override {
    for (auto* x : e_)
      if (x->in_flight()) return true;
    return false;
  }
  size_t size_known() override {
    size_t s = 0;
    for (auto* x : e_) s += x->size_known();
    return s;
  }
  size_t size_exportable() override {
    size_t s = 0;
    for (auto* x : e_) s += x->size_exportable();
    return s;
  }
  int best_known() override {
    int b = e_[0]->best_known();
    for (auto* x : e_) b = std::min(b, x->best_known());
    return std::min(b, best_.load(std::memory_order_acquire));
  }
  bool split_pending_known() override { return e_[0]->split_pending_known(); }
  void offer_best(int b) override {
    for (auto* x : e_) x->offer_best(b);
  }
  unsigned long long tree_known() override {
    unsigned long long t = 0;
    for (auto* x : e_) t += x->tree_known();
    return t;
  }
  int best() override {
    int b = e_[0]->best();
    for (auto* x : e_) b = std::min(b, x->best());
    return b;
  }
  void set_best(int b) override {
    for (auto* x : e_) x->set_best(b);
  }
  void reset_counters() override {
    for (auto* x : e_) x->reset_counters();
  }
  double pool_weight(const std::vector<double>& w) override {
    double s = 0;
    for (auto* x : e_) s += x->pool_weight(w);
    return s;
  }
  void push_host(const void* nodes, size_t n) override { e_[0]->push_host(nodes, n); }
  size_t pop_host(void* out, size_t max_n) override {
    size_t got = 0;
    for (auto* x : e_)
      if (got < max_n) got += x->pop_host(static_cast<uint8_t*>(out) + got * node_bytes(), max_n - got);
    return got;
  }
  // Largest pools first; the sub-engines other than 0 are fenced so that a send
  // enqueued on sub-engine 0's transfer stream sees their copies.
  // With replays in flight each sub-engine gives at most what it can export from under
  // its replay (no wait); sizes come from the last completed replays either way (the
  // known sizes: no per-sub-engine synchronisation).
  size_t export_device(void* dst, size_t max_n) override {
    std::vector<int> order(e_.size());
    std::iota(order.begin(), order.end(), 0);
    std::vector<size_t> sz(e_.size());
    const bool flying = overlap_ && in_flight();
    for (size_t i = 0; i < e_.size(); ++i) sz[i] = flying ? e_[i]->size_exportable() : e_[i]->size_known();
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return sz[a] > sz[b]; });
    size_t got = 0;
    for (int i : order) {
      if (got >= max_n) break;
      const size_t want = flying ? std::min(max_n - got, sz[i]) : max_n - got;
      if (want == 0) continue;
      const size_t n = e_[i]->export_device(static_cast<uint8_t*>(dst) + got * node_bytes(), want);
      if (n && i != 0) e_[i]->fence();
      got += n;
    }
    return got;
  }
  void import_device(const void* src, size_t n) override { e_[0]->import_device(src, n); }

  void begin(const void* nodes, size_t n, int best) override {
    const int K = static_cast<int>(e_.size());
    split_mode_ = cfg_.split_min > 0 && K > 1;
    if (split_mode_) {
      const int r = arm_ ? arank_ : 0, W = arm_ ? aworld_ : 1;
      const size_t mp = std::max(arm_ ? amin_ / static_cast<size_t>(std::max(1, W)) : size_t(0), cfg_.split_min) *
                        static_cast<size_t>(W * K);
      for (int k = 0; k < K; ++k) {
        e_[k]->set_split(r * K + k, W * K, mp);
        e_[k]->begin(nodes, n, best);
      }
      arm_ = false;
      return;
    }
    e_[0]->begin(nodes, n, best);
    for (size_t i = 1; i < e_.size(); ++i) e_[i]->begin(nodes, 0, best);
  }
  EngineStats solve_from(const void* nodes, size_t n, int best) override {
    begin(nodes, n, best);
    run(-1, 0.0, 0);
    return stats();
  }
  size_t warm_split(int rank, int world, size_t window, int passes) override {
    return e_[0]->warm_split(rank, world, window, passes);
  }
  void set_split(int rank, int world, size_t min_parents) override {
    if (cfg_.split_min == 0 || e_.size() == 1) {
      e_[0]->set_split(rank, world, min_parents);
      return;
    }
    arm_ = true;  // applied by the next begin(), combined with the sub-engine split
    arank_ = rank;
    aworld_ = world;
    amin_ = min_parents;
  }
  bool split_pending() override { return e_[0]->split_pending(); }

  EngineStats stats() override {
    EngineStats s = e_[0]->stats();
    for (size_t i = 1; i < e_.size(); ++i) {
      const EngineStats x = e_[i]->stats();
      s.tree += x.tree;
      s.sol += x.sol;
      s.parents += x.parents;
      s.iters += x.iters;
      s.launches += x.launches;
      s.syncs += x.syncs;
      s.spilled += x.spilled;
      s.refilled += x.refilled;
      s.best = std::min(s.best, x.best);
      s.device_nodes += x.device_nodes;
      s.host_nodes += x.host_nodes;
      s.t_memcpy += x.t_memcpy;
      s.t_malloc += x.t_malloc;
      s.cpu_tree += x.cpu_tree;
      s.cpu_sol += x.cpu_sol;
    }
    return s;
  }
  unsigned long long handovers() const { return handovers_; }

  long run(long max_launches, double max_seconds, size_t stop_below) override {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    auto over = [&]() {
      return max_seconds > 0 && std::chrono::duration<double>(clock::now() - t0).count() >= max_seconds;
    };
    if (e_.size() == 1 || (!split_mode_ && e_[0]->split_pending())) {  // rank split: sub-engine 0 alone
      e_[0]->set_progress_hook(hook_);
      struct Unhook {
        IEngine* e;
        ~Unhook() { e->set_progress_hook(nullptr); }
      } uh{e_[0]};
      return e_[0]->run(max_launches, max_seconds, stop_below);
    }
    long launches = 0;
    for (;;) {
      rebalance();
      size_t total = 0;
      for (size_t i = 0; i < e_.size(); ++i) total += (sizes_[i] = sub_size(i), sizes_[i].load());
      if (total == 0 || total < stop_below) break;
      // ---- one slice: every sub-engine on its own thread ----
      double left = 0;
      if (max_seconds > 0) left = std::max(1e-6, max_seconds - std::chrono::duration<double>(clock::now() - t0).count());
      best_.store(best());
      end_.store(false);
      running_.store(static_cast<int>(e_.size()));
      caller_stop_ = false;
      slice_stop_below_ = stop_below;
      {
        std::lock_guard<std::mutex> lk(mu_);
        slice_left_ = left;
        pending_ = static_cast<int>(e_.size()) - 1;
        errors_.clear();
        ++slice_id_;
        cv_.notify_all();
      }
      try {
        launches += run_sub(0, left);
      } catch (...) {
        // end the slice for the worker threads and let them drain before unwinding:
        // the caller must not touch the sub-engines while they still run
        e_[0]->set_progress_hook(nullptr);
        end_.store(true, std::memory_order_release);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
        throw;
      }
      {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
        if (!errors_.empty()) std::rethrow_exception(errors_.front());
      }
      const int b = best_.load();
      for (auto* x : e_) {
        if (overlap_)
          x->offer_best(b);  // applied after a replay still in flight (no wait)
        else if (b < x->best())
          x->set_best(b);
      }
      if (caller_stop_ || over() || (max_launches >= 0 && launches >= max_launches)) break;
    }
    return launches;
  }

 private:
  // Sub-engine i runs until its pool is empty, the slice ends, or another one asks
  // for the slice to end (a dry sub-engine with a donor, or the caller's hook).
  long run_sub(int i, double left) {
    IEngine* x = e_[i];
    x->set_progress_hook([this, i](size_t pool, int& b) {
      sizes_[i].store(pool, std::memory_order_relaxed);
      int cur = best_.load(std::memory_order_acquire);
      while (b < cur && !best_.compare_exchange_weak(cur, b, std::memory_order_acq_rel)) {
      }
      if (cur < b) b = cur;
      if ((i == 0 && hook_) || slice_stop_below_ > 1) {
        size_t tot = 0;
        for (auto& s : sizes_) tot += s.load(std::memory_order_relaxed);
        // the caller's stop_below holds inside a slice too (summed live pool sizes)
        if (slice_stop_below_ > 1 && tot < slice_stop_below_) end_.store(true, std::memory_order_release);
        if (i == 0 && hook_ && hook_(tot, b)) {
          caller_stop_ = true;
          end_.store(true, std::memory_order_release);
        }
      }
      return end_.load(std::memory_order_acquire);
    });
    // Leave the replay loop below needy_below nodes while another sub-engine can
    // donate (it is then asked for work at once), else run the pool down to empty.
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    auto remaining = [&]() -> double {
      if (left <= 0) return 0.0;
      return std::max(1e-6, left - std::chrono::duration<double>(clock::now() - t0).count());
    };
    auto can_donate = [&]() {
      for (size_t k = 0; k < e_.size(); ++k)
        if (static_cast<int>(k) != i && sizes_[k].load(std::memory_order_relaxed) >= cfg_.donor_min) return true;
      return false;
    };
    long l = 0;
    size_t s = 0;
    for (;;) {
      l += x->run(-1, remaining(), can_donate() ? cfg_.needy_below : 1);
      s = sub_size(i);
      sizes_[i].store(s, std::memory_order_relaxed);
      if (end_.load(std::memory_order_acquire) || s == 0) break;
      if (left > 0 && std::chrono::duration<double>(clock::now() - t0).count() >= left) break;
      if (s < cfg_.needy_below && can_donate()) {
        end_.store(true, std::memory_order_release);
        break;
      }
    }
    x->set_progress_hook(nullptr);
    running_.fetch_sub(1, std::memory_order_acq_rel);
    // dry: watch the others' live pool sizes and end the slice as soon as one of them
    // can donate (it stops at its next replay boundary), or until they are all done
    if (s < cfg_.needy_below) {
      for (;;) {
        bool donor = false;
        for (size_t k = 0; k < e_.size(); ++k)
          if (static_cast<int>(k) != i && sizes_[k].load(std::memory_order_relaxed) >= cfg_.donor_min) donor = true;
        if (donor) {
          end_.store(true, std::memory_order_release);
          break;
        }
        if (running_.load(std::memory_order_acquire) == 0 || end_.load(std::memory_order_acquire)) break;
        if (i == 0 && hook_) {  // the caller's hook keeps being answered (early rounds, incumbent)
          size_t tot = 0;
          for (auto& z : sizes_) tot += z.load(std::memory_order_relaxed);
          int b = best_.load(std::memory_order_acquire);
          const bool stop = hook_(tot, b);
          int cur = best_.load(std::memory_order_acquire);
          while (b < cur && !best_.compare_exchange_weak(cur, b, std::memory_order_acq_rel)) {
          }
          if (stop) {
            caller_stop_ = true;
            end_.store(true, std::memory_order_release);
            break;
          }
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
    return l;
  }

  void worker(int i) {
    unsigned long long seen = 0;
    for (;;) {
      double left;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return quit_ || slice_id_ != seen; });
        if (quit_) return;
        seen = slice_id_;
        left = slice_left_;
      }
      try {
        run_sub(i, left);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        errors_.push_back(std::current_exception());
        end_.store(true);
      }
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }

  // Between slices (no sub-engine running): every dry sub-engine receives half of the
  // largest pool, device to device through the staging buffer.
  void rebalance() {
    const size_t K = e_.size();
    // no hand-over while the sub-engines still hold the same replicated pool
    if (split_mode_)
      for (auto* x : e_)
        if (x->split_pending()) return;
    std::vector<size_t> sz(K);
    for (size_t i = 0; i < K; ++i) sz[i] = sub_size(i);
    for (size_t r = 0; r < K; ++r) {
      if (sz[r] >= cfg_.needy_below) continue;
      size_t d = K;
      for (size_t k = 0; k < K; ++k)
        if (k != r && sz[k] >= cfg_.donor_min && (d == K || sz[k] > sz[d])) d = k;
      if (d == K) continue;
      const size_t n = std::min(sz[d] / 2, cfg_.cap);
      if (n == 0) continue;
      void* buf = stage(n * node_bytes());
      const size_t got = e_[d]->export_device(buf, n);
      e_[d]->fence();
      if (got) {
        e_[r]->import_device(buf, got);
        e_[r]->fence();  // the buffer is free again
        ++handovers_;
      }
      sz[d] -= got;
      sz[r] += got;
    }
  }
  // a sub-engine's pool: with overlap on, as of its last completed replay (a replay in
  // flight counts as work), so no slice boundary waits for the device
  size_t sub_size(size_t i) { return overlap_ ? e_[i]->size_known() : e_[i]->size(); }
  bool overlap_ = false;
  bool split_mode_ = false;  // the current solve is split between the sub-engines
  bool arm_ = false;         // a rank split armed for the next begin()
  int arank_ = 0, aworld_ = 1;
  size_t amin_ = 0;
  void* stage(size_t bytes) {
    if (bytes <= buf_bytes_) return buf_;
    if (staging_) {
      if (buf_) staging_->release(e_[0]->device(), buf_);
      buf_ = staging_->alloc(e_[0]->device(), bytes);
    } else {
      host_buf_.resize(bytes);
      buf_ = host_buf_.data();
    }
    buf_bytes_ = bytes;
    return buf_;
  }

  std::vector<IEngine*> e_;
  std::unique_ptr<DeviceStaging> own_staging_;
  MultiConfig cfg_;
  std::vector<std::atomic<size_t>> sizes_;
  DeviceStaging* staging_ = nullptr;
  ProgressHook hook_;
  std::atomic<int> best_{0x7fffffff};
  std::atomic<bool> end_{false};
  std::atomic<int> running_{0};  // sub-engines still inside their run() this slice
  bool caller_stop_ = false;  // written by sub-engine 0's thread = the caller's thread
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool quit_ = false;
  unsigned long long slice_id_ = 0;
  double slice_left_ = 0;
  std::atomic<size_t> slice_stop_below_{0};  // run()'s stop_below, applied inside a slice
  int pending_ = 0;
  std::vector<std::exception_ptr> errors_;
  void* buf_ = nullptr;
  size_t buf_bytes_ = 0;
  std::vector<uint8_t> host_buf_;
  unsigned long long handovers_ = 0;
};

}  // namespace tts
