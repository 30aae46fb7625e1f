// Host (CPU) implementation of the engine contract of csrc/hip/engine.hpp.
//
// It lets the distributed runtime (parallel/) and its termination / work-sharing
// logic run unchanged on CPU-only machines over the gloo backend (the reference has
// no loopback harness at all), and it is the CPU worker used next to
// the GPUs for -C 1. "Device" pointers are host pointers here.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

#include "engine_api.hpp"
#include "pfsp_instance.hpp"
#include "search_cpu.hpp"

namespace tts {

template <class Problem>
class CpuEngine final : public IEngine {
 public:
  using Node = typename Problem::Node;

  CpuEngine(Problem prob, size_t batch, int threads) : prob_(std::move(prob)), batch_(std::max<size_t>(1, batch)),
                                                        threads_(std::max(1, threads)) {}
  ~CpuEngine() override {
    try {
      join_bg();
    } catch (...) {  // a failed background batch: nothing left to report it to
    }
  }

  size_t node_bytes() const override { return sizeof(Node); }
  size_t size() override {
    join_bg();
    return pool_.size();
  }
  int best() override {
    join_bg();
    return best_;
  }
  void set_best(int b) override {
    join_bg();
    best_ = b;
  }
  void reset_counters() override {
    join_bg();
    tree_ = sol_ = parents_ = launches_ = 0;
  }
  void synchronize() override { join_bg(); }
  uintptr_t stream() const override { return 0; }
  int device() const override { return -1; }

  void push_host(const void* nodes, size_t n) override {
    join_bg();
    pool_.push_back_bulk_free(static_cast<const Node*>(nodes), n);
  }
  // (may run next to a batch in flight: the pool is locked, the batch's children join
  // it when the batch ends)
  void import_device(const void* src, size_t n) override {
    std::lock_guard<std::mutex> lk(mu_);
    pool_.push_back_bulk_free(static_cast<const Node*>(src), n);
  }

  // Oldest (bottom) nodes first, like the GPU engine's export.
  size_t pop_host(void* out, size_t max_n) override {
    join_bg();
    return pop_front_locked(out, max_n);
  }
  // (may run next to a batch in flight, like the GPU engine's export from under a replay)
  size_t export_device(void* dst, size_t max_n) override {
    if (bg_.joinable()) ++overlapped_exports_;
    return pop_front_locked(dst, max_n);
  }

  // ---- overlapped rounds (engine_api.hpp): one batch "in flight" on a host thread ----
  void set_overlap(bool on) override {
    overlap_ = on;
    if (!on) join_bg();
  }
  bool in_flight() override { return bg_.joinable(); }
  // (the pool without the batch in flight: exports can always take half of it)
  size_t size_known() override {
    std::lock_guard<std::mutex> lk(mu_);
    return std::max<size_t>(pool_.size(), bg_n_ ? 1 : 0);
  }
  int best_known() override {
    std::lock_guard<std::mutex> lk(mu_);
    return std::min(best_, pending_best_);
  }
  bool split_pending_known() override { return split_world_ > 1 && !split_done_; }
  void offer_best(int b) override {
    std::lock_guard<std::mutex> lk(mu_);
    pending_best_ = std::min(pending_best_, b);
    if (!bg_.joinable() && pending_best_ < best_) best_ = pending_best_;
  }
  unsigned long long overlapped_exports() const { return overlapped_exports_; }

  // One "launch" expands up to `batch` parents from the top of the pool.
  long run(long max_launches, double max_seconds, size_t stop_below) override {
    join_bg();  // a batch the previous (overlapped) run left in flight
    const double t0 = now_s();
    long launches = 0;
    if (split_world_ > 1 && !split_done_) {
      do_split(t0, max_seconds);
      if (!split_done_ && !pool_.empty()) {  // time slice over while still replicated
        t_run_ += now_s() - t0;
        return 0;
      }
    }
    std::vector<Node> parents(batch_);
    while (!pool_.empty() && pool_.size() >= std::max<size_t>(stop_below, 1)) {
      if (max_launches >= 0 && launches >= max_launches) break;
      if (max_seconds > 0 && now_s() - t0 >= max_seconds) {
        leave_one();
        break;
      }
      if (hook_) {
        int b = best_;
        const bool stop = hook_(pool_.size(), b);
        best_ = std::min(best_, b);
        if (stop) {
          leave_one();
          break;
        }
      }
      const size_t n = pool_.pop_back_bulk_free(1, batch_, parents.data(), 1);
      expand(parents.data(), n);
      parents_ += n;
      ++launches;
    }
    launches_ += launches;
    t_run_ += now_s() - t0;
    return launches;
  }

  void begin(const void* nodes, size_t n, int best) override {
    reset_counters();
    pool_.clear();
    best_ = best;
    push_host(nodes, n);
    split_world_ = arm_world_;
    split_rank_ = arm_rank_;
    split_min_ = arm_min_;
    split_done_ = false;
    arm_world_ = 0;
  }
  void set_split(int rank, int world, size_t min_parents) override {
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("set_split: bad rank/world");
    arm_world_ = world;
    arm_rank_ = rank;
    arm_min_ = std::max<size_t>(1, min_parents);
  }
  bool split_pending() override { return split_world_ > 1 && !split_done_; }
  void set_progress_hook(ProgressHook hook) override { hook_ = std::move(hook); }
  double pool_weight(const std::vector<double>& w) override {
    join_bg();  // the background batch may reallocate the pool
    double s = 0;
    if (w.empty()) return s;
    for (size_t i = 0; i < pool_.size(); ++i)
      s += w[std::min<size_t>(static_cast<size_t>(pool_.data()[i].depth), w.size() - 1)];
    return s;
  }
  EngineStats solve_from(const void* nodes, size_t n, int best) override {
    begin(nodes, n, best);
    run(-1, 0.0, 0);
    return stats();
  }

  size_t warm_split(int rank, int world, size_t window, int passes) override {
    join_bg();
    const double t0 = now_s();
    std::vector<Node> parents(std::max<size_t>(1, window));
    for (int i = 0; i < passes * 6 && !pool_.empty(); ++i) {
      const size_t n = pool_.pop_back_bulk_free(1, parents.size(), parents.data(), 1);
      expand(parents.data(), n);
      parents_ += n;
      ++launches_;
    }
    if (world > 1) {
      std::vector<Node> mine;
      const size_t n = pool_.size();
      for (size_t i = static_cast<size_t>(rank); i < n; i += static_cast<size_t>(world)) mine.push_back(pool_.data()[i]);
      pool_.clear();
      pool_.push_back_bulk_free(mine.data(), mine.size());
      if (rank != 0) reset_counters();
    }
    t_run_ += now_s() - t0;
    return pool_.size();
  }

  EngineStats stats() override {
    join_bg();
    EngineStats s;
    s.tree = tree_;
    s.sol = sol_;
    if (split_pending() && split_rank_ != 0 && pool_.empty()) s.tree = s.sol = 0;  // see set_split
    s.parents = parents_;
    s.iters = launches_;
    s.launches = launches_;
    s.best = best_;
    s.device_nodes = pool_.size();
    s.t_run = t_run_;
    s.overlapped_exports = overlapped_exports_;
    s.left_inflight = left_inflight_;
    return s;
  }

 private:
  size_t pop_front_locked(void* out, size_t max_n) {
    std::lock_guard<std::mutex> lk(mu_);
    const size_t n = std::min(max_n, pool_.size());
    Node tmp;
    Node* dst = static_cast<Node*>(out);
    for (size_t i = 0; i < n; ++i) {
      pool_.pop_front_free(tmp);
      dst[i] = tmp;
    }
    return n;
  }
  // Overlapped rounds: with at least two batches pooled, one more batch goes to a host
  // thread that expands it while the caller runs its round; its children, counts and
  // incumbent join the engine when it ends (join_bg). Exports meanwhile take the pool's
  // oldest nodes under the lock.
  void leave_one() {
    if (!overlap_ || bg_.joinable() || pool_.size() < 2 * batch_) return;
    std::vector<Node> mine(batch_);
    size_t n = 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      n = pool_.pop_back_bulk_free(1, batch_, mine.data(), 1);
      bg_n_ = n;
    }
    mine.resize(n);
    ++left_inflight_;
    const int b0 = best_;
    bg_ = std::thread([this, mine = std::move(mine), b0]() {
      int b = b0;
      u64 tr = 0, so = 0;
      std::vector<Node> kids;
      try {
        for (const Node& p : mine) prob_.decompose(p, b, tr, so, [&](const Node& c) { kids.push_back(c); });
      } catch (...) {  // rethrown to the caller by join_bg (never std::terminate)
        std::lock_guard<std::mutex> lk(mu_);
        bg_error_ = std::current_exception();
        bg_n_ = 0;
        return;
      }
      std::lock_guard<std::mutex> lk(mu_);
      pool_.push_back_bulk_free(kids.data(), kids.size());
      tree_ += tr;
      sol_ += so;
      parents_ += mine.size();
      ++launches_;
      bg_best_ = b;
      bg_n_ = 0;
    });
  }
  void join_bg() {
    if (!bg_.joinable()) return;
    bg_.join();
    std::exception_ptr err;
    {
      std::lock_guard<std::mutex> lk(mu_);
      best_ = std::min({best_, bg_best_, pending_best_});
      bg_best_ = pending_best_ = 0x7fffffff;
      std::swap(err, bg_error_);
    }
    if (err) std::rethrow_exception(err);
  }

  // Same contract as the device split: identical breadth-first expansion on every
  // rank until the pool holds split_min_ nodes, then a strided 1/world share;
  // ranks != 0 drop the replicated counts. A tree that dies out first is left to
  // rank 0 (stats()).
  void do_split(double t0, double max_seconds) {
    std::vector<Node> level;
    while (!pool_.empty() && pool_.size() < split_min_) {
      if (max_seconds > 0 && now_s() - t0 >= max_seconds) return;  // resumed by the next run()
      level.resize(pool_.size());
      const size_t n = pool_.pop_back_bulk_free(1, level.size(), level.data(), 1);
      expand(level.data(), n);
      parents_ += n;
    }
    if (pool_.empty()) return;  // pending forever: rank 0 reports the whole tree
    std::vector<Node> mine;
    const size_t n = pool_.size();
    for (size_t i = static_cast<size_t>(split_rank_); i < n; i += static_cast<size_t>(split_world_))
      mine.push_back(pool_.data()[i]);
    pool_.clear();
    pool_.push_back_bulk_free(mine.data(), mine.size());
    if (split_rank_ != 0) tree_ = sol_ = 0;
    split_done_ = true;
  }

  void expand(const Node* parents, size_t n) {
    if (threads_ == 1 || n < 256) {
      for (size_t i = 0; i < n; ++i)
        prob_.decompose(parents[i], best_, tree_, sol_, [&](const Node& c) { pool_.push_back_free(c); });
      return;
    }
    // static split of the batch over threads, children merged afterwards
    std::vector<std::vector<Node>> out(threads_);
    std::vector<u64> tr(threads_, 0), so(threads_, 0);
    std::vector<int> bl(threads_, best_);
    std::vector<std::thread> th;
    for (int t = 0; t < threads_; ++t)
      th.emplace_back([&, t]() {
        for (size_t i = t; i < n; i += threads_)
          prob_.decompose(parents[i], bl[t], tr[t], so[t], [&](const Node& c) { out[t].push_back(c); });
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < threads_; ++t) {
      tree_ += tr[t];
      sol_ += so[t];
      best_ = std::min(best_, bl[t]);
      pool_.push_back_bulk_free(out[t].data(), out[t].size());
    }
  }

  Problem prob_;
  size_t batch_;
  int threads_;
  Pool<Node> pool_;
  int best_ = 0x7fffffff;
  u64 tree_ = 0, sol_ = 0, parents_ = 0, launches_ = 0;
  double t_run_ = 0;
  int arm_world_ = 0, arm_rank_ = 0, split_world_ = 0, split_rank_ = 0;
  size_t arm_min_ = 1, split_min_ = 1;
  bool split_done_ = false;
  ProgressHook hook_;
  // overlapped rounds (leave_one / join_bg)
  std::mutex mu_;
  std::thread bg_;
  std::exception_ptr bg_error_;  // an exception of the background batch (join_bg rethrows it)
  size_t bg_n_ = 0;
  int bg_best_ = 0x7fffffff, pending_best_ = 0x7fffffff;
  bool overlap_ = false;
  unsigned long long overlapped_exports_ = 0, left_inflight_ = 0;
};

// CPU engine that keeps its PFSP instance alive (for callers that build the
// instance on the fly, e.g. the HIP module's CPU workers).
template <class Problem>
class OwningCpuEngine final : public IEngine {
 public:
  OwningCpuEngine(std::shared_ptr<const PfspInstance> inst, Problem prob, size_t batch, int threads)
      : inst_(std::move(inst)), eng_(std::move(prob), batch, threads) {}
  size_t node_bytes() const override { return eng_.node_bytes(); }
  void push_host(const void* n, size_t k) override { eng_.push_host(n, k); }
  size_t pop_host(void* o, size_t k) override { return eng_.pop_host(o, k); }
  size_t export_device(void* d, size_t k) override { return eng_.export_device(d, k); }
  void import_device(const void* s, size_t k) override { eng_.import_device(s, k); }
  size_t size() override { return eng_.size(); }
  long run(long a, double b, size_t c) override { return eng_.run(a, b, c); }
  void begin(const void* n, size_t k, int b) override { eng_.begin(n, k, b); }
  EngineStats solve_from(const void* n, size_t k, int b) override { return eng_.solve_from(n, k, b); }
  size_t warm_split(int r, int w, size_t win, int p) override { return eng_.warm_split(r, w, win, p); }
  void set_split(int r, int w, size_t mp) override { eng_.set_split(r, w, mp); }
  bool split_pending() override { return eng_.split_pending(); }
  void set_progress_hook(ProgressHook h) override { eng_.set_progress_hook(std::move(h)); }
  void set_overlap(bool on) override { eng_.set_overlap(on); }
  bool in_flight() override { return eng_.in_flight(); }
  size_t size_known() override { return eng_.size_known(); }
  int best_known() override { return eng_.best_known(); }
  bool split_pending_known() override { return eng_.split_pending_known(); }
  void offer_best(int b) override { eng_.offer_best(b); }
  double pool_weight(const std::vector<double>& w) override { return eng_.pool_weight(w); }
  void set_best(int b) override { eng_.set_best(b); }
  int best() override { return eng_.best(); }
  void reset_counters() override { eng_.reset_counters(); }
  EngineStats stats() override { return eng_.stats(); }
  void synchronize() override {}
  uintptr_t stream() const override { return 0; }
  int device() const override { return -1; }

 private:
  std::shared_ptr<const PfspInstance> inst_;
  CpuEngine<Problem> eng_;
};

}  // namespace tts
