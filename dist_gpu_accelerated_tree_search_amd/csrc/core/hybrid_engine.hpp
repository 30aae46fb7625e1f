// One rank = one GPU engine + one (multithreaded) CPU worker sharing the rank's work.
//
// Parity: ref pfsp_dist_multigpu_cuda.c:161-162,471-575 — every MPI rank runs GPU
// driving threads and CPU B&B worker threads (-C 1) on its own pools, with
// intra-rank steals (m / 2m thresholds, a CPU thief takes at most 4*T) and the comm
// thread exchanging work between ranks. Here the rank's engine in the
// one-process-per-GPU runtime (core/dist_rounds.hpp) is this composite: the round
// loop sees one pool (GPU + CPU) and moves nodes between ranks through the GPU side
// (device staging + RCCL), while inside the rank
//   * the GPU engine runs on the calling thread, the CPU engine on a worker thread;
//   * a CPU worker that runs dry asks for work: the GPU leaves its replay loop at the
//     next replay boundary (progress hook) and hands over the bottom of its pool
//     (min(half, 4*T) nodes, ref popBackBulk ratio 2 + 4*T cap) through a mailbox;
//   * a GPU that runs dry takes half of the CPU pool when it holds at least 2m;
//   * both pull and push the incumbent through one atomic (ref checkBest).
// Nodes only ever move while the engine that gives them is not running, so neither
// engine needs to be thread-safe.
//
// Overlapped rounds (set_overlap; ref pfsp_dist_multigpu_cuda.c:364-469 against
// :471-575, the comm thread's collectives beside every GPU and CPU thread): run()
// returns with the GPU's last replay still running and the CPU worker's last batch
// still expanding on its host thread (CpuEngine::leave_one), so the round's all-gather,
// plan and transfers run while both keep searching; the *_known calls answer from what
// completed, and exports go through the GPU side only (from under its replay).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <stdexcept>
#include <mutex>
#include <thread>
#include <vector>

#include "engine_api.hpp"

namespace tts {

struct HybridConfig {
  size_t m = 25;              // CPU side: needy below m, donates from 2m (ref -m)
  size_t cpu_cap = 20000;     // at most this many nodes per hand-over to the CPU (ref 4*T)
  size_t gpu_needy = 25;      // GPU side: takes CPU work below this many nodes
};

class HybridEngine final : public IEngine {
 public:
  HybridEngine(IEngine* gpu, IEngine* cpu, const HybridConfig& cfg) : g_(gpu), c_(cpu), cfg_(cfg) {
    if (!g_ || !c_) throw std::invalid_argument("HybridEngine: two engines needed");
    if (g_->node_bytes() != c_->node_bytes()) throw std::invalid_argument("HybridEngine: node layouts differ");
  }

  size_t node_bytes() const override { return g_->node_bytes(); }
  uintptr_t transfer_stream() const override { return g_->transfer_stream(); }
  uintptr_t stream() const override { return g_->stream(); }
  int device() const override { return g_->device(); }
  void fence() override { g_->fence(); }
  void record_event(uintptr_t ev) override { g_->record_event(ev); }
  void wait_event(uintptr_t ev) override { g_->wait_event(ev); }
  void synchronize() override { g_->synchronize(); }
  void set_progress_hook(ProgressHook hook) override { hook_ = std::move(hook); }

  size_t size() override { return g_->size() + c_->size(); }
  // ---- overlapped rounds (engine_api.hpp) ----
  void set_overlap(bool on) override {
    overlap_ = on;
    g_->set_overlap(on);
    c_->set_overlap(on);
  }
  bool in_flight() override { return g_->in_flight() || c_->in_flight(); }
  size_t size_known() override { return g_->size_known() + c_->size_known(); }
  size_t size_exportable() override { return overlap_ && in_flight() ? g_->size_exportable() : size_known(); }
  int best_known() override { return std::min(g_->best_known(), c_->best_known()); }
  bool split_pending_known() override { return g_->split_pending_known(); }
  void offer_best(int b) override {
    g_->offer_best(b);
    c_->offer_best(b);
  }
  unsigned long long tree_known() override { return g_->tree_known() + c_->tree_known(); }
  int best() override { return std::min(g_->best(), c_->best()); }
  void set_best(int b) override {
    g_->set_best(b);
    c_->set_best(b);
  }
  void reset_counters() override {
    g_->reset_counters();
    c_->reset_counters();
  }
  double pool_weight(const std::vector<double>& w) override { return g_->pool_weight(w) + c_->pool_weight(w); }

  void push_host(const void* nodes, size_t n) override { g_->push_host(nodes, n); }
  size_t pop_host(void* out, size_t max_n) override {
    size_t got = g_->pop_host(out, max_n);
    if (got < max_n) got += c_->pop_host(static_cast<uint8_t*>(out) + got * node_bytes(), max_n - got);
    return got;
  }
  // Transfers between ranks go through the GPU side; CPU nodes join it first when the
  // GPU pool alone cannot cover a planned export.
  size_t export_device(void* dst, size_t max_n) override {
    if (overlap_ && in_flight()) return g_->export_device(dst, max_n);  // the plan asked <= size_exportable
    const size_t have = g_->size();
    if (have < max_n && c_->size() > 0) move(c_, g_, std::min(c_->size(), max_n - have));
    return g_->export_device(dst, max_n);
  }
  void import_device(const void* src, size_t n) override { g_->import_device(src, n); }

  void begin(const void* nodes, size_t n, int best) override {
    g_->begin(nodes, n, best);
    c_->begin(nodes, 0, best);
  }
  EngineStats solve_from(const void* nodes, size_t n, int best) override {
    begin(nodes, n, best);
    run(-1, 0.0, 0);
    return stats();
  }
  size_t warm_split(int rank, int world, size_t window, int passes) override {
    return g_->warm_split(rank, world, window, passes);
  }
  void set_split(int rank, int world, size_t min_parents) override { g_->set_split(rank, world, min_parents); }
  bool split_pending() override { return g_->split_pending(); }

  EngineStats stats() override {
    EngineStats s = g_->stats();
    const EngineStats c = c_->stats();
    s.tree += c.tree;
    s.sol += c.sol;
    s.parents += c.parents;
    s.best = std::min(s.best, c.best);
    s.host_nodes += c.device_nodes + c.host_nodes;
    s.cpu_tree = c.tree;
    s.cpu_sol = c.sol;
    return s;
  }
  EngineStats gpu_stats() { return g_->stats(); }
  EngineStats cpu_stats() { return c_->stats(); }
  unsigned long long to_cpu() const { return to_cpu_; }
  unsigned long long to_gpu() const { return to_gpu_; }

  long run(long max_launches, double max_seconds, size_t stop_below) override {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    auto left = [&]() -> double {
      if (max_seconds <= 0) return 0.0;
      const double e = std::chrono::duration<double>(clock::now() - t0).count();
      return std::max(1e-6, max_seconds - e);
    };
    auto over = [&]() {
      return max_seconds > 0 && std::chrono::duration<double>(clock::now() - t0).count() >= max_seconds;
    };
    // replicated phase of an in-search rank split: the GPU alone (the CPU side is empty)
    if (g_->split_pending()) {
      g_->set_progress_hook(hook_);
      struct Unhook {
        IEngine* e;
        ~Unhook() { e->set_progress_hook(nullptr); }
      } uh{g_};
      return g_->run(max_launches, max_seconds, stop_below);
    }
    std::atomic<int> shared_best{std::min(g_->best(), c_->best())};
    auto pull_push = [&](int& b) {
      int cur = shared_best.load(std::memory_order_acquire);
      while (b < cur && !shared_best.compare_exchange_weak(cur, b, std::memory_order_acq_rel)) {
      }
      if (cur < b) b = cur;
    };
    // ---- CPU worker thread; everything below `mu` is shared with it ----
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false, cpu_hungry = false, gpu_hungry = false, to_cpu_ready = false, to_gpu_ready = false;
    std::vector<uint8_t> to_cpu_mail, to_gpu_mail;
    std::atomic<bool> interrupt{false};  // the CPU leaves c_->run() at its next batch
    std::exception_ptr worker_err;
    c_size_hint_.store(c_size());
    c_->set_progress_hook([&](size_t pool, int& b) {
      c_size_hint_.store(pool, std::memory_order_relaxed);
      pull_push(b);
      return interrupt.load(std::memory_order_acquire);
    });
    struct Unhook2 {  // declared before the worker's Join: destroyed after the worker is joined
      IEngine* a;
      IEngine* b;
      ~Unhook2() {
        a->set_progress_hook(nullptr);
        b->set_progress_hook(nullptr);
      }
    } uh2{g_, c_};
    const size_t nb = node_bytes();
    std::thread worker([&] {
      try {
        for (;;) {
          if (!interrupt.load() && c_size() > 0) c_->run(-1, 0.0, 1);
          c_size_hint_.store(c_size(), std::memory_order_relaxed);
          std::unique_lock<std::mutex> lk(mu);
          if (gpu_hungry) {  // hand half of the CPU pool to the GPU when it holds at least 2m
            const size_t n = c_->size() >= 2 * cfg_.m ? c_->size() / 2 : 0;
            to_gpu_mail.resize(n * nb);
            const size_t got = n ? c_->pop_host(to_gpu_mail.data(), n) : 0;
            to_gpu_mail.resize(got * nb);
            gpu_hungry = false;
            interrupt.store(stop);
            to_gpu_ready = true;
            cv.notify_all();
            continue;
          }
          if (stop) break;
          if (c_size() > 0) continue;
          cpu_hungry = true;  // dry: wait for the GPU's hand-over, a request, or the end
          cv.wait(lk, [&] { return stop || to_cpu_ready || gpu_hungry; });
          if (to_cpu_ready) {
            if (!to_cpu_mail.empty()) c_->push_host(to_cpu_mail.data(), to_cpu_mail.size() / nb);
            to_cpu_mail.clear();
            to_cpu_ready = false;
          }
          if (stop && !gpu_hungry) break;
        }
      } catch (...) {
        worker_err = std::current_exception();
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
        cpu_hungry = true;
        to_gpu_ready = true;
        cv.notify_all();
      }
    });
    struct Join {  // the worker is stopped and joined on every exit path
      std::mutex& mu;
      std::condition_variable& cv;
      bool& stop;
      std::atomic<bool>& interrupt;
      std::thread& th;
      void operator()() {
        {
          std::lock_guard<std::mutex> lk(mu);
          stop = true;
          interrupt.store(true);
          cv.notify_all();
        }
        if (th.joinable()) th.join();
      }
      ~Join() { (*this)(); }
    } join{mu, cv, stop, interrupt, worker};
    // ---- GPU side on this thread ----
    bool caller_stop = false;
    g_->set_progress_hook([&](size_t pool, int& b) {
      pull_push(b);
      const bool s = hook_ ? hook_(pool + c_size_hint_.load(std::memory_order_relaxed), b) : false;
      if (s) caller_stop = true;
      std::lock_guard<std::mutex> lk(mu);
      return s || (cpu_hungry && pool >= 2 * cfg_.m);
    });
    const size_t floor = std::max<size_t>(stop_below, 1);
    long launches = 0;
    for (;;) {
      const long l = g_->run(max_launches < 0 ? -1 : std::max(0L, max_launches - launches), left(), stop_below);
      launches += l;
      if (caller_stop || over() || (max_launches >= 0 && launches >= max_launches)) break;
      std::unique_lock<std::mutex> lk(mu);
      if (worker_err) break;
      const size_t gsz = g_->size();
      if (cpu_hungry && gsz >= 2 * cfg_.m) {  // feed the CPU worker from the GPU pool's bottom
        const size_t n = std::min(gsz / 2, cfg_.cpu_cap);
        to_cpu_mail.resize(n * nb);
        const size_t got = g_->pop_host(to_cpu_mail.data(), n);
        to_cpu_mail.resize(got * nb);
        to_cpu_ += got;
        cpu_hungry = false;
        to_cpu_ready = true;
        cv.notify_all();
        continue;
      }
      if (gsz >= floor) continue;
      // the GPU is dry: take half of the CPU pool (>= 2m), else let the CPU work and ask again
      bool done = false;
      for (;;) {
        if (cpu_hungry || worker_err) {  // both dry
          done = true;
          break;
        }
        gpu_hungry = true;
        interrupt.store(true);
        cv.wait(lk, [&] { return to_gpu_ready; });
        to_gpu_ready = false;
        const size_t n = to_gpu_mail.size() / nb;
        if (n) {
          g_->push_host(to_gpu_mail.data(), n);
          to_gpu_ += n;
          to_gpu_mail.clear();
          break;
        }
        lk.unlock();
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        lk.lock();
        if (over()) {
          done = true;
          break;
        }
      }
      if (done) break;
    }
    join();  // the CPU worker has stopped: both engines belong to this thread again
    if (worker_err) std::rethrow_exception(worker_err);
    const int b = shared_best.load();
    if (overlap_) {  // work may be in flight on both sides: applied when it completes
      g_->offer_best(b);
      c_->offer_best(b);
    } else {
      if (b < g_->best()) g_->set_best(b);
      if (b < c_->best()) c_->set_best(b);
    }
    return launches;
  }

 private:
  // n nodes from the bottom of `from` onto `to` (neither engine running)
  void move(IEngine* from, IEngine* to, size_t n) {
    std::vector<uint8_t> buf(n * node_bytes());
    const size_t got = from->pop_host(buf.data(), n);
    if (got) to->push_host(buf.data(), got);
  }

  // the CPU pool; with overlap on, without joining a batch left in flight (it counts)
  size_t c_size() { return overlap_ ? c_->size_known() : c_->size(); }

  IEngine* g_;
  IEngine* c_;
  bool overlap_ = false;
  HybridConfig cfg_;
  ProgressHook hook_;
  std::atomic<size_t> c_size_hint_{0};
  unsigned long long to_cpu_ = 0, to_gpu_ = 0;
};

}  // namespace tts
