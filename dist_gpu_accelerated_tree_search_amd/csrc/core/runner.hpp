// Single-process multi-worker runner: several engines (GPUs and/or CPU workers)
// driven by one host thread each, sharing work in lock-step rounds.
//
// Parity: ref pfsp/pfsp_multigpu_cuda.c:55-511 — one OpenMP thread per GPU, optional
// CPU worker threads (-C 1), random steal-half work stealing under spin locks,
// BUSY/IDLE termination, checkBest incumbent sharing. Here the same roles run as:
//   * each worker runs its engine for a time slice (device-resident search);
//   * a round = barrier -> leader reads every pool size + incumbent, takes the
//     MIN incumbent, detects termination (all pools empty: exact, nothing is in
//     flight between rounds), plans steal-half transfers (same plan as
//     parallel/comm.py::plan_sharing) -> barrier -> donors move nodes into
//     staging -> barrier -> receivers load them -> next slice.
// The multi-process equivalent over RCCL is parallel/runtime.py; this runner is
// the native path (no Python, no collectives library) for one node.
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "engine_api.hpp"

namespace tts {

struct RunnerConfig {
  size_t m = 25;               // needy below m nodes, donors need >= 2m
  size_t steal_cap = 250000;   // ref 5*M
  double slice_min = 0.0005;   // seconds of local search between rounds (adaptive)
  double slice_max = 0.05;
  bool work_sharing = true;    // ref -w
};

struct WorkerReport {
  EngineStats st;
  unsigned long long rounds = 0, sent = 0, received = 0, transfers_in = 0, transfers_out = 0;
  double t_run = 0, t_comm = 0, t_idle = 0;
};

// Deterministic steal-half matching (identical to parallel/comm.py::plan_sharing
// with a single node).
inline std::vector<std::tuple<int, int, size_t>> plan_sharing(const std::vector<size_t>& sizes, size_t m,
                                                              size_t cap) {
  const int n = static_cast<int>(sizes.size());
  std::vector<size_t> left = sizes;
  std::vector<char> needy(n, 0);
  for (int r = 0; r < n; ++r) needy[r] = sizes[r] < m;
  std::vector<std::tuple<int, int, size_t>> plan;
  for (int r = 0; r < n; ++r) {
    if (!needy[r]) continue;
    int d = -1;
    for (int x = 0; x < n; ++x) {
      if (x == r || needy[x] || left[x] < 2 * m) continue;
      if (d < 0 || left[x] > left[d]) d = x;
    }
    if (d < 0) continue;
    const size_t k = std::min(left[d] / 2, cap);
    if (k == 0) continue;
    left[d] -= k;
    left[r] += k;
    plan.emplace_back(d, r, k);
  }
  return plan;
}

class RoundBarrier {
 public:
  explicit RoundBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const unsigned long long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen != gen_; });
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  unsigned long long gen_ = 0;
};

// Runs all workers to exhaustion. initial[w] holds worker w's starting nodes
// (node_bytes each). Returns per-worker reports; `best` is updated to the final
// incumbent. Engines must share one node layout.
inline std::vector<WorkerReport> run_workers(const std::vector<IEngine*>& engines,
                                             const std::vector<std::vector<uint8_t>>& initial, int& best,
                                             const RunnerConfig& cfg) {
  const int W = static_cast<int>(engines.size());
  if (W == 0) return {};
  const size_t nb = engines[0]->node_bytes();
  for (auto* e : engines)
    if (e->node_bytes() != nb) throw std::invalid_argument("workers disagree on the node layout");
  std::vector<WorkerReport> rep(W);
  std::vector<size_t> sizes(W, 0);
  std::vector<int> bests(W, best);
  std::vector<std::vector<uint8_t>> staging(W);  // staging[r]: nodes bound for worker r
  std::vector<std::tuple<int, int, size_t>> plan;
  bool done = false;
  int gbest = best;
  double slice = cfg.slice_min;
  RoundBarrier bar(W);
  std::mutex stage_mu;

  auto now = [] { return std::chrono::steady_clock::now(); };
  auto secs = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };

  // A worker whose engine throws keeps taking part in the rounds with an empty
  // pool (so no thread waits forever at a barrier); the first error is rethrown.
  std::exception_ptr err;
  std::mutex err_mu;
  auto fail = [&](std::exception_ptr p) {
    std::lock_guard<std::mutex> lk(err_mu);
    if (!err) err = p;
  };

  auto worker = [&](int w) {
    IEngine* e = engines[w];
    WorkerReport& r = rep[w];
    bool dead = false;
    auto guarded = [&](auto&& f) {
      if (dead) return;
      try {
        f();
      } catch (...) {
        fail(std::current_exception());
        dead = true;
      }
    };
    const std::vector<uint8_t>& init = initial[w];
    guarded([&] { e->begin(init.data(), init.size() / nb, best); });
    for (;;) {
      const auto t0 = now();
      guarded([&] { e->run(-1, slice, 1); });
      const auto t1 = now();
      r.t_run += secs(t0, t1);
      sizes[w] = 0;
      guarded([&] {
        sizes[w] = e->size();
        bests[w] = e->best();
      });
      bar.wait();
      if (w == 0) {  // leader: incumbent, termination, plan
        gbest = *std::min_element(bests.begin(), bests.end());
        size_t total = 0;
        bool starving = false;
        for (size_t s : sizes) {
          total += s;
          starving |= s < cfg.m;
        }
        done = total == 0;
        plan.clear();
        if (!done && cfg.work_sharing && W > 1 && starving) plan = plan_sharing(sizes, cfg.m, cfg.steal_cap);
        slice = starving ? cfg.slice_min : std::min(cfg.slice_max, slice * 2);
      }
      bar.wait();
      ++r.rounds;
      if (done) {
        r.t_comm += secs(t1, now());
        break;
      }
      if (gbest < bests[w]) guarded([&] { e->set_best(gbest); });
      if (!plan.empty()) {
        // donors: pool bottom -> staging of each receiver
        for (const auto& t : plan) {
          const int d = std::get<0>(t), rc = std::get<1>(t);
          const size_t k = std::get<2>(t);
          if (d != w) continue;
          std::vector<uint8_t> buf(k * nb);
          size_t got = 0;
          guarded([&] { got = e->pop_host(buf.data(), k); });
          buf.resize(got * nb);
          {
            std::lock_guard<std::mutex> lk(stage_mu);
            staging[rc].insert(staging[rc].end(), buf.begin(), buf.end());
          }
          r.sent += got;
          ++r.transfers_out;
        }
        bar.wait();
        if (!staging[w].empty()) {
          guarded([&] { e->push_host(staging[w].data(), staging[w].size() / nb); });
          r.received += staging[w].size() / nb;
          ++r.transfers_in;
          staging[w].clear();
        }
        bar.wait();
      }
      if (sizes[w] == 0) r.t_idle += secs(t0, now());
      r.t_comm += secs(t1, now());
    }
    guarded([&] { r.st = e->stats(); });
  };

  std::vector<std::thread> th;
  th.reserve(W);
  for (int w = 0; w < W; ++w) th.emplace_back(worker, w);
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
  best = gbest;
  for (auto& r : rep) best = std::min(best, r.st.best);
  return rep;
}

}  // namespace tts
