// CPU search drivers shared by both problems:
//   * bfs_warmup         Step 1: breadth-first until the pool holds `target` nodes
//                        (ref pfsp_multigpu_cuda.c:111-118, popFrontFree + decompose)
//   * dfs_drain          Step 3 / sequential: depth-first until the pool is empty
//                        (ref pfsp_c.c:55-63)
//   * multicore_search   Step 2 on C threads: per-thread pools, batch pop of up to
//                        `batch` parents (ratio 1, threshold m), random steal-half
//                        (victim >= 2m, cap 5*M), BUSY/IDLE termination with a
//                        sticky all-idle flag (ref pfsp_omp_c.c:54-370,
//                        common/util.c:4-58).
// The incumbent is a std::atomic<int> read once per batch and lowered with a CAS
// loop (the reference's checkBest spin lock, pfsp_multigpu_cuda.c:30-50; CPU
// workers there also race on *best, SURVEY §5.2 item 2 — not here).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <random>
#include <thread>
#include <vector>

#include "pool.hpp"
#include "problems.hpp"

namespace tts {

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Per-worker counters and phase timers; same buckets as the reference CSV
// (ref pfsp/lib/PFSP_statistic.c:82-84).
struct WorkerStats {
  u64 tree = 0, sol = 0, gen_child = 0, steals = 0, success_steals = 0, terminations = 0;
  double t_memcpy = 0, t_malloc = 0, t_kernel = 0, t_gen_child = 0, t_pool_ops = 0, t_idle = 0, t_termination = 0;
};

inline void atomic_min(std::atomic<int>& a, int v) {
  int cur = a.load(std::memory_order_relaxed);
  while (v < cur && !a.compare_exchange_weak(cur, v, std::memory_order_acq_rel)) {
  }
}

template <class Problem>
void bfs_warmup(const Problem& prob, Pool<typename Problem::Node>& pool, size_t target, int& best, u64& tree,
                u64& sol) {
  using Node = typename Problem::Node;
  Node parent;
  while (pool.size() < target) {
    if (!pool.pop_front_free(parent)) break;
    prob.decompose(parent, best, tree, sol, [&](const Node& c) { pool.push_back_free(c); });
  }
}

template <class Problem>
void dfs_drain(const Problem& prob, Pool<typename Problem::Node>& pool, int& best, u64& tree, u64& sol) {
  using Node = typename Problem::Node;
  Node parent;
  while (pool.pop_back_free(parent))
    prob.decompose(parent, best, tree, sol, [&](const Node& c) { pool.push_back_free(c); });
}

struct MulticoreConfig {
  int threads = 1;
  size_t m = 25;        // min pool size to pop a batch / steal unit
  size_t batch = 20000; // max parents per pop (ref falseM, pfsp_omp_c.c:158)
  size_t steal_cap = 250000;  // 5*M (ref pfsp_omp_c.c:256)
  bool work_stealing = true;
  uint64_t seed = 0x5eedULL;
};

// Step 2 on `cfg.threads` workers. Consumes `pool` (round-robin split), leaves any
// node a worker could not process (pool < m and nothing to steal) back in `pool`.
template <class Problem>
void multicore_search(const Problem& prob, Pool<typename Problem::Node>& pool, const MulticoreConfig& cfg,
                      std::atomic<int>& best, std::vector<WorkerStats>& stats) {
  using Node = typename Problem::Node;
  const int C = std::max(1, cfg.threads);
  stats.assign(C, WorkerStats{});
  std::vector<Pool<Node>> pools(C);
  for (int i = 0; i < C; ++i) pools[i].round_robin_from(pool, i, C);
  pool.clear();

  std::vector<std::atomic<bool>> idle(C);
  for (auto& s : idle) s.store(false);
  std::atomic<bool> all_idle{false};

  auto all_idle_check = [&]() {
    if (all_idle.load(std::memory_order_acquire)) return true;
    for (int i = 0; i < C; ++i)
      if (!idle[i].load(std::memory_order_acquire)) return false;
    all_idle.store(true, std::memory_order_release);
    return true;
  };

  auto worker = [&](int id) {
    WorkerStats& st = stats[id];
    Pool<Node>& mine = pools[id];
    std::vector<Node> parents(cfg.batch);
    std::vector<Node> stolen(cfg.steal_cap);
    Pool<Node> children;
    std::vector<int> victims(C);
    std::mt19937_64 rng(cfg.seed * 0x9E3779B97F4A7C15ULL + id);
    bool busy = true;
    for (;;) {
      double t0 = now_s();
      const size_t n = mine.pop_back_bulk(cfg.m, cfg.batch, parents.data(), 1);
      st.t_pool_ops += now_s() - t0;
      if (n > 0) {
        if (!busy) {
          busy = true;
          idle[id].store(false, std::memory_order_release);
        }
        int best_l = best.load(std::memory_order_acquire);
        t0 = now_s();
        // The batch is processed depth-first through a private stack, as the
        // reference does with parentsPool/childrenPool (pfsp_omp_c.c:169-190).
        for (size_t i = 0; i < n; ++i)
          prob.decompose(parents[i], best_l, st.tree, st.sol, [&](const Node& c) { children.push_back_free(c); });
        st.t_kernel += now_s() - t0;
        atomic_min(best, best_l);
        t0 = now_s();
        st.gen_child += children.size();
        mine.push_back_bulk(children.data(), children.size());
        children.clear();
        st.t_pool_ops += now_s() - t0;
        continue;
      }
      if (!cfg.work_stealing) break;
      // ---- random steal-half ----
      t0 = now_s();
      for (int i = 0; i < C; ++i) victims[i] = i;
      std::shuffle(victims.begin(), victims.end(), rng);
      bool got = false;
      for (int t = 0; t < C && !got; ++t) {
        const int v = victims[t];
        if (v == id) continue;
        ++st.steals;
        Pool<Node>& vp = pools[v];
        for (int tries = 0; tries < 10; ++tries) {
          if (!vp.lock().try_lock()) continue;
          size_t k = 0;
          if (vp.size() >= 2 * cfg.m) k = vp.pop_back_bulk_free(cfg.m, cfg.steal_cap, stolen.data(), 2);
          vp.lock().unlock();
          if (k > 0) {
            const double tp = now_s();
            mine.push_back_bulk(stolen.data(), k);
            st.t_pool_ops += now_s() - tp;
            ++st.success_steals;
            got = true;
          }
          break;
        }
      }
      st.t_idle += now_s() - t0;
      if (got) continue;
      t0 = now_s();
      ++st.terminations;
      if (busy) {
        busy = false;
        idle[id].store(true, std::memory_order_release);
      }
      const bool done = all_idle_check();
      st.t_termination += now_s() - t0;
      if (done) break;
      std::this_thread::yield();
    }
  };

  std::vector<std::thread> th;
  th.reserve(C);
  for (int i = 0; i < C; ++i) th.emplace_back(worker, i);
  for (auto& t : th) t.join();
  for (int i = 0; i < C; ++i) pool.push_back_bulk_free(pools[i].data(), pools[i].size());
}

}  // namespace tts
