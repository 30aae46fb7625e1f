// CPU-only end-to-end drivers (sequential and multi-core), shared by the native
// CLIs (csrc/apps) and the Python bindings.
//   run_pfsp_sequential   ref pfsp/pfsp_c.c:26-73
//   run_pfsp_multicore    ref pfsp/pfsp_omp_c.c:54-370 (Step 1 BFS to C*m nodes,
//                         Step 2 WS threads, Step 3 sequential tail)
//   run_queens_*          ref nqueens/nqueens_c.c:120-148
#pragma once

#include <climits>
#include <cstdio>
#include <type_traits>
#include <utility>

#include "pfsp_front.hpp"
#include "report.hpp"

namespace tts {

struct RunResult {
  int best = INT_MAX;
  u64 tree = 0, sol = 0;
  double t_init = 0, t_search = 0, t_tail = 0, elapsed = 0;
  std::vector<WorkerStats> workers;
};

template <class Problem>
RunResult run_sequential(const Problem& prob, int best_init) {
  using Node = typename Problem::Node;
  RunResult r;
  r.best = best_init;
  Pool<Node> pool;
  pool.push_back(prob.root());
  const double t0 = now_s();
  dfs_drain(prob, pool, r.best, r.tree, r.sol);
  r.t_search = now_s() - t0;
  r.elapsed = r.t_search;
  return r;
}

template <class Problem>
RunResult run_multicore(const Problem& prob, int best_init, const MulticoreConfig& cfg, bool verbose) {
  using Node = typename Problem::Node;
  RunResult r;
  r.best = best_init;
  Pool<Node> pool;
  pool.push_back(prob.root());
  double t0 = now_s();
  bfs_warmup(prob, pool, static_cast<size_t>(cfg.threads) * cfg.m, r.best, r.tree, r.sol);
  r.t_init = now_s() - t0;
  if (verbose) print_phase("Initial search on CPU completed", r.tree, r.sol, r.t_init);

  t0 = now_s();
  std::atomic<int> best{r.best};
  multicore_search(prob, pool, cfg, best, r.workers);
  r.best = best.load();
  for (auto& w : r.workers) {
    r.tree += w.tree;
    r.sol += w.sol;
  }
  r.t_search = now_s() - t0;
  if (verbose) print_phase("Search on Parallel CPU completed", r.tree, r.sol, r.t_search);

  t0 = now_s();
  dfs_drain(prob, pool, r.best, r.tree, r.sol);
  r.t_tail = now_s() - t0;
  if (verbose) {
    print_phase("Search on CPU completed", r.tree, r.sol, r.t_tail);
    std::printf("\nExploration terminated.\n");
  }
  r.elapsed = r.t_init + r.t_search + r.t_tail;
  return r;
}

inline RunResult run_pfsp_cpu(const PfspInstance& in, int lb, int best_init, int threads, const MulticoreConfig& cfg,
                              bool verbose) {
  return with_pfsp_problem(in, lb, [&](auto prob) {
    if (threads <= 0) return run_sequential(prob, best_init);
    MulticoreConfig c = cfg;
    c.threads = threads;
    return run_multicore(prob, best_init, c, verbose);
  });
}

inline RunResult run_queens_cpu(int N, int G, int threads, const MulticoreConfig& cfg, bool verbose) {
  QueensProblem prob(N, G);
  if (threads <= 0) return run_sequential(prob, 0);
  MulticoreConfig c = cfg;
  c.threads = threads;
  return run_multicore(prob, 0, c, verbose);
}

}  // namespace tts
