// One native call per cooperative solve (the default multi-rank Step 1): host warm-up,
// in-search rank split, native rounds, final reductions — no Python between them.
//
// Parity: ref pfsp_dist_multigpu_cuda.c:142-905 (Step 1 redundant BFS on every rank,
// Step 2 rounds, reductions). The Python runtime (parallel/runtime.py) keeps the other
// Step-1 variants (host round-robin share, engine warm-up, resume) and calls
// run_dist_rounds directly; this session is what bench.py times at N > 1, so a solve
// of a 0.3-ms tree does not pay tens of microseconds of interpreter work per rank.
#pragma once

#include <chrono>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "dist_rounds.hpp"
#include "search_cpu.hpp"

namespace tts {

struct WarmupResult {
  std::vector<uint8_t> nodes;  // n nodes in the engine's layout
  size_t n = 0;
  unsigned long long tree = 0, sol = 0;
  int best = 0;
};
using WarmupFn = std::function<WarmupResult(int best, size_t target)>;

// Step 1 of `prob` (host breadth-first to `target` nodes); `keep` holds what the
// problem refers to (the instance) alive.
template <class Problem>
WarmupFn make_warmup(std::shared_ptr<const void> keep, Problem prob) {
  return [keep, prob](int best, size_t target) {
    using Node = typename Problem::Node;
    Pool<Node> pool;
    pool.push_back_free(prob.root());
    WarmupResult r;
    r.best = best;
    bfs_warmup(prob, pool, target, r.best, r.tree, r.sol);
    r.n = pool.size();
    const uint8_t* p = reinterpret_cast<const uint8_t*>(pool.data());
    r.nodes.assign(p, p + r.n * sizeof(Node));
    return r;
  };
}

struct DistSolveResult {
  int best = 0;
  unsigned long long tree = 0, sol = 0, rounds = 0;
  bool complete = true;
  double t_init = 0, t_search = 0, elapsed = 0;
  DistOutcome outcome;
};

// Rank-strided share of the warm-up nodes: i = rank, rank + world, ...; the last rank
// also takes the tail (ref Pool_atom.c:14-36 roundRobin_distribution).
inline void keep_round_robin(WarmupResult& w, size_t node_bytes, int rank, int world) {
  const size_t c = w.n / static_cast<size_t>(world);
  std::vector<uint8_t> mine;
  mine.reserve((c + static_cast<size_t>(world)) * node_bytes);
  auto take = [&](size_t i) { mine.insert(mine.end(), w.nodes.begin() + i * node_bytes, w.nodes.begin() + (i + 1) * node_bytes); };
  for (size_t k = 0; k < c; ++k) take(static_cast<size_t>(rank) + k * static_cast<size_t>(world));
  if (rank == world - 1)
    for (size_t i = c * static_cast<size_t>(world); i < w.n; ++i) take(i);
  w.n = mine.size() / node_bytes;
  w.nodes.swap(mine);
}

// Every rank: the same warm-up to `warm_target` nodes, then either the split armed at
// `split_min` pool nodes (IEngine::set_split, split = true) or the round-robin share
// of the warm-up nodes (split = false, ref roundRobin_distribution), the rounds, then
// global counts (Step-1 counts once). A world of one is the engine's fused solve from
// the warm-up (bench.py at N = 1); with o.time_limit it is a time box instead
// (complete = false when the pool was not exhausted).
inline DistSolveResult dist_solve_split(IEngine& e, RoundControl& ctl, const DistOptions& o, const WarmupFn& warm,
                                        int best, size_t warm_target, size_t split_min, const TransferFn& xfer,
                                        const RoundHook& hook, bool split = true) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  WarmupResult w = warm(best, warm_target);
  if (ctl.world() == 1) {
    // one rank: the engine's own fused solve (no rounds, no control plane)
    const auto t1 = clock::now();
    EngineStats st;
    bool complete = true;
    if (o.time_limit > 0) {
      e.begin(w.nodes.data(), w.n, w.best);
      e.run(-1, o.time_limit, 0);
      st = e.stats();
      complete = e.size() == 0;
    } else {
      st = e.solve_from(w.nodes.data(), w.n, w.best);
    }
    const auto t2 = clock::now();
    DistSolveResult r;
    r.complete = complete;
    r.outcome.complete = complete;
    r.best = std::min(st.best, w.best);
    r.tree = w.tree + st.tree;
    r.sol = w.sol + st.sol;
    r.t_init = std::chrono::duration<double>(t1 - t0).count();
    r.t_search = std::chrono::duration<double>(t2 - t1).count();
    r.elapsed = std::chrono::duration<double>(t2 - t0).count();
    DistOutcome& o1 = r.outcome;
    o1.best = r.best;
    auto one = [](auto& v, auto x) { v.assign(1, x); };
    one(o1.tree, st.tree);
    one(o1.sol, st.sol);
    for (auto* v : {&o1.sent, &o1.received, &o1.transfers_in, &o1.transfers_out, &o1.steals, &o1.success_steals,
                    &o1.idle_rounds, &o1.early_rounds, &o1.dropped})
      one(*v, 0ull);
    one(o1.cpu_tree, st.cpu_tree);
    one(o1.cpu_sol, st.cpu_sol);
    one(o1.t_run, st.t_run);
    one(o1.t_memcpy, st.t_memcpy);
    one(o1.t_malloc, st.t_malloc);
    for (auto* v : {&o1.t_comm, &o1.t_idle, &o1.t_termination, &o1.t_load_bal}) one(*v, 0.0);
    return r;
  }
  if (split)
    e.set_split(ctl.rank(), ctl.world(), split_min);
  else
    keep_round_robin(w, e.node_bytes(), ctl.rank(), ctl.world());
  e.begin(w.nodes.data(), w.n, w.best);
  const auto t1 = clock::now();
  DistSolveResult r;
  r.outcome = run_dist_rounds(e, ctl, o, xfer, hook, 0);
  const auto t2 = clock::now();
  r.tree = w.tree;
  r.sol = w.sol;
  for (auto x : r.outcome.tree) r.tree += x;
  for (auto x : r.outcome.sol) r.sol += x;
  r.best = std::min(r.outcome.best, w.best);
  r.rounds = r.outcome.rounds;
  r.complete = r.outcome.complete;
  r.t_init = std::chrono::duration<double>(t1 - t0).count();
  r.t_search = std::chrono::duration<double>(t2 - t1).count();
  r.elapsed = std::chrono::duration<double>(t2 - t0).count();
  return r;
}

}  // namespace tts
