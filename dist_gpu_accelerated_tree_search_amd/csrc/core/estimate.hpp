// Tree-size estimation for long solves (ta056 LB2 and the like): Knuth's random-probe
// estimator on the host (D. E. Knuth, "Estimating the efficiency of backtrack
// programs", Math. Comp. 1975). A probe walks from the root, at every node expands
// all children with the problem's own decompose (same bound, same incumbent, same
// counting rules as the search), multiplies a weight by the number of pushed
// children and follows one of them uniformly at random. The sum of the weights is
// an unbiased estimate of the explored tree (the reference's "tree" count) for a
// fixed incumbent, i.e. for -u 1 runs. The reference has no estimator; this is what
// projects a time-to-solution from a measured nodes/s rate.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <random>
#include <thread>
#include <vector>

#include "problems.hpp"

namespace tts {

struct TreeEstimate {
  double tree = 0;        // mean estimate of the explored tree
  double stderr_ = 0;     // standard error of the mean
  double depth = 0;       // mean probe depth
  unsigned long long probes = 0;
  std::vector<double> per_level;  // mean estimated nodes per tree level
};

template <class Problem>
TreeEstimate knuth_estimate(const Problem& prob, int best, unsigned long long probes, unsigned long long seed,
                            int threads = 1) {
  using Node = typename Problem::Node;
  threads = std::max(1, threads);
  struct Acc {
    double s = 0, s2 = 0, depth = 0;
    std::vector<double> lvl;
  };
  std::vector<Acc> acc(threads);
  auto worker = [&](int t) {
    std::mt19937_64 rng(seed * 0x9e3779b97f4a7c15ull + static_cast<unsigned long long>(t));
    Acc& a = acc[t];
    std::vector<Node> kids;
    for (unsigned long long p = static_cast<unsigned long long>(t); p < probes; p += static_cast<unsigned long long>(threads)) {
      Node x = prob.root();
      double w = 1, est = 0;
      int lvl = 0;
      for (;;) {
        kids.clear();
        int b = best;
        u64 tree = 0, sol = 0;
        prob.decompose(x, b, tree, sol, [&](const Node& c) { kids.push_back(c); });
        if (kids.empty()) break;
        w *= static_cast<double>(kids.size());
        est += w;
        if (static_cast<int>(a.lvl.size()) <= lvl) a.lvl.resize(lvl + 1, 0.0);
        a.lvl[lvl] += w;
        ++lvl;
        x = kids[std::uniform_int_distribution<size_t>(0, kids.size() - 1)(rng)];
      }
      a.s += est;
      a.s2 += est * est;
      a.depth += lvl;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  TreeEstimate r;
  r.probes = probes;
  double s = 0, s2 = 0, dep = 0;
  for (auto& a : acc) {
    s += a.s;
    s2 += a.s2;
    dep += a.depth;
    if (a.lvl.size() > r.per_level.size()) r.per_level.resize(a.lvl.size(), 0.0);
    for (size_t i = 0; i < a.lvl.size(); ++i) r.per_level[i] += a.lvl[i];
  }
  const double n = static_cast<double>(std::max<unsigned long long>(1, probes));
  r.tree = s / n;
  const double var = std::max(0.0, s2 / n - r.tree * r.tree);
  r.stderr_ = std::sqrt(var / n);
  r.depth = dep / n;
  for (auto& v : r.per_level) v /= n;
  return r;
}

}  // namespace tts
