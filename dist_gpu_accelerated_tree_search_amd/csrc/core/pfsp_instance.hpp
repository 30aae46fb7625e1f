// PFSP instance + constant bounding tables (host side).
//
// Parity:
//   LB1 tables (min heads / min tails)      ref pfsp/lib/c_bound_simple.c:278-322
//   LB2 tables (pairs, lags, Johnson order) ref pfsp/lib/c_bound_johnson.c:8-178
//                                           (LB2_FULL variant, all M(M-1)/2 pairs)
//
// Everything here is computed once per instance and then uploaded read-only to every
// GPU (csrc/hip/device_instance.hpp) where it lives in LDS / the scalar cache.
#pragma once

#include <algorithm>
#include <climits>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "taillard.hpp"

namespace tts {

enum class LowerBound : int { LB1_D = 0, LB1 = 1, LB2 = 2 };

inline const char* lower_bound_name(int lb) {
  switch (lb) {
    case 0: return "lb1_d";
    case 1: return "lb1";
    default: return "lb2";
  }
}

struct PfspInstance {
  int id = 0;           // Taillard id (1..120) or 0 for a synthetic instance
  int jobs = 0;         // N
  int machines = 0;     // M
  int best_known = INT_MAX;
  std::vector<int> p;   // machine-major  p[m*N + j]
  std::vector<int> pj;  // job-major      pj[j*M + m]
  std::vector<int> min_heads, min_tails;  // [M]
  // LB2 (two-machine Johnson bound) tables
  int npairs = 0;
  std::vector<int> pair_m0, pair_m1;  // [P]
  std::vector<int> lags;              // [P][N]  sum of p strictly between the pair
  std::vector<int> johnson;           // [P][N]  Johnson order (job ids)

  int pt(int machine, int job) const { return p[static_cast<size_t>(machine) * jobs + job]; }
};

namespace detail {

inline void fill_heads_tails(PfspInstance& in) {
  const int N = in.jobs, M = in.machines;
  in.min_heads.assign(M, INT_MAX);
  in.min_tails.assign(M, INT_MAX);
  in.min_heads[0] = 0;
  in.min_tails[M - 1] = 0;
  std::vector<int> acc(M);
  for (int j = 0; j < N; ++j) {
    // head of machine k = time job j needs on machines 0..k-1 when run alone
    acc[0] = in.pt(0, j);
    for (int k = 1; k < M; ++k) acc[k] = acc[k - 1] + in.pt(k, j);
    for (int k = 1; k < M; ++k) in.min_heads[k] = std::min(in.min_heads[k], acc[k - 1]);
    // tail of machine k = time job j needs on machines k+1..M-1
    acc[M - 1] = in.pt(M - 1, j);
    for (int k = M - 2; k >= 0; --k) acc[k] = acc[k + 1] + in.pt(k, j);
    for (int k = M - 2; k >= 0; --k) in.min_tails[k] = std::min(in.min_tails[k], acc[k + 1]);
  }
}

inline void fill_lb2_tables(PfspInstance& in) {
  const int N = in.jobs, M = in.machines;
  in.npairs = M * (M - 1) / 2;
  in.pair_m0.clear();
  in.pair_m1.clear();
  for (int a = 0; a < M - 1; ++a)
    for (int b = a + 1; b < M; ++b) {
      in.pair_m0.push_back(a);
      in.pair_m1.push_back(b);
    }
  in.lags.assign(static_cast<size_t>(in.npairs) * N, 0);
  in.johnson.assign(static_cast<size_t>(in.npairs) * N, 0);

  struct Item {
    int job, part, a, b;
  };
  std::vector<Item> items(N);
  for (int q = 0; q < in.npairs; ++q) {
    const int m0 = in.pair_m0[q], m1 = in.pair_m1[q];
    for (int j = 0; j < N; ++j) {
      int lag = 0;
      for (int k = m0 + 1; k < m1; ++k) lag += in.pt(k, j);
      in.lags[static_cast<size_t>(q) * N + j] = lag;
      const int a = in.pt(m0, j) + lag, b = in.pt(m1, j) + lag;
      items[j] = Item{j, a < b ? 0 : 1, a, b};
    }
    // Johnson's rule: set {a<b} by increasing a, then set {a>=b} by decreasing b.
    // A stable sort reproduces the tie order of the reference's (merge-sort) qsort.
    std::stable_sort(items.begin(), items.end(), [](const Item& x, const Item& y) {
      if (x.part != y.part) return x.part < y.part;
      return x.part == 0 ? x.a < y.a : x.b > y.b;
    });
    for (int r = 0; r < N; ++r) in.johnson[static_cast<size_t>(q) * N + r] = items[r].job;
  }
}

}  // namespace detail

inline PfspInstance make_instance(int jobs, int machines, std::vector<int> p_machine_major, int id = 0,
                                  int best_known = INT_MAX) {
  if (jobs < 2 || machines < 2) throw std::invalid_argument("PFSP instance needs >= 2 jobs and >= 2 machines");
  if (static_cast<int>(p_machine_major.size()) != jobs * machines)
    throw std::invalid_argument("processing-time matrix has the wrong size");
  PfspInstance in;
  in.id = id;
  in.jobs = jobs;
  in.machines = machines;
  in.best_known = best_known;
  in.p = std::move(p_machine_major);
  in.pj.resize(in.p.size());
  for (int m = 0; m < machines; ++m)
    for (int j = 0; j < jobs; ++j) in.pj[static_cast<size_t>(j) * machines + m] = in.pt(m, j);
  detail::fill_heads_tails(in);
  detail::fill_lb2_tables(in);
  return in;
}

inline PfspInstance make_taillard_instance(int id) {
  return make_instance(taillard_jobs(id), taillard_machines(id), taillard_processing_times(id), id,
                       taillard_best_ub(id));
}

}  // namespace tts
