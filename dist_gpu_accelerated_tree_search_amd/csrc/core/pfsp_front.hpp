// LB1 / LB1_d search on front-carrying nodes (core/pfsp_node.hpp PfspFrontNode):
// padded bound tables, the host problem (Step 1, Step 3, CPU workers, CPU drivers,
// oracle of the GPU kernel) and the layout dispatch every engine and driver uses.
//
// Parity: same bounds, same tree and solution counts as ref decompose_lb1 /
// decompose_lb1_d (PFSP_lib.c:7-90, c_bound_simple.c:127-244): the child appending
// job j gets
//     lb = max_m ( start_m + remain_m + tail_m ),   start_m = max(front'_{m-1}, front_m)
// where remain is the parent's unscheduled work (job j included) and tail the minimum
// tails — ref add_front_and_bound (c_bound_simple.c:219-244), i.e. LB1 == LB1_d
// (SURVEY §2.4). Only the node representation differs: the prefix's completion
// times are carried instead of recomputed from the permutation.
#pragma once

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstdint>
#include <stdexcept>
#include <type_traits>
#include <utility>

#include "pfsp_instance.hpp"
#include "pfsp_node.hpp"
#include "problems.hpp"

namespace tts {

// Machine-count bucket of the front layout / GPU kernels: 5, 10 or 20; smaller counts
// run with zero-time padding machines (their terms never exceed a real machine's).
inline int pfsp_machine_bucket(int machines) {
  if (machines >= 1 && machines <= 5) return 5;
  if (machines > 5 && machines <= 10) return 10;
  if (machines > 10 && machines <= 20) return 20;
  return 0;
}

// Per-machine tables padded to MB machines (the layout the GPU kernels use too):
// a padding machine has zero processing times, no tail, and the whole real route of
// the cheapest job as its head, so every bound and every real front is unchanged.
struct PfspPadded {
  int heads[20], tails[20], sum_all[20];
};
inline PfspPadded pfsp_padded_tables(const PfspInstance& in, int MB) {
  if (in.machines > MB || MB > 20) throw std::invalid_argument("machine count exceeds the bucket");
  PfspPadded t{};
  int route = INT_MAX;
  for (int j = 0; j < in.jobs; ++j) {
    int s = 0;
    for (int k = 0; k < in.machines; ++k) s += in.pt(k, j);
    route = std::min(route, s);
  }
  for (int m = 0; m < MB; ++m) {
    const bool real = m < in.machines;
    t.heads[m] = real ? in.min_heads[m] : route;
    t.tails[m] = real ? in.min_tails[m] : 0;
    long s = 0;
    if (real)
      for (int j = 0; j < in.jobs; ++j) s += in.pt(m, j);
    t.sum_all[m] = static_cast<int>(s);
  }
  return t;
}

// The front layout applies: LB1 / LB1_d, at most 50 jobs (job sets of 32 bits up to 20
// jobs, 64 bits up to 50) and 20 machines, and every front fits 16 bits (the sum of all
// processing times does).
// TTS_FRONT=0 turns it off (permutation nodes everywhere: A/B runs); the CPU and the
// HIP module read the variable alike, so every engine of a process agrees.
inline bool pfsp_front_ok(const PfspInstance& in, int lb) {
  if (lb != 0 && lb != 1) return false;
  if (const char* e = std::getenv("TTS_FRONT"))
    if (e[0] == '0') return false;
  if (in.jobs > 50 || in.machines > 20 || pfsp_machine_bucket(in.machines) == 0) return false;
  long tot = 0;
  for (int v : in.p) tot += v;
  return tot < 65536;
}

// job bucket of the front layout: 20 (32-bit job sets) or 50 (64-bit)
inline int pfsp_front_jobs(int jobs) { return jobs <= 20 ? 20 : 50; }

template <int MB, int NJ = 20>
struct PfspFrontProblem {
  using Node = PfspFrontNode<MB, NJ>;
  using Mask = typename Node::Mask;
  static constexpr int kJobs = NJ;
  static constexpr int kMaxJ = NJ <= 32 ? 32 : 64;
  const PfspInstance* inst = nullptr;
  int lb = 1;
  int jobs = 0;
  PfspPadded tab{};
  int p[kMaxJ][MB];  // job-major, padded machines 0

  PfspFrontProblem(const PfspInstance& in, int lb_kind) : inst(&in), lb(lb_kind), jobs(in.jobs) {
    if (!pfsp_front_ok(in, lb_kind)) throw std::invalid_argument("front layout does not apply to this instance");
    if (pfsp_machine_bucket(in.machines) != MB) throw std::invalid_argument("wrong machine bucket");
    if (pfsp_front_jobs(in.jobs) != NJ) throw std::invalid_argument("wrong front job bucket");
    tab = pfsp_padded_tables(in, MB);
    for (int j = 0; j < kMaxJ; ++j)
      for (int m = 0; m < MB; ++m) p[j][m] = (j < in.jobs && m < in.machines) ? in.pt(m, j) : 0;
  }

  Mask all_jobs() const {
    return jobs >= static_cast<int>(8 * sizeof(Mask)) ? ~Mask(0) : ((Mask(1) << jobs) - Mask(1));
  }

  Node root() const {
    Node r{};
    r.depth = 0;
    r.rest = all_jobs();
    for (int m = 0; m < MB; ++m) r.front[m] = static_cast<uint16_t>(tab.heads[m]);
    return r;
  }

  // remain + tail of the parent's unscheduled jobs, per machine
  void remain_tail(const Node& n, int* r) const {
    for (int m = 0; m < MB; ++m) r[m] = tab.tails[m];
    for (Mask x = n.rest; x; x &= x - 1) {
      const int j = mask_ctz(x);
      for (int m = 0; m < MB; ++m) r[m] += p[j][m];
    }
  }

  // Bound of the child appending job j; its front in cf (when non-null).
  int child(const Node& n, const int* r, int j, uint16_t* cf) const {
    const int* pj = p[j];
    int f0 = n.front[0];
    int lb = f0 + r[0];
    int tt = f0 + pj[0];
    // the root's front is the minimum heads (bound only); a child's front starts from 0
    int ft = (n.depth == 0 ? 0 : f0) + pj[0];
    if (cf) cf[0] = static_cast<uint16_t>(ft);
    for (int m = 1; m < MB; ++m) {
      const int fm = n.front[m];
      const int sv = std::max(tt, fm);
      lb = std::max(lb, sv + r[m]);
      tt = sv + pj[m];
      ft = std::max(ft, n.depth == 0 ? 0 : fm) + pj[m];
      if (cf) cf[m] = static_cast<uint16_t>(ft);
    }
    return lb;
  }

  // Bounds of every child, by job (lb_by_job[j] for j in n.rest).
  void children_bounds(const Node& n, int* lb_by_job) const {
    int r[MB];
    remain_tail(n, r);
    for (Mask x = n.rest; x; x &= x - 1) {
      const int j = mask_ctz(x);
      lb_by_job[j] = child(n, r, j, nullptr);
    }
  }

  template <class Push>
  void decompose(const Node& parent, int& best, unsigned long long& tree, unsigned long long& sol, Push&& push) const {
    int r[MB];
    remain_tail(parent, r);
    const bool leaf = parent.depth + 1 == jobs;
    for (Mask x = parent.rest; x; x &= x - 1) {
      const int j = mask_ctz(x);
      Node c{};
      const int b = child(parent, r, j, leaf ? nullptr : c.front);
      if (leaf) {
        ++sol;
        if (b < best) best = b;
      } else if (b < best) {
        c.depth = static_cast<uint8_t>(parent.depth + 1);
        c.rest = parent.rest & ~(Mask(1) << j);
        push(c);
        ++tree;
      }
    }
  }
};

template <class P>
struct is_front_problem : std::false_type {};
template <int MB, int NJ>
struct is_front_problem<PfspFrontProblem<MB, NJ>> : std::true_type {};

// Front node of a permutation node (scheduled prefix prmu[0..depth)).
template <int MB, int NJ, class PermNode>
inline PfspFrontNode<MB, NJ> pfsp_front_from_perm(const PfspFrontProblem<MB, NJ>& prob, const PermNode& n) {
  using Mask = typename PfspFrontNode<MB, NJ>::Mask;
  PfspFrontNode<MB, NJ> f{};
  f.depth = static_cast<uint8_t>(n.depth);
  f.rest = prob.all_jobs();
  if (n.depth == 0) {
    for (int m = 0; m < MB; ++m) f.front[m] = static_cast<uint16_t>(prob.tab.heads[m]);
    return f;
  }
  int fr[MB] = {};
  for (int i = 0; i < n.depth; ++i) {
    const int j = n.prmu[i];
    f.rest &= ~(Mask(1) << j);
    fr[0] += prob.p[j][0];
    for (int m = 1; m < MB; ++m) fr[m] = std::max(fr[m - 1], fr[m]) + prob.p[j][m];
  }
  for (int m = 0; m < MB; ++m) f.front[m] = static_cast<uint16_t>(fr[m]);
  return f;
}

// Calls f(problem) with the problem in the node layout every engine, driver and host
// step uses for (instance, lb): the front layout where it applies, else the
// permutation layout of the job-count bucket.
template <class F>
decltype(auto) with_pfsp_problem(const PfspInstance& in, int lb, F&& f) {
  if (pfsp_front_ok(in, lb)) {
    if (in.jobs <= 20) {
      switch (pfsp_machine_bucket(in.machines)) {
        case 5: return f(PfspFrontProblem<5>(in, lb));
        case 10: return f(PfspFrontProblem<10>(in, lb));
        default: return f(PfspFrontProblem<20>(in, lb));
      }
    }
    switch (pfsp_machine_bucket(in.machines)) {
      case 5: return f(PfspFrontProblem<5, 50>(in, lb));
      case 10: return f(PfspFrontProblem<10, 50>(in, lb));
      default: return f(PfspFrontProblem<20, 50>(in, lb));
    }
  }
  return with_pfsp_bucket(in.jobs, [&](auto nj) -> decltype(auto) {
    return f(PfspProblem<decltype(nj)::value>(in, lb));
  });
}

}  // namespace tts
