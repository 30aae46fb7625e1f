// Host (CPU) implementations of the three PFSP lower bounds.
//
// Parity (same values, same early-exit semantics):
//   LB1    one-machine bound, full recompute per child   ref c_bound_simple.c:52-158
//   LB1_d  all children of a parent from one prefix      ref c_bound_simple.c:160-244
//   LB2    two-machine Johnson bound with early exit      ref c_bound_johnson.c:180-254
// They serve Step 1 (BFS warm-up), Step 3 (CPU tail), the CPU-only drivers and the
// CPU workers (-C 1), and are the oracle every GPU kernel is tested against.
#pragma once

#include <utility>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <vector>

#include "pfsp_instance.hpp"

namespace tts {

// Completion times on each machine of the scheduled prefix perm[0..len).
// An empty prefix uses the per-machine minimum heads (ref schedule_front, limit1==-1).
template <typename Id>
inline void cpu_front(const PfspInstance& in, const Id* perm, int len, int* front) {
  const int N = in.jobs, M = in.machines;
  if (len == 0) {
    for (int k = 0; k < M; ++k) front[k] = in.min_heads[k];
    return;
  }
  for (int k = 0; k < M; ++k) front[k] = 0;
  for (int i = 0; i < len; ++i) {
    const int j = perm[i];
    front[0] += in.p[j];
    for (int k = 1; k < M; ++k) front[k] = std::max(front[k - 1], front[k]) + in.p[static_cast<size_t>(k) * N + j];
  }
}

// Sum of processing times of perm[from..N) on each machine.
template <typename Id>
inline void cpu_remain(const PfspInstance& in, const Id* perm, int from, int* remain) {
  const int N = in.jobs, M = in.machines;
  for (int k = 0; k < M; ++k) remain[k] = 0;
  for (int i = from; i < N; ++i) {
    const int j = perm[i];
    for (int k = 0; k < M; ++k) remain[k] += in.p[static_cast<size_t>(k) * N + j];
  }
}

// max over machines of (running max of front+remain) + back; ref machine_bound_from_parts.
inline int cpu_machine_bound(const int* front, const int* back, const int* remain, int M) {
  int run = front[0] + remain[0];
  int lb = run + back[0];
  for (int k = 1; k < M; ++k) {
    run = std::max(run, front[k] + remain[k]);
    lb = std::max(lb, run + back[k]);
  }
  return lb;
}

// LB1 of a node whose scheduled prefix is perm[0..len) (len = limit1+1).
template <typename Id>
inline int cpu_lb1(const PfspInstance& in, const Id* perm, int len) {
  int front[64], remain[64];
  cpu_front(in, perm, len, front);
  cpu_remain(in, perm, len, remain);
  return cpu_machine_bound(front, in.min_tails.data(), remain, in.machines);
}

// LB1_d: bounds of every child of a parent with prefix perm[0..len).
// lb_by_job[job] receives the bound of the child that appends `job`.
template <typename Id>
inline void cpu_lb1_children(const PfspInstance& in, const Id* perm, int len, int* lb_by_job) {
  const int N = in.jobs, M = in.machines;
  int front[64], remain[64];
  cpu_front(in, perm, len, front);
  cpu_remain(in, perm, len, remain);
  const int* back = in.min_tails.data();
  for (int i = len; i < N; ++i) {
    const int j = perm[i];
    // s is the child's start on machine k, and the parent's remain still holds
    // p[k][j], so s + remain[k] == front'(k) + remain'(k) of the child
    // (ref add_front_and_bound, c_bound_simple.c:219-244).
    int lb = front[0] + remain[0] + back[0];
    int t = front[0] + in.p[j];
    for (int k = 1; k < M; ++k) {
      const int s = std::max(t, front[k]);
      lb = std::max(lb, s + remain[k] + back[k]);
      t = s + in.p[static_cast<size_t>(k) * N + j];
    }
    lb_by_job[j] = lb;
  }
}

// LB2 of a node with prefix perm[0..len); stops once the partial max exceeds `best`
// (the returned value is then only guaranteed to be > best).
template <typename Id>
inline int cpu_lb2(const PfspInstance& in, const Id* perm, int len, int best) {
  const int N = in.jobs, M = in.machines;
  int front[64];
  cpu_front(in, perm, len, front);
  const int* back = in.min_tails.data();
  // scheduled flags
  uint8_t sched[512];
  for (int j = 0; j < N; ++j) sched[j] = 0;
  for (int i = 0; i < len; ++i) sched[perm[i]] = 1;
  (void)M;
  int lb = 0;
  for (int q = 0; q < in.npairs; ++q) {
    const int m0 = in.pair_m0[q], m1 = in.pair_m1[q];
    int t0 = front[m0], t1 = front[m1];
    const int* order = &in.johnson[static_cast<size_t>(q) * N];
    const int* lag = &in.lags[static_cast<size_t>(q) * N];
    for (int r = 0; r < N; ++r) {
      const int j = order[r];
      if (sched[j]) continue;
      t0 += in.p[static_cast<size_t>(m0) * N + j];
      t1 = std::max(t1, t0 + lag[j]) + in.p[static_cast<size_t>(m1) * N + j];
    }
    lb = std::max(lb, std::max(t1 + back[m1], t0 + back[m0]));
    if (lb > best) break;
  }
  return lb;
}

// Machine-pair evaluation order for LB2's early exit. LB2 is a max over pairs, so
// any order gives the same value and the same prune decision; the order only sets
// how many pairs a pruned child costs before its partial max exceeds `best`. The
// reference walks pairs lexicographically (ref c_bound_johnson.c:48-91, 211-237);
// a few bottleneck-machine pairs usually decide. Pairs are ranked by how often
// they attain a child's LB2 over a sample of the first tree levels (every child of
// up to `sample` nodes of the first level holding that many). On ta056 this cuts
// the pairs a pruned child evaluates from ~16 to ~4 (depths 2-3).
inline std::vector<int> lb2_pair_order(const PfspInstance& in, int sample = 48) {
  const int N = in.jobs, P = in.npairs;
  std::vector<int> order(P);
  for (int q = 0; q < P; ++q) order[q] = q;
  if (P <= 1 || N < 3) return order;
  std::vector<std::vector<int>> level(1, std::vector<int>(N));
  for (int j = 0; j < N; ++j) level[0][j] = j;
  int depth = 0;
  while (static_cast<int>(level.size()) < sample && depth < N - 2) {
    std::vector<std::vector<int>> next;
    for (const auto& perm : level)
      for (int k = depth; k < N; ++k) {
        std::vector<int> c = perm;
        std::swap(c[depth], c[k]);
        next.push_back(std::move(c));
      }
    level.swap(next);
    ++depth;
  }
  const size_t stride = std::max<size_t>(1, level.size() / static_cast<size_t>(sample));
  std::vector<long> score(P, 0);
  std::vector<int> val(P);
  int front[64];
  std::vector<uint8_t> sched(N);
  for (size_t s = 0; s < level.size(); s += stride) {
    std::vector<int> perm = level[s];
    for (int k = depth; k < N; ++k) {
      std::swap(perm[depth], perm[k]);
      cpu_front(in, perm.data(), depth + 1, front);
      std::fill(sched.begin(), sched.end(), 0);
      for (int i = 0; i <= depth; ++i) sched[perm[i]] = 1;
      int mx = 0;
      for (int q = 0; q < P; ++q) {
        const int m0 = in.pair_m0[q], m1 = in.pair_m1[q];
        int t0 = front[m0], t1 = front[m1];
        const int* ord = &in.johnson[static_cast<size_t>(q) * N];
        const int* lag = &in.lags[static_cast<size_t>(q) * N];
        for (int r = 0; r < N; ++r) {
          const int j = ord[r];
          if (sched[j]) continue;
          t0 += in.p[static_cast<size_t>(m0) * N + j];
          t1 = std::max(t1, t0 + lag[j]) + in.p[static_cast<size_t>(m1) * N + j];
        }
        val[q] = std::max(t1 + in.min_tails[m1], t0 + in.min_tails[m0]);
        mx = std::max(mx, val[q]);
      }
      for (int q = 0; q < P; ++q) score[q] += (val[q] == mx);
      std::swap(perm[depth], perm[k]);
    }
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return score[a] > score[b]; });
  return order;
}

// Makespan of a complete permutation (used by tests as the ground truth).
template <typename Id>
inline int cpu_makespan(const PfspInstance& in, const Id* perm) {
  int front[64];
  const int N = in.jobs, M = in.machines;
  for (int k = 0; k < M; ++k) front[k] = 0;
  for (int i = 0; i < N; ++i) {
    const int j = perm[i];
    front[0] += in.p[j];
    for (int k = 1; k < M; ++k) front[k] = std::max(front[k - 1], front[k]) + in.p[static_cast<size_t>(k) * N + j];
  }
  return front[M - 1];
}


// Beam dive for an initial incumbent of a search started without one (-u 0): from the
// root, keep the `beam` partial schedules of smallest LB1 at every depth (their children
// bounded incrementally, LB1_d) down to complete schedules, and return the best makespan
// reached (a leaf's bound is its makespan). The reference's -u 0 search starts from
// INT_MAX and its depth-first order reaches leaves at once (ref pfsp_c.c:55-63); a
// breadth-first device window reaches none for tens of millions of nodes, so the
// device drivers start from this dive's value instead. O(N * beam * N * M).
inline int pfsp_dive_makespan(const PfspInstance& in, int beam) {
  const int N = in.jobs;
  if (N <= 0) return 0;
  beam = std::max(1, beam);
  struct Cand {
    int lb;
    std::vector<int16_t> prmu;
  };
  std::vector<Cand> cur(1);
  cur[0].lb = 0;
  cur[0].prmu.resize(N);
  for (int j = 0; j < N; ++j) cur[0].prmu[j] = static_cast<int16_t>(j);
  std::vector<int> lbj(N);
  for (int d = 0; d < N; ++d) {
    std::vector<Cand> nxt;
    nxt.reserve(static_cast<size_t>(cur.size()) * (N - d));
    for (const Cand& c : cur) {
      cpu_lb1_children(in, c.prmu.data(), d, lbj.data());
      for (int k = d; k < N; ++k) {
        Cand x{lbj[c.prmu[k]], c.prmu};
        std::swap(x.prmu[d], x.prmu[k]);
        nxt.push_back(std::move(x));
      }
    }
    const size_t keep = std::min<size_t>(static_cast<size_t>(beam), nxt.size());
    std::partial_sort(nxt.begin(), nxt.begin() + static_cast<std::ptrdiff_t>(keep), nxt.end(),
                      [](const Cand& a, const Cand& b) { return a.lb < b.lb; });
    nxt.resize(keep);
    cur = std::move(nxt);
  }
  int best = cur[0].lb;
  for (const Cand& c : cur) best = std::min(best, c.lb);
  return best;
}


// ---- Constructive incumbent for -u 0: NEH + iterated greedy (host, deterministic) ----
// NEH (Nawaz, Enscore, Ham 1983): jobs by decreasing total processing time, each
// inserted where the partial sequence's makespan is smallest, every position priced at
// once from the sequence's heads / tails (Taillard 1990, O(L * M) per insertion); then
// iterated greedy (Ruiz, Stuetzle 2007): remove d jobs, re-insert them greedily, improve
// by insertion local search, keep the result when it is not worse, until `budget` cell
// updates are spent. Returns the best makespan (a complete schedule's: >= the optimum).
class PfspNeh {
 public:
  explicit PfspNeh(const PfspInstance& in) : in_(in), N_(in.jobs), M_(in.machines) {}

  int makespan(const std::vector<int>& seq) const {
    std::vector<int> c(static_cast<size_t>(M_), 0);
    for (int j : seq)
      for (int k = 0; k < M_; ++k) c[k] = std::max(c[k], k ? c[k - 1] : 0) + p(k, j);
    return M_ ? c[M_ - 1] : 0;
  }

  // best position of job `job` in `seq` and the makespan there
  std::pair<int, int> best_insert(const std::vector<int>& seq, int job) {
    const int L = static_cast<int>(seq.size());
    e_.assign(static_cast<size_t>(L + 1) * M_, 0);
    q_.assign(static_cast<size_t>(L + 2) * M_, 0);
    for (int i = 0; i < L; ++i)
      for (int k = 0; k < M_; ++k)
        E(i + 1, k) = std::max(E(i, k), k ? E(i + 1, k - 1) : 0) + p(k, seq[i]);
    for (int i = L - 1; i >= 0; --i)
      for (int k = M_ - 1; k >= 0; --k)
        Q(i, k) = std::max(Q(i + 1, k), k + 1 < M_ ? Q(i, k + 1) : 0) + p(k, seq[i]);
    int best = INT32_MAX, pos = 0;
    for (int i = 0; i <= L; ++i) {
      int f = 0, cmax = 0;
      for (int k = 0; k < M_; ++k) {
        f = std::max(f, E(i, k)) + p(k, job);
        cmax = std::max(cmax, f + Q(i, k));
      }
      if (cmax < best) {
        best = cmax;
        pos = i;
      }
    }
    cells_ += static_cast<long long>(3 * (L + 1)) * M_;
    return {pos, best};
  }

  std::vector<int> neh() {
    std::vector<int> order(static_cast<size_t>(N_));
    for (int j = 0; j < N_; ++j) order[j] = j;
    std::vector<long> tot(static_cast<size_t>(N_), 0);
    for (int j = 0; j < N_; ++j)
      for (int k = 0; k < M_; ++k) tot[j] += p(k, j);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return tot[a] > tot[b]; });
    std::vector<int> seq;
    for (int j : order) {
      const auto bi = best_insert(seq, j);
      seq.insert(seq.begin() + bi.first, j);
    }
    return seq;
  }

  // insertion local search: every job in turn removed and re-inserted at its best place
  int local_search(std::vector<int>& seq, int cur) {
    for (bool improved = true; improved;) {
      improved = false;
      for (int t = 0; t < N_; ++t) {
        const int j = seq[static_cast<size_t>(t)];
        std::vector<int> rest = seq;
        rest.erase(rest.begin() + t);
        const auto bi = best_insert(rest, j);
        if (bi.second < cur) {
          rest.insert(rest.begin() + bi.first, j);
          seq.swap(rest);
          cur = bi.second;
          improved = true;
        }
      }
    }
    return cur;
  }

  int solve(long long budget, unsigned seed = 12345u) {
    if (N_ == 0) return 0;
    std::vector<int> seq = neh();
    int cur = local_search(seq, makespan(seq));
    std::vector<int> best_seq = seq;
    int best = cur;
    const int d = std::min(4, std::max(1, N_ / 2));
    unsigned long long x = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&](int n) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      return static_cast<int>(x % static_cast<unsigned long long>(n));
    };
    while (cells_ < budget && N_ > 1) {
      std::vector<int> s2 = seq, removed;
      for (int r = 0; r < d; ++r) {
        const int at = rnd(static_cast<int>(s2.size()));
        removed.push_back(s2[static_cast<size_t>(at)]);
        s2.erase(s2.begin() + at);
      }
      int c2 = 0;
      for (int j : removed) {
        const auto bi = best_insert(s2, j);
        s2.insert(s2.begin() + bi.first, j);
        c2 = bi.second;
      }
      c2 = local_search(s2, c2);
      if (c2 <= cur) {  // accept equal moves: walks plateaus
        seq.swap(s2);
        cur = c2;
        if (cur < best) {
          best = cur;
          best_seq = seq;
        }
      }
    }
    return best;
  }

 private:
  int p(int k, int j) const { return in_.p[static_cast<size_t>(k) * N_ + j]; }
  int& E(int i, int k) { return e_[static_cast<size_t>(i) * M_ + k]; }
  int& Q(int i, int k) { return q_[static_cast<size_t>(i) * M_ + k]; }
  const PfspInstance& in_;
  int N_, M_;
  std::vector<int> e_, q_;
  long long cells_ = 0;
};

}  // namespace tts
