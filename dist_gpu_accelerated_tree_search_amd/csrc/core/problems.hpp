// The two tree-search problems behind one host-side "problem" interface:
//   using Node = ...;  Node root() const;
//   template <class Push> void decompose(const Node&, int& best, u64& tree, u64& sol, Push&&) const;
// Counting rules are the reference's:
//   PFSP   tree = pushed children (non-leaf with lb < best); sol = every leaf child
//          evaluated (pruned or not); a leaf with lb < best improves best.
//          ref pfsp/lib/PFSP_lib.c:7-129
//   Queens tree = pushed safe children (leaves included); sol = popped node at depth N.
//          ref nqueens/nqueens_c.c:80-117
#pragma once

#include <cstdint>
#include <stdexcept>

#include "pfsp_bounds_cpu.hpp"
#include "pfsp_node.hpp"

namespace tts {

using u64 = unsigned long long;

template <int NJ>
struct PfspProblem {
  using Node = PfspNode<NJ>;
  const PfspInstance* inst = nullptr;
  int lb = 1;  // 0 = LB1_d, 1 = LB1, 2 = LB2

  PfspProblem(const PfspInstance& in, int lb_kind) : inst(&in), lb(lb_kind) {
    if (in.jobs > NJ) throw std::invalid_argument("instance has more jobs than the node bucket");
    if (lb_kind < 0 || lb_kind > 2) throw std::invalid_argument("lower bound must be 0, 1 or 2");
  }

  Node root() const {
    Node r;
    pfsp_init_root(r, inst->jobs);
    return r;
  }

  template <class Push>
  void decompose(const Node& parent, int& best, u64& tree, u64& sol, Push&& push) const {
    const PfspInstance& in = *inst;
    const int N = in.jobs;
    const int d = parent.depth;
    const bool leaf = (d + 1 == N);
    if (lb == 0) {
      int lbj[512];
      cpu_lb1_children(in, parent.prmu, d, lbj);
      for (int k = d; k < N; ++k) {
        const int b = lbj[parent.prmu[k]];
        if (leaf) {
          ++sol;
          if (b < best) best = b;
        } else if (b < best) {
          push(pfsp_child(parent, k));
          ++tree;
        }
      }
      return;
    }
    for (int k = d; k < N; ++k) {
      const Node c = pfsp_child(parent, k);
      const int b = (lb == 1) ? cpu_lb1(in, c.prmu, d + 1) : cpu_lb2(in, c.prmu, d + 1, best);
      if (leaf) {
        ++sol;
        if (b < best) best = b;
      } else if (b < best) {
        push(c);
        ++tree;
      }
    }
  }
};

struct QueensProblem {
  using Node = QueensNode;
  int N = 14;
  int G = 1;

  QueensProblem(int n, int g) : N(n), G(g) {
    if (n < 1 || n > 32) throw std::invalid_argument("N-Queens supports 1 <= N <= 32");
    if (g < 1) throw std::invalid_argument("g must be >= 1");
  }

  uint32_t full() const { return N == 32 ? 0xffffffffu : ((1u << N) - 1u); }

  Node root() const { return Node{0u, 0u, 0u, 0u}; }

  template <class Push>
  void decompose(const Node& parent, int& /*best*/, u64& tree, u64& sol, Push&& push) const {
    if (static_cast<int>(parent.depth) == N) {
      ++sol;
      return;
    }
    uint32_t safe = ~(parent.cols | parent.diag | parent.anti) & full();
    // -g > 1: the reference's artificial work (ref nqueens_c.c:80-96): each candidate
    // row is tested G times against the `depth` placed queens — G * depth dependent
    // compares per candidate, kept by the barrier (see queens_free_rows on the GPU).
    if (G > 1) {
      const uint32_t att = parent.diag | parent.anti;
      uint32_t cand = ~parent.cols & full();
      while (cand) {
        const uint32_t bit = cand & (0u - cand);
        cand ^= bit;
        uint32_t hit = 0;
        for (int g = 0; g < G; ++g)
          for (uint32_t i = 0; i < parent.depth; ++i) {
            hit |= att & bit;
            asm volatile("" : "+r"(hit));
          }
        safe &= ~hit;
      }
    }
    while (safe) {
      const uint32_t bit = safe & (0u - safe);
      safe ^= bit;
      push(Node{parent.cols | bit, (parent.diag | bit) << 1, (parent.anti | bit) >> 1, parent.depth + 1});
      ++tree;
    }
  }
};

}  // namespace tts
