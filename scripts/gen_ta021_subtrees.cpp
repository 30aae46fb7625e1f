// Generates tests/fixtures/ta021_subtrees.json: sampled ta021 (20x20) LB1_d subtrees
// with their -u 1 tree / sol counts from the host engine (PfspFrontProblem, the same
// oracle the CPU drivers use). The GPU test solves each subtree on the device and
// compares (tests/test_gpu_front_probe.py). The whole ta021 tree (260,069,628,524
// nodes) has no count in the reference to compare with; these samples pin the GPU
// against the host on disjoint parts of it.
//   g++ -O2 -std=c++17 -I dist_gpu_accelerated_tree_search_amd/csrc scripts/gen_ta021_subtrees.cpp -o /tmp/gen
#include <cstdio>
#include <random>
#include <vector>

#include "core/pfsp_front.hpp"
#include "core/taillard.hpp"

using namespace tts;
using Node = PfspFrontNode<20>;

int main() {
  const PfspInstance in = make_taillard_instance(21);
  const PfspFrontProblem<20> pr(in, 0);
  const int best = in.best_known;
  std::vector<std::vector<Node>> level(7);
  level[0] = {pr.root()};
  unsigned long long t0 = 0, s0 = 0;
  for (int d = 0; d < 6; ++d) {
    int b = best;
    for (const Node& n : level[d]) pr.decompose(n, b, t0, s0, [&](const Node& c) { level[d + 1].push_back(c); });
  }
  std::mt19937_64 rng(20261017);
  std::printf("{\"instance\": 21, \"lb\": 0, \"best\": %d, \"node_bytes\": %zu, \"samples\": [\n", best, sizeof(Node));
  int emitted = 0;
  for (int depth : {4, 6}) {
    int got = 0;
    while (got < 32) {
      const Node n = level[depth][rng() % level[depth].size()];
      std::vector<Node> st{n};
      unsigned long long t = 0, s = 0;
      int b = best;
      while (!st.empty() && t <= 20000000ull) {
        const Node x = st.back();
        st.pop_back();
        pr.decompose(x, b, t, s, [&](const Node& c) { st.push_back(c); });
      }
      // keep subtrees large enough to take several GPU iterations, small enough for the host
      if (t > 20000000ull || t < (depth == 4 ? 10000ull : 500ull)) continue;
      const unsigned char* p = reinterpret_cast<const unsigned char*>(&n);
      std::printf("%s  {\"depth\": %d, \"tree\": %llu, \"sol\": %llu, \"node\": \"", emitted ? ",\n" : "", depth, t, s);
      for (size_t i = 0; i < sizeof(Node); ++i) std::printf("%02x", p[i]);
      std::printf("\"}");
      ++got;
      ++emitted;
    }
  }
  std::printf("\n]}\n");
}
