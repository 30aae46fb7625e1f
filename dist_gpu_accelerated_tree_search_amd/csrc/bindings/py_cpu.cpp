// _tts_cpu: host-side native core (no HIP dependency; builds and runs anywhere).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <climits>

#include "../core/cpu_engine.hpp"
#include "../core/drivers_cpu.hpp"
#include "../core/estimate.hpp"
#include "../core/pfsp_front.hpp"
#include "../core/shm_control.hpp"
#include "engine_binding.hpp"

namespace py = pybind11;
using namespace tts;

namespace {

using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

template <class Node>
U8 nodes_to_array(const Node* p, size_t n) {
  U8 out({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(sizeof(Node))});
  if (n) std::memcpy(out.mutable_data(), p, n * sizeof(Node));
  return out;
}

template <class Node>
const Node* array_nodes(const U8& a, size_t& n) {
  if (a.ndim() != 2 || static_cast<size_t>(a.shape(1)) != sizeof(Node))
    throw std::invalid_argument("nodes must be a (n, node_bytes) uint8 array");
  n = static_cast<size_t>(a.shape(0));
  return reinterpret_cast<const Node*>(a.data());
}

py::dict worker_dict(const WorkerStats& w) {
  py::dict d;
  d["tree"] = w.tree;
  d["sol"] = w.sol;
  d["gen_child"] = w.gen_child;
  d["steals"] = w.steals;
  d["success_steals"] = w.success_steals;
  d["terminations"] = w.terminations;
  d["t_memcpy"] = w.t_memcpy;
  d["t_malloc"] = w.t_malloc;
  d["t_kernel"] = w.t_kernel;
  d["t_gen_child"] = w.t_gen_child;
  d["t_pool_ops"] = w.t_pool_ops;
  d["t_idle"] = w.t_idle;
  d["t_termination"] = w.t_termination;
  return d;
}

py::dict result_dict(const RunResult& r) {
  py::dict d;
  d["best"] = r.best;
  d["tree"] = r.tree;
  d["sol"] = r.sol;
  d["t_init"] = r.t_init;
  d["t_search"] = r.t_search;
  d["t_tail"] = r.t_tail;
  d["elapsed"] = r.elapsed;
  py::list ws;
  for (auto& w : r.workers) ws.append(worker_dict(w));
  d["workers"] = ws;
  return d;
}

MulticoreConfig mc_config(size_t m, size_t batch, size_t steal_cap, bool ws) {
  MulticoreConfig c;
  c.m = m;
  c.batch = batch;
  c.steal_cap = steal_cap;
  c.work_stealing = ws;
  return c;
}

}  // namespace

PYBIND11_MODULE(_tts_cpu, m) {
  m.doc() = "Native host core of the MI355X tree-search engine (Taillard, bounds, pools, CPU drivers).";
  bind_engine(m);
  bind_runner(m);

  // ---- Taillard ----
  m.def("taillard_jobs", &taillard_jobs);
  m.def("taillard_machines", &taillard_machines);
  m.def("taillard_best_ub", &taillard_best_ub);
  m.def("taillard_processing_times", &taillard_processing_times, "machine-major p[m*N+j]");
  m.def("synthetic_processing_times", &synthetic_processing_times, py::arg("jobs"), py::arg("machines"),
        py::arg("seed"));

  py::class_<PfspInstance>(m, "PfspInstance")
      .def_static("taillard", &make_taillard_instance, py::arg("id"))
      .def_static(
          "from_matrix",
          [](int jobs, int machines, std::vector<int> p, int best_known) {
            return make_instance(jobs, machines, std::move(p), 0, best_known);
          },
          py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("best_known") = INT_MAX)
      .def_readonly("id", &PfspInstance::id)
      .def_readonly("jobs", &PfspInstance::jobs)
      .def_readonly("machines", &PfspInstance::machines)
      .def_readonly("best_known", &PfspInstance::best_known)
      .def_readonly("p", &PfspInstance::p)
      .def_readonly("min_heads", &PfspInstance::min_heads)
      .def_readonly("min_tails", &PfspInstance::min_tails)
      .def_readonly("npairs", &PfspInstance::npairs)
      .def_readonly("pair_m0", &PfspInstance::pair_m0)
      .def_readonly("pair_m1", &PfspInstance::pair_m1)
      .def_readonly("lags", &PfspInstance::lags)
      .def_readonly("johnson", &PfspInstance::johnson);

  // ---- bounds (oracle for the GPU kernels) ----
  m.def("lb1", [](const PfspInstance& in, std::vector<int> prmu, int len) { return cpu_lb1(in, prmu.data(), len); });
  m.def("lb1_children", [](const PfspInstance& in, std::vector<int> prmu, int len) {
    std::vector<int> out(in.jobs, 0);
    cpu_lb1_children(in, prmu.data(), len, out.data());
    return out;
  });
  m.def("lb2", [](const PfspInstance& in, std::vector<int> prmu, int len, int best) {
    return cpu_lb2(in, prmu.data(), len, best);
  });
  m.def("makespan", [](const PfspInstance& in, std::vector<int> perm) { return cpu_makespan(in, perm.data()); });

  m.def("pfsp_node_bytes", [](int jobs) {
    return with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
  });
  m.def("pfsp_bucket", &pfsp_bucket);
  // node layout of the engines for (instance, lb): front nodes where they apply
  // (core/pfsp_front.hpp), else the permutation node of the job-count bucket
  m.def("pfsp_engine_node_bytes", [](const PfspInstance& in, int lb) {
    return with_pfsp_problem(in, lb, [](auto prob) { return sizeof(typename decltype(prob)::Node); });
  });
  m.def("pfsp_front_layout", [](const PfspInstance& in, int lb) { return pfsp_front_ok(in, lb); });
  m.def(
      "pfsp_root",
      [](const PfspInstance& in, int lb) {
        return with_pfsp_problem(in, lb, [](auto prob) {
          const auto r = prob.root();
          return nodes_to_array(&r, 1);
        });
      },
      py::arg("inst"), py::arg("lb"), "Root node in the engines' layout, shape (1, node_bytes).");
  m.def(
      "pfsp_to_engine_layout",
      [](const PfspInstance& in, int lb, U8 nodes) {
        // permutation-layout nodes (utils/nodes.pfsp_pack) -> the engines' layout
        return with_pfsp_bucket(in.jobs, [&](auto nj) -> U8 {
          constexpr int NJ = decltype(nj)::value;
          size_t n = 0;
          const PfspNode<NJ>* p = array_nodes<PfspNode<NJ>>(nodes, n);
          if (!pfsp_front_ok(in, lb)) return nodes_to_array(p, n);
          return with_pfsp_problem(in, lb, [&](auto prob) -> U8 {
            using P = decltype(prob);
            if constexpr (is_front_problem<P>::value) {
              if constexpr (NJ == P::kJobs) {
                std::vector<typename P::Node> out(n);
                for (size_t i = 0; i < n; ++i) out[i] = pfsp_front_from_perm(prob, p[i]);
                return nodes_to_array(out.data(), n);
              } else {
                return nodes_to_array(p, n);
              }
            } else {
              return nodes_to_array(p, n);
            }
          });
        });
      },
      py::arg("inst"), py::arg("lb"), py::arg("nodes"));
  m.def(
      "pfsp_children_bounds",
      [](const PfspInstance& in, int lb, U8 nodes) {
        // bounds of every child of engine-layout nodes, by ascending job id per node
        // (front layout) or child position (permutation layout): the host twin of the
        // front kernel, for tests
        std::vector<int> out;
        with_pfsp_problem(in, lb, [&](auto prob) {
          using P = decltype(prob);
          using Node = typename P::Node;
          size_t n = 0;
          const Node* p = array_nodes<Node>(nodes, n);
          for (size_t i = 0; i < n; ++i) {
            if constexpr (is_front_problem<P>::value) {
              int by_job[64];
              prob.children_bounds(p[i], by_job);
              for (auto x = p[i].rest; x; x &= x - 1) out.push_back(by_job[mask_ctz(x)]);
            } else {
              throw std::invalid_argument("pfsp_children_bounds: front layout only");
            }
          }
          return 0;
        });
        return out;
      },
      py::arg("inst"), py::arg("lb"), py::arg("nodes"));
  m.def("queens_node_bytes", []() { return sizeof(QueensNode); });

  // ---- end-to-end CPU drivers ----
  m.def(
      "run_pfsp",
      [](const PfspInstance& in, int lb, int best, int threads, size_t m_, size_t batch, size_t steal_cap, bool ws,
         bool verbose) {
        py::gil_scoped_release nogil;
        RunResult r = run_pfsp_cpu(in, lb, best, threads, mc_config(m_, batch, steal_cap, ws), verbose);
        py::gil_scoped_acquire gil;
        return result_dict(r);
      },
      py::arg("inst"), py::arg("lb"), py::arg("best"), py::arg("threads") = 0, py::arg("m") = 25,
      py::arg("batch") = 20000, py::arg("steal_cap") = 250000, py::arg("ws") = true, py::arg("verbose") = false);
  m.def(
      "run_queens",
      [](int N, int G, int threads, size_t m_, size_t batch, size_t steal_cap, bool ws, bool verbose) {
        py::gil_scoped_release nogil;
        RunResult r = run_queens_cpu(N, G, threads, mc_config(m_, batch, steal_cap, ws), verbose);
        py::gil_scoped_acquire gil;
        return result_dict(r);
      },
      py::arg("N"), py::arg("G") = 1, py::arg("threads") = 0, py::arg("m") = 25, py::arg("batch") = 20000,
      py::arg("steal_cap") = 250000, py::arg("ws") = true, py::arg("verbose") = false);

  m.def(
      "pfsp_dive",
      [](const PfspInstance& in, int beam) {
        py::gil_scoped_release nogil;
        return pfsp_dive_makespan(in, beam);
      },
      py::arg("inst"), py::arg("beam") = 32,
      "Makespan of the best complete schedule a beam dive of LB1 reaches (initial incumbent for -u 0).");
  m.def(
      "pfsp_neh",
      [](const PfspInstance& in, long long budget, unsigned seed) {
        py::gil_scoped_release nogil;
        PfspNeh h(in);
        return h.solve(budget, seed);
      },
      py::arg("inst"), py::arg("budget") = 5000000LL, py::arg("seed") = 12345u,
      "NEH + iterated greedy makespan (a complete schedule's) within `budget` cell updates.");
  // ---- Step 1 (BFS warm-up) and Step 3 (DFS drain) for the GPU/distributed drivers ----
  m.def(
      "pfsp_bfs",
      [](const PfspInstance& in, int lb, int best, size_t target) {
        return with_pfsp_problem(in, lb, [&](auto prob) {
          Pool<typename decltype(prob)::Node> pool;
          pool.push_back_free(prob.root());
          u64 tree = 0, sol = 0;
          bfs_warmup(prob, pool, target, best, tree, sol);
          return py::make_tuple(nodes_to_array(pool.data(), pool.size()), tree, sol, best);
        });
      },
      py::arg("inst"), py::arg("lb"), py::arg("best"), py::arg("target"));
  m.def(
      "pfsp_bfs_level",
      [](const PfspInstance& in, int lb, int best, int depth) {
        // every node of tree level `depth` (engine layout), level by level from the root
        // with a fixed incumbent (analysis and kernel timing windows)
        return with_pfsp_problem(in, lb, [&](auto prob) {
          using Node = typename decltype(prob)::Node;
          std::vector<Node> cur{prob.root()}, nxt;
          u64 tree = 0, sol = 0;
          int b = best;
          for (int d = 0; d < depth && !cur.empty(); ++d) {
            nxt.clear();
            for (const Node& x : cur) prob.decompose(x, b, tree, sol, [&](const Node& c) { nxt.push_back(c); });
            std::swap(cur, nxt);
          }
          return nodes_to_array(cur.data(), cur.size());
        });
      },
      py::arg("inst"), py::arg("lb"), py::arg("best"), py::arg("depth"));
  m.def(
      "lb2_child_profile",
      [](const PfspInstance& in, U8 nodes, int best) {
        // analysis helper: for every child of every node (LB2 work model of the expand
        // kernel): LB1, the number of pairs in the learned order until the partial LB2
        // exceeds best (P if never), and the full LB2
        const std::vector<int> ord = lb2_pair_order(in);
        std::vector<int> out;
        with_pfsp_bucket(in.jobs, [&](auto nj) {
          constexpr int NJ = decltype(nj)::value;
          using Node = PfspNode<NJ>;
          size_t n = 0;
          const Node* p = array_nodes<Node>(nodes, n);
          const int N = in.jobs;
          for (size_t i = 0; i < n; ++i) {
            const int d = p[i].depth;
            for (int k = d; k < N; ++k) {
              Node c = pfsp_child(p[i], k);
              int front[64];
              cpu_front(in, c.prmu, d + 1, front);
              uint8_t sched[512] = {0};
              for (int x = 0; x <= d; ++x) sched[c.prmu[x]] = 1;
              int lb = 0, until = in.npairs;
              for (int qi = 0; qi < in.npairs; ++qi) {
                const int q = ord[qi];
                const int m0 = in.pair_m0[q], m1 = in.pair_m1[q];
                int t0 = front[m0], t1 = front[m1];
                for (int r = 0; r < N; ++r) {
                  const int j = in.johnson[static_cast<size_t>(q) * N + r];
                  if (sched[j]) continue;
                  t0 += in.pt(m0, j);
                  t1 = std::max(t1, t0 + in.lags[static_cast<size_t>(q) * N + j]) + in.pt(m1, j);
                }
                lb = std::max(lb, std::max(t1 + in.min_tails[m1], t0 + in.min_tails[m0]));
                if (lb >= best && until == in.npairs) until = qi + 1;
              }
              out.push_back(cpu_lb1(in, c.prmu, d + 1));
              out.push_back(until);
              out.push_back(lb);
            }
          }
          return 0;
        });
        py::array_t<int> r({static_cast<py::ssize_t>(out.size() / 3), static_cast<py::ssize_t>(3)});
        std::memcpy(r.mutable_data(), out.data(), out.size() * sizeof(int));
        return r;
      },
      py::arg("inst"), py::arg("nodes"), py::arg("best"));
  m.def(
      "tree_estimate",
      [](py::object problem, int best, unsigned long long probes, unsigned long long seed, int threads) {
        auto pack = [](const TreeEstimate& e) {
          py::dict d;
          d["tree"] = e.tree;
          d["stderr"] = e.stderr_;
          d["depth"] = e.depth;
          d["probes"] = e.probes;
          d["per_level"] = e.per_level;
          return d;
        };
        TreeEstimate e;
        if (py::hasattr(problem, "native") && py::isinstance<PfspInstance>(problem.attr("native"))) {
          const PfspInstance& in = problem.attr("native").cast<const PfspInstance&>();
          const int lb = problem.attr("host_lb").cast<int>();
          py::gil_scoped_release nogil;
          e = with_pfsp_problem(in, lb, [&](auto prob) { return knuth_estimate(prob, best, probes, seed, threads); });
        } else {
          QueensProblem q(problem.attr("N").cast<int>(), problem.attr("G").cast<int>());
          py::gil_scoped_release nogil;
          e = knuth_estimate(q, best, probes, seed, threads);
        }
        return pack(e);
      },
      py::arg("model"), py::arg("best"), py::arg("probes") = 1000, py::arg("seed") = 1, py::arg("threads") = 1,
      "Knuth random-probe estimate of the explored tree for a fixed incumbent (core/estimate.hpp).");
  m.def(
      "pfsp_drain",
      [](const PfspInstance& in, int lb, int best, U8 nodes) {
        return with_pfsp_problem(in, lb, [&](auto prob) {
          using Node = typename decltype(prob)::Node;
          size_t n = 0;
          const Node* p = array_nodes<Node>(nodes, n);
          Pool<Node> pool;
          pool.push_back_bulk_free(p, n);
          u64 tree = 0, sol = 0;
          {
            py::gil_scoped_release nogil;
            dfs_drain(prob, pool, best, tree, sol);
          }
          return py::make_tuple(tree, sol, best);
        });
      },
      py::arg("inst"), py::arg("lb"), py::arg("best"), py::arg("nodes"));
  m.def(
      "queens_bfs",
      [](int N, int G, size_t target) {
        QueensProblem prob(N, G);
        Pool<QueensNode> pool;
        pool.push_back_free(prob.root());
        u64 tree = 0, sol = 0;
        int best = 0;
        bfs_warmup(prob, pool, target, best, tree, sol);
        return py::make_tuple(nodes_to_array(pool.data(), pool.size()), tree, sol);
      },
      py::arg("N"), py::arg("G"), py::arg("target"));
  m.def(
      "queens_drain",
      [](int N, int G, U8 nodes) {
        QueensProblem prob(N, G);
        size_t n = 0;
        const QueensNode* p = array_nodes<QueensNode>(nodes, n);
        Pool<QueensNode> pool;
        pool.push_back_bulk_free(p, n);
        u64 tree = 0, sol = 0;
        int best = 0;
        {
          py::gil_scoped_release nogil;
          dfs_drain(prob, pool, best, tree, sol);
        }
        return py::make_tuple(tree, sol);
      },
      py::arg("N"), py::arg("G"), py::arg("nodes"));

  // ---- CPU engines (same contract as the GPU engines) ----
  m.def(
      "make_pfsp_cpu_engine",
      [](const PfspInstance& in, int lb, size_t batch, int threads) -> std::unique_ptr<IEngine> {
        return with_pfsp_problem(in, lb, [&](auto prob) -> std::unique_ptr<IEngine> {
          return std::make_unique<CpuEngine<decltype(prob)>>(prob, batch, threads);
        });
      },
      py::arg("inst"), py::arg("lb"), py::arg("batch") = 4096, py::arg("threads") = 1, py::keep_alive<0, 1>());
  m.def(
      "make_queens_cpu_engine",
      [](int N, int G, size_t batch, int threads) -> std::unique_ptr<IEngine> {
        return std::make_unique<CpuEngine<QueensProblem>>(QueensProblem(N, G), batch, threads);
      },
      py::arg("N"), py::arg("G") = 1, py::arg("batch") = 4096, py::arg("threads") = 1);

  bind_shm_control(m);
  bind_dist_rounds(m, [](py::object model) -> WarmupFn {
    if (py::hasattr(model, "native")) {
      auto inst = std::make_shared<PfspInstance>(model.attr("native").cast<const PfspInstance&>());
      const int lb = model.attr("host_lb").cast<int>();
      return with_pfsp_problem(*inst, lb, [&](auto prob) -> WarmupFn { return make_warmup(inst, prob); });
    }
    return make_warmup(nullptr, QueensProblem(model.attr("N").cast<int>(), model.attr("G").cast<int>()));
  });
}
