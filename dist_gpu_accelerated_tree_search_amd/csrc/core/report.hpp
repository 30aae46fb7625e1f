// Command line, stdout blocks and CSV statistics, byte-compatible with the reference.
//
// Parity:
//   parse_parameters   ref pfsp/lib/PFSP_lib.c:173-320 (flags, defaults, messages)
//   print_settings     ref PFSP_lib.c:133-158          print_results ref :160-170
//   CSV writers        ref pfsp/lib/PFSP_statistic.c:7-167 (quoted "[a,b]", arrays,
//                      trailing comma before the newline on multi/dist rows)
//   N-Queens CLI       ref nqueens/nqueens_multigpu_cuda.c:25-89, 106-124
#pragma once

#include <getopt.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "search_cpu.hpp"

namespace tts {

struct PfspArgs {
  int inst = 14, lb = 1, ub = 1, m = 25, M = 50000, T = 5000, D = 1, C = 1, ws = 1, L = 1;
  double perc = 0.5;
};

inline PfspArgs parse_pfsp_args(int argc, char* argv[]) {
  PfspArgs a;
  static struct option long_options[] = {{"inst", required_argument, nullptr, 'i'}, {"lb", required_argument, nullptr, 'l'},
                                         {"ub", required_argument, nullptr, 'u'},   {"m", required_argument, nullptr, 'm'},
                                         {"M", required_argument, nullptr, 'M'},    {"T", required_argument, nullptr, 'T'},
                                         {"D", required_argument, nullptr, 'D'},    {"C", required_argument, nullptr, 'C'},
                                         {"ws", required_argument, nullptr, 'w'},   {"L", required_argument, nullptr, 'L'},
                                         {"perc", required_argument, nullptr, 'p'}, {nullptr, 0, nullptr, 0}};
  int opt, idx = 0;
  auto fail = [](const char* msg) {
    std::fprintf(stderr, "%s\n", msg);
    std::exit(EXIT_FAILURE);
  };
  optind = 1;
  while ((opt = getopt_long(argc, argv, "i:l:u:m:M:T:D:C:w:L:p:", long_options, &idx)) != -1) {
    const int v = optarg ? std::atoi(optarg) : 0;
    switch (opt) {
      case 'i': if (v < 1 || v > 120) fail("Error: unsupported Taillard's instance"); a.inst = v; break;
      case 'l': if (v < 0 || v > 2) fail("Error: unsupported lower bound function"); a.lb = v; break;
      case 'u': if (v != 0 && v != 1) fail("Error: unsupported upper bound initialization"); a.ub = v; break;
      case 'm': if (v < 1) fail("Error: unsupported minimal pool for GPU initialization"); a.m = v; break;
      case 'M': if (v < a.m) fail("Error: unsupported maximal pool for GPU initialization"); a.M = v; break;
      case 'T': if (v < a.m) fail("Error: unsupported maximal pool for CPU multi-core"); a.T = v; break;
      case 'D': if (v < 0) fail("Error: unsupported number of GPU(s)"); a.D = v; break;
      case 'C': if (v < 0) fail("Error: unsupported number of CPU Core(s)"); a.C = v; break;
      case 'w': if (v < 0 || v > 1) fail("Error: unsupported Intra-node Work Stealing option"); a.ws = v; break;
      case 'L': if (v < 0 || v > 1) fail("Error: unsupported distributed dynamic load balancing option"); a.L = v; break;
      case 'p': if (v <= 0 || v > 100) fail("Error: unsupported WS percentage for popFrontBulkFree"); a.perc = v / 100.0; break;
      default:
        std::fprintf(stderr,
                     "Usage: %s --inst <value> --lb <value> --ub <value> --m <value> --M <value> --T <value> --D <value> "
                     "--C <value> --w <value> --L <value> --perc <value>\n",
                     argv[0]);
        std::exit(EXIT_FAILURE);
    }
  }
  return a;
}

// version: 0 sequential, 1 single GPU, 2 multi-GPU / multi-core, 3 distributed.
inline void print_pfsp_settings(int inst, int machines, int jobs, int ub, int lb, int D, int C, int ws, int comm_size,
                                int LB, int version) {
  std::printf("\n=================================================\n");
  if (version == 0)
    std::printf("Sequential C++\n\n");
  else if (version == 1)
    std::printf("Single-GPU C++/HIP (MI355X)\n\n");
  else if (version == 2)
    std::printf("Multi-core Multi-GPU C++/HIP (%d GPU(s) - [%d] Multi-core - [%d] Work Stealing)\n\n", D, C, ws);
  else
    std::printf("Distributed Multi-GPU C++/HIP+RCCL (%d processes x ( %d GPU(s) - [%d] Multi-core ) - [%d] LB)\n\n",
                comm_size, D, C, LB);
  std::printf("Resolution of PFSP Taillard's instance: ta%d (m = %d, n = %d)\n", inst, machines, jobs);
  std::printf(ub == 0 ? "Initial upper bound: inf\n" : "Initial upper bound: opt\n");
  std::printf("Lower bound function: %s\n", lower_bound_name(lb));
  std::printf("Branching rule: fwd\n");
  std::printf("=================================================\n");
}

inline void print_pfsp_results(int optimum, u64 tree, u64 sol, double timer) {
  std::printf("\n=================================================\n");
  std::printf("Size of the explored tree: %llu\n", tree);
  std::printf("Number of explored solutions: %llu\n", sol);
  std::printf("Optimal makespan: %d\n", optimum);
  std::printf("Elapsed time: %.4f [s]\n", timer);
  std::printf("=================================================\n");
}

inline void print_phase(const char* title, u64 tree, u64 sol, double t) {
  std::printf("\n%s\n", title);
  std::printf("Size of the explored tree: %llu\n", tree);
  std::printf("Number of explored solutions: %llu\n", sol);
  std::printf("Elapsed time: %f [s]\n", t);
}

// ---- N-Queens ----
struct QueensArgs {
  int N = 14, g = 1, m = 25, M = 50000, D = 1;
};

inline QueensArgs parse_queens_args(int argc, char* argv[], bool gpu_flags) {
  QueensArgs a;
  int opt;
  optind = 1;
  const char* spec = gpu_flags ? "N:g:m:M:D:" : "N:g:";
  while ((opt = getopt(argc, argv, spec)) != -1) {
    const int v = std::atoi(optarg);
    switch (opt) {
      case 'N': if (v < 1) { std::fprintf(stderr, "Error: N must be a positive integer.\n"); std::exit(EXIT_FAILURE); } a.N = v; break;
      case 'g': if (v < 1) { std::fprintf(stderr, "Error: g must be a positive integer.\n"); std::exit(EXIT_FAILURE); } a.g = v; break;
      case 'm': if (v < 1) { std::fprintf(stderr, "Error: m must be a positive integer.\n"); std::exit(EXIT_FAILURE); } a.m = v; break;
      case 'M': if (v < a.m) { std::fprintf(stderr, "Error: M must be a positive integer, greater or equal to m.\n"); std::exit(EXIT_FAILURE); } a.M = v; break;
      case 'D': if (v < 1) { std::fprintf(stderr, "Error: D must be a positive integer.\n"); std::exit(EXIT_FAILURE); } a.D = v; break;
      default:
        std::fprintf(stderr, gpu_flags ? "Usage: %s -N value -g value -m value -M value -D value\n" : "Usage: %s -N value -g value\n", argv[0]);
        std::exit(EXIT_FAILURE);
    }
  }
  return a;
}

inline void print_queens_settings(int N, int G, const char* backend) {
  std::printf("\n=================================================\n");
  std::printf("%s\n\n", backend);
  std::printf("Resolution of the %d-Queens instance\n", N);
  std::printf("  with %d safety check(s) per evaluation\n", G);
  std::printf("=================================================\n");
}

inline void print_queens_results(u64 tree, u64 sol, double timer) {
  std::printf("\n=================================================\n");
  std::printf("Size of the explored tree: %llu\n", tree);
  std::printf("Number of explored solutions: %llu\n", sol);
  std::printf("Elapsed time: %.4f [s]\n", timer);
  std::printf("=================================================\n");
}

// ---- CSV (append-only; header written when the file is empty) ----
namespace csv_detail {
inline FILE* open_with_header(const char* path, const char* header) {
  FILE* f = std::fopen(path, "a");
  if (!f) return nullptr;
  std::fseek(f, 0, SEEK_END);
  if (std::ftell(f) == 0) std::fputs(header, f);
  return f;
}
inline void ull_array(FILE* f, const std::vector<u64>& v) {
  std::fputs("\"[", f);
  for (size_t i = 0; i < v.size(); ++i) std::fprintf(f, i + 1 < v.size() ? "%llu," : "%llu", v[i]);
  std::fputs("]\",", f);
}
inline void dbl_array(FILE* f, const std::vector<double>& v) {
  std::fputs("\"[", f);
  for (size_t i = 0; i < v.size(); ++i) std::fprintf(f, i + 1 < v.size() ? "%.4f," : "%.4f", v[i]);
  std::fputs("]\",", f);
}
template <class F>
std::vector<u64> col_u(const std::vector<WorkerStats>& w, F f) {
  std::vector<u64> r;
  for (auto& s : w) r.push_back(f(s));
  return r;
}
template <class F>
std::vector<double> col_d(const std::vector<WorkerStats>& w, F f) {
  std::vector<double> r;
  for (auto& s : w) r.push_back(f(s));
  return r;
}
inline void worker_arrays(FILE* f, const std::vector<WorkerStats>& w) {
  ull_array(f, col_u(w, [](const WorkerStats& s) { return s.tree; }));
  ull_array(f, col_u(w, [](const WorkerStats& s) { return s.sol; }));
  ull_array(f, col_u(w, [](const WorkerStats& s) { return s.gen_child; }));
  ull_array(f, col_u(w, [](const WorkerStats& s) { return s.steals; }));
  ull_array(f, col_u(w, [](const WorkerStats& s) { return s.success_steals; }));
  ull_array(f, col_u(w, [](const WorkerStats& s) { return s.terminations; }));
}
inline void worker_times(FILE* f, const std::vector<WorkerStats>& w) {
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_memcpy; }));
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_malloc; }));
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_kernel; }));
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_gen_child; }));
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_pool_ops; }));
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_idle; }));
  dbl_array(f, col_d(w, [](const WorkerStats& s) { return s.t_termination; }));
}
}  // namespace csv_detail

inline void write_csv_single_gpu(const char* path, int inst, int lb, int optimum, int m, int M, u64 tree, u64 sol,
                                 double timer, double t_memcpy, double t_malloc, double t_kernel, double t_gen_child) {
  FILE* f = csv_detail::open_with_header(path,
      "instance_id,lower_bound,optimum,m,M,total_time,gpu_memcpy_time,gpu_malloc_time,gpu_kernel_time,gen_child_time,"
      "explored_tree,explored_sol\n");
  if (!f) return;
  std::fprintf(f, "%d,%d,%d,%d,%d,%.4f,%.4f,%.4f,%.4f,%.4f,%llu,%llu\n", inst, lb, optimum, m, M, timer, t_memcpy, t_malloc,
               t_kernel, t_gen_child, tree, sol);
  std::fclose(f);
}

inline void write_csv_multi_gpu(const char* path, int inst, int lb, int D, int C, int ws, int optimum, int m, int M, int T,
                                u64 tree, u64 sol, double timer, const std::vector<WorkerStats>& w) {
  FILE* f = csv_detail::open_with_header(path,
      "instance_id,D,C,lower_bound,work_stealing,optimum,m,M,T,total_time,total_tree,total_sol,"
      "exp_tree_gpu,exp_sol_gpu,gen_child_gpu,steals_gpu,success_steals_gpu,termination_gpu,"
      "gpu_memcpy_time,gpu_malloc_time,gpu_kernel_time,gpu_gen_child_time,pool_ops_time,gpu_idle_time,termination_time\n");
  if (!f) return;
  std::fprintf(f, "%d,%d,%d,%d,%d,%d,%d,%d,%d,%.4f,%llu,%llu,", inst, D, C, lb, ws, optimum, m, M, T, timer, tree, sol);
  csv_detail::worker_arrays(f, w);
  csv_detail::worker_times(f, w);
  std::fputs("\n", f);
  std::fclose(f);
}

}  // namespace tts
