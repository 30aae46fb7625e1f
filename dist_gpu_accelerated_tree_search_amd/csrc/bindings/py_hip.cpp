// _tts_hip: gfx950 device engines and kernels. Instances are passed as plain
// (jobs, machines, machine-major p) data so this module shares no C++ types with
// _tts_cpu (the two are built by different compilers).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <climits>
#include <string>

#include "../core/cpu_engine.hpp"
#include "../core/pfsp_front.hpp"
#include "../core/problems.hpp"
#include "../hip/host_support.hpp"
#include "../hip/pfsp_engine.hpp"
#include "../hip/queens_engine.hpp"
#include "../hip/rccl_transport.hpp"
#include "engine_binding.hpp"

namespace py = pybind11;
using namespace tts;

namespace {

using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

EngineConfig make_cfg(int device, size_t max_parents, size_t ring_bytes, int iters_small, int iters_large,
                      bool use_graphs, uintptr_t stream, int iters_first, int dyn_us = 0, int dive_window = 0,
                      int dive_shift = 2) {
  EngineConfig c;
  c.dyn_us = dyn_us;
  c.dive_window = dive_window;
  c.dive_shift = dive_shift;
  c.device = device;
  c.max_parents = max_parents;
  c.ring_bytes = ring_bytes;
  c.iters_small = iters_small;
  c.iters_large = iters_large;
  c.use_graphs = use_graphs;
  c.external_stream = stream;
  c.iters_first = iters_first;
  return c;
}

}  // namespace

PYBIND11_MODULE(_tts_hip, m) {
  m.doc() = "gfx950 (MI355X) device engines: device-resident pools, fused bound/prune/compact kernels, hipGraphs.";
  bind_engine(m);
  bind_shm_control(m);
  py::class_<RcclTransport>(m, "RcclTransport")
      .def(py::init([](py::bytes id, int rank, int world, int device) {
             const std::string s = id;
             const std::vector<uint8_t> v(s.begin(), s.end());
             py::gil_scoped_release nogil;  // ncclCommInitRank waits for every rank
             return std::make_unique<RcclTransport>(v, rank, world, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_static("new_id", []() {
        const std::vector<uint8_t> v = RcclTransport::new_id();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def(
          "execute",
          [](RcclTransport& t, py::list plan, IEngine& e) {
            Plan pl;
            for (auto x : plan) {
              auto tt = x.cast<py::tuple>();
              pl.push_back({tt[0].cast<int>(), tt[1].cast<int>(), tt[2].cast<size_t>()});
            }
            py::gil_scoped_release nogil;
            return t.execute(pl, e);
          },
          py::arg("plan"), py::arg("engine"),
          "This rank's part of a transfer plan: export -> grouped ncclSend/ncclRecv on the engine's transfer "
          "stream -> import; (sent, received).")
      .def(
          "self_loop",
          [](RcclTransport& t, IEngine& e, size_t n) {
            py::gil_scoped_release nogil;
            return t.self_loop(e, n);
          },
          py::arg("engine"), py::arg("n"))
      .def(
          "preflight",
          [](RcclTransport& t, size_t nbytes, bool corrupt) {
            std::pair<int, double> r;
            {
              py::gil_scoped_release nogil;
              r = t.preflight(nbytes, corrupt);
            }
            py::dict d;
            d["ok"] = true;
            d["peers"] = r.first;
            d["bytes_per_peer"] = nbytes / 4 * 4;
            d["seconds"] = r.second;
            d["GBps"] = r.second > 0 ? r.first * static_cast<double>(nbytes) / r.second / 1e9 : 0.0;
            d["native"] = true;
            return d;
          },
          py::arg("nbytes") = size_t(4) << 20, py::arg("corrupt") = false)
      .def_property_readonly("rank", &RcclTransport::rank)
      .def_property_readonly("world", &RcclTransport::world)
      .def_property_readonly("device", &RcclTransport::device)
      .def_property_readonly("transfers", &RcclTransport::transfers)
      .def_property_readonly("bytes_sent", &RcclTransport::bytes_sent)
      .def_property_readonly("bytes_recv", &RcclTransport::bytes_recv)
      .def_property_readonly("collectives", &RcclTransport::collectives)
      .def_property("timeout_s", &RcclTransport::timeout_s, &RcclTransport::set_timeout_s)
      .def(
          "allgather_i64",
          [](RcclTransport& t, std::vector<int64_t> v, IEngine& e) {
            py::array_t<int64_t> out({static_cast<py::ssize_t>(t.world()), static_cast<py::ssize_t>(v.size())});
            {
              py::gil_scoped_release nogil;
              t.allgather_i64(v.data(), static_cast<int>(v.size()), out.mutable_data(), e);
            }
            return out;
          },
          py::arg("values"), py::arg("engine"),
          "Status all-gather over the communicator on the engine's transfer stream -> (world, n) int64.");
  const NativeTransfer native_rccl = [](py::object obj, IEngine* e) -> TransferFn {
    if (!py::isinstance<RcclTransport>(obj)) return {};
    RcclTransport* t = obj.cast<RcclTransport*>();
    // the Python object stays referenced by the caller (DistSolver / dist_rounds call)
    return [t, e](const Plan& p) { return t->execute(p, *e); };
  };
  bind_dist_rounds(m, [](py::object model) -> WarmupFn {
    if (py::hasattr(model, "native")) {
      auto inst = std::make_shared<PfspInstance>(make_instance(model.attr("jobs").cast<int>(),
                                                               model.attr("machines").cast<int>(),
                                                               model.attr("native").attr("p").cast<std::vector<int>>()));
      const int lb = model.attr("host_lb").cast<int>();
      return with_pfsp_problem(*inst, lb, [&](auto prob) -> WarmupFn { return make_warmup(inst, prob); });
    }
    return make_warmup(nullptr, QueensProblem(model.attr("N").cast<int>(), model.attr("G").cast<int>()));
  }, native_rccl, [](py::object obj, IEngine* e) -> std::unique_ptr<RoundControl> {
    // the RCCL transport as the round loop's control plane (ncclAllGather, no Python)
    if (!py::isinstance<RcclTransport>(obj) || !e) return nullptr;
    return std::make_unique<RcclRoundControl>(obj.cast<RcclTransport*>(), e);
  });
  bind_runner(
      m, []() -> std::unique_ptr<DeviceStaging> { return std::make_unique<HipStaging>(); }, &device_cpus);
  if (!std::getenv("TTS_NO_ROCTX")) install_roctx_hooks();
  // release every engine / RCCL communicator while the HIP runtime is alive (atexit
  // handlers run before interpreter teardown; csrc/hip/device_resource.hpp)
  m.def("release_all", &DeviceResource::release_all,
        "Free the device resources of every live engine and RCCL transport (also run at exit).");
  m.def("live_resources", &DeviceResource::live_count);
  py::module_::import("atexit").attr("register")(py::cpp_function([]() {
    if (const char* e = std::getenv("TTS_EXIT_MODE"))  // profiler exit-crash diagnosis (scripts/profile_workload.py)
      if (std::string(e) == "keep") return;
    DeviceResource::release_all();
  }));
  m.def("device_pci_bus_id", &device_pci_bus_id);
  m.def("device_cpus", &device_cpus, "CPUs of the NUMA node closest to the GPU (empty if unknown).");

  // CPU workers that can be mixed with GPU engines in run_workers (-C 1)
  m.def(
      "make_pfsp_cpu_engine",
      [](int jobs, int machines, std::vector<int> p, int lb, size_t batch, int threads) -> std::unique_ptr<IEngine> {
        auto inst = std::make_shared<PfspInstance>(make_instance(jobs, machines, std::move(p)));
        // LB1 is evaluated with the incremental LB1_d on the CPU (same values); the node
        // layout is the GPU engines' (front nodes where they apply)
        return with_pfsp_problem(*inst, lb == 1 ? 0 : lb, [&](auto prob) -> std::unique_ptr<IEngine> {
          return std::make_unique<OwningCpuEngine<decltype(prob)>>(inst, prob, batch, threads);
        });
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("batch") = 4096,
      py::arg("threads") = 1);
  m.def(
      "make_queens_cpu_engine",
      [](int N, int G, size_t batch, int threads) -> std::unique_ptr<IEngine> {
        return std::make_unique<CpuEngine<QueensProblem>>(QueensProblem(N, G), batch, threads);
      },
      py::arg("N"), py::arg("G") = 1, py::arg("batch") = 4096, py::arg("threads") = 1);

  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("device_info", [](int device) {
    hipDeviceProp_t p;
    TTS_HIP_CHECK(hipGetDeviceProperties(&p, device));
    py::dict d;
    d["name"] = std::string(p.name);
    d["arch"] = std::string(p.gcnArchName);
    d["compute_units"] = p.multiProcessorCount;
    d["clock_khz"] = p.clockRate;
    d["total_mem"] = static_cast<size_t>(p.totalGlobalMem);
    d["lds_per_block"] = static_cast<size_t>(p.sharedMemPerBlock);
    d["warp_size"] = p.warpSize;
    return d;
  });

  m.def(
      "make_pfsp_engine",
      [](int jobs, int machines, std::vector<int> p, int lb, int device, size_t max_parents, size_t ring_bytes,
         int iters_small, int iters_large, bool use_graphs, uintptr_t stream, int taillard_id, int iters_first,
         int dyn_us, int dive_window, int dive_shift) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p), taillard_id);
        py::gil_scoped_release nogil;
        return make_pfsp_engine(in, lb,
                                make_cfg(device, max_parents, ring_bytes, iters_small, iters_large, use_graphs, stream,
                                         iters_first, dyn_us, dive_window, dive_shift));
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("device") = 0,
      py::arg("max_parents") = size_t(1) << 18, py::arg("ring_bytes") = size_t(16) << 30, py::arg("iters_small") = 6,
      py::arg("iters_large") = 48, py::arg("use_graphs") = true, py::arg("stream") = 0, py::arg("taillard_id") = 0,
      py::arg("iters_first") = 18, py::arg("dyn_us") = 0, py::arg("dive_window") = 0, py::arg("dive_shift") = 2);

  m.def(
      "make_queens_engine",
      [](int N, int G, int device, size_t max_parents, size_t ring_bytes, int iters_small, int iters_large,
         bool use_graphs, uintptr_t stream, int iters_first) {
        py::gil_scoped_release nogil;
        return make_queens_engine(
            N, G, make_cfg(device, max_parents, ring_bytes, iters_small, iters_large, use_graphs, stream, iters_first));
      },
      py::arg("N"), py::arg("G") = 1, py::arg("device") = 0, py::arg("max_parents") = size_t(1) << 20,
      py::arg("ring_bytes") = size_t(16) << 30, py::arg("iters_small") = 6, py::arg("iters_large") = 48,
      py::arg("use_graphs") = true, py::arg("stream") = 0, py::arg("iters_first") = 24);

  m.def(
      "pfsp_bounds",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 parents, int best, int device) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        std::vector<int> out;
        {
          py::gil_scoped_release nogil;
          out = pfsp_gpu_bounds(in, lb, parents.data(), static_cast<size_t>(parents.shape(0)), best, device);
        }
        py::array_t<int> r(static_cast<py::ssize_t>(out.size()));
        std::memcpy(r.mutable_data(), out.data(), out.size() * sizeof(int));
        return r;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("parents"), py::arg("best") = INT_MAX,
      py::arg("device") = 0);

  m.def(
      "pfsp_expand_probe",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 parents, int best, int device, int variant) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        std::vector<int> out;
        {
          py::gil_scoped_release nogil;
          out = pfsp_expand_probe(in, lb, parents.data(), static_cast<size_t>(parents.shape(0)), best, device, variant);
        }
        py::array_t<int> r(static_cast<py::ssize_t>(out.size()));
        std::memcpy(r.mutable_data(), out.data(), out.size() * sizeof(int));
        return r;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("parents"), py::arg("best") = INT_MAX,
      py::arg("device") = 0, py::arg("variant") = 0,
      "One production expand iteration over these parents with the debug output on: every child's bound "
      "(exact LB2 below best, else >= best). variant 1 rounds, 2 dense, 4 rounds of packed two-child walks.");
  m.def(
      "pfsp_expand_probe_out",
      [](int jobs, int machines, std::vector<int> p, U8 parents, int best, int device, int variant) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        ExpandProbeResult r;
        {
          py::gil_scoped_release nogil;
          r.bounds = pfsp_expand_probe(in, 2, parents.data(), static_cast<size_t>(parents.shape(0)), best, device, variant,
                                       0, nullptr, &r);
        }
        py::array_t<int> b(static_cast<py::ssize_t>(r.bounds.size()));
        std::memcpy(b.mutable_data(), r.bounds.data(), r.bounds.size() * sizeof(int));
        py::array_t<uint8_t> c({static_cast<py::ssize_t>(r.children.size() / nb), static_cast<py::ssize_t>(nb)});
        if (!r.children.empty()) std::memcpy(c.mutable_data(), r.children.data(), r.children.size());
        py::dict d;
        d["bounds"] = b;
        d["children"] = c;
        d["leaves"] = r.leaves;
        d["best"] = r.best;
        return d;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("parents"), py::arg("best") = INT_MAX,
      py::arg("device") = 0, py::arg("variant") = 4,
      "pfsp_expand_probe (LB2) plus what the iteration wrote: children (lb < best), leaves, incumbent.");
  m.def(
      "pfsp_lb1_expand_probe",
      [](int jobs, int machines, std::vector<int> p, U8 parents, int best, int device) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        ExpandProbeResult r;
        {
          py::gil_scoped_release nogil;
          r = pfsp_lb1_expand_probe(in, parents.data(), static_cast<size_t>(parents.shape(0)), best, device);
        }
        py::array_t<int> b(static_cast<py::ssize_t>(r.bounds.size()));
        std::memcpy(b.mutable_data(), r.bounds.data(), r.bounds.size() * sizeof(int));
        py::array_t<uint8_t> c({static_cast<py::ssize_t>(r.children.size() / nb), static_cast<py::ssize_t>(nb)});
        if (!r.children.empty()) std::memcpy(c.mutable_data(), r.children.data(), r.children.size());
        py::dict d;
        d["bounds"] = b;
        d["children"] = c;
        d["leaves"] = r.leaves;
        d["best"] = r.best;
        return d;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("parents"), py::arg("best") = INT_MAX,
      py::arg("device") = 0,
      "One iteration of the permutation-node LB1 / LB1_d expand kernel over these parents: every child's bound, "
      "the children it wrote (lb < best), the leaves it counted and the incumbent after it.");
  m.def(
      "pfsp_expand_time",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 parents, int best, int device, int variant, int reps) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        std::vector<double> t;
        {
          py::gil_scoped_release nogil;
          (void)pfsp_expand_probe(in, lb, parents.data(), static_cast<size_t>(parents.shape(0)), best, device, variant,
                                  reps, &t);
        }
        py::dict d;
        d["ms_min"] = t[0];
        d["ms_median"] = t[1];
        d["clk_a"] = t[2];
        d["clk_b1"] = t[3];
        d["clk_b2"] = t[4];
        d["clk_c"] = t[5];
        d["chunks"] = t[6];
        d["clk_block_max"] = t[7];
        d["clk_block_mean"] = t[8];
        d["grid"] = t[9];
        const size_t nblk = (t.size() - 10) / 3;
        py::array_t<double> tl({static_cast<py::ssize_t>(nblk), static_cast<py::ssize_t>(3)});
        std::memcpy(tl.mutable_data(), t.data() + 10, nblk * 3 * sizeof(double));
        d["timeline_us"] = tl;
        return d;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("parents"), py::arg("best"),
      py::arg("device") = 0, py::arg("variant") = 1, py::arg("reps") = 10,
      "Time one expand iteration over this window (LB2): min/median ms over reps launches on the engine's grid, "
      "and per-chunk shader clocks of phases A, B1, B2, B3+C from one instrumented launch.");

  m.def(
      "pfsp_front_probe",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 nodes, int best, int device, size_t max_parents,
         int fuse_max, int deep_levels, int deep_per3, int deep_per4, int local_steps, unsigned cap, int split_rank,
         int split_world, size_t split_min, int wide_levels, int local_min, int dyn_us) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        EngineConfig c;
        c.dyn_us = dyn_us;
        c.local_min = local_min;
        c.device = device;
        c.max_parents = max_parents;
        c.ring_bytes = size_t(1) << 30;
        c.fuse_max = fuse_max;
        c.deep_levels = deep_levels;
        c.deep_per3 = deep_per3;
        c.deep_per4 = deep_per4;
        c.local_steps = local_steps;
        c.wide_levels = wide_levels;
        FrontProbeResult r;
        {
          py::gil_scoped_release nogil;
          r = pfsp_front_probe(in, lb, nodes.data(), static_cast<size_t>(nodes.shape(0)), best, c, cap, split_rank,
                               split_world, split_min);
        }
        py::dict d;
        d["records"] = r.records;
        d["checked"] = r.checked;
        py::dict k;
        const char* names[6] = {"one_level", "child_parallel", "thread_per_node", "local_dfs", "split", "dynamic"};
        for (int i = 0; i < 6; ++i) k[names[i]] = r.by_kind[i];
        d["by_kind"] = k;
        d["bad_lb"] = r.bad_lb;
        d["bad_remain"] = r.bad_remain;
        d["bad_job"] = r.bad_job;
        d["first_bad"] = r.first_bad;
        d["tree"] = r.st.tree;
        d["sol"] = r.st.sol;
        d["best"] = r.st.best;
        d["iters"] = r.st.iters;
        return d;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("nodes"), py::arg("best"),
      py::arg("device") = 0, py::arg("max_parents") = size_t(1) << 16, py::arg("fuse_max") = 1 << 30,
      py::arg("deep_levels") = 2, py::arg("deep_per3") = 8, py::arg("deep_per4") = 2, py::arg("local_steps") = 4,
      py::arg("cap") = 1u << 22, py::arg("split_rank") = 0, py::arg("split_world") = 1, py::arg("split_min") = 0,
      py::arg("wide_levels") = 1, py::arg("local_min") = -1, py::arg("dyn_us") = 0,
      "A complete front-kernel engine solve from these (front-layout) nodes with probe records on: every child "
      "bound of every iteration shape checked against the host oracle (counts of records and mismatches).");
  m.def(
      "pfsp_front_time",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 nodes, int best, int device, size_t max_parents,
         int fuse_max, int deep_levels, int deep_per3, int deep_per4, int reps, int wide_levels, int local_min,
         int local_steps, int dyn_us) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        EngineConfig c;
        c.dyn_us = dyn_us;
        c.device = device;
        c.local_min = local_min;
        c.local_steps = local_steps;
        c.max_parents = max_parents;
        c.fuse_max = fuse_max;
        c.deep_levels = deep_levels;
        c.deep_per3 = deep_per3;
        c.deep_per4 = deep_per4;
        c.wide_levels = wide_levels;
        std::vector<double> t;
        {
          py::gil_scoped_release nogil;
          t = pfsp_front_time(in, lb, nodes.data(), static_cast<size_t>(nodes.shape(0)), best, c, reps);
        }
        py::dict d;
        d["ms_min"] = t[0];
        d["ms_median"] = t[1];
        d["grid"] = static_cast<int>(t[2]);
        d["nch_out"] = static_cast<int>(t[3]);
        const size_t nblk = (t.size() - 4) / 16;
        py::array_t<double> tl({static_cast<py::ssize_t>(nblk), static_cast<py::ssize_t>(16)});
        std::memcpy(tl.mutable_data(), t.data() + 4, nblk * 16 * sizeof(double));
        d["stamps_us"] = tl;
        return d;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("nodes"), py::arg("best"),
      py::arg("device") = 0, py::arg("max_parents") = size_t(1) << 19, py::arg("fuse_max") = 1 << 30,
      py::arg("deep_levels") = 2, py::arg("deep_per3") = 8, py::arg("deep_per4") = 2, py::arg("reps") = 20,
      py::arg("wide_levels") = 1, py::arg("local_min") = 0, py::arg("local_steps") = 4, py::arg("dyn_us") = 0,
      "Time one front-kernel iteration over this window: min / median ms, and the per-workgroup phase stamps.");
  m.def(
      "queens_labels",
      [](int N, int G, U8 parents, int device) {
        if (parents.ndim() != 2 || parents.shape(1) != static_cast<py::ssize_t>(sizeof(QueensNode)))
          throw std::invalid_argument("parents must be a (n, 16) uint8 array");
        const size_t n = static_cast<size_t>(parents.shape(0));
        std::vector<uint8_t> out;
        {
          py::gil_scoped_release nogil;
          out = queens_gpu_labels(N, G, reinterpret_cast<const QueensNode*>(parents.data()), n, device);
        }
        U8 r({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(N)});
        std::memcpy(r.mutable_data(), out.data(), out.size());
        return r;
      },
      py::arg("N"), py::arg("G"), py::arg("parents"), py::arg("device") = 0);
}
