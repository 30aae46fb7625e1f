// PFSP device engine: instance tables on the GPU + engine traits + factories.
//
// Parity: ref lb1_alloc_gpu / lb2_alloc_gpu (PFSP_gpu_lib.cu:154-200) deep-copy the
// bound tables once per GPU thread (and leak them). Here the tables
// are built once in the layout the kernels stage into LDS:
//   ptab  job-major u16 rows padded to 16 B        (LB1 / LB1_d / LB2 fronts)
//   recs  per machine pair, the Johnson order as {job, p0, p1, lag} u16 records,
//         so one wave-uniform 8-B read drives one Johnson step for 64 children.
// and are owned (freed) by the engine.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <type_traits>
#include <vector>

#include "../core/pfsp_bounds_cpu.hpp"
#include "../core/pfsp_front.hpp"
#include "../core/pfsp_instance.hpp"
#include "engine.hpp"
#include "pfsp_front_kernels.hpp"
#include "pfsp_kernels.hpp"

namespace tts {

template <int NJ, int M, int LBK>
struct PfspTraits {
  using Node = PfspNode<NJ>;
  using Args = dev::PfspArgs<NJ, M>;
  using G = dev::PfspGeom<NJ, LBK, M>;
  static constexpr int kParentsPerChunk = G::BP;
  static constexpr int kChildrenPerChunk = G::SLOT;  // slot region per chunk
  static constexpr int kMaxChildren = NJ;            // children per parent (one level)
  static constexpr int kLocalSteps = G::LT;
  static constexpr int kLocalMin = 0;
  static constexpr int kMaxChunks = G::MAXCHUNKS;
  static void launch(const Args& a, int t, int grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::pfsp_expand_kernel<NJ, M, LBK>), dim3(grid), dim3(dev::kBlock), 0, s, a, t);
  }
  static void flatten(const dev::PoolArgs<Node>& pa, int b, int grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::pool_flatten_kernel<Node, G::SLOT, G::MAXCHUNKS>), dim3(grid), dim3(dev::kBlock), 0, s,
                       pa, b);
  }
  static void finalize(const dev::PoolArgs<Node>& pa, int b, int slot, hipStream_t s) {
    hipLaunchKernelGGL((dev::pool_finalize_kernel<Node, G::MAXCHUNKS>), dim3(1), dim3(dev::kBlock), 0, s, pa, b, slot);
  }
  static int blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::pfsp_expand_kernel<NJ, M, LBK>, dev::kBlock, 0) !=
        hipSuccess)
      return 1;
    // 106 SGPRs: 6 resident per CU. The packed LB2 walks of 50+-job instances run on 3 of
    // their 4 (LDS-bound) resident workgroups: fewer walks contend for the record lines
    // (ta056 0.1748 -> 0.1773 G nodes/s, 2 per CU 0.1765; profiles/r5/grid_ab.txt)
    return dev::resident_blocks(n, (LBK == 5 && NJ >= 50) ? 3 : dev::kSgprResidentCap);
  }
};

// LB1 / LB1_d on front-carrying nodes (pfsp_front_kernels.hpp), machine bucket M.
template <int M, int NJ = 20>
struct PfspFrontTraits {
  using Node = PfspFrontNode<M, NJ>;
  using Args = dev::PfspFrontArgs<M, NJ>;
  using G = dev::FrontGeom<M, NJ>;
  static constexpr int kParentsPerChunk = G::BP;
  static constexpr int kChildrenPerChunk = G::SLOT;
  static constexpr int kMaxChildren = G::NJ;
  static constexpr int kLocalSteps = G::LT;
  // local DFS from 16K-parent windows: the wide levels of a 20-job tree take up to
  // local_steps levels per dependent kernel (ta014 -u 1, one MI355X: 0.234 -> 0.221 ms;
  // rank shares of 2/4/8-way splits 9-12 % faster; ta021 unchanged — its pool is a
  // backlog anyway; 4K-parent windows were slower again: profiles/r4/local_min.txt)
  static constexpr int kLocalMin = 16384;
  static constexpr int kMaxChunks = G::MAXCHUNKS;
  static constexpr bool kDyn = true;  // dynamic local DFS iterations (front_dyn)
  static void launch(const Args& a, int t, int grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::pfsp_front_kernel<M, NJ>), dim3(grid), dim3(dev::kBlock), 0, s, a, t);
  }
  static void flatten(const dev::PoolArgs<Node>& pa, int b, int grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::pool_flatten_kernel<Node, G::SLOT, G::MAXCHUNKS>), dim3(grid), dim3(dev::kBlock), 0, s,
                       pa, b);
  }
  static void finalize(const dev::PoolArgs<Node>& pa, int b, int slot, hipStream_t s) {
    hipLaunchKernelGGL((dev::pool_finalize_kernel<Node, G::MAXCHUNKS>), dim3(1), dim3(dev::kBlock), 0, s, pa, b, slot);
  }
  static int blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::pfsp_front_kernel<M, NJ>, dev::kBlock, 0) != hipSuccess)
      return 1;
    return std::min(n, G::GRID_WGS);  // FrontGeom::GRID_WGS (the API over-reports by one)
  }
};

// Front-layout tables: job-major u16 p rows padded to the LDS stride, padded tails.
template <int M, int NJ>
inline std::vector<uint16_t> pfsp_front_fill_args(const PfspInstance& in, dev::PfspFrontArgs<M, NJ>& a) {
  if (!pfsp_front_ok(in, 1) || pfsp_machine_bucket(in.machines) != M || pfsp_front_jobs(in.jobs) != NJ)
    throw std::invalid_argument("front layout does not apply to this instance");
  constexpr int MS = dev::FrontGeom<M, NJ>::MS;
  const PfspPadded t = pfsp_padded_tables(in, M);
  std::vector<uint16_t> ptab(static_cast<size_t>(in.jobs) * MS, 0);
  for (int j = 0; j < in.jobs; ++j)
    for (int m = 0; m < in.machines; ++m) ptab[static_cast<size_t>(j) * MS + m] = static_cast<uint16_t>(in.pt(m, j));
  a.jobs = in.jobs;
  for (int m = 0; m < M; ++m) a.min_tails[m] = t.tails[m];
  a.bpf = dev::FrontGeom<M, NJ>::BPF;
  a.cp_max = dev::FrontGeom<M, NJ>::CPMAX;
  if (const char* f = std::getenv("TTS_CP_MAX")) a.cp_max = std::max(0, std::atoi(f));  // A/B runs
  if (const char* f = std::getenv("TTS_FUSED_BPF"))  // A/B runs
    a.bpf = std::min(std::max(1, std::atoi(f)), dev::FrontGeom<M, NJ>::BPF_CP);
  return ptab;
}

// Host-side images of the device tables.
struct PfspTableImages {
  std::vector<uint16_t> ptab;  // [N][MS]
  std::vector<uint2> recs;     // [P][N]
  std::vector<uint2> pinfo;    // [P]
  std::vector<uint4> recs4;    // [P][rs4]: recs padded with zero records (lb2_walk_pipe)
  int rs4 = 0;
};

// Software-pipelined record loads in the LB2 walks (lb2_walk_pipe): on unless
// TTS_LB2_PIPE=0 (A/B).
inline int lb2_pipe_wanted() {
  const char* f = std::getenv("TTS_LB2_PIPE");
  return f ? (std::atoi(f) != 0) : 1;
}

// The LB2 kernel with two children per lane in packed u16 walks (LBK 5): every walk
// value must fit 16 bits (any job count: wide job sets read their words from LDS). A walk value (a child
// front, t0 + p0, t0 + lag, t1 + p1) is the length of a monotone staircase path
// through the machine x job grid (prefix columns, then Johnson-order columns; a lag
// is the column segment between the pair's machines), so it visits at most
// jobs + machines - 1 cells: (jobs + machines - 1) * max p bounds it (50 x 20 with
// p <= 99: 6,831). The tails are added in 32 bits after the walk. On when it applies
// unless TTS_LB2_PK=0 (A/B).
inline bool lb2_pk_ok(const PfspInstance& in) {
  long pmax = 0;
  for (int v : in.p) pmax = std::max<long>(pmax, v);
  return (in.jobs + in.machines - 1) * pmax < 65536;
}
inline bool lb2_pk_wanted(const PfspInstance& in) {
  const char* f = std::getenv("TTS_LB2_PK");
  return (f ? std::atoi(f) != 0 : true) && lb2_pk_ok(in);
}

// Strided LB2 chunks (parents ch + i * nchunks): on unless TTS_LB2_STRIDE=0 (A/B).
inline int lb2_stride_wanted() {
  const char* f = std::getenv("TTS_LB2_STRIDE");
  return f ? (std::atoi(f) != 0) : 1;
}

// Machine counts below the kernel's M are padded with trailing machines of zero
// processing time: the makespan, every LB1 machine term and the fronts of the real
// machines are unchanged (a zero machine after the last one completes with it), and
// LB2 walks only the instance's own pairs (npairs), so the bounds equal the host
// oracle's for the real instance.
template <int NJ, int M>
inline PfspTableImages pfsp_fill_args(const PfspInstance& in, dev::PfspArgs<NJ, M>& a, bool pair_order = false) {
  using C = dev::PfspConsts<M>;
  if (in.machines > M || in.machines < 1) throw std::invalid_argument("machine count exceeds kernel instantiation");
  if (in.jobs > NJ) throw std::invalid_argument("job count exceeds kernel bucket");
  const int MR = in.machines;
  const int PR = MR * (MR - 1) / 2;
  PfspTableImages img;
  img.ptab.assign(static_cast<size_t>(in.jobs) * C::MS, 0);
  for (int j = 0; j < in.jobs; ++j)
    for (int m = 0; m < MR; ++m) img.ptab[static_cast<size_t>(j) * C::MS + m] = static_cast<uint16_t>(in.pt(m, j));
  img.recs.resize(static_cast<size_t>(PR) * in.jobs);
  for (int q = 0; q < PR; ++q) {
    const int m0 = in.pair_m0[q], m1 = in.pair_m1[q];
    for (int r = 0; r < in.jobs; ++r) {
      const int job = in.johnson[static_cast<size_t>(q) * in.jobs + r];
      const int lag = in.lags[static_cast<size_t>(q) * in.jobs + job];
      if (lag > 0xffff) throw std::invalid_argument("LB2 lag does not fit 16 bits");
      uint2 rc;
      rc.x = static_cast<uint32_t>(job) | (static_cast<uint32_t>(in.pt(m0, job)) << 16);
      rc.y = static_cast<uint32_t>(in.pt(m1, job)) | (static_cast<uint32_t>(lag) << 16);
      img.recs[static_cast<size_t>(q) * in.jobs + r] = rc;
    }
  }
  {
    const int ndouble = (in.jobs + 7) / 8;
    img.rs4 = 4 * ndouble + 4;  // walks of ndouble x 8 records + one double group of prefetch
    img.recs4.assign(static_cast<size_t>(PR) * img.rs4, make_uint4(0, 0, 0, 0));
    for (int q = 0; q < PR; ++q)
      for (int r = 0; r < in.jobs; ++r) {
        const uint2 rc = img.recs[static_cast<size_t>(q) * in.jobs + r];
        uint4& v = img.recs4[static_cast<size_t>(q) * img.rs4 + r / 2];
        if (r & 1) {
          v.z = rc.x;
          v.w = rc.y;
        } else {
          v.x = rc.x;
          v.y = rc.y;
        }
      }
  }
  // expand kernel's pair table in the learned early-exit order (lb2_pair_order);
  // recs stay in the reference order (the bounds kernel keeps its exact partial
  // values) and pinfo points each slot at its pair's records
  img.pinfo.resize(PR);
  {
    std::vector<int> ord(PR);
    for (int q = 0; q < PR; ++q) ord[q] = q;
    if (pair_order && PR > 0) ord = lb2_pair_order(in);
    for (int i = 0; i < PR; ++i) {
      const int q = ord[i];
      const int m0 = in.pair_m0[q], m1 = in.pair_m1[q];
      if (in.min_tails[m0] > 0xffff || in.min_tails[m1] > 0xffff)
        throw std::invalid_argument("LB2 tail does not fit 16 bits");
      img.pinfo[i].x = static_cast<uint32_t>(m0) | (static_cast<uint32_t>(m1) << 8) | (static_cast<uint32_t>(q) << 16);
      img.pinfo[i].y = static_cast<uint32_t>(in.min_tails[m0]) | (static_cast<uint32_t>(in.min_tails[m1]) << 16);
    }
  }
  a.jobs = in.jobs;
  a.npairs = PR;
  a.rs4 = img.rs4;
  a.lb2_pipe = lb2_pipe_wanted();
  a.lb2_stride = lb2_stride_wanted();
  for (int m = 0; m < M; ++m) {
    if (m < MR) {
      a.min_heads[m] = in.min_heads[m];
      a.min_tails[m] = in.min_tails[m];
    } else {  // padding machine: head = whole real route of the cheapest job, no tail
      int h = INT_MAX;
      for (int j = 0; j < in.jobs; ++j) {
        int t = 0;
        for (int k = 0; k < MR; ++k) t += in.pt(k, j);
        h = std::min(h, t);
      }
      a.min_heads[m] = h;
      a.min_tails[m] = 0;
    }
    long s = 0;
    if (m < MR)
      for (int j = 0; j < in.jobs; ++j) s += in.pt(m, j);
    // front and remain are packed as two u16 per machine in LDS
    if (s > 0xffff) throw std::invalid_argument("instance too large for 16-bit schedule packing");
    a.sum_all[m] = static_cast<int>(s);
  }
  for (int q = 0; q < PR; ++q) {
    a.pm0[q] = static_cast<uint8_t>(in.pair_m0[q]);
    a.pm1[q] = static_cast<uint8_t>(in.pair_m1[q]);
  }
  return img;
}

template <class T>
inline T* upload_vec(const std::vector<T>& v) {
  T* d = nullptr;
  TTS_HIP_CHECK(hipMalloc(&d, std::max<size_t>(1, v.size()) * sizeof(T)));
  if (!v.empty()) TTS_HIP_CHECK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

template <int NJ, int M, int LBK>
std::unique_ptr<IEngine> make_pfsp_engine_t(const PfspInstance& in, const EngineConfig& cfg) {
  TTS_HIP_CHECK(hipSetDevice(cfg.device));
  dev::PfspArgs<NJ, M> a{};
  const PfspTableImages img = pfsp_fill_args(in, a, LBK >= 2);
  a.ptab = upload_vec(img.ptab);
  a.recs = upload_vec(img.recs);
  a.pinfo = upload_vec(img.pinfo);
  a.recs4 = upload_vec(img.recs4);
  // B2 in rounds of pairs: ta056 (50x20) 0.060 -> 0.081 G nodes/s, ta020 (20x10)
  // 11.1 -> 8.0 ms, ta014 (20x10) even; ta010 (20x5, 10 pairs) 4.0 -> 4.6 ms
  // (profiles/r1/r1ak): on from 10 machines (45 pairs)
  a.lb2_rounds = M >= 10 ? 1 : 0;
  if (const char* f = std::getenv("TTS_LB2_ROUNDS")) a.lb2_rounds = std::atoi(f) != 0;  // A/B runs
  auto eng = std::make_unique<DeviceEngine<PfspTraits<NJ, M, LBK>>>(cfg, a);
  eng->adopt(const_cast<uint16_t*>(a.ptab));
  eng->adopt(const_cast<uint2*>(a.recs));
  eng->adopt(const_cast<uint2*>(a.pinfo));
  eng->adopt(const_cast<uint4*>(a.recs4));
  return eng;
}

// Reference-style batch evaluation on the GPU (host arrays in and out):
// bounds of every child of every parent, in parent order, children k = depth..N-1.
template <int NJ, int M, int LBK>
std::vector<int> pfsp_gpu_bounds_t(const PfspInstance& in, const void* parents, size_t n, int best, int device) {
  using Node = PfspNode<NJ>;
  TTS_HIP_CHECK(hipSetDevice(device));
  dev::PfspArgs<NJ, M> a{};
  const PfspTableImages img = pfsp_fill_args(in, a);
  const Node* ph = static_cast<const Node*>(parents);
  std::vector<int> offsets(n + 1, 0);
  for (size_t i = 0; i < n; ++i) offsets[i + 1] = offsets[i] + (in.jobs - ph[i].depth);
  const size_t nb = static_cast<size_t>(offsets[n]);
  std::vector<int> out(nb, 0);
  if (n == 0) return out;
  a.ptab = upload_vec(img.ptab);
  a.recs = upload_vec(img.recs);
  a.offsets = upload_vec(offsets);
  Node* dparents = nullptr;
  int* dbounds = nullptr;
  TTS_HIP_CHECK(hipMalloc(&dparents, n * sizeof(Node)));
  TTS_HIP_CHECK(hipMalloc(&dbounds, std::max<size_t>(1, nb) * sizeof(int)));
  TTS_HIP_CHECK(hipMemcpy(dparents, ph, n * sizeof(Node), hipMemcpyHostToDevice));
  a.parents_in = dparents;
  a.bounds_out = dbounds;
  a.nparents = static_cast<int>(n);
  a.best_in = best;
  constexpr int BP = dev::PfspGeom<NJ, LBK, M>::BP;
  const int nchunks = static_cast<int>((n + BP - 1) / BP);
  hipLaunchKernelGGL((dev::pfsp_bounds_kernel<NJ, M, LBK>), dim3(std::min(nchunks, 2048)), dim3(dev::kBlock), 0, 0, a);
  TTS_HIP_CHECK(hipGetLastError());
  TTS_HIP_CHECK(hipDeviceSynchronize());
  TTS_HIP_CHECK(hipMemcpy(out.data(), dbounds, nb * sizeof(int), hipMemcpyDeviceToHost));
  (void)hipFree(dparents);
  (void)hipFree(dbounds);
  (void)hipFree(const_cast<int*>(a.offsets));
  (void)hipFree(const_cast<uint16_t*>(a.ptab));
  (void)hipFree(const_cast<uint2*>(a.recs));
  return out;
}

// Output of the expand probes beyond the bounds: the children an iteration wrote (chunk
// order), the leaves it counted and the incumbent after it.
struct ExpandProbeResult {
  std::vector<int> bounds;
  std::vector<uint8_t> children;
  long long leaves = 0;
  int best = 0;
};

// Element-wise probe of the production expand kernel (LB2 only): ONE iteration
// over `n` parents loaded as the window, with the kernel's debug output on. Returns
// every child's bound in parent order (children k = depth..N-1): the exact LB2 when
// it is below `best`, otherwise a value >= best (the kernel's prune decision).
// variant: 1 rounds of dense walks, 2 dense walks, 4 rounds of packed two-child walks
// (kernel LBK 5, the default search path where lb2_pk_ok).
// With `timing`: `reps` more launches without the debug output, each from the same
// window (ring and control block restored), on the engine's grid (resident
// workgroups), then one launch with the phase timers; timing = {min ms, median ms,
// phase A, B1, B2, B3+C shader clocks per chunk, chunks}.
template <int NJ, int M, int LBK>
std::vector<int> pfsp_expand_probe_t(const PfspInstance& in, const void* parents, size_t n, int best, int device,
                                     int variant, int reps = 0, std::vector<double>* timing = nullptr,
                                     ExpandProbeResult* extra = nullptr) {
  using Node = PfspNode<NJ>;
  using G = dev::PfspGeom<NJ, LBK, M>;
  if constexpr (LBK != 2) {
    throw std::invalid_argument("expand probe: LB2 kernels only");
  } else {
    TTS_HIP_CHECK(hipSetDevice(device));
    const Node* ph = static_cast<const Node*>(parents);
    std::vector<int> offsets(n + 1, 0);
    for (size_t i = 0; i < n; ++i) offsets[i + 1] = offsets[i] + (in.jobs - ph[i].depth);
    const size_t nb = static_cast<size_t>(offsets[n]);
    std::vector<int> out(nb, -1);
    if (n == 0) return out;
    const size_t nchunks = (n + G::BP - 1) / G::BP;
    if (nchunks > static_cast<size_t>(G::MAXCHUNKS)) throw std::invalid_argument("expand probe: too many parents");
    dev::PfspArgs<NJ, M> a{};
    const PfspTableImages img = pfsp_fill_args(in, a, true);
    std::vector<void*> owned;
    auto up = [&](const auto& v) {
      auto* d = upload_vec(v);
      owned.push_back(const_cast<void*>(static_cast<const void*>(d)));
      return d;
    };
    auto dalloc = [&](size_t bytes) {
      void* d = nullptr;
      TTS_HIP_CHECK(hipMalloc(&d, std::max<size_t>(bytes, 16)));
      TTS_HIP_CHECK(hipMemset(d, 0, std::max<size_t>(bytes, 16)));
      owned.push_back(d);
      return d;
    };
    a.ptab = up(img.ptab);
    a.recs = up(img.recs);
    a.pinfo = up(img.pinfo);
    a.recs4 = up(img.recs4);
    a.dbg_off = up(offsets);
    a.dbg_lb = up(out);
    if (variant != 1 && variant != 2 && variant != 4) throw std::invalid_argument("expand probe: variant 1, 2 or 4");
    a.lb2_rounds = variant == 1 || variant == 4;
    size_t cap = 1;
    while (cap < n) cap *= 2;
    auto& pa = a.pool;
    pa.ring = static_cast<Node*>(dalloc(cap * sizeof(Node)));
    TTS_HIP_CHECK(hipMemcpy(pa.ring, ph, n * sizeof(Node), hipMemcpyHostToDevice));
    for (int b = 0; b < 2; ++b) {
      pa.buf[b] = static_cast<Node*>(dalloc(nchunks * G::SLOT * sizeof(Node)));
      pa.cnt[b] = static_cast<int*>(dalloc(nchunks * sizeof(int)));
      pa.lcnt[b] = static_cast<int*>(dalloc(nchunks * sizeof(int)));
    }
    dev::PoolCtl h{};
    h.slot[0].stack = n;
    h.best.v = best;
    pa.ctl = static_cast<dev::PoolCtl*>(dalloc(sizeof(dev::PoolCtl)));
    TTS_HIP_CHECK(hipMemcpy(pa.ctl, &h, sizeof(h), hipMemcpyHostToDevice));
    pa.mirror = nullptr;
    pa.cap_mask = cap - 1;
    pa.max_parents = static_cast<int>(nchunks * G::BP);
    pa.max_chunks = static_cast<int>(nchunks);
    if (variant == 4 && !lb2_pk_ok(in)) throw std::invalid_argument("expand probe: packed walks do not apply");
    auto launch = [&](const dim3& grid) {
      if (variant == 4)
        hipLaunchKernelGGL((dev::pfsp_expand_kernel<NJ, M, 5>), grid, dim3(dev::kBlock), 0, 0, a, 0);
      else
        hipLaunchKernelGGL((dev::pfsp_expand_kernel<NJ, M, LBK>), grid, dim3(dev::kBlock), 0, 0, a, 0);
      TTS_HIP_CHECK(hipGetLastError());
    };
    launch(dim3(static_cast<unsigned>(std::min<size_t>(nchunks, 1024))));
    TTS_HIP_CHECK(hipDeviceSynchronize());
    TTS_HIP_CHECK(hipMemcpy(out.data(), a.dbg_lb, nb * sizeof(int), hipMemcpyDeviceToHost));
    if (extra) {  // what the iteration wrote: per-chunk children (buffer 1), leaves, incumbent
      std::vector<int> cnt(nchunks), lcnt(nchunks);
      TTS_HIP_CHECK(hipMemcpy(cnt.data(), pa.cnt[1], nchunks * sizeof(int), hipMemcpyDeviceToHost));
      TTS_HIP_CHECK(hipMemcpy(lcnt.data(), pa.lcnt[1], nchunks * sizeof(int), hipMemcpyDeviceToHost));
      extra->children.clear();
      extra->leaves = 0;
      for (size_t c = 0; c < nchunks; ++c) {
        if (cnt[c] < 0 || static_cast<size_t>(cnt[c]) > static_cast<size_t>(G::SLOT))
          throw std::runtime_error("expand probe: chunk count out of range");
        const size_t at = extra->children.size();
        extra->children.resize(at + static_cast<size_t>(cnt[c]) * sizeof(Node));
        if (cnt[c])
          TTS_HIP_CHECK(hipMemcpy(extra->children.data() + at, pa.buf[1] + c * G::SLOT,
                                  static_cast<size_t>(cnt[c]) * sizeof(Node), hipMemcpyDeviceToHost));
        extra->leaves += lcnt[c] & 0xffff;
      }
      dev::PoolCtl hc{};
      TTS_HIP_CHECK(hipMemcpy(&hc, pa.ctl, sizeof(hc), hipMemcpyDeviceToHost));
      extra->best = hc.best.v;
    }
    if (timing) {
      int bpc = 0, cus = 0;
      if (variant == 4)
        TTS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::pfsp_expand_kernel<NJ, M, 5>,
                                                                   dev::kBlock, 0));
      else
        TTS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::pfsp_expand_kernel<NJ, M, LBK>,
                                                                   dev::kBlock, 0));
      TTS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
      const dim3 grid(static_cast<unsigned>(std::min<size_t>(nchunks, static_cast<size_t>(std::max(1, bpc * cus)))));
      a.dbg_lb = nullptr;
      auto restore = [&] {
        TTS_HIP_CHECK(hipMemcpy(pa.ring, ph, n * sizeof(Node), hipMemcpyHostToDevice));
        TTS_HIP_CHECK(hipMemcpy(pa.ctl, &h, sizeof(h), hipMemcpyHostToDevice));
      };
      hipEvent_t e0, e1;
      TTS_HIP_CHECK(hipEventCreate(&e0));
      TTS_HIP_CHECK(hipEventCreate(&e1));
      std::vector<double> ms;
      for (int r = 0; r < std::max(1, reps); ++r) {
        restore();
        TTS_HIP_CHECK(hipEventRecord(e0, 0));
        launch(grid);
        TTS_HIP_CHECK(hipEventRecord(e1, 0));
        TTS_HIP_CHECK(hipEventSynchronize(e1));
        float t = 0;
        TTS_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
      }
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      std::sort(ms.begin(), ms.end());
      restore();
      a.dbg_time = static_cast<unsigned long long*>(dalloc(8 * sizeof(unsigned long long)));
      launch(grid);
      TTS_HIP_CHECK(hipDeviceSynchronize());
      unsigned long long tm[8] = {};
      TTS_HIP_CHECK(hipMemcpy(tm, a.dbg_time, sizeof(tm), hipMemcpyDeviceToHost));
      // workgroup timeline, from its own launch (no phase timers)
      restore();
      a.dbg_time = nullptr;
      a.dbg_blk = static_cast<unsigned long long*>(dalloc(3 * grid.x * sizeof(unsigned long long)));
      launch(grid);
      TTS_HIP_CHECK(hipDeviceSynchronize());
      std::vector<unsigned long long> blk(3 * grid.x);
      TTS_HIP_CHECK(hipMemcpy(blk.data(), a.dbg_blk, blk.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      a.dbg_blk = nullptr;
      int rate_khz = 0;
      TTS_HIP_CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device));
      unsigned long long t0 = ~0ull;
      for (size_t i = 0; i < grid.x; ++i) t0 = std::min(t0, blk[3 * i]);
      const double nc = static_cast<double>(std::max<unsigned long long>(1, tm[4]));
      *timing = {ms.front(), ms[ms.size() / 2], tm[0] / nc, tm[1] / nc, tm[2] / nc, tm[3] / nc, nc,
                 static_cast<double>(tm[5]), static_cast<double>(tm[6]) / std::max<unsigned long long>(1, tm[7]),
                 static_cast<double>(grid.x)};
      const double us = 1e3 / std::max(1, rate_khz);
      for (unsigned long long x : blk) timing->push_back(static_cast<double>(x - t0) * us);
    }
    for (void* d : owned) (void)hipFree(d);
    return out;
  }
}

// Element-wise probe of the permutation-node LB1 / LB1_d expand kernel (instances of
// more than 50 jobs; 20 / 50 jobs under TTS_FRONT=0): ONE iteration over `n` parents
// loaded as the window. Returns every child's bound (parent order, children
// k = depth..N-1), the children the kernel wrote (chunk order; lb < best, the leaves of
// depth N-1 parents excluded), the leaves it counted and the incumbent after the launch.
template <int NJ, int M>
ExpandProbeResult pfsp_lb1_expand_probe_t(const PfspInstance& in, const void* parents, size_t n, int best, int device) {
  using Node = PfspNode<NJ>;
  using G = dev::PfspGeom<NJ, 1, M>;
  TTS_HIP_CHECK(hipSetDevice(device));
  const Node* ph = static_cast<const Node*>(parents);
  ExpandProbeResult res;
  std::vector<int> offsets(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    if (ph[i].depth >= in.jobs) throw std::invalid_argument("lb1 expand probe: parents must have children");
    offsets[i + 1] = offsets[i] + (in.jobs - ph[i].depth);
  }
  res.bounds.assign(static_cast<size_t>(offsets[n]), -1);
  res.best = best;
  if (n == 0) return res;
  const size_t nchunks = (n + G::BP - 1) / G::BP;
  if (nchunks > static_cast<size_t>(G::MAXCHUNKS)) throw std::invalid_argument("lb1 expand probe: too many parents");
  dev::PfspArgs<NJ, M> a{};
  const PfspTableImages img = pfsp_fill_args(in, a);
  std::vector<void*> owned;
  auto up = [&](const auto& v) {
    auto* d = upload_vec(v);
    owned.push_back(const_cast<void*>(static_cast<const void*>(d)));
    return d;
  };
  auto dalloc = [&](size_t bytes) {
    void* d = nullptr;
    TTS_HIP_CHECK(hipMalloc(&d, std::max<size_t>(bytes, 16)));
    TTS_HIP_CHECK(hipMemset(d, 0, std::max<size_t>(bytes, 16)));
    owned.push_back(d);
    return d;
  };
  a.ptab = up(img.ptab);
  a.dbg_off = up(offsets);
  a.dbg_lb = up(res.bounds);
  size_t cap = 1;
  while (cap < n) cap *= 2;
  auto& pa = a.pool;
  pa.ring = static_cast<Node*>(dalloc(cap * sizeof(Node)));
  TTS_HIP_CHECK(hipMemcpy(pa.ring, ph, n * sizeof(Node), hipMemcpyHostToDevice));
  for (int b = 0; b < 2; ++b) {
    pa.buf[b] = static_cast<Node*>(dalloc(nchunks * G::SLOT * sizeof(Node)));
    pa.cnt[b] = static_cast<int*>(dalloc(nchunks * sizeof(int)));
    pa.lcnt[b] = static_cast<int*>(dalloc(nchunks * sizeof(int)));
  }
  dev::PoolCtl h{};
  h.slot[0].stack = n;
  h.best.v = best;
  pa.ctl = static_cast<dev::PoolCtl*>(dalloc(sizeof(dev::PoolCtl)));
  TTS_HIP_CHECK(hipMemcpy(pa.ctl, &h, sizeof(h), hipMemcpyHostToDevice));
  pa.mirror = nullptr;
  pa.cap_mask = cap - 1;
  pa.max_parents = static_cast<int>(nchunks * G::BP);
  pa.max_chunks = static_cast<int>(nchunks);
  hipLaunchKernelGGL((dev::pfsp_expand_kernel<NJ, M, 1>), dim3(static_cast<unsigned>(std::min<size_t>(nchunks, 1024))),
                     dim3(dev::kBlock), 0, 0, a, 0);
  TTS_HIP_CHECK(hipGetLastError());
  TTS_HIP_CHECK(hipDeviceSynchronize());
  TTS_HIP_CHECK(hipMemcpy(res.bounds.data(), a.dbg_lb, res.bounds.size() * sizeof(int), hipMemcpyDeviceToHost));
  std::vector<int> cnt(nchunks), lcnt(nchunks);
  TTS_HIP_CHECK(hipMemcpy(cnt.data(), pa.cnt[1], nchunks * sizeof(int), hipMemcpyDeviceToHost));
  TTS_HIP_CHECK(hipMemcpy(lcnt.data(), pa.lcnt[1], nchunks * sizeof(int), hipMemcpyDeviceToHost));
  for (size_t c = 0; c < nchunks; ++c) {
    if (cnt[c] < 0 || static_cast<size_t>(cnt[c]) > static_cast<size_t>(G::SLOT))
      throw std::runtime_error("lb1 expand probe: chunk count out of range");
    const size_t at = res.children.size();
    res.children.resize(at + static_cast<size_t>(cnt[c]) * sizeof(Node));
    if (cnt[c])
      TTS_HIP_CHECK(hipMemcpy(res.children.data() + at, pa.buf[1] + c * G::SLOT, static_cast<size_t>(cnt[c]) * sizeof(Node),
                              hipMemcpyDeviceToHost));
    res.leaves += lcnt[c] & 0xffff;
  }
  TTS_HIP_CHECK(hipMemcpy(&h, pa.ctl, sizeof(h), hipMemcpyDeviceToHost));
  res.best = h.best.v;
  for (void* d : owned) (void)hipFree(d);
  return res;
}

template <int M, int NJ = 20>
std::unique_ptr<IEngine> make_pfsp_front_engine_t(const PfspInstance& in, const EngineConfig& cfg) {
  TTS_HIP_CHECK(hipSetDevice(cfg.device));
  dev::PfspFrontArgs<M, NJ> a{};
  const std::vector<uint16_t> ptab = pfsp_front_fill_args(in, a);
  a.ptab = upload_vec(ptab);
  auto eng = std::make_unique<DeviceEngine<PfspFrontTraits<M, NJ>>>(cfg, a);
  eng->adopt(const_cast<uint16_t*>(a.ptab));
  return eng;
}

// Element-wise probe of the production LB1 / LB1_d front kernel (tests):
// a complete engine solve from `nodes` (front layout) with the kernel's probe records
// on, so every iteration shape the solve takes — one level per kernel, the split
// iteration, multi-level chunks (child-parallel and thread-per-node levels with carried
// remains), local DFS — records each child it bounds: the parent's words, the parent's
// remain as the kernel holds it, the job and the bound. Every record is checked here
// against the host oracle (PfspFrontProblem: ref add_front_and_bound,
// c_bound_simple.c:219-244). At most `cap` records are kept and checked; the count of
// all records is returned too.
struct FrontProbeResult {
  unsigned long long records = 0, checked = 0;
  unsigned long long by_kind[6] = {};
  unsigned long long bad_lb = 0, bad_remain = 0, bad_job = 0;
  EngineStats st;
  std::vector<uint32_t> first_bad;
};
template <int M, int NJ = 20>
FrontProbeResult pfsp_front_probe_t(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                    const EngineConfig& cfg, unsigned cap, int split_rank, int split_world,
                                    size_t split_min) {
  using G = dev::FrontGeom<M, NJ>;
  using Node = PfspFrontNode<M, NJ>;
  TTS_HIP_CHECK(hipSetDevice(cfg.device));
  const PfspFrontProblem<M, NJ> prob(in, lb);
  dev::PfspFrontArgs<M, NJ> a{};
  const std::vector<uint16_t> ptab = pfsp_front_fill_args(in, a);
  a.ptab = upload_vec(ptab);
  uint32_t* drec = nullptr;
  unsigned* dn = nullptr;
  TTS_HIP_CHECK(hipMalloc(&drec, std::max<size_t>(1, cap) * G::DBGW * sizeof(uint32_t)));
  TTS_HIP_CHECK(hipMalloc(&dn, sizeof(unsigned)));
  TTS_HIP_CHECK(hipMemset(dn, 0, sizeof(unsigned)));
  a.dbg_rec = drec;
  a.dbg_n = dn;
  a.dbg_cap = cap;
  FrontProbeResult res;
  {
    DeviceEngine<PfspFrontTraits<M, NJ>> eng(cfg, a);
    if (split_world > 1) eng.set_split(split_rank, split_world, split_min);
    res.st = eng.solve_from(nodes, n, best);
  }
  unsigned total = 0;
  TTS_HIP_CHECK(hipMemcpy(&total, dn, sizeof(unsigned), hipMemcpyDeviceToHost));
  res.records = total;
  const size_t keep = std::min<size_t>(total, cap);
  std::vector<uint32_t> rec(keep * G::DBGW);
  if (keep) TTS_HIP_CHECK(hipMemcpy(rec.data(), drec, rec.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  (void)hipFree(drec);
  (void)hipFree(dn);
  (void)hipFree(const_cast<uint16_t*>(a.ptab));
  res.checked = keep;
  for (size_t i = 0; i < keep; ++i) {
    const uint32_t* r = &rec[i * G::DBGW];
    const int j = static_cast<int>(r[0] & 0xffu), kind = static_cast<int>((r[0] >> 8) & 0xffu);
    if (kind < 6) ++res.by_kind[kind];
    Node parent;
    std::memcpy(&parent, r + 2, sizeof(Node));
    bool bad = false;
    if (j >= NJ || !((parent.rest >> j) & 1u)) {
      ++res.bad_job;
      bad = true;
    } else {
      int rt[M];
      prob.remain_tail(parent, rt);
      for (int m = 0; m < M; ++m) {
        const int got = static_cast<int>((r[2 + G::NW + (m >> 1)] >> ((m & 1) * 16)) & 0xffffu);
        if (got != rt[m] - prob.tab.tails[m]) {
          ++res.bad_remain;
          bad = true;
          break;
        }
      }
      if (prob.child(parent, rt, j, nullptr) != static_cast<int>(r[1])) {
        ++res.bad_lb;
        bad = true;
      }
    }
    if (bad && res.first_bad.empty()) res.first_bad.assign(r, r + G::DBGW);
  }
  return res;
}

// Timing probe of ONE front-kernel iteration over a given window (the nodes loaded as
// the pool), on the engine's grid: `reps` launches from the same state (min / median
// ms), then one launch with the per-workgroup phase stamps (front_stamp). Returns
// {ms_min, ms_median, grid, iteration levels, then grid x 16 stamps in us from the first
// workgroup entry (0 where a stamp was not reached)}.
template <int M, int NJ = 20>
std::vector<double> pfsp_front_time_t(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                      const EngineConfig& cfg, int reps) {
  using G = dev::FrontGeom<M, NJ>;
  using Node = PfspFrontNode<M, NJ>;
  TTS_HIP_CHECK(hipSetDevice(cfg.device));
  (void)lb;
  dev::PfspFrontArgs<M, NJ> a{};
  const std::vector<uint16_t> ptab = pfsp_front_fill_args(in, a);
  std::vector<void*> owned;
  auto dalloc = [&](size_t bytes) {
    void* d = nullptr;
    TTS_HIP_CHECK(hipMalloc(&d, std::max<size_t>(bytes, 16)));
    TTS_HIP_CHECK(hipMemset(d, 0, std::max<size_t>(bytes, 16)));
    owned.push_back(d);
    return d;
  };
  a.ptab = upload_vec(ptab);
  owned.push_back(const_cast<uint16_t*>(a.ptab));
  const size_t max_chunks = std::min<size_t>((cfg.max_parents + G::BP - 1) / G::BP, G::MAXCHUNKS);
  size_t cap = 1;
  while (cap < n) cap *= 2;
  auto& pa = a.pool;
  pa.ring = static_cast<Node*>(dalloc(cap * sizeof(Node)));
  for (int b = 0; b < 2; ++b) {
    pa.buf[b] = static_cast<Node*>(dalloc(max_chunks * G::SLOT * sizeof(Node)));
    pa.cnt[b] = static_cast<int*>(dalloc(max_chunks * sizeof(int)));
    pa.lcnt[b] = static_cast<int*>(dalloc(max_chunks * sizeof(int)));
  }
  dev::PoolCtl h{};
  h.slot[0].stack = n;
  h.best.v = best;
  pa.ctl = static_cast<dev::PoolCtl*>(dalloc(sizeof(dev::PoolCtl)));
  pa.mirror = nullptr;
  pa.cap_mask = cap - 1;
  pa.max_parents = static_cast<int>(max_chunks * G::BP);
  pa.max_chunks = static_cast<int>(max_chunks);
  pa.fuse_max = cfg.fuse_max;
  pa.local_steps = std::min(cfg.local_steps, G::LT);
  pa.local_min = std::max(0, cfg.local_min);
  pa.local_stride = 0;
  pa.local_wide_steps = 0;
  if (const char* f = std::getenv("TTS_LOCAL_STRIDE")) pa.local_stride = std::atoi(f);
  pa.deep_levels = cfg.deep_levels;
  pa.deep_per[0] = cfg.deep_per3;
  pa.deep_per[1] = cfg.deep_per4;
  pa.wide_levels = cfg.wide_levels;
  if (const char* f = std::getenv("TTS_WIDE_LEVELS")) pa.wide_levels = std::atoi(f);
  int bpc = 0, cus = 0;
  bpc = PfspFrontTraits<M, NJ>::blocks_per_cu();
  if (const char* g = std::getenv("TTS_BLOCKS_PER_CU")) bpc = std::max(1, std::atoi(g));  // as DeviceEngine
  TTS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg.device));
  const int grid = static_cast<int>(std::min<size_t>(max_chunks, static_cast<size_t>(std::max(1, bpc)) * cus));
  // dynamic local DFS (as DeviceEngine): 3 control sets, the budget in wall-clock ticks
  int dyn_us = cfg.dyn_us;
  if (const char* f = std::getenv("TTS_DYN_US")) dyn_us = std::max(0, std::atoi(f));
  const int dq = static_cast<int>(std::min<size_t>(dev::kDynQMax, max_chunks - std::min<size_t>(max_chunks, grid))) / 8 * 8;
  if (dyn_us > 0 && dq >= 8) {
    int rk = 0;
    TTS_HIP_CHECK(hipDeviceGetAttribute(&rk, hipDeviceAttributeWallClockRate, cfg.device));
    pa.dyn = static_cast<dev::DynCtl*>(dalloc(3 * sizeof(dev::DynCtl)));
    pa.dyn_ticks = static_cast<int>(static_cast<long long>(dyn_us) * std::max(1, rk) / 1000);
    pa.dyn_q = dq;
  }
  auto restore = [&] {
    TTS_HIP_CHECK(hipMemcpy(pa.ring, nodes, n * sizeof(Node), hipMemcpyHostToDevice));
    TTS_HIP_CHECK(hipMemcpy(pa.ctl, &h, sizeof(h), hipMemcpyHostToDevice));
    if (pa.dyn) TTS_HIP_CHECK(hipMemset(pa.dyn, 0, 3 * sizeof(dev::DynCtl)));
  };
  hipEvent_t e0, e1;
  TTS_HIP_CHECK(hipEventCreate(&e0));
  TTS_HIP_CHECK(hipEventCreate(&e1));
  std::vector<double> ms;
  for (int r = 0; r < std::max(1, reps); ++r) {
    restore();
    TTS_HIP_CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((dev::pfsp_front_kernel<M, NJ>), dim3(grid), dim3(dev::kBlock), 0, 0, a, 0);
    TTS_HIP_CHECK(hipGetLastError());
    TTS_HIP_CHECK(hipEventRecord(e1, 0));
    TTS_HIP_CHECK(hipEventSynchronize(e1));
    float t = 0;
    TTS_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  std::sort(ms.begin(), ms.end());
  restore();
  a.dbg_blk = static_cast<unsigned long long*>(dalloc(static_cast<size_t>(grid) * 16 * sizeof(unsigned long long)));
  hipLaunchKernelGGL((dev::pfsp_front_kernel<M, NJ>), dim3(grid), dim3(dev::kBlock), 0, 0, a, 0);
  TTS_HIP_CHECK(hipGetLastError());
  TTS_HIP_CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> blk(static_cast<size_t>(grid) * 16);
  TTS_HIP_CHECK(hipMemcpy(blk.data(), a.dbg_blk, blk.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  dev::PoolCtl after{};
  TTS_HIP_CHECK(hipMemcpy(&after, pa.ctl, sizeof(after), hipMemcpyDeviceToHost));
  for (void* d : owned) (void)hipFree(d);
  int rate_khz = 0;
  TTS_HIP_CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, cfg.device));
  unsigned long long t0 = ~0ull;
  for (int i = 0; i < grid; ++i)
    if (blk[16 * i]) t0 = std::min(t0, blk[16 * i]);
  const double us = 1e3 / std::max(1, rate_khz);
  std::vector<double> out = {ms.front(), ms[ms.size() / 2], static_cast<double>(grid),
                             static_cast<double>(after.slot[1].nch)};
  // words 9-10 and 12-14 of a workgroup are raw (dynamic DFS counters and idle ticks,
  // HW_ID, XCC_ID, local DFS counts: front_stamp / front_dyn)
  for (size_t i = 0; i < blk.size(); ++i) {
    const unsigned long long x = blk[i];
    const size_t k = i % 16;
    const bool raw = (k >= 12 && k <= 14) || k == 9 || k == 10;
    out.push_back(raw ? static_cast<double>(x) : (x ? static_cast<double>(x - t0) * us : 0.0));
  }
  return out;
}

// Bounds of permutation-layout parents through the front kernel (tests): parents are
// converted on the host, bounds come back in the permutation's child order k = depth..N-1.
template <int M, int NJ = 20>
std::vector<int> pfsp_front_bounds_t(const PfspInstance& in, const PfspNode<NJ>* ph, size_t n, int device) {
  using FNode = PfspFrontNode<M, NJ>;
  using Mask = typename FNode::Mask;
  TTS_HIP_CHECK(hipSetDevice(device));
  const PfspFrontProblem<M, NJ> prob(in, 1);
  std::vector<FNode> fn(n);
  std::vector<int> offsets(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    fn[i] = pfsp_front_from_perm(prob, ph[i]);
    offsets[i + 1] = offsets[i] + (in.jobs - ph[i].depth);
  }
  const size_t nb = static_cast<size_t>(offsets[n]);
  std::vector<int> by_job(nb, 0), out(nb, 0);
  if (n == 0) return out;
  dev::PfspFrontArgs<M, NJ> a{};
  const std::vector<uint16_t> ptab = pfsp_front_fill_args(in, a);
  a.ptab = upload_vec(ptab);
  a.offsets = upload_vec(offsets);
  a.parents_in = upload_vec(fn);
  int* dbounds = nullptr;
  TTS_HIP_CHECK(hipMalloc(&dbounds, std::max<size_t>(1, nb) * sizeof(int)));
  a.bounds_out = dbounds;
  a.nparents = static_cast<int>(n);
  const int blocks = static_cast<int>(std::min<size_t>((n + dev::kBlock - 1) / dev::kBlock, 2048));
  hipLaunchKernelGGL((dev::pfsp_front_bounds_kernel<M, NJ>), dim3(blocks), dim3(dev::kBlock), 0, 0, a);
  TTS_HIP_CHECK(hipGetLastError());
  TTS_HIP_CHECK(hipDeviceSynchronize());
  TTS_HIP_CHECK(hipMemcpy(by_job.data(), dbounds, nb * sizeof(int), hipMemcpyDeviceToHost));
  (void)hipFree(dbounds);
  (void)hipFree(const_cast<int*>(a.offsets));
  (void)hipFree(const_cast<FNode*>(a.parents_in));
  (void)hipFree(const_cast<uint16_t*>(a.ptab));
  for (size_t i = 0; i < n; ++i) {
    const int d = ph[i].depth;
    for (int k = d; k < in.jobs; ++k) {
      const int job = ph[i].prmu[k];
      out[offsets[i] + (k - d)] =
          by_job[offsets[i] + __builtin_popcountll(static_cast<unsigned long long>(fn[i].rest & ((Mask(1) << job) - 1)))];
    }
  }
  return out;
}

// Kernel machine bucket: 5, 10 or 20 (Taillard's counts); other counts up to 20 run
// in the next bucket with zero-time padding machines (pfsp_fill_args).
template <class F>
decltype(auto) with_machine_bucket(int machines, F&& f) {
  if (machines >= 1 && machines <= 5) return f(std::integral_constant<int, 5>{});
  if (machines > 5 && machines <= 10) return f(std::integral_constant<int, 10>{});
  if (machines > 10 && machines <= 20) return f(std::integral_constant<int, 20>{});
  throw std::invalid_argument("GPU kernels support 1 to 20 machines");
}

// ---- run-time dispatch (definitions in pfsp_engine_nj*.hip, one TU per bucket) ----
std::unique_ptr<IEngine> make_pfsp_engine(const PfspInstance& in, int lb, const EngineConfig& cfg);
std::vector<int> pfsp_gpu_bounds(const PfspInstance& in, int lb, const void* parents, size_t n, int best, int device);
std::vector<int> pfsp_expand_probe(const PfspInstance& in, int lb, const void* parents, size_t n, int best, int device,
                                   int variant, int reps = 0, std::vector<double>* timing = nullptr,
                                   ExpandProbeResult* extra = nullptr);
std::vector<double> pfsp_front_time(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                    const EngineConfig& cfg, int reps);
// front-layout instances only (pfsp_front_ok), defined with the 20-job bucket (the
// 50-job front bucket's in its own TU)
ExpandProbeResult pfsp_lb1_expand_probe(const PfspInstance& in, const void* parents, size_t n, int best, int device);
FrontProbeResult pfsp_front_probe(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                  const EngineConfig& cfg, unsigned cap, int split_rank = 0, int split_world = 1,
                                  size_t split_min = 0);
FrontProbeResult pfsp_front_probe_nj50(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                       const EngineConfig& cfg, unsigned cap, int split_rank, int split_world,
                                       size_t split_min);
std::vector<double> pfsp_front_time_nj50(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                         const EngineConfig& cfg, int reps);

#define TTS_PFSP_DECLARE_BUCKET(NJ)                                                                   \
  std::unique_ptr<IEngine> make_pfsp_engine_nj##NJ(const PfspInstance& in, int lb, const EngineConfig& cfg); \
  std::vector<int> pfsp_gpu_bounds_nj##NJ(const PfspInstance& in, int lb, const void* parents, size_t n, int best, \
                                          int device);                                                \
  std::vector<int> pfsp_expand_probe_nj##NJ(const PfspInstance& in, int lb, const void* parents, size_t n, int best, \
                                            int device, int variant, int reps, std::vector<double>* timing, \
                                            ExpandProbeResult* extra); \
  ExpandProbeResult pfsp_lb1_expand_probe_nj##NJ(const PfspInstance& in, const void* parents, size_t n, int best, int device);
TTS_PFSP_DECLARE_BUCKET(20)
TTS_PFSP_DECLARE_BUCKET(50)
TTS_PFSP_DECLARE_BUCKET(100)
TTS_PFSP_DECLARE_BUCKET(200)
TTS_PFSP_DECLARE_BUCKET(500)

// Body of one bucket's TU: machine buckets (with_machine_bucket), LB kernels 1 (LB1
// and LB1_d) / 2.
#define TTS_PFSP_DEFINE_BUCKET(NJ)                                                                     \
  std::unique_ptr<IEngine> make_pfsp_engine_nj##NJ(const PfspInstance& in, int lb, const EngineConfig& cfg) { \
    return with_machine_bucket(in.machines, [&](auto mm) -> std::unique_ptr<IEngine> {               \
      constexpr int M = decltype(mm)::value;                                                         \
      if constexpr (NJ == 20 || NJ == 50)                                                            \
        if (pfsp_front_ok(in, lb)) return make_pfsp_front_engine_t<M, NJ>(in, cfg);                  \
      if (lb != 2) return make_pfsp_engine_t<NJ, M, 1>(in, cfg);                                    \
      if (M >= 10 && lb2_pk_wanted(in)) return make_pfsp_engine_t<NJ, M, 5>(in, cfg);                 \
      return make_pfsp_engine_t<NJ, M, 2>(in, cfg);                                                  \
    });                                                                                              \
  }                                                                                                  \
  std::vector<int> pfsp_gpu_bounds_nj##NJ(const PfspInstance& in, int lb, const void* parents, size_t n, int best, \
                                          int device) {                                              \
    return with_machine_bucket(in.machines, [&](auto mm) {                                           \
      constexpr int M = decltype(mm)::value;                                                         \
      if constexpr (NJ == 20 || NJ == 50)                                                            \
        if (pfsp_front_ok(in, lb))                                                                   \
          return pfsp_front_bounds_t<M, NJ>(in, static_cast<const PfspNode<NJ>*>(parents), n, device); \
      return lb == 2 ? pfsp_gpu_bounds_t<NJ, M, 2>(in, parents, n, best, device)                    \
                     : pfsp_gpu_bounds_t<NJ, M, 1>(in, parents, n, best, device);                   \
    });                                                                                              \
  }                                                                                                  \
  std::vector<int> pfsp_expand_probe_nj##NJ(const PfspInstance& in, int lb, const void* parents, size_t n, int best, \
                                            int device, int variant, int reps, std::vector<double>* timing, \
                                            ExpandProbeResult* extra) {                                     \
    if (lb != 2) throw std::invalid_argument("expand probe: LB2 only");                             \
    return with_machine_bucket(in.machines, [&](auto mm) {                                           \
      constexpr int M = decltype(mm)::value;                                                         \
      return pfsp_expand_probe_t<NJ, M, 2>(in, parents, n, best, device, variant, reps, timing, extra); \
    });                                                                                              \
  }                                                                                                  \
  ExpandProbeResult pfsp_lb1_expand_probe_nj##NJ(const PfspInstance& in, const void* parents, size_t n, int best, \
                                              int device) {                                          \
    return with_machine_bucket(in.machines, [&](auto mm) {                                           \
      constexpr int M = decltype(mm)::value;                                                         \
      return pfsp_lb1_expand_probe_t<NJ, M>(in, parents, n, best, device);                           \
    });                                                                                              \
  }

}  // namespace tts
