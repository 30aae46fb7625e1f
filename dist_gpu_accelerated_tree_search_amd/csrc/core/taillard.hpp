// Taillard PFSP benchmark instances ta001..ta120, regenerated from their seeds.
//
// Parity: reference pfsp/lib/c_taillard.c:6-105 (seeds, best-known makespans,
// class geometry, Lehmer LCG with a *float* division). The generator must be
// bit-exact because every golden tree size in tests/ depends on it.
//
// Layout choice (MI355X-first): besides the reference's machine-major matrix
// p[m*N + j] we also produce a job-major copy (p[j*M + m]) — a job's M processing
// times are then one contiguous row, which is what the GPU kernels stage into LDS
// and read with a single vector load per job.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace tts {

namespace taillard_detail {
inline constexpr long kSeeds[120] = {
    873654221,  379008056,  1866992158, 216771124,  495070989,  402959317,  1369363414, 2021925980,
    573109518,  88325120,   587595453,  1401007982, 873136276,  268827376,  1634173168, 691823909,
    73807235,   1273398721, 2065119309, 1672900551, 479340445,  268827376,  1958948863, 918272953,
    555010963,  2010851491, 1519833303, 1748670931, 1923497586, 1829909967, 1328042058, 200382020,
    496319842,  1203030903, 1730708564, 450926852,  1303135678, 1273398721, 587288402,  248421594,
    1958948863, 575633267,  655816003,  1977864101, 93805469,   1803345551, 49612559,   1899802599,
    2013025619, 578962478,  1539989115, 691823909,  655816003,  1315102446, 1949668355, 1923497586,
    1805594913, 1861070898, 715643788,  464843328,  896678084,  1179439976, 1122278347, 416756875,
    267829958,  1835213917, 1328833962, 1418570761, 161033112,  304212574,  1539989115, 655816003,
    960914243,  1915696806, 2013025619, 1168140026, 1923497586, 167698528,  1528387973, 993794175,
    450926852,  1462772409, 1021685265, 83696007,   508154254,  1861070898, 26482542,   444956424,
    2115448041, 118254244,  471503978,  1215892992, 135346136,  1602504050, 160037322,  551454346,
    519485142,  383947510,  1968171878, 540872513,  2013025619, 475051709,  914834335,  810642687,
    1019331795, 2056065863, 1342855162, 1325809384, 1988803007, 765656702,  1368624604, 450181436,
    1927888393, 1759567256, 606425239,  19268348,   1298201670, 2041736264, 379756761,  28837162};

// Best-known makespans (optimal for every instance solved to date).
inline constexpr int kBestKnown[120] = {
    1278,  1359,  1081,  1293,  1235,  1195,  1234,  1206,  1230,  1108,  1582,  1659,  1496,  1377,
    1419,  1397,  1484,  1538,  1593,  1591,  2297,  2099,  2326,  2223,  2291,  2226,  2273,  2200,
    2237,  2178,  2724,  2834,  2621,  2751,  2863,  2829,  2725,  2683,  2552,  2782,  2991,  2867,
    2839,  3063,  2976,  3006,  3093,  3037,  2897,  3065,  3846,  3699,  3640,  3719,  3610,  3679,
    3704,  3691,  3741,  3755,  5493,  5268,  5175,  5014,  5250,  5135,  5246,  5094,  5448,  5322,
    5770,  5349,  5676,  5781,  5467,  5303,  5595,  5617,  5871,  5845,  6173,  6183,  6252,  6254,
    6285,  6331,  6223,  6372,  6247,  6404,  10862, 10480, 10922, 10889, 10524, 10329, 10854, 10730,
    10438, 10675, 11158, 11160, 11281, 11275, 11259, 11176, 11337, 11301, 11146, 11284, 26040, 26500,
    26371, 26456, 26334, 26469, 26389, 26560, 26005, 26457};

// Park–Miller minimal standard generator, Schrage's decomposition; the [0,1)
// sample is formed with single-precision division exactly as Taillard's code.
inline long lcg_uniform(long& seed, long low, long high) {
  constexpr long m = 2147483647, a = 16807, q = 127773, r = 2836;
  const long k = seed / q;
  seed = a * (seed % q) - k * r;
  if (seed < 0) seed += m;
  const float u = static_cast<float>(seed) / static_cast<float>(m);
  const double value01 = static_cast<double>(u);
  return low + static_cast<long>(value01 * static_cast<double>(high - low + 1));
}
}  // namespace taillard_detail

inline void check_taillard_id(int id) {
  if (id < 1 || id > 120) throw std::out_of_range("Taillard instance id must be in 1..120");
}

inline int taillard_jobs(int id) {
  check_taillard_id(id);
  if (id > 110) return 500;
  if (id > 90) return 200;
  if (id > 60) return 100;
  if (id > 30) return 50;
  return 20;
}

inline int taillard_machines(int id) {
  check_taillard_id(id);
  // 20x5 20x10 20x20 | 50x5 50x10 50x20 | 100x5 100x10 100x20 | 200x10 200x20 | 500x20
  static constexpr int kBlockMachines[12] = {5, 10, 20, 5, 10, 20, 5, 10, 20, 10, 20, 20};
  return kBlockMachines[(id - 1) / 10];
}

inline int taillard_best_ub(int id) {
  check_taillard_id(id);
  return taillard_detail::kBestKnown[id - 1];
}

// Machine-major processing times p[m*N + j] (reference layout).
inline std::vector<int> taillard_processing_times(int id) {
  const int N = taillard_jobs(id), M = taillard_machines(id);
  long seed = taillard_detail::kSeeds[id - 1];
  std::vector<int> p(static_cast<size_t>(N) * M);
  for (int m = 0; m < M; ++m)
    for (int j = 0; j < N; ++j) p[static_cast<size_t>(m) * N + j] = static_cast<int>(taillard_detail::lcg_uniform(seed, 1, 99));
  return p;
}

// Synthetic Taillard-shaped instance (same LCG, caller-chosen seed and shape):
// used for scaling studies on shapes the benchmark set does not contain.
inline std::vector<int> synthetic_processing_times(int jobs, int machines, long seed) {
  if (jobs < 2 || machines < 2) throw std::invalid_argument("synthetic instance needs >=2 jobs and >=2 machines");
  if (seed <= 0) seed = 1;
  std::vector<int> p(static_cast<size_t>(jobs) * machines);
  for (int m = 0; m < machines; ++m)
    for (int j = 0; j < jobs; ++j) p[static_cast<size_t>(m) * jobs + j] = static_cast<int>(taillard_detail::lcg_uniform(seed, 1, 99));
  return p;
}

}  // namespace tts
