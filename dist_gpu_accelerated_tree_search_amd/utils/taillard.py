"""Pure-Python Taillard generator: an independent oracle for the native one.

Parity: ref pfsp/lib/c_taillard.c:46-105 (class geometry, seeds, Lehmer LCG where
the [0,1) sample is a *single-precision* quotient). Used by tests to pin the C++
generator bit-for-bit and by tools that must not load native code.
"""
from __future__ import annotations

import numpy as np

# Seeds and best-known makespans of ta001..ta120 (public benchmark data).
SEEDS = [
    873654221, 379008056, 1866992158, 216771124, 495070989, 402959317, 1369363414, 2021925980, 573109518, 88325120,
    587595453, 1401007982, 873136276, 268827376, 1634173168, 691823909, 73807235, 1273398721, 2065119309, 1672900551,
    479340445, 268827376, 1958948863, 918272953, 555010963, 2010851491, 1519833303, 1748670931, 1923497586, 1829909967,
    1328042058, 200382020, 496319842, 1203030903, 1730708564, 450926852, 1303135678, 1273398721, 587288402, 248421594,
    1958948863, 575633267, 655816003, 1977864101, 93805469, 1803345551, 49612559, 1899802599, 2013025619, 578962478,
    1539989115, 691823909, 655816003, 1315102446, 1949668355, 1923497586, 1805594913, 1861070898, 715643788, 464843328,
    896678084, 1179439976, 1122278347, 416756875, 267829958, 1835213917, 1328833962, 1418570761, 161033112, 304212574,
    1539989115, 655816003, 960914243, 1915696806, 2013025619, 1168140026, 1923497586, 167698528, 1528387973, 993794175,
    450926852, 1462772409, 1021685265, 83696007, 508154254, 1861070898, 26482542, 444956424, 2115448041, 118254244,
    471503978, 1215892992, 135346136, 1602504050, 160037322, 551454346, 519485142, 383947510, 1968171878, 540872513,
    2013025619, 475051709, 914834335, 810642687, 1019331795, 2056065863, 1342855162, 1325809384, 1988803007, 765656702,
    1368624604, 450181436, 1927888393, 1759567256, 606425239, 19268348, 1298201670, 2041736264, 379756761, 28837162,
]
BEST_KNOWN = [
    1278, 1359, 1081, 1293, 1235, 1195, 1234, 1206, 1230, 1108, 1582, 1659, 1496, 1377, 1419, 1397, 1484, 1538, 1593,
    1591, 2297, 2099, 2326, 2223, 2291, 2226, 2273, 2200, 2237, 2178, 2724, 2834, 2621, 2751, 2863, 2829, 2725, 2683,
    2552, 2782, 2991, 2867, 2839, 3063, 2976, 3006, 3093, 3037, 2897, 3065, 3846, 3699, 3640, 3719, 3610, 3679, 3704,
    3691, 3741, 3755, 5493, 5268, 5175, 5014, 5250, 5135, 5246, 5094, 5448, 5322, 5770, 5349, 5676, 5781, 5467, 5303,
    5595, 5617, 5871, 5845, 6173, 6183, 6252, 6254, 6285, 6331, 6223, 6372, 6247, 6404, 10862, 10480, 10922, 10889,
    10524, 10329, 10854, 10730, 10438, 10675, 11158, 11160, 11281, 11275, 11259, 11176, 11337, 11301, 11146, 11284,
    26040, 26500, 26371, 26456, 26334, 26469, 26389, 26560, 26005, 26457,
]
_CLASS_MACHINES = [5, 10, 20, 5, 10, 20, 5, 10, 20, 10, 20, 20]


def _check(i: int) -> None:
    if not 1 <= i <= 120:
        raise ValueError("Taillard instance id must be in 1..120")


def jobs(i: int) -> int:
    _check(i)
    return 500 if i > 110 else 200 if i > 90 else 100 if i > 60 else 50 if i > 30 else 20


def machines(i: int) -> int:
    _check(i)
    return _CLASS_MACHINES[(i - 1) // 10]


def best_known(i: int) -> int:
    _check(i)
    return BEST_KNOWN[i - 1]


def _lcg(seed: int, n: int) -> tuple[np.ndarray, int]:
    m, a, q, r = 2147483647, 16807, 127773, 2836
    out = np.empty(n, dtype=np.int64)
    for t in range(n):
        k = seed // q
        seed = a * (seed % q) - k * r
        if seed < 0:
            seed += m
        u = np.float32(seed) / np.float32(m)  # single-precision quotient, as Taillard's code
        out[t] = 1 + int(float(u) * 99.0)
    return out, seed


def processing_times(i: int) -> np.ndarray:
    """(machines, jobs) int matrix, row = machine (reference's machine-major layout)."""
    n, mm = jobs(i), machines(i)
    vals, _ = _lcg(SEEDS[i - 1], n * mm)
    return vals.reshape(mm, n).astype(np.int32)


def synthetic(jobs_: int, machines_: int, seed: int) -> np.ndarray:
    """Taillard-shaped synthetic instance (same LCG, chosen seed and shape)."""
    vals, _ = _lcg(max(1, seed), jobs_ * machines_)
    return vals.reshape(machines_, jobs_).astype(np.int32)
