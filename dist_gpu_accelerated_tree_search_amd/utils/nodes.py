"""numpy views of the node layouts shared by host and device pools.

PFSP node (csrc/core/pfsp_node.hpp): id_t depth; id_t prmu[NJ]; padded to 16 B,
id_t = uint8 for NJ <= 255 else uint16. PFSP front node (LB1 / LB1_d engines on up to
20 jobs): uint8 depth, 3 pad, uint32 unscheduled-job mask, uint16 front[MB] (21-50 jobs:
7 pad and a uint64 mask), padded
to 16 B (32 B for MB <= 10 machines, 48 B for 20). N-Queens node: 4 x uint32
{cols, diag, anti, depth}. Parity: ref pfsp/lib/PFSP_node.h:15-20 (44-B node with
limit1 stored), nqueens/lib/NQueens_node.h:13-17 (board).
"""
from __future__ import annotations

import numpy as np

BUCKETS = (20, 50, 100, 200, 500)


def pfsp_bucket(jobs: int) -> int:
    for b in BUCKETS:
        if jobs <= b:
            return b
    return 500


def pfsp_id_dtype(jobs: int):
    return np.uint16 if pfsp_bucket(jobs) > 255 else np.uint8


def pfsp_node_bytes(jobs: int) -> int:
    nj = pfsp_bucket(jobs)
    isz = np.dtype(pfsp_id_dtype(jobs)).itemsize
    raw = (nj + 1) * isz
    return (raw + 15) // 16 * 16


def pfsp_pack(depths, perms, jobs: int) -> np.ndarray:
    """Pack (depth, permutation) pairs into an (n, node_bytes) uint8 array."""
    depths = np.asarray(depths)
    perms = np.asarray(perms)
    n = len(depths)
    nb = pfsp_node_bytes(jobs)
    dt = pfsp_id_dtype(jobs)
    isz = np.dtype(dt).itemsize
    out = np.zeros((n, nb // isz), dtype=dt)
    out[:, 0] = depths
    out[:, 1 : 1 + jobs] = perms
    return out.view(np.uint8).reshape(n, nb)


def pfsp_unpack(nodes: np.ndarray, jobs: int):
    """Inverse of pfsp_pack: (depths[n], perms[n, jobs])."""
    dt = pfsp_id_dtype(jobs)
    v = np.ascontiguousarray(nodes).view(dt)
    return v[:, 0].astype(np.int64), v[:, 1 : 1 + jobs].astype(np.int64)


def pfsp_root(jobs: int) -> np.ndarray:
    return pfsp_pack([0], [np.arange(jobs)], jobs)


def pfsp_front_unpack(nodes: np.ndarray, machines_bucket: int, jobs: int = 20):
    """Front nodes -> (depths[n], rest masks[n], fronts[n, machines_bucket]). Up to 20
    jobs the unscheduled set is 32 bits at byte 4 and the fronts start at byte 8; up to
    50 jobs it is 64 bits at byte 8 and the fronts start at byte 16."""
    a = np.ascontiguousarray(nodes, dtype=np.uint8)
    depths = a[:, 0].astype(np.int64)
    if jobs <= 20:
        rest = a[:, 4:8].copy().view(np.uint32).reshape(-1).astype(np.int64)
        f0 = 8
    else:
        rest = a[:, 8:16].copy().view(np.uint64).reshape(-1)
        f0 = 16
    fronts = a[:, f0:f0 + 2 * machines_bucket].copy().view(np.uint16).astype(np.int64)
    return depths, rest, fronts


QUEENS_NODE_BYTES = 16


def queens_pack(cols, diag, anti, depth) -> np.ndarray:
    a = np.stack([np.asarray(cols), np.asarray(diag), np.asarray(anti), np.asarray(depth)], axis=1).astype(np.uint32)
    return a.view(np.uint8).reshape(len(a), QUEENS_NODE_BYTES)


def queens_unpack(nodes: np.ndarray):
    v = np.ascontiguousarray(nodes).view(np.uint32).reshape(-1, 4)
    return v[:, 0], v[:, 1], v[:, 2], v[:, 3]
