"""Checkpoint / resume of a distributed solve (the reference has none).

Pools are flat arrays of POD nodes, so a checkpoint taken at a round boundary —
when no node is in flight — is exact: per rank, its pool content plus the
counters and incumbent it has accumulated. Files are plain `.npz` (no pickles):

    <dir>/ckpt_rank<r>_of<w>.npz   nodes (n, node_bytes) uint8
                                   meta  int64 [tree, sol, best, rounds, node_bytes, rank, world]
                                   model JSON string of model.describe()

Resume may use a different world size: every rank reads all files, concatenates
their nodes in rank order and keeps the strided share i % world == rank; the
saved counters are summed once (rank 0) and the incumbent is the minimum.
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np


def _path(directory: str, rank: int, world: int) -> str:
    return os.path.join(directory, f"ckpt_rank{rank}_of{world}.npz")


def save(directory: str, rank: int, world: int, model, engine, tree: int, sol: int, best: int,
         rounds: int) -> str:
    """Snapshot this rank's pool without changing it (pop everything, push it back
    in the same order) and write it with the counters."""
    os.makedirs(directory, exist_ok=True)
    n = int(engine.size())
    nodes = engine.pop(n) if n else np.zeros((0, model.node_bytes), np.uint8)
    if len(nodes):
        engine.push(nodes)
    meta = np.asarray([tree, sol, best, rounds, model.node_bytes, rank, world], dtype=np.int64)
    path = _path(directory, rank, world)
    tmp = path + ".tmp.npz"
    np.savez(tmp, nodes=np.ascontiguousarray(nodes, dtype=np.uint8), meta=meta,
             model=np.asarray(json.dumps(model.describe())))
    os.replace(tmp, path)
    return path


def prune(directory: str, keep_world: int) -> None:
    """Remove checkpoint files of other world sizes (after every rank of the current
    world has written its file), so a later resume never sees mixed worlds."""
    for f in glob.glob(os.path.join(directory, "ckpt_rank*_of*.npz")):
        w = int(os.path.basename(f).split("_of")[1].split(".")[0])
        if w != keep_world:
            os.remove(f)


def load_all(directory: str, model) -> tuple[np.ndarray, int, int, int, int]:
    """All saved pools (concatenated in rank order) + summed counters, min incumbent,
    max rounds. Validates that the checkpoint belongs to `model`."""
    files = glob.glob(os.path.join(directory, "ckpt_rank*_of*.npz"))
    if not files:
        raise FileNotFoundError(f"no checkpoint in {directory}")
    worlds = {int(os.path.basename(f).split("_of")[1].split(".")[0]) for f in files}
    if len(worlds) != 1:
        raise ValueError(f"mixed checkpoints in {directory}: worlds {sorted(worlds)}")
    world = worlds.pop()
    nodes, tree, sol, best, rounds = [], 0, 0, 2**31 - 1, 0
    seen_rounds = set()
    for r in range(world):
        f = _path(directory, r, world)
        with np.load(f, allow_pickle=False) as z:
            meta = z["meta"]
            desc = json.loads(str(z["model"]))
            if desc != json.loads(json.dumps(model.describe())):
                raise ValueError(f"checkpoint {f} is for {desc}, not {model.describe()}")
            if int(meta[4]) != model.node_bytes:
                raise ValueError("node layout mismatch")
            nodes.append(np.array(z["nodes"]))
            tree += int(meta[0])
            sol += int(meta[1])
            best = min(best, int(meta[2]))
            rounds = max(rounds, int(meta[3]))
            seen_rounds.add(int(meta[3]))
    if len(seen_rounds) > 1:
        # a crash between two ranks' writes of one periodic checkpoint leaves files of
        # different rounds: resuming from them would lose or duplicate subtrees
        raise ValueError(f"inconsistent checkpoint in {directory}: ranks saved different rounds "
                         f"{sorted(seen_rounds)}")
    allnodes = np.concatenate(nodes) if nodes else np.zeros((0, model.node_bytes), np.uint8)
    return allnodes, tree, sol, best, rounds
