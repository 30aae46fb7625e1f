"""N-Queens backtracking model (the reference's proof of concept).

Parity: ref nqueens/nqueens_c.c (isSafe + decompose, :80-117), nqueens_gpu_cuda.cu
(evaluate_gpu labels kernel, :143-171), nqueens_multigpu_cuda.cu (multi-GPU
driver). Counting rules are the reference's: every pushed safe child counts in the
tree, a node popped at depth N counts as a solution; -g repeats the safety test.
"""
from __future__ import annotations

import numpy as np

from .. import ops
from ..utils import nodes as nodes_mod
from .pfsp import EngineOptions, make_multi


class QueensModel:
    kind = "nqueens"

    def __init__(self, N: int = 14, G: int = 1):
        if not 1 <= N <= 32:
            raise ValueError("N-Queens supports 1 <= N <= 32")
        if G < 1:
            raise ValueError("g must be >= 1")
        self.N = int(N)
        self.G = int(G)
        self.node_bytes = nodes_mod.QUEENS_NODE_BYTES
        self.lb = 0

    def initial_best(self, ub: int = 1) -> int:  # no incumbent in a counting problem
        return 0

    def search_best(self, ub: int = 1) -> int:
        return 0

    def root(self) -> np.ndarray:
        return nodes_mod.queens_pack([0], [0], [0], [0])

    def warmup(self, best: int, target: int):
        nodes, tree, sol = ops.cpu().queens_bfs(self.N, self.G, int(target))
        return nodes, tree, sol, best

    def drain(self, best: int, nodes: np.ndarray):
        tree, sol = ops.cpu().queens_drain(self.N, self.G, np.ascontiguousarray(nodes, dtype=np.uint8))
        return tree, sol, best

    def make_engine(self, backend: str = "gpu", device: int = 0, opts: EngineOptions | None = None):
        opts = opts or EngineOptions(max_parents=1 << 20)
        if opts.streams > 1:
            return make_multi(self, backend, device, opts)
        if backend == "cpu":
            return ops.cpu().make_queens_cpu_engine(self.N, self.G, opts.cpu_batch, opts.cpu_threads)
        if backend != "gpu":
            raise ValueError(f"unknown backend {backend!r}")
        H = ops.require_gpu(device)
        return H.make_queens_engine(self.N, self.G, device=device, max_parents=opts.max_parents,
                                    ring_bytes=opts.ring_bytes, iters_small=opts.iters_small,
                                    iters_large=opts.iters_large, use_graphs=opts.use_graphs,
                                    iters_first=opts.iters_first)

    def make_hybrid(self, engine, backend: str, threads: int, m: int = 25, cap: int = 20000, batch: int = 5000):
        """`engine` plus a CPU worker of `threads` threads as one rank engine
        (csrc/core/hybrid_engine.hpp)."""
        mod = ops.hip() if backend == "gpu" else ops.cpu()
        cpu = mod.make_queens_cpu_engine(self.N, self.G, batch, threads)
        return mod.make_hybrid_engine(engine, cpu, m, cap)

    def labels_cpu(self, nodes: np.ndarray) -> np.ndarray:
        """labels[i, r] = 1 iff row r is free and diagonal-safe for parent i."""
        cols, diag, anti, depth = nodes_mod.queens_unpack(nodes)
        full = (1 << self.N) - 1
        out = np.zeros((len(cols), self.N), np.uint8)
        for i in range(len(cols)):
            if int(depth[i]) == self.N:
                continue
            av = ~(int(cols[i]) | int(diag[i]) | int(anti[i])) & full
            for r in range(self.N):
                out[i, r] = (av >> r) & 1
        return out

    def labels_gpu(self, nodes: np.ndarray, device: int = 0) -> np.ndarray:
        return ops.require_gpu(device).queens_labels(self.N, self.G, np.ascontiguousarray(nodes, np.uint8), device)

    def describe(self) -> dict:
        return {"problem": "nqueens", "N": self.N, "G": self.G, "layout": "bitmask"}
