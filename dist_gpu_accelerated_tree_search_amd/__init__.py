"""MI355X-native distributed GPU-accelerated tree search (Branch-and-Bound).

Problems: PFSP on Taillard's instances (LB1, LB1_d, LB2) and N-Queens.
Backends: C++ host core (sequential / multi-core work stealing), gfx950 HIP device
engines (device-resident pools, fused bound/prune/compact kernels, hipGraphs), and
a one-process-per-GPU distributed runtime over torch.distributed (RCCL / gloo).

Quick start:
    from dist_gpu_accelerated_tree_search_amd import PfspModel, solve_gpu
    r = solve_gpu(PfspModel(14, lb=1))     # tree 2,573,652, makespan 1377
"""
__version__ = "0.1.0"

from .models.nqueens import QueensModel  # noqa: E402,F401
from .models.pfsp import EngineOptions, PfspModel  # noqa: E402,F401
from .search import SolveResult, solve_cpu, solve_engine, solve_gpu, solve_workers  # noqa: E402,F401
