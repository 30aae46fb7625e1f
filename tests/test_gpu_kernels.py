"""gfx950 kernels vs the host oracle (exact integer equality), ref evaluate_gpu semantics."""
import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.nqueens import QueensModel
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel
from dist_gpu_accelerated_tree_search_amd.utils import nodes as nd

pytestmark = pytest.mark.gpu
INT_MAX = 2**31 - 1


def random_nodes(jobs, n, seed):
    rng = np.random.default_rng(seed)
    depths = rng.integers(0, jobs, size=n)
    perms = np.stack([rng.permutation(jobs) for _ in range(n)])
    return nd.pfsp_pack(depths, perms, jobs)


def test_extension_is_native_and_on_gfx950():
    H = ops.require_gpu(0)
    info = H.device_info(0)
    assert info["arch"].startswith("gfx950"), info
    assert info["compute_units"] >= 256 and info["warp_size"] == 64
    assert H.__file__.endswith(".so") and "dist_gpu_accelerated_tree_search_amd" in H.__file__


# instances covering every node bucket up to 100 jobs and all machine counts
@pytest.mark.parametrize("inst", [1, 14, 21, 31, 45, 56, 61, 75, 85])
@pytest.mark.parametrize("lb", [0, 1, 2])
def test_pfsp_bounds_match_cpu(inst, lb):
    model = PfspModel(inst, lb)
    n = 400 if model.jobs <= 50 else 60
    nodes = random_nodes(model.jobs, n, inst * 10 + lb)
    for best in (INT_MAX, model.best_known):
        if lb != 2 and best != INT_MAX:
            continue
        cpu = model.child_bounds_cpu(nodes, best)
        gpu = model.child_bounds_gpu(nodes, best)
        assert gpu.shape == cpu.shape
        assert np.array_equal(gpu, cpu), f"ta{inst} lb{lb} best={best}: {(gpu != cpu).sum()} mismatches"


@pytest.mark.parametrize("inst", [101, 111])
def test_pfsp_bounds_large_buckets(inst):
    model = PfspModel(inst, 1)
    nodes = random_nodes(model.jobs, 8, inst)
    assert np.array_equal(model.child_bounds_gpu(nodes), model.child_bounds_cpu(nodes))


def test_pfsp_bounds_root_and_leaf_parents():
    model = PfspModel(14, 1)
    root = nd.pfsp_root(20)
    assert np.array_equal(model.child_bounds_gpu(root), model.child_bounds_cpu(root))
    deep = random_nodes(20, 50, 1)
    deep[:, 0] = 19  # one child each, all leaves
    assert np.array_equal(model.child_bounds_gpu(deep), model.child_bounds_cpu(deep))


@pytest.mark.parametrize("N,G", [(8, 1), (14, 1), (20, 3), (32, 1)])
def test_queens_labels_match_cpu(N, G):
    C = ops.cpu()
    nodes, _, _ = C.queens_bfs(min(N, 12), 1, 2000)
    model = QueensModel(min(N, 12), G)
    assert np.array_equal(model.labels_gpu(nodes), model.labels_cpu(nodes))
