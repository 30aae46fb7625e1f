"""The production permutation-node LB1 / LB1_d expand kernel (instances of more than 50
jobs — 100 / 200 / 500-job buckets — and 20 / 50 jobs when front nodes are off), one
iteration over a window of random parents, against the host oracle: every child's bound
exactly, the surviving children the kernel wrote (lb < best, as a multiset of node bytes),
the leaves it counted and the incumbent after it (ref generate_children,
PFSP_lib.h:51-95; bounds c_bound_simple.c:144-244)."""
import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel
from dist_gpu_accelerated_tree_search_amd.utils import nodes as nd

pytestmark = pytest.mark.gpu
INT_MAX = 2**31 - 1


def _parents(jobs, n, seed, leaf_parents=3):
    rng = np.random.default_rng(seed)
    depths = rng.integers(0, jobs - 1, size=n)
    depths[:leaf_parents] = jobs - 1  # parents whose children are leaves
    perms = np.stack([rng.permutation(jobs) for _ in range(n)])
    return depths, perms


def _host_expand(model, depths, perms, best):
    """(bounds in parent order, surviving child nodes, leaves, incumbent) on the host."""
    jobs = model.jobs
    nodes = nd.pfsp_pack(depths, perms, jobs)
    bounds = model.child_bounds_cpu(nodes, INT_MAX)
    kids, leaves, inc, i = [], 0, best, 0
    for d, q in zip(depths, perms):
        d = int(d)
        for k in range(d, jobs):
            b = int(bounds[i])
            i += 1
            if d + 1 == jobs:
                leaves += 1
                inc = min(inc, b)
            elif b < best:
                c = q.copy()
                c[d], c[k] = c[k], c[d]
                kids.append((d + 1, c))
    kid_nodes = nd.pfsp_pack([k[0] for k in kids], [k[1] for k in kids], jobs) if kids else \
        np.zeros((0, nodes.shape[1]), np.uint8)
    return nodes, bounds, kid_nodes, leaves, inc


def _rows(a):
    return sorted(bytes(r) for r in np.ascontiguousarray(a))


@pytest.mark.parametrize("inst,n", [(61, 40), (75, 40), (85, 24), (95, 12), (105, 8), (111, 6), (14, 60), (35, 40)])
@pytest.mark.parametrize("mode", ["inf", "median"])
def test_lb1_expand_kernel_matches_host(inst, n, mode):
    model = PfspModel(inst, 1)
    depths, perms = _parents(model.jobs, n, inst)
    nodes = nd.pfsp_pack(depths, perms, model.jobs)
    all_b = model.child_bounds_cpu(nodes, INT_MAX)
    best = INT_MAX if mode == "inf" else int(np.median(all_b))
    nodes, bounds, kids, leaves, inc = _host_expand(model, depths, perms, best)
    H = ops.require_gpu(0)
    r = H.pfsp_lb1_expand_probe(model.jobs, model.machines, list(model.native.p), nodes, best, 0)
    assert np.array_equal(r["bounds"], bounds), f"ta{inst}: {(r['bounds'] != bounds).sum()} bound mismatches"
    assert r["children"].shape == kids.shape, (r["children"].shape, kids.shape)
    assert _rows(r["children"]) == _rows(kids)
    assert r["leaves"] == leaves and r["best"] == inc


def test_lb1_expand_kernel_chunk_boundaries():
    # more parents than one chunk holds (100-job chunks take 128 parents): children of every
    # chunk land in its own slot region and the per-chunk counts cover them all
    model = PfspModel(65, 1)
    depths, perms = _parents(model.jobs, 300, 5, leaf_parents=0)
    depths[:] = np.clip(depths, 80, 98)  # deep parents: few children each
    nodes, bounds, kids, leaves, inc = _host_expand(model, depths, perms, INT_MAX)
    r = ops.require_gpu(0).pfsp_lb1_expand_probe(model.jobs, model.machines, list(model.native.p), nodes, INT_MAX, 0)
    assert np.array_equal(r["bounds"], bounds)
    assert _rows(r["children"]) == _rows(kids) and r["leaves"] == 0
