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


@pytest.mark.parametrize("N,G", [(8, 1), (14, 1), (20, 3), (32, 1), (32, 4)])
def test_queens_labels_match_cpu(N, G):
    C = ops.cpu()
    nodes, _, _ = C.queens_bfs(N, 1, 2000 if N > 10 else 100)
    assert len(nodes) > 0 and int(nd.queens_unpack(nodes)[3].max()) >= 2
    model = QueensModel(N, G)
    assert np.array_equal(model.labels_gpu(nodes), model.labels_cpu(nodes))


@pytest.mark.parametrize("inst,best_from", [(3, None), (14, None), (21, None), (56, None), (81, None), (91, None),
                                            (101, None), (111, None), (14, "opt"), (56, "opt"), (21, "opt"),
                                            (111, "opt")])
@pytest.mark.parametrize("variant", [1, 2, 4])
def test_lb2_expand_path_matches_cpu(inst, best_from, variant):
    # the production LB2 expand kernel (B1 LB1 filter, learned pair order, B2 walks:
    # rounds (1), dense (2), rounds of packed two-child walks (4);
    # B3 decision) against cpu_lb2 child by child: exact values when best = INT_MAX,
    # the lb < best decision otherwise
    model = PfspModel(inst, 2)
    if variant == 4 and (model.jobs + model.machines - 1) * max(model.native.p) >= 65536:
        pytest.skip("packed walks need 16-bit walk values (lb2_pk_ok)")
    n = {20: 600, 50: 200, 100: 40}.get(model.jobs, 12)
    nodes = random_nodes(model.jobs, n, inst * 7 + variant)
    best = INT_MAX if best_from is None else model.best_known
    H = ops.require_gpu(0)
    gpu = H.pfsp_expand_probe(model.jobs, model.machines, list(model.native.p), 2, nodes, best, 0, variant)
    cpu = model.child_bounds_cpu(nodes, INT_MAX)
    assert gpu.shape == cpu.shape
    if best == INT_MAX:
        assert np.array_equal(gpu, cpu), f"{(gpu != cpu).sum()} mismatches"
    else:
        assert np.array_equal(gpu < best, cpu < best), f"{((gpu < best) != (cpu < best)).sum()} decisions differ"
        below = cpu < best
        assert np.array_equal(gpu[below], cpu[below])


@pytest.mark.parametrize("inst", [101, 111])
def test_lb2_bounds_large_buckets(inst):
    model = PfspModel(inst, 2)
    nodes = random_nodes(model.jobs, 4, inst)
    assert np.array_equal(model.child_bounds_gpu(nodes), model.child_bounds_cpu(nodes))
    H = ops.require_gpu(0)
    gpu = H.pfsp_expand_probe(model.jobs, model.machines, list(model.native.p), 2, nodes, INT_MAX, 0, 1)
    assert np.array_equal(gpu, model.child_bounds_cpu(nodes))


@pytest.mark.parametrize("machines", [2, 3, 7, 13, 17])
@pytest.mark.parametrize("lb", [1, 2])
def test_other_machine_counts_match_cpu(machines, lb):
    # machine counts outside Taillard's 5/10/20 run in the next kernel bucket with
    # zero-time padding machines: bounds, the LB2 expand path and whole trees must
    # equal the host oracle's for the real instance
    from dist_gpu_accelerated_tree_search_amd import solve_cpu, solve_gpu

    model = PfspModel.synthetic(12, machines, 100 + machines, lb=lb)
    nodes = random_nodes(12, 300, machines)
    assert np.array_equal(model.child_bounds_gpu(nodes), model.child_bounds_cpu(nodes))
    if lb == 2:
        H = ops.require_gpu(0)
        gpu = H.pfsp_expand_probe(12, machines, list(model.native.p), 2, nodes, INT_MAX, 0, 1)
        assert np.array_equal(gpu, model.child_bounds_cpu(nodes))
    ref = solve_cpu(model, ub=0)
    got = solve_gpu(model, ub=0)
    assert got.best == ref.best
    bk = PfspModel.synthetic(12, machines, 100 + machines, lb=lb)
    bk.best_known = ref.best  # -u 1 with the optimum: deterministic tree
    r1, g1 = solve_cpu(bk, ub=1), solve_gpu(bk, ub=1)
    assert (g1.tree, g1.sol, g1.best) == (r1.tree, r1.sol, r1.best)


@pytest.mark.parametrize("inst,n", [(3, 300), (14, 300), (56, 120), (81, 40), (95, 16), (111, 6)])
@pytest.mark.parametrize("variant", [1, 4])
def test_lb2_expand_writes_the_surviving_children(inst, n, variant):
    # what the LB2 expand iteration WRITES (phase C compaction), not only its bounds: the
    # children with LB2 < best as a multiset of node bytes, the leaves counted, the incumbent
    model = PfspModel(inst, 2)
    if variant == 4 and (model.jobs + model.machines - 1) * max(model.native.p) >= 65536:
        pytest.skip("packed walks need 16-bit walk values (lb2_pk_ok)")
    rng = np.random.default_rng(inst * 3 + variant)
    depths = rng.integers(0, model.jobs - 1, size=n)
    depths[:2] = model.jobs - 1  # two parents of leaves
    perms = np.stack([rng.permutation(model.jobs) for _ in range(n)])
    nodes = nd.pfsp_pack(depths, perms, model.jobs)
    cpu = model.child_bounds_cpu(nodes, INT_MAX)
    best = int(np.median(cpu))
    kids, leaves, inc, i = [], 0, best, 0
    for d, q in zip(depths, perms):
        for k in range(int(d), model.jobs):
            b = int(cpu[i])
            i += 1
            if d + 1 == model.jobs:
                leaves += 1
                inc = min(inc, b)
            elif b < best:
                c = q.copy()
                c[d], c[k] = c[k], c[d]
                kids.append(bytes(nd.pfsp_pack([d + 1], [c], model.jobs)[0]))
    r = ops.require_gpu(0).pfsp_expand_probe_out(model.jobs, model.machines, list(model.native.p), nodes, best, 0, variant)
    got = sorted(bytes(x) for x in np.ascontiguousarray(r["children"]))
    assert got == sorted(kids), (len(got), len(kids))
    assert r["leaves"] == leaves and r["best"] == inc
    below = cpu < best
    assert np.array_equal(r["bounds"][below], cpu[below])
