"""Front-carrying PFSP nodes (csrc/core/pfsp_front.hpp): the layout every engine uses
for LB1 / LB1_d on instances of up to 20 jobs. The host problem is the oracle of the
GPU kernel (pfsp_front_kernels.hpp); here it is checked against the permutation-node
bounds (themselves checked against brute force in test_bounds.py) and for identical
trees with the permutation layout (TTS_FRONT=0)."""
import os

import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel
from dist_gpu_accelerated_tree_search_amd.utils import nodes as nd


def random_perm_nodes(jobs, n, seed, dmax=None):
    rng = np.random.default_rng(seed)
    depths = rng.integers(0, (dmax or jobs - 1) + 1, size=n)
    perms = np.stack([rng.permutation(jobs) for _ in range(n)])
    return nd.pfsp_pack(depths, perms, jobs), depths, perms


def test_layout_sizes():
    C = ops.cpu()
    assert PfspModel(14, 1).node_bytes == 32 and PfspModel(14, 1).front_layout   # 20 x 10
    assert PfspModel(7, 0).node_bytes == 32                                        # 20 x 5
    assert PfspModel(21, 0).node_bytes == 48                                       # 20 x 20
    assert PfspModel(14, 2).node_bytes == 32 and not PfspModel(14, 2).front_layout  # LB2: permutation
    assert PfspModel(56, 1).node_bytes == 64 and PfspModel(56, 1).front_layout      # 50 x 20: 64-bit job set
    assert PfspModel(31, 0).node_bytes == 32 and PfspModel(31, 0).front_layout      # 50 x 5
    assert PfspModel(41, 1).node_bytes == 48                                        # 50 x 10
    assert PfspModel(56, 2).node_bytes == 64 and not PfspModel(56, 2).front_layout  # LB2: permutation
    assert PfspModel(61, 1).node_bytes == 112 and not PfspModel(61, 1).front_layout  # 100 jobs: permutation
    r50 = PfspModel(51, 0).root()
    d, rest, fr = nd.pfsp_front_unpack(r50, 20, jobs=50)
    assert d[0] == 0 and int(rest[0]) == (1 << 50) - 1
    assert list(fr[0]) == list(C.PfspInstance.taillard(51).min_heads)
    root = PfspModel(21, 0).root()
    d, rest, fr = nd.pfsp_front_unpack(root, 20)
    inst = C.PfspInstance.taillard(21)
    assert d[0] == 0 and rest[0] == (1 << 20) - 1 and list(fr[0]) == list(inst.min_heads)


@pytest.mark.parametrize("spec", [(14, None), (7, None), (21, None), (None, (20, 7, 3)), (None, (20, 13, 4)),
                                  (None, (16, 2, 5)), (None, (12, 20, 6)), (31, None), (41, None), (51, None),
                                  (None, (21, 4, 8)), (None, (35, 9, 9)), (None, (50, 17, 10))])
def test_front_bounds_equal_permutation_bounds(spec):
    inst, syn = spec
    model = PfspModel(inst, 0) if inst else PfspModel.synthetic(*syn, lb=0)
    assert model.front_layout
    C = ops.cpu()
    perm_nodes, depths, perms = random_perm_nodes(model.jobs, 200, 11)
    ref = model.child_bounds_cpu(perm_nodes)  # child order k = depth..N-1
    front = model.to_engine_layout(perm_nodes)
    got = np.asarray(C.pfsp_children_bounds(model.native, 0, front))  # ascending job order
    off = 0
    for d, q in zip(depths, perms):
        kids = list(q[d:])
        mine = ref[off:off + len(kids)]
        by_job = dict(zip(kids, mine))
        assert list(got[off:off + len(kids)]) == [by_job[j] for j in sorted(kids)]
        off += len(kids)
    assert off == len(got)


@pytest.mark.parametrize("inst,lb,gold", [(14, 1, (2573652, 2648, 1377)), (7, 0, (271602, 28447, 1234)),
                                          (4, 1, (1163892, 941, 1293))])
def test_front_trees_equal_permutation_trees(inst, lb, gold, monkeypatch):
    C = ops.cpu()
    native = C.PfspInstance.taillard(inst)
    got = {}
    for front in ("1", "0"):
        monkeypatch.setenv("TTS_FRONT", front)
        r = C.run_pfsp(native, lb, native.best_known, threads=0)
        got[front] = (r["tree"], r["sol"], r["best"])
    assert got["1"] == got["0"] == gold


def test_front_trees_twenty_machines():
    # 12 jobs x 20 machines: the 48-byte node, same tree as the permutation layout
    # (with the optimum as the initial bound: with +inf the tree depends on the child order)
    model = PfspModel.synthetic(12, 20, 9, lb=0)
    C = ops.cpu()
    opt = C.run_pfsp(model.native, 0, 2**31 - 1, threads=0)["best"]
    res = []
    for front in ("1", "0"):
        os.environ["TTS_FRONT"] = front
        try:
            r = C.run_pfsp(model.native, 0, opt, threads=0)
        finally:
            os.environ.pop("TTS_FRONT", None)
        res.append((r["tree"], r["sol"], r["best"]))
    assert res[0] == res[1] and res[0][0] > 1000 and res[0][2] == opt


def test_front_children_of_the_root_start_from_zero():
    # the root's front holds the minimum heads (its children's bounds use them) but a
    # child's front is the job's own completion times from 0 (ref schedule_front)
    C = ops.cpu()
    model = PfspModel(14, 1)
    e = model.make_engine("cpu")
    e.begin(model.root(), 2**31 - 1)
    e.run(max_launches=1)
    kids = e.pop(100)
    d, rest, fr = nd.pfsp_front_unpack(kids, 10)
    p = np.asarray(model.native.p).reshape(model.machines, model.jobs)
    assert len(kids) == 20 and (d == 1).all()
    for r, f in zip(rest, fr):
        j = [x for x in range(20) if not (int(r) >> x) & 1][0]
        assert list(f) == list(np.cumsum(p[:, j]))


@pytest.mark.parametrize("gap,gold", [(170, 5553), (160, None)])
def test_front_trees_fifty_jobs(gap, gold, monkeypatch):
    # 50-job front nodes (64-bit job sets) against the permutation layout on ta051 LB1_d
    # with an incumbent below the optimum (the -u 1 tree is far too large for a test)
    C = ops.cpu()
    native = C.PfspInstance.taillard(51)
    got = {}
    for front in ("1", "0"):
        monkeypatch.setenv("TTS_FRONT", front)
        r = C.run_pfsp(native, 0, native.best_known - gap, threads=2)
        got[front] = (r["tree"], r["sol"], r["best"])
    assert got["1"] == got["0"]
    if gold is not None:
        assert got["1"][0] == gold
