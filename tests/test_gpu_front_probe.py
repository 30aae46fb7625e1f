"""Element-wise probe of the production LB1 / LB1_d front kernel.

`pfsp_front_probe` runs a complete engine solve with the kernel's probe records on:
every child bound evaluated by any iteration shape — one level per kernel, the rank
split iteration, multi-level chunks (child-parallel and thread-per-node levels with
carried packed-u16 remains), local DFS — is recorded with its parent and the parent's
remain as the kernel holds it, and checked on the host against PfspFrontProblem (ref
add_front_and_bound, c_bound_simple.c:219-244). The solve's tree / sol must equal the
CPU drain of the same start nodes.
"""
import os

import numpy as np
import pytest

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel

pytestmark = pytest.mark.gpu


def probe(model, nodes, best, **kw):
    H = ops.require_gpu(0)
    return H.pfsp_front_probe(model.jobs, model.machines, list(model.native.p), model.lb,
                              np.ascontiguousarray(nodes, dtype=np.uint8), best, **kw)


def check(r, kinds):
    assert r["records"] > 0
    assert r["checked"] == r["records"], "probe buffer too small"
    assert r["bad_job"] == 0 and r["bad_remain"] == 0 and r["bad_lb"] == 0, r
    for k in kinds:
        assert r["by_kind"][k] > 0, (k, r["by_kind"])


def start(model, best, target, take=None):
    nodes, t, s, b = model.warmup(best, target)
    if take is not None:  # the deepest (last) nodes: small subtrees
        nodes = nodes[-take:]
        t = s = 0
    return nodes, t, s, b


# (local_min 0: local DFS only on a backlog of four grid windows, so the wide levels run
# one level per kernel; the default local_min takes them local on a window of at least a
# resident grid of chunks, as the headline's 2^19)
@pytest.mark.parametrize("cfg,kinds", [
    ({}, ["child_parallel", "local_dfs"]),
    ({"local_min": 0}, ["child_parallel", "one_level"]),
    ({"deep_levels": 4, "local_min": 0}, ["child_parallel", "thread_per_node", "one_level"]),
    ({"fuse_max": 0}, ["one_level", "local_dfs"]),
    ({"deep_levels": 2}, ["child_parallel", "local_dfs"]),
    ({"deep_levels": 4, "deep_per3": 64, "deep_per4": 16, "max_parents": 1 << 13}, ["child_parallel", "thread_per_node"]),
    ({"wide_levels": 3, "local_min": 0}, ["one_level", "thread_per_node"]),
    ({"wide_levels": 2, "local_min": 0}, ["one_level", "thread_per_node"]),
])
def test_front_probe_ta014_every_shape(cfg, kinds):
    model = PfspModel(14, 1)
    nodes, t0, s0, best = start(model, 1377, 25)
    r = probe(model, nodes, best, cap=1 << 25, **{"max_parents": 1 << 19, **cfg})  # the headline window
    check(r, kinds)
    assert (r["tree"] + t0, r["sol"] + s0, r["best"]) == (2573652, 2648, 1377)


def test_front_probe_local_dfs():
    # local DFS iterations when the pool holds a backlog (TTS_LOCAL_MIN: from 1 parent)
    model = PfspModel(14, 0)
    nodes, t0, s0, best = start(model, 1377, 25)
    os.environ["TTS_LOCAL_MIN"] = "1"
    try:
        r = probe(model, nodes, best, cap=1 << 25, max_parents=1 << 12, fuse_max=0)
    finally:
        del os.environ["TTS_LOCAL_MIN"]
    check(r, ["local_dfs"])
    assert (r["tree"] + t0, r["sol"] + s0) == (2573652, 2648)


def test_front_probe_split_iteration():
    # two ranks of an in-graph split: both shares together are the whole tree
    model = PfspModel(14, 1)
    nodes, t0, s0, best = start(model, 1377, 25)
    tot_t = tot_s = 0
    for rank in (0, 1):
        r = probe(model, nodes, best, cap=1 << 25, split_rank=rank, split_world=2, split_min=2000)
        check(r, ["split"])
        tot_t += r["tree"]
        tot_s += r["sol"]
    assert (tot_t + t0, tot_s + s0) == (2573652, 2648)


@pytest.mark.parametrize("inst,target,take", [(21, 20000, 24), (1, 200000, 1), (11, 5000, 64), (61, 0, 0)])
def test_front_probe_machine_buckets(inst, target, take):
    # M = 20 (ta021), 5 (ta001), 10 (ta011) on deep subtrees; ta061 (100 jobs) has no front
    # layout (50-job instances do: test_front_probe_fifty_jobs)
    model = PfspModel(inst, 0)
    if not model.front_layout:
        with pytest.raises(Exception):
            probe(model, model.root(), model.best_known)
        return
    nodes, _, _, best = start(model, model.best_known, target, take)
    r = probe(model, nodes, best, cap=1 << 25)
    check(r, [])
    tree, sol, _ = model.drain(best, nodes)
    assert (r["tree"], r["sol"]) == (tree, sol)


def test_front_probe_synthetic_machine_padding():
    # 7 machines run in the 10-machine bucket with zero-time padding machines
    model = PfspModel.synthetic(14, 7, seed=3, lb=1)
    opt = model.drain(2**31 - 1, model.root())[2]  # the optimum, then a -u 1 style solve
    nodes, _, _, best = start(model, opt, 25)
    r = probe(model, nodes, best, cap=1 << 24)
    check(r, [])
    tree, sol, _ = model.drain(best, nodes)
    assert (r["tree"], r["sol"], r["best"]) == (tree, sol, opt)


def _ta021_samples():
    import json
    from pathlib import Path

    d = json.loads((Path(__file__).parent / "fixtures" / "ta021_subtrees.json").read_text())
    nodes = np.stack([np.frombuffer(bytes.fromhex(s["node"]), dtype=np.uint8) for s in d["samples"]])
    return d, nodes


def test_ta021_subtree_parity_gpu_vs_host():
    # 64 sampled ta021 LB1_d subtrees (32 at depth 4, 32 at depth 6; 71.6 M nodes in all)
    # whose -u 1 counts the host engine computed (scripts/gen_ta021_subtrees.cpp): the
    # device solve of each must give the same tree and solution counts
    from dist_gpu_accelerated_tree_search_amd.models.pfsp import EngineOptions

    d, nodes = _ta021_samples()
    model = PfspModel(21, 0)
    assert model.node_bytes == d["node_bytes"] == nodes.shape[1]
    eng = model.make_engine("gpu", 0, EngineOptions(max_parents=1 << 16, ring_bytes=4 << 30))
    bad = []
    for i, s in enumerate(d["samples"]):
        eng.begin(nodes[i:i + 1], d["best"])
        eng.run()
        st = eng.stats()
        if (st["tree"], st["sol"]) != (s["tree"], s["sol"]):
            bad.append((i, s["depth"], (st["tree"], st["sol"]), (s["tree"], s["sol"])))
    assert not bad, bad
    # all 64 at once, with the probe records on for the depth-6 half
    r = probe(model, nodes[32:], d["best"], cap=1 << 25)
    check(r, [])
    assert (r["tree"], r["sol"]) == (sum(s["tree"] for s in d["samples"][32:]), sum(s["sol"] for s in d["samples"][32:]))


@pytest.mark.parametrize("gap,dyn_us", [(170, 0), (155, 0), (155, 40)])
def test_front_probe_fifty_jobs(gap, dyn_us):
    # 50-job front nodes (64-bit job sets, 64-B nodes for 20 machines) on ta051 LB1_d with
    # an incumbent below the optimum: every bound the kernel evaluates against the host
    # oracle, and the tree against the host drain of the same start nodes
    model = PfspModel(51, 0)
    assert model.front_layout and model.node_bytes == 64
    nodes, _, _, best = model.warmup(model.best_known - gap, 25)
    r = probe(model, nodes, best, cap=1 << 25, max_parents=1 << 19, dyn_us=dyn_us)
    check(r, [])
    tree, sol, _ = model.drain(best, nodes)
    assert (r["tree"], r["sol"]) == (tree, sol)
