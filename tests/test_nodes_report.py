"""Node layouts and reference-format outputs (CSV schemas, stdout blocks)."""
import numpy as np

from dist_gpu_accelerated_tree_search_amd import ops
from dist_gpu_accelerated_tree_search_amd.utils import nodes as nd
from dist_gpu_accelerated_tree_search_amd.utils import report


def test_node_bytes_match_native():
    C = ops.cpu()
    for jobs in (5, 20, 21, 50, 100, 200, 500):
        assert nd.pfsp_node_bytes(jobs) == C.pfsp_node_bytes(jobs)
    assert nd.pfsp_node_bytes(20) == 32 and nd.pfsp_node_bytes(500) == 1008
    assert C.queens_node_bytes() == nd.QUEENS_NODE_BYTES == 16


def test_pack_roundtrip():
    rng = np.random.default_rng(0)
    for jobs in (20, 50, 500):
        perms = np.stack([rng.permutation(jobs) for _ in range(5)])
        depths = rng.integers(0, jobs, 5)
        a = nd.pfsp_pack(depths, perms, jobs)
        assert a.shape == (5, nd.pfsp_node_bytes(jobs))
        d, p = nd.pfsp_unpack(a, jobs)
        assert np.array_equal(d, depths) and np.array_equal(p, perms)
    q = nd.queens_pack([1, 2], [3, 4], [5, 6], [7, 8])
    assert [x.tolist() for x in nd.queens_unpack(q)] == [[1, 2], [3, 4], [5, 6], [7, 8]]


def test_bfs_nodes_are_valid_children():
    C = ops.cpu()
    inst = C.PfspInstance.taillard(14)
    nodes, tree, sol, best = C.pfsp_bfs(inst, 0, 1377, 100)
    assert len(nodes) >= 100 and tree > 0 and best == 1377
    # LB1_d on 20 jobs: front nodes (depth, unscheduled set, fronts)
    d, rest, fr = nd.pfsp_front_unpack(nodes, 10)
    for depth, r in zip(d, rest):
        assert bin(int(r)).count("1") == 20 - depth
    assert (fr[:, 1:] >= fr[:, :-1]).all()  # completion times grow along the machines
    # draining the warm-up frontier completes the golden tree
    t2, s2, b2 = C.pfsp_drain(inst, 0, 1377, nodes)
    assert (tree + t2, sol + s2, b2) == (2573652, 2648, 1377)


def test_cpu_engine_contract():
    C = ops.cpu()
    inst = C.PfspInstance.taillard(14)
    e = C.make_pfsp_cpu_engine(inst, 0, 512, 2)
    nodes, tree, sol, _ = C.pfsp_bfs(inst, 0, 1377, 64)
    e.best = 1377
    e.push(nodes)
    assert e.size() == len(nodes)
    part = e.pop(10)
    assert part.shape == (10, 32) and e.size() == len(nodes) - 10
    e.push(part)
    e.run(max_launches=3)
    e.run()
    st = e.stats()
    assert (st["tree"] + tree, st["sol"] + sol, e.size()) == (2573652, 2648, 0)


def test_stdout_blocks():
    s = report.pfsp_results(1377, 2573652, 2648, 0.12345)
    assert s.splitlines()[2:6] == ["Size of the explored tree: 2573652", "Number of explored solutions: 2648",
                                   "Optimal makespan: 1377", "Elapsed time: 0.1235 [s]"]
    st = report.pfsp_settings(14, 10, 20, 1, 1, 0, 0, 0, 1, 0, 0)
    assert "Resolution of PFSP Taillard's instance: ta14 (m = 10, n = 20)" in st
    assert "Lower bound function: lb1" in st and "Initial upper bound: opt" in st and "Branching rule: fwd" in st


def test_csv_formats(tmp_path):
    w = [report.WorkerStats(tree=5, sol=1, gen_child=5, steals=2, success_steals=1, terminations=3, t_kernel=0.5),
         report.WorkerStats(tree=7)]
    p = tmp_path / "multigpu.csv"
    report.write_multi_gpu_csv(str(p), 14, 1, 2, 0, 1, 1377, 25, 50000, 5000, 1.23456, 12, 1, w)
    report.write_multi_gpu_csv(str(p), 14, 1, 2, 0, 1, 1377, 25, 50000, 5000, 1.0, 12, 1, w)
    lines = p.read_text().splitlines()
    assert lines[0] == report.MULTI_HEADER.strip()
    assert len(lines) == 3
    assert lines[1].startswith('14,2,0,1,1,1377,25,50000,5000,1.2346,12,1,"[5,7]","[1,0]","[5,0]","[2,0]","[1,0]",')
    assert lines[1].endswith('"[0.0000,0.0000]",')  # reference rows end with a trailing comma
    s = tmp_path / "singlegpu.csv"
    report.write_single_gpu_csv(str(s), 14, 1, 1377, 25, 50000, 0.5, 0.1, 0.2, 0.3, 0.4, 10, 2)
    assert s.read_text().splitlines()[1] == "14,1,1377,25,50000,0.5000,0.1000,0.2000,0.3000,0.4000,10,2"
    d = tmp_path / "dist.csv"
    report.write_dist_multi_gpu_csv(str(d), 14, 1, 1, 0, 1, 2, 1377, 25, 50000, 5000, 1.0, 12, 1, w, [3, 4], [0.1, 0.2])
    row = d.read_text().splitlines()[1]
    assert row.startswith("14,1,0,2,1,1,1377,25,50000,5000,1.0000,12,1,") and '"[3,4]"' in row


def test_cli_defaults_match_the_reference():
    # ref pfsp/lib/PFSP_lib.c:175-185: inst 14, lb 1, ub 1, m 25, M 50000, T 5000, D 1, C 1, ws 1, L 1, perc 50
    from dist_gpu_accelerated_tree_search_amd.cli import _pfsp_parser

    a = _pfsp_parser().parse_args([])
    assert (a.inst, a.lb, a.ub, a.m, a.M, a.T, a.D, a.C, a.ws, a.L, a.perc) == \
        (14, 1, 1, 25, 50000, 5000, 1, 1, 1, 1, 50)


def test_dist_csv_uses_measured_load_balancing(tmp_path):
    from dist_gpu_accelerated_tree_search_amd.utils import report

    ws = [report.WorkerStats(tree=10, sol=1, gen_child=10, steals=3, success_steals=2, terminations=1,
                             dist_load_bal=2, t_load_bal=0.25),
          report.WorkerStats(tree=20, sol=0, gen_child=20, steals=0, success_steals=0, terminations=0,
                             dist_load_bal=0, t_load_bal=0.0)]
    path = tmp_path / "dist.csv"
    report.write_dist_multi_gpu_csv(str(path), 14, 1, 1, 0, 1, 2, 1377, 25, 50000, 5000, 0.5, 30, 1, ws,
                                    [w.dist_load_bal for w in ws], [w.t_load_bal for w in ws])
    row = path.read_text().splitlines()[1]
    assert '"[2,0]",' in row and '"[0.2500,0.0000]",' in row and '"[3,0]",' in row
