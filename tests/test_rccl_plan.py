"""Transfer plan -> grouped point-to-point calls (csrc/core/dist_rounds.hpp p2p_calls), the
mapping the native RCCL transport issues inside one ncclGroupStart/End per round
(csrc/hip/rccl_transport.hpp). CPU only: every rank must derive matching sends and
receives from the same plan."""
import random

import pytest

from dist_gpu_accelerated_tree_search_amd import ops


def test_p2p_calls_single_pair():
    C = ops.cpu()
    plan = [(2, 0, 100)]
    assert C.p2p_calls(plan, 2) == [("send", 0, 0, 100)]
    assert C.p2p_calls(plan, 0) == [("recv", 2, 0, 100)]
    assert C.p2p_calls(plan, 1) == []


def test_p2p_calls_offsets_follow_plan_order():
    C = ops.cpu()
    # rank 1 donates to 0 and 3, receives from 2 (a rank may both send and receive
    # across different pairs of one plan)
    plan = [(1, 0, 10), (2, 1, 7), (1, 3, 5), (0, 0, 9), (4, 2, 0)]
    assert C.p2p_calls(plan, 1) == [("send", 0, 0, 10), ("recv", 2, 0, 7), ("send", 3, 10, 5)]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_p2p_calls_match_across_ranks(world):
    # from random steal-half plans (the native planner): every send of rank d to r has
    # exactly one receive on r from d of the same size, and each rank's blocks are dense
    C = ops.cpu()
    rng = random.Random(world)
    for _ in range(50):
        sizes = [rng.choice([0, 0, 3, 500, 10**6]) for _ in range(world)]
        plan = [tuple(t) for t in C.plan_transfers(sizes, 25, 50, 250000, 0, True, True)]
        calls = {r: C.p2p_calls(plan, r) for r in range(world)}
        sends = sorted((r, c[1], c[3]) for r in calls for c in calls[r] if c[0] == "send")
        recvs = sorted((c[1], r, c[3]) for r in calls for c in calls[r] if c[0] == "recv")
        assert sends == recvs
        for r in range(world):
            for kind in ("send", "recv"):
                offs = [(c[2], c[3]) for c in calls[r] if c[0] == kind]
                pos = 0
                for o, n in offs:
                    assert o == pos
                    pos += n
        # totals equal what the plan moves
        assert sum(c[3] for r in calls for c in calls[r] if c[0] == "send") == sum(t[2] for t in plan)


def test_plan_caps_donation_at_exportable_amount():
    # a rank with a replay in flight reports its real pool (8000: a donor) and what it
    # can export without waiting (1000): the plan asks no more than that of it
    C = ops.cpu()
    sizes = [8000, 0, 6000, 0]
    free = C.plan_transfers(sizes, 1000, 2000, 100000)
    assert free == [(0, 1, 4000), (2, 3, 3000)]
    capped = C.plan_transfers(sizes, 1000, 2000, 100000, give=[1000, 0, 6000, 0])
    assert capped == [(0, 1, 1000), (2, 3, 3000)]
    # the cap is per donor over the whole plan: a second receiver gets the rest of it
    twice = C.plan_transfers([9000, 0, 0], 1000, 2000, 100000, give=[3000, 0, 0])
    assert twice == [(0, 1, 3000)]
    with pytest.raises(ValueError):
        C.plan_transfers(sizes, 1000, 2000, 100000, give=[1, 2])
