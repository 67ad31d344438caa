"""The oracle simulator on the scenarios the GPU parity tests use: every
scenario runs, behavioural invariants restated from the reference's
integration tests hold, and two runs are identical (determinism)."""
import numpy as np
import pytest

import scenarios


@pytest.mark.parametrize("name", sorted(set(scenarios.SCENARIOS) - set(scenarios.HEAVY)))
def test_scenario_runs_and_is_deterministic(oracle_path, name):
    a = scenarios.run(oracle_path, name)
    b = scenarios.run(oracle_path, name)
    assert scenarios.compare(a, b) == []
    c = a["counters"]
    assert c["hops"] > 0
    if name not in ("spam_graft", "spam_ihave", "spam_ihave_2t", "spam_invalid", "promise_flood",
                    "promise_flood_long"):  # no valid publishes
        assert c["published"] > 0 and c["deliveries"] > 0


def test_dense_gossipsub_delivers_everything(oracle_path):
    """TestDenseGossipsub (gossipsub_test.go:84-123): every subscriber receives
    every one of the 100 messages, exactly once."""
    a = scenarios.run(oracle_path, "gossipsub_dense")
    assert a["counters"]["published"] == 100
    assert a["counters"]["deliveries"] == 100 * 19
    for hops, frm in a["deliv"]:
        assert (hops >= 0).all()


def test_floodsub_delivers_everything(oracle_path):
    """TestBasicFloodsub-style (floodsub_test.go:130-167): all hosts get all messages."""
    a = scenarios.run(oracle_path, "floodsub_dense")
    assert a["counters"]["deliveries"] == 100 * 19


def test_gossipsub_mesh_degree_bounds(oracle_path):
    """After heartbeats every mesh has at most Dhi peers and, given >= Dlo
    candidates, at least Dlo (gossipsub.go:1359-1436)."""
    import ctypes
    from pubsub_amd import graphs
    e, hops = scenarios.SCENARIOS["gossipsub_dense_dhi"](oracle_path)
    e.step(hops)
    m = e.mesh()
    deg = np.array([int(np.sum(m[e.rowptr[u]:e.rowptr[u + 1]] & np.uint64(1))) for u in range(e.N)])
    assert deg.max() <= 12 + 6  # handleGraft accepts outbound GRAFTs past Dhi until the next heartbeat
    assert np.median(deg) >= 5


def test_negative_app_score_peers_are_graylisted(oracle_path):
    a = scenarios.run(oracle_path, "gossipsub_negative_app")
    # app score -150 gives score -150 < gossip threshold -100 but > graylist -300
    assert a["counters"]["deliveries"] > 0
    assert (a["scores"] <= -150).any()


def test_cut_honest_4t_reaches_the_sender_cut_mode(oracle_path):
    """cut_honest_4t is built to run the honest engine's phase B in its
    sender-cut instantiation (gs_engine.hip stepOne: cutMode bit 1 when more
    than MaxIHaveLength ids were published within the gossip bound of
    (HistoryGossip + 1) heartbeats + the delivery age + 2 hops, bit 0 only if
    one topic alone exceeds it).  The schedule must reach bit 1 for many hops
    and never bit 0, and the run must carry IHAVE/IWANT traffic there."""
    e, hops = scenarios.SCENARIOS["cut_honest_4t"](oracle_path)
    top, hop = e.sched_top, e.sched_hops
    bound = (5 + 1) * 10 + 3 * 10 + 2
    cut_hops = 0
    for h in range(hops):
        live = (hop >= h - bound) & (hop <= h)
        if live.sum() > 5000:
            cut_hops += 1
            assert np.bincount(top[live], minlength=4).max() <= 5000
    assert cut_hops >= 60, cut_hops
    e.step(hops)
    c = e.counters()
    assert c["ihave_sent"] > 0 and c["iwant_sent"] > 0 and c["deliveries"] == 9000 * 199


def test_cut_spill_16t_cuts_more_items_than_lds_holds(oracle_path):
    """cut_spill_16t must bring more over-length IHAVE items to one node in one
    hop than phase B keeps in LDS (GS_CUTS = 64), so the GPU runs its cut-table
    spill.  Traced IHAVE lists are cut to MaxIHaveLength (3) ids by the host
    (include/gs_trace.h); the gossip windows of this schedule hold ~11 ids per
    topic, so an item of 3 ids is a cut one."""
    from test_trace_rpc import run as trace_run, blocks, RECV
    from pubsub_amd import _abi
    _, _, ev = trace_run(oracle_path, "cut_spill_16t", [0, 7])
    per = {}
    for head, items in blocks(ev):
        if head["type"] != RECV:
            continue
        n = np.bincount(items["topic"][items["reason"] == _abi.GS_RPC_ITEM_IHAVE].astype(np.int64), minlength=16)
        key = (int(head["node"]), int(head["hop"]))
        per[key] = per.get(key, 0) + int((n >= 3).sum())
    assert max(per.values()) > 2 * 64, max(per.values())
