"""Connection churn and subscription changes on the oracle (gs_schedule_events):
the reference's own assertions restated on the simulator.
  TestGossipsubRemovePeer (gossipsub_test.go:629-676): hosts 0-4 close; every
    later message reaches hosts 5-19.
  TestGossipsubPrune (gossipsub_test.go:535-582): hosts 0-4 leave the topic; every
    later message reaches hosts 5-19, and the ones that left get nothing new.
  TestGossipsubGraft (gossipsub_test.go:584-627): hosts subscribe one by one on a
    sparse graph; every message reaches every host.
  TestScoreRetention (score_test.go:861-903) at the simulator level: a dropped
    connection's record stays (with its negative score) for RetainScore, then
    reads 0.
The GPU engine is compared with the oracle on the same scenarios in
tests/test_parity_gpu.py."""
import numpy as np
import pytest

import scenarios
from pubsub_amd import GS_EV_CONNECT, GS_EV_DISCONNECT, GS_EV_LEAVE, NewGossipSub, Second, WithHop, \
    WithPeerScore, WithRecordDeliveries, eth2_peer_score_params, eth2_thresholds
from pubsub_amd import graphs


def _received(e, ids, nodes):
    got = np.zeros((len(ids), len(nodes)), dtype=bool)
    for i, m in enumerate(ids):
        hop, _ = e.deliveries(int(m))
        got[i] = hop[list(nodes)] >= 0
    return got


def test_remove_peer(oracle_path):
    e, hops = scenarios.SCENARIOS["churn_remove_peer"](oracle_path)
    e.step(hops)
    assert _received(e, range(10), range(5, 20)).all()
    # the closed hosts are out of every mesh: no mesh bit on any of their edges
    mesh = e.mesh()
    src = np.repeat(np.arange(e.N), np.diff(e.rowptr))
    touch = (src < 5) | (e.col < 5)
    assert not mesh[touch].any()


def test_prune_after_leave(oracle_path):
    e, hops = scenarios.SCENARIOS["churn_prune"](oracle_path)
    e.step(hops)
    assert _received(e, range(10), range(5, 20)).all()
    for m in range(10):                                   # unsubscribed: only their own publishes
        hop, frm = e.deliveries(m)
        assert all(frm[u] == -1 for u in range(5) if hop[u] >= 0)
    mesh = e.mesh()
    src = np.repeat(np.arange(e.N), np.diff(e.rowptr))
    assert not mesh[(src < 5) | (e.col < 5)].any()       # PRUNEd on both ends


def test_graft_on_late_join(oracle_path):
    e, hops = scenarios.SCENARIOS["churn_graft"](oracle_path)
    e.step(hops)
    assert _received(e, range(100), range(20)).all()
    deg = np.bitwise_count(e.mesh()).reshape(-1)
    assert deg.sum() > 0


def test_score_retention(oracle_path):
    """A peer with AppSpecificScore -1000 disconnects: its record is retained
    (score -1000 x weight) until RetainScore passes, then reads 0."""
    n = 2
    rowptr = np.array([0, 1, 2], dtype=np.int64)
    col = np.array([1, 0], dtype=np.int32)
    out = np.array([1, 0], dtype=np.uint8)
    sp = eth2_peer_score_params(1)
    sp.RetainScore = 1 * Second
    sp.AppSpecificWeight = 1.0
    app = np.array([0.0, -1000.0])
    e = NewGossipSub(n, 1, (rowptr, col, out), graphs.all_subscribed(n, 1), WithPeerScore(sp, eth2_thresholds()),
                     WithHop(100 * 1000 * 1000), app_score=app, lib=oracle_path)
    e.schedule_events([GS_EV_DISCONNECT], [0], [1], [3])
    e.step(3)
    assert e.scores()[0] < -900          # connected
    e.step(1)
    assert e.scores()[0] < -900          # disconnected, retained
    e.step(16)
    assert e.scores()[0] < -900          # hop 20: the refresh at 2.0 s has not run yet
    e.step(1)
    assert e.scores()[0] == 0.0          # the refresh at 2.0 s > expire (1.3 s) dropped the record


def test_reconnect_restores_mesh(oracle_path):
    e, hops = scenarios.SCENARIOS["churn_scored"](oracle_path)
    e.step(hops)
    c = e.counters()
    assert c["deliveries"] > 0.9 * 400 * e.N * 0.5
    # every connection is back up at the end of the schedule: meshes are formed
    assert np.bitwise_count(e.mesh()).sum() > e.N


def test_bad_events(oracle_path):
    from pubsub_amd import GossipEngineError
    e, _ = scenarios.SCENARIOS["churn_prune"](oracle_path)
    with pytest.raises(GossipEngineError):
        e.schedule_events([GS_EV_DISCONNECT], [0], [0], [30])   # not a connection
    with pytest.raises(GossipEngineError):
        e.schedule_events([GS_EV_LEAVE], [0], [5], [30])        # no topic 5
    with pytest.raises(GossipEngineError):
        e.schedule_events([GS_EV_CONNECT], [0], [1], [1])       # before the last scheduled hop


def test_churn_with_the_peer_gater(oracle_path):
    """Connection churn with the peer gater (peer_gater.go:366-383 AddPeer /
    RemovePeer, decayStats :219-259 with a 2 s RetainStats): the adversarial
    mix keeps throttling and gating while connections come and go."""
    e, hops = scenarios.SCENARIOS["churn_gater"](oracle_path)
    e.step(hops)
    c = e.counters()
    assert c["throttled"] > 0 and c["gated"] > 0 and c["graylisted"] > 0, c
    assert c["deliveries"] > 0
