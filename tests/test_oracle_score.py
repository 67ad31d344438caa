"""Restates the reference's peerScore known-answer tests (score_test.go) on the
oracle's PeerScore object with a virtual clock: time.Sleep(d) becomes now += d.
Each test names the reference test it restates; expected values are the
reference's own literal/derived expectations (exact float equality where the
reference asserts equality)."""
import ctypes as C
import math

from pubsub_amd import _abi
from pubsub_amd.params import Millisecond, PeerScoreParams, Second, TopicScoreParams

A, B, Cp, D = 0, 1, 2, 3
MYTOPIC = 0


def mk(olib, params, topics):
    ps = olib.ops_new(C.byref(params.to_c()))
    for t, tp in topics.items():
        olib.ops_set_topic(ps, t, C.byref(tp.to_c()))
    return ps


def deliver_n(olib, ps, peer, n, now, start=0):
    for i in range(start, start + n):
        olib.ops_validate(ps, i, MYTOPIC, peer, now)
        olib.ops_deliver(ps, i, MYTOPIC, peer, now)


def test_score_time_in_mesh(olib):  # score_test.go:13-50
    p = PeerScoreParams(AppSpecificScore=True)
    tp = TopicScoreParams(TopicWeight=0.5, TimeInMeshWeight=1, TimeInMeshQuantum=Millisecond, TimeInMeshCap=3600)
    ps = mk(olib, p, {MYTOPIC: tp})
    olib.ops_add_peer(ps, A)
    assert olib.ops_score(ps, A) == 0
    olib.ops_graft(ps, A, MYTOPIC, 0)
    elapsed = 200 * Millisecond
    olib.ops_refresh(ps, elapsed)
    expected = 0.5 * 1 * float(elapsed // Millisecond)
    assert olib.ops_score(ps, A) >= expected
    assert olib.ops_score(ps, A) == expected  # virtual clock: exact
    olib.ops_free(ps)


def test_score_time_in_mesh_cap(olib):  # score_test.go:52-84
    p = PeerScoreParams(AppSpecificScore=True)
    tp = TopicScoreParams(TopicWeight=0.5, TimeInMeshWeight=1, TimeInMeshQuantum=Millisecond, TimeInMeshCap=10)
    ps = mk(olib, p, {MYTOPIC: tp})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    olib.ops_refresh(ps, 40 * Millisecond)
    expected = 0.5 * 1 * 10
    s = olib.ops_score(ps, A)
    assert expected * 0.5 < s < expected * 1.5
    olib.ops_free(ps)


def _fmd_params(decay, cap):
    return TopicScoreParams(TopicWeight=1, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=decay,
                            FirstMessageDeliveriesCap=cap, TimeInMeshQuantum=Second)


def test_score_first_message_deliveries(olib):  # score_test.go:86-124
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _fmd_params(1.0, 2000)})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    deliver_n(olib, ps, A, 100, 0)
    olib.ops_refresh(ps, 0)
    assert olib.ops_score(ps, A) == 1 * 1 * 100.0
    olib.ops_free(ps)


def test_score_first_message_deliveries_cap(olib):  # score_test.go:126-164
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _fmd_params(1.0, 50)})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    deliver_n(olib, ps, A, 100, 0)
    olib.ops_refresh(ps, 0)
    assert olib.ops_score(ps, A) == 50.0
    olib.ops_free(ps)


def test_score_first_message_deliveries_decay(olib):  # score_test.go:166-215
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _fmd_params(0.9, 2000)})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    deliver_n(olib, ps, A, 100, 0)
    olib.ops_refresh(ps, 0)
    expected = 1 * 1 * 0.9 * 100.0
    assert olib.ops_score(ps, A) == expected
    for _ in range(10):
        olib.ops_refresh(ps, 0)
        expected *= 0.9
    assert olib.ops_score(ps, A) == expected
    olib.ops_free(ps)


def _mmd_params(activation, decay, window=10 * Millisecond):
    return TopicScoreParams(TopicWeight=1, MeshMessageDeliveriesWeight=-1,
                            MeshMessageDeliveriesActivation=activation,
                            MeshMessageDeliveriesWindow=window, MeshMessageDeliveriesThreshold=20,
                            MeshMessageDeliveriesCap=100, MeshMessageDeliveriesDecay=decay,
                            FirstMessageDeliveriesWeight=0, TimeInMeshQuantum=Second)


def test_score_mesh_message_deliveries(olib):  # score_test.go:217-308
    tp = _mmd_params(Second, 1.0)
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: tp})
    now = 0
    for p in (A, B, Cp):
        olib.ops_add_peer(ps, p)
        olib.ops_graft(ps, p, MYTOPIC, now)
    olib.ops_refresh(ps, now)
    for p in (A, B, Cp):
        assert olib.ops_score(ps, p) >= 0
    now += Second  # time.Sleep(activation)
    late = tp.MeshMessageDeliveriesWindow + 20 * Millisecond
    for i in range(100):
        olib.ops_validate(ps, i, MYTOPIC, A, now)
        olib.ops_deliver(ps, i, MYTOPIC, A, now)
        olib.ops_duplicate(ps, i, MYTOPIC, B, now)
    for i in range(100):  # time.AfterFunc(window + 20ms): C's duplicates
        olib.ops_duplicate(ps, i, MYTOPIC, Cp, now + late)
    now += late
    olib.ops_refresh(ps, now)
    assert olib.ops_score(ps, A) >= 0
    assert olib.ops_score(ps, B) >= 0
    penalty = 20.0 * 20.0
    assert olib.ops_score(ps, Cp) == 1 * -1 * penalty
    olib.ops_free(ps)


def test_score_mesh_message_deliveries_decay(olib):  # score_test.go:310-369
    tp = _mmd_params(0, 0.9)
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: tp})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    deliver_n(olib, ps, A, 40, 0)
    # Activation is 0: the reference relies on wall time having advanced
    # past graftTime when refreshScores runs (meshTime > 0); so does this.
    olib.ops_refresh(ps, Millisecond)
    assert olib.ops_score(ps, A) >= 0
    decayed = 40.0 * 0.9
    for i in range(20):
        olib.ops_refresh(ps, (i + 2) * Millisecond)
        decayed *= 0.9
    deficit = 20 - decayed
    assert olib.ops_score(ps, A) == 1 * -1 * (deficit * deficit)
    olib.ops_free(ps)


def test_score_mesh_failure_penalty(olib):  # score_test.go:371-450
    tp = TopicScoreParams(TopicWeight=1, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=1.0,
                          MeshMessageDeliveriesActivation=0, MeshMessageDeliveriesWindow=10 * Millisecond,
                          MeshMessageDeliveriesThreshold=20, MeshMessageDeliveriesCap=100,
                          MeshMessageDeliveriesDecay=1.0, MeshMessageDeliveriesWeight=0,
                          FirstMessageDeliveriesWeight=0, TimeInMeshQuantum=Second)
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: tp})
    for p in (A, B):
        olib.ops_add_peer(ps, p)
        olib.ops_graft(ps, p, MYTOPIC, 0)
    deliver_n(olib, ps, A, 100, 0)
    olib.ops_refresh(ps, Millisecond)  # wall time advanced past graftTime (Activation 0)
    assert olib.ops_score(ps, A) == 0
    assert olib.ops_score(ps, B) == 0
    olib.ops_prune(ps, B, MYTOPIC)
    olib.ops_refresh(ps, 2 * Millisecond)
    assert olib.ops_score(ps, A) == 0
    assert olib.ops_score(ps, B) == 1 * -1 * (20.0 * 20.0)
    olib.ops_free(ps)


def _imd_params(decay, weight=-1):
    return TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second, InvalidMessageDeliveriesWeight=weight,
                            InvalidMessageDeliveriesDecay=decay)


REJECT = {n: i for i, n in enumerate([
    "blacklisted peer", "blacklisted source", "missing signature", "unexpected signature",
    "unexpected auth info", "invalid signature", "validation queue full", "validation throttled",
    "validation failed", "validation ignored", "self originated message"])}


def test_score_invalid_message_deliveries(olib):  # score_test.go:452-487
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _imd_params(1.0)})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    for i in range(100):
        olib.ops_reject(ps, i, MYTOPIC, A, REJECT["invalid signature"], 0)
    olib.ops_refresh(ps, 0)
    assert olib.ops_score(ps, A) == 1 * -1 * float(100 * 100)
    olib.ops_free(ps)


def test_score_invalid_message_deliveries_decay(olib):  # score_test.go:489-534
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _imd_params(0.9)})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    for i in range(100):
        olib.ops_reject(ps, i, MYTOPIC, A, REJECT["invalid signature"], 0)
    olib.ops_refresh(ps, 0)
    expected = 1 * -1 * math.pow(0.9 * 100.0, 2)
    assert olib.ops_score(ps, A) == expected
    for _ in range(10):
        olib.ops_refresh(ps, 0)
        expected *= math.pow(0.9, 2)
    assert olib.ops_score(ps, A) == expected
    olib.ops_free(ps)


def test_score_reject_message_deliveries(olib):  # score_test.go:536-666
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _imd_params(1.0)})
    olib.ops_add_peer(ps, A)
    olib.ops_add_peer(ps, B)
    now = 0
    for r in ("blacklisted peer", "blacklisted source", "validation queue full"):
        olib.ops_reject(ps, 0, MYTOPIC, A, REJECT[r], now)
    assert olib.ops_score(ps, A) == 0.0

    def clear():
        nonlocal now
        olib.ops_expire_head(ps, now)
        now += Millisecond
        olib.ops_gc(ps, now)

    olib.ops_validate(ps, 0, MYTOPIC, A, now)
    olib.ops_reject(ps, 0, MYTOPIC, A, REJECT["validation throttled"], now)
    olib.ops_duplicate(ps, 0, MYTOPIC, B, now)
    assert olib.ops_score(ps, A) == 0.0 and olib.ops_score(ps, B) == 0.0
    clear()
    olib.ops_validate(ps, 0, MYTOPIC, A, now)
    olib.ops_reject(ps, 0, MYTOPIC, A, REJECT["validation ignored"], now)
    olib.ops_duplicate(ps, 0, MYTOPIC, B, now)
    assert olib.ops_score(ps, A) == 0.0 and olib.ops_score(ps, B) == 0.0
    clear()
    olib.ops_validate(ps, 0, MYTOPIC, A, now)
    olib.ops_reject(ps, 0, MYTOPIC, A, REJECT["validation failed"], now)
    olib.ops_duplicate(ps, 0, MYTOPIC, B, now)
    assert olib.ops_score(ps, A) == -1.0 and olib.ops_score(ps, B) == -1.0
    clear()
    olib.ops_validate(ps, 0, MYTOPIC, A, now)
    olib.ops_duplicate(ps, 0, MYTOPIC, B, now)
    olib.ops_reject(ps, 0, MYTOPIC, A, REJECT["validation failed"], now)
    assert olib.ops_score(ps, A) == -4.0 and olib.ops_score(ps, B) == -4.0
    olib.ops_free(ps)


def test_score_application_score(olib):  # score_test.go:668-694
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True, AppSpecificWeight=0.5), {})
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    for i in range(-100, 100):
        olib.ops_set_app_score(ps, A, float(i))
        olib.ops_refresh(ps, 0)
        assert olib.ops_score(ps, A) == float(i) * 0.5
    olib.ops_free(ps)


def _ip(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def _set_ips(olib, ps, p, *ips):
    arr = (C.c_uint32 * len(ips))(*[_ip(x) for x in ips])
    olib.ops_set_ips(ps, p, len(ips), arr)


def test_score_ip_colocation(olib):  # score_test.go:696-744
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True, IPColocationFactorThreshold=1,
                                  IPColocationFactorWeight=-1), {})
    for p in (A, B, Cp, D):
        olib.ops_add_peer(ps, p)
        olib.ops_graft(ps, p, MYTOPIC, 0)
    _set_ips(olib, ps, A, "1.2.3.4")
    _set_ips(olib, ps, B, "2.3.4.5")
    _set_ips(olib, ps, Cp, "2.3.4.5", "3.4.5.6")
    _set_ips(olib, ps, D, "2.3.4.5")
    olib.ops_refresh(ps, 0)
    assert olib.ops_score(ps, A) == 0
    expected = -1 * float((3 - 1) ** 2)
    for p in (B, Cp, D):
        assert olib.ops_score(ps, p) == expected
    olib.ops_free(ps)


def test_score_ip_colocation_whitelist(olib):  # score_test.go:746-803
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True, IPColocationFactorThreshold=1,
                                  IPColocationFactorWeight=-1), {})
    olib.ops_add_whitelist(ps, _ip("2.3.0.0"), 0xFFFF0000)
    for p in (A, B, Cp, D):
        olib.ops_add_peer(ps, p)
        olib.ops_graft(ps, p, MYTOPIC, 0)
    _set_ips(olib, ps, A, "1.2.3.4")
    _set_ips(olib, ps, B, "2.3.4.5")
    _set_ips(olib, ps, Cp, "2.3.4.5", "3.4.5.6")
    _set_ips(olib, ps, D, "2.3.4.5")
    olib.ops_refresh(ps, 0)
    for p in (A, B, Cp, D):
        assert olib.ops_score(ps, p) == 0
    olib.ops_free(ps)


def test_score_behaviour_penalty(olib):  # score_test.go:805-859
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True, BehaviourPenaltyWeight=-1,
                                  BehaviourPenaltyDecay=0.99), {})
    olib.ops_add_penalty(ps, A, 1)  # non-existent peer: no effect
    assert olib.ops_score(ps, A) == 0
    olib.ops_add_peer(ps, A)
    assert olib.ops_score(ps, A) == 0
    olib.ops_add_penalty(ps, A, 1)
    assert olib.ops_score(ps, A) == -1
    olib.ops_add_penalty(ps, A, 1)
    assert olib.ops_score(ps, A) == -4
    olib.ops_refresh(ps, 0)
    assert olib.ops_score(ps, A) == -3.9204
    olib.ops_free(ps)


def test_score_retention(olib):  # score_test.go:861-903
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True, AppSpecificWeight=1.0, RetainScore=Second), {})
    olib.ops_set_app_score(ps, A, -1000)
    olib.ops_add_peer(ps, A)
    olib.ops_graft(ps, A, MYTOPIC, 0)
    now = 0
    olib.ops_refresh(ps, now)
    assert olib.ops_score(ps, A) == -1000.0
    olib.ops_remove_peer(ps, A, now)
    delay = Second // 2
    now += delay
    olib.ops_refresh(ps, now)
    assert olib.ops_score(ps, A) == -1000.0
    now += delay + 50 * Millisecond
    olib.ops_refresh(ps, now)
    assert olib.ops_score(ps, A) == 0
    olib.ops_free(ps)


def test_score_recap_topic_params(olib):  # score_test.go:905-1000
    tp = TopicScoreParams(TopicWeight=1, MeshMessageDeliveriesWeight=-1,
                          MeshMessageDeliveriesActivation=Second, MeshMessageDeliveriesWindow=10 * Millisecond,
                          MeshMessageDeliveriesThreshold=20, MeshMessageDeliveriesCap=100,
                          MeshMessageDeliveriesDecay=1.0, FirstMessageDeliveriesWeight=10,
                          FirstMessageDeliveriesDecay=1.0, FirstMessageDeliveriesCap=100,
                          TimeInMeshQuantum=Second)
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: tp})
    for p in (A, B):
        olib.ops_add_peer(ps, p)
        olib.ops_graft(ps, p, MYTOPIC, 0)
    for i in range(100):
        olib.ops_validate(ps, i, MYTOPIC, A, 0)
        olib.ops_deliver(ps, i, MYTOPIC, A, 0)
        olib.ops_duplicate(ps, i, MYTOPIC, B, 0)
    st = (C.c_double * 4)()
    olib.ops_topic_stats(ps, A, MYTOPIC, st)
    assert st[0] == 100
    olib.ops_topic_stats(ps, B, MYTOPIC, st)
    assert st[1] == 100
    tp2 = TopicScoreParams(**{**tp.__dict__, "MeshMessageDeliveriesCap": 50, "FirstMessageDeliveriesCap": 50})
    olib.ops_set_topic_score_params(ps, MYTOPIC, C.byref(tp2.to_c()))
    olib.ops_topic_stats(ps, A, MYTOPIC, st)
    assert st[0] == 50
    olib.ops_topic_stats(ps, B, MYTOPIC, st)
    assert st[1] == 50
    olib.ops_free(ps)


def test_score_reset_topic_params(olib):  # score_test.go:1002-1062
    ps = mk(olib, PeerScoreParams(AppSpecificScore=True), {MYTOPIC: _imd_params(1.0)})
    olib.ops_add_peer(ps, A)
    for i in range(100):
        olib.ops_validate(ps, i, MYTOPIC, A, 0)
        olib.ops_reject(ps, i, MYTOPIC, A, REJECT["validation failed"], 0)
    assert olib.ops_score(ps, A) == -10000
    olib.ops_set_topic_score_params(ps, MYTOPIC, C.byref(_imd_params(1.0, weight=-10).to_c()))
    assert olib.ops_score(ps, A) == -100000
    olib.ops_free(ps)
