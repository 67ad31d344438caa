"""Restates mcache_test.go, gossip_tracer_test.go and peer_gater_test.go on the
oracle's MessageCache / GossipTracer / PeerGater objects (virtual clock)."""
import ctypes as C

from pubsub_amd import _abi
from pubsub_amd.params import Millisecond, NewPeerGaterParams, Second

TOPIC = 0


def gossip_ids(olib, mc, topic=TOPIC):
    buf = (C.c_int64 * 1024)()
    n = olib.omc_gossip_ids(mc, topic, buf, 1024)
    return list(buf[:n])


def test_message_cache(olib):  # mcache_test.go:11-154
    mc = olib.omc_new(3, 5)
    msgs = list(range(60))
    for i in range(10):
        olib.omc_put(mc, msgs[i], TOPIC)
    for i in range(10):
        assert olib.omc_get(mc, msgs[i])
    gids = gossip_ids(olib, mc)
    assert gids == msgs[:10]
    olib.omc_shift(mc)
    for i in range(10, 20):
        olib.omc_put(mc, msgs[i], TOPIC)
    for i in range(20):
        assert olib.omc_get(mc, msgs[i])
    gids = gossip_ids(olib, mc)
    assert len(gids) == 20
    assert gids[10:] == msgs[:10] and gids[:10] == msgs[10:20]
    for lo in (20, 30, 40, 50):
        olib.omc_shift(mc)
        for i in range(lo, lo + 10):
            olib.omc_put(mc, msgs[i], TOPIC)
    assert olib.omc_len(mc) == 50
    for i in range(10):
        assert not olib.omc_get(mc, msgs[i])
    for i in range(10, 60):
        assert olib.omc_get(mc, msgs[i])
    gids = gossip_ids(olib, mc)
    assert len(gids) == 30
    assert gids[0:10] == msgs[50:60]
    assert gids[10:20] == msgs[40:50]
    assert gids[20:30] == msgs[30:40]
    olib.omc_free(mc)


def test_message_cache_invalid_params(olib):  # mcache.go:24-28 panics; we refuse
    assert not olib.omc_new(6, 5)


def test_message_cache_get_for_peer_counts(olib):  # mcache.go:66-80 (IWANT retransmission counts)
    mc = olib.omc_new(3, 5)
    olib.omc_put(mc, 7, TOPIC)
    assert [olib.omc_get_for_peer(mc, 7, 1) for _ in range(4)] == [1, 2, 3, 4]
    assert olib.omc_get_for_peer(mc, 7, 2) == 1
    assert olib.omc_get_for_peer(mc, 8, 1) == -1
    olib.omc_free(mc)


def _broken(olib, gt, now):
    peers = (C.c_int * 16)()
    counts = (C.c_int * 16)()
    n = olib.ogt_broken(gt, now, peers, counts, 16)
    return {peers[i]: counts[i] for i in range(n)}


def test_broken_promises(olib):  # gossip_tracer_test.go:12-61
    A, B, Cp = 0, 1, 2
    gt = olib.ogt_new(100 * Millisecond)
    mids = (C.c_int64 * 100)(*range(100))
    now = 0
    for p, idx in ((A, 17), (B, 42), (Cp, 3)):  # rand.Intn(len) index: any
        olib.ogt_add_promise(gt, p, 100, mids, idx, now)
    assert _broken(olib, gt, now) == {}
    olib.ogt_throttle(gt, Cp)
    now += 3 * Second + 10 * Millisecond  # GossipSubIWantFollowupTime + 10ms
    assert _broken(olib, gt, now) == {A: 1, B: 1}
    olib.ogt_free(gt)


def test_no_broken_promises(olib):  # gossip_tracer_test.go:63-101
    A, B = 0, 1
    gt = olib.ogt_new(100 * Millisecond)
    mids = (C.c_int64 * 100)(*range(100))
    olib.ogt_add_promise(gt, A, 100, mids, 5, 0)
    olib.ogt_add_promise(gt, B, 100, mids, 77, 0)
    for m in range(100):
        olib.ogt_deliver(gt, m)
    assert _broken(olib, gt, 110 * Millisecond) == {}
    olib.ogt_free(gt)


REJ_QUEUE_FULL, REJ_THROTTLED, REJ_FAILED, REJ_IGNORED = 6, 7, 8, 9
ACCEPT_NONE, ACCEPT_CONTROL, ACCEPT_ALL = 0, 1, 2


def test_peer_gater(olib):  # peer_gater_test.go:11-128
    import numpy as np
    A = 0
    ip_a = (1 << 24) | (2 << 16) | (3 << 8) | 4
    params = NewPeerGaterParams(.1, .9, .999)
    pc = params.to_c()
    assert _abi.bind(olib._name).gs_validate_peer_gater_params(C.byref(pc)) == 0
    ips = (C.c_uint32 * 1)(ip_a)
    pg = olib.opg_new(C.byref(pc), ips, 1)
    rng = np.random.default_rng(11)  # stands in for rand.Float64()
    now = 0
    olib.opg_add_peer(pg, A)
    assert olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_ALL
    olib.opg_validate(pg)
    assert olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_ALL
    olib.opg_reject(pg, A, REJ_QUEUE_FULL, now)
    assert olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_ALL
    olib.opg_reject(pg, A, REJ_THROTTLED, now)
    assert olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_ALL
    for _ in range(100):
        olib.opg_reject(pg, A, REJ_IGNORED, now)
        olib.opg_reject(pg, A, REJ_FAILED, now)
    assert any(olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_CONTROL for _ in range(1000))
    for _ in range(100):
        olib.opg_deliver(pg, A)
    assert any(olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_ALL for _ in range(1000))
    for _ in range(100):
        olib.opg_decay(pg, now)
    assert olib.opg_accept_from(pg, A, now, rng.random()) == ACCEPT_ALL
    olib.opg_remove_peer(pg, A, now)
    assert not olib.opg_has_peer_stats(pg, A)
    assert olib.opg_has_ip_stats(pg, ip_a)
    olib.opg_set_ip_expire(pg, ip_a, now)
    now += 2 * Second
    olib.opg_decay(pg, now)
    assert not olib.opg_has_ip_stats(pg, ip_a)
    olib.opg_free(pg)
