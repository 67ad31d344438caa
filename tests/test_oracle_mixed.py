"""Mixed networks on the oracle (CPU): hosts running different routers and
connections running different protocols (gs_set_routers / gs_set_graph_ex,
PubSubRouter.AddPeer(peer.ID, protocol.ID) pubsub.go:165, gossipsub_feat.go).
The reference's own TestMixedGossipsub assertion plus the per-protocol rules
of gossipsub.go (floodsub peers at publish :969-975, GossipSubFeatureMesh in
getPeers :1849 / emitGossip :1681, v1.0 PRUNEs :1804-1807, EnoughPeers
:549-576) and randomsub.go (floodsub peers always sent :117-118, EnoughPeers
:59-89), floodsub.go (EnoughPeers :52-66)."""
import numpy as np
import pytest

import scenarios
from pubsub_amd import (GS_PROTO_FLOODSUB, GS_PROTO_GOSSIPSUB_V10, GS_PROTO_GOSSIPSUB_V11, GS_PROTO_RANDOMSUB,
                        GS_ROUTER_FLOODSUB, GS_ROUTER_GOSSIPSUB, GS_ROUTER_GOSSIPSUB_V10, GS_ROUTER_RANDOMSUB,
                        GossipEngineError, NewGossipSub, NewRandomSub, Second, WithEventTracer,
                        WithGossipSubParams, WithHop, WithPeerExchange, WithPeerScore, WithProtocols,
                        WithRecordDeliveries, WithRouters, WithSeed, eth2_peer_score_params, eth2_thresholds, graphs)
from pubsub_amd.params import GossipSubParams, Millisecond

HOP = 100 * Millisecond


def _src(e):
    return np.repeat(np.arange(e.N), np.diff(e.rowptr))


def negotiated(routers, rowptr, col):
    """The protocol both hosts of each connection run (multistream-select
    over the dialer's Protocols(), floodsub.go:26, randomsub.go:40,
    gossipsub_feat.go:24, 41)."""
    protos = {GS_ROUTER_FLOODSUB: [GS_PROTO_FLOODSUB], GS_ROUTER_RANDOMSUB: [GS_PROTO_RANDOMSUB, GS_PROTO_FLOODSUB],
              GS_ROUTER_GOSSIPSUB_V10: [GS_PROTO_GOSSIPSUB_V10, GS_PROTO_FLOODSUB],
              GS_ROUTER_GOSSIPSUB: [GS_PROTO_GOSSIPSUB_V11, GS_PROTO_GOSSIPSUB_V10, GS_PROTO_FLOODSUB]}
    src = np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr))
    out = np.empty(len(col), np.uint8)
    for e, (u, v) in enumerate(zip(src, col)):
        b = protos[int(routers[v])]
        out[e] = next(p for p in protos[int(routers[u])] if p in b)
    return out


def test_mixed_gossipsub_every_host_gets_every_message(oracle_path):
    """TestMixedGossipsub (gossipsub_test.go:834-850): each of the 100
    messages reaches all 30 hosts; floodsub hosts keep no mesh and no
    gossipsub host grafts a floodsub peer."""
    e, hops = scenarios.mixed_gossip_flood(oracle_path)
    e.step(hops)
    c = e.counters()
    assert c["published"] == 100 and c["deliveries"] == 100 * 29, c
    mesh = e.mesh()
    src = _src(e)
    routers = np.array([GS_ROUTER_GOSSIPSUB] * 20 + [GS_ROUTER_FLOODSUB] * 10)
    assert not mesh[routers[src] == GS_ROUTER_FLOODSUB].any()          # floodsub hosts: no mesh
    assert not mesh[routers[e.col] == GS_ROUTER_FLOODSUB].any()        # nobody grafts a floodsub peer
    assert mesh[routers[src] == GS_ROUTER_GOSSIPSUB].any()
    # the gossipsub <-> floodsub connections exist, so both forwarding paths ran
    assert ((routers[src] == GS_ROUTER_GOSSIPSUB) & (routers[e.col] == GS_ROUTER_FLOODSUB)).any()


def test_mixed_scored_mesh_and_scores(oracle_path):
    e, hops = scenarios.mixed_scored(oracle_path)
    e.step(hops)
    routers = e.routers_h
    src = _src(e)
    proto = negotiated(routers, e.rowptr, e.col)
    mesh, scores = e.mesh(), e.scores()
    gossip_host = (routers == GS_ROUTER_GOSSIPSUB) | (routers == GS_ROUTER_GOSSIPSUB_V10)
    assert not mesh[proto < GS_PROTO_GOSSIPSUB_V10].any()   # GossipSubFeatureMesh (gossipsub.go:1849)
    assert not mesh[~gossip_host[src]].any()
    assert (scores[~gossip_host[src]] == 0).all()          # floodsub / randomsub hosts keep no score
    assert mesh[proto == GS_PROTO_GOSSIPSUB_V10].any() and mesh[proto == GS_PROTO_GOSSIPSUB_V11].any()
    c = e.counters()
    assert c["prunes_sent"] > 0 and c["grafts_sent"] > 0 and c["ihave_sent"] > 0
    # gossipsub hosts score their floodsub peers too (P2 from first deliveries)
    fs = gossip_host[src] & (proto == GS_PROTO_FLOODSUB)
    assert (e.topic_stats()["fmd"][:, fs] > 0).any()


def _star(lib, n_leaves, leaf_routers, leaf_app=None, extra=()):
    """Host 0 (gossipsub v1.1) connected to leaves 1..n (leaf_routers); no
    leaf-leaf connections; host 0 dialled nobody (so the Dhi GRAFT check
    applies to every leaf)."""
    n = n_leaves + 1
    rowptr = np.concatenate([[0, n_leaves], n_leaves + np.arange(1, n_leaves + 1)]).astype(np.int64)
    col = np.concatenate([np.arange(1, n), np.zeros(n_leaves)]).astype(np.int32)
    outbound = np.concatenate([np.zeros(n_leaves), np.ones(n_leaves)]).astype(np.uint8)
    routers = np.concatenate([[GS_ROUTER_GOSSIPSUB], leaf_routers]).astype(np.uint8)
    app = None if leaf_app is None else np.concatenate([[0.0], leaf_app])
    return NewGossipSub(n, 1, (rowptr, col, outbound), graphs.all_subscribed(n, 1), WithRouters(routers),
                        WithRecordDeliveries(), WithSeed(5), WithHop(HOP), *extra, app_score=app, lib=lib)


def test_v10_prune_has_no_backoff_and_no_px(oracle_path):
    """20 leaves GRAFT the centre at Join; beyond Dhi the centre rejects them
    with a PRUNE (gossipsub.go:778-785).  PruneBackoff = 61.5 s: a v1.1 leaf
    backs off for the PRUNE's whole seconds (61 s, handlePrune :819-825), a
    v1.0 leaf for its own PruneBackoff (the PRUNE carries no backoff,
    makePrune :1804-1807).  With PX on, only the v1.1 leaves' PRUNEs carry
    peers, and those peers are mesh-capable (getPeers :1849)."""
    leaves = 20
    lr = np.array([GS_ROUTER_GOSSIPSUB_V10 if i % 2 else GS_ROUTER_GOSSIPSUB for i in range(leaves)])
    lr[:2] = GS_ROUTER_FLOODSUB  # floodsub leaves: never grafted, never in PX lists
    gp = GossipSubParams(PruneBackoff=61500 * Millisecond)
    e = _star(oracle_path, leaves, lr,
              extra=(WithGossipSubParams(gp), WithPeerExchange(True), WithEventTracer([0], rpc=True)))
    e.step(4)
    bo = e.backoff().reshape(-1)[leaves:]  # leaf -> centre edges (topic 0)
    rejected = np.flatnonzero(bo)
    assert len(rejected) >= 4
    got = {}
    ev = e.trace_events()
    for i in rejected:
        leaf = i + 1
        prune_hop = next(int(x["hop"]) for x in ev if x["type"] == 7 and x["peer"] == leaf)  # SendRPC
        got[leaf] = int(bo[i]) - (prune_hop + 1) * HOP
    for leaf, d in got.items():
        assert d == (61500 if lr[leaf - 1] == GS_ROUTER_GOSSIPSUB_V10 else 61000) * Millisecond, (leaf, d)
    assert {lr[leaf - 1] for leaf in got} == {GS_ROUTER_GOSSIPSUB, GS_ROUTER_GOSSIPSUB_V10}
    # PX items follow PRUNE items of SendRPC blocks of the centre
    px_to = {}
    for x in ev:
        if x["type"] == 32 and x["node"] == 0 and x["reason"] == 7:
            px_to.setdefault(int(x["peer"]), []).append(int(x["msg"]))
    assert px_to, "no PX sent"
    for leaf, peers in px_to.items():
        assert lr[leaf - 1] == GS_ROUTER_GOSSIPSUB
        assert all(lr[p - 1] != GS_ROUTER_FLOODSUB for p in peers)


@pytest.mark.parametrize("app,received", [(-250.0, False), (-150.0, True)])
def test_floodsub_peer_needs_publish_threshold(oracle_path, app, received):
    """gossipsub.go:969-975: a gossipsub host sends to a floodsub peer only if
    the peer's score >= PublishThreshold (-200 here).  Leaf 1 (floodsub, app
    score `app`) hangs off the centre only; leaf 2 is a gossipsub host."""
    lr = np.array([GS_ROUTER_FLOODSUB, GS_ROUTER_GOSSIPSUB])
    e = _star(oracle_path, 2, lr, leaf_app=np.array([app, 0.0]),
              extra=(WithPeerScore(eth2_peer_score_params(1), eth2_thresholds()),))
    e.publish(np.zeros(5, np.int32), np.zeros(5, np.int32), np.arange(20, 25))
    e.step(40)
    hop1, _ = e.deliveries(0)
    assert (hop1[1] >= 0) == received
    assert hop1[2] >= 0


def test_randomsub_always_sends_to_floodsub_peers(oracle_path):
    """randomsub.go:99-150 closed form over the recorded first deliveries:
    every holder of a message (its author, then each first receiver) sends it
    to all of its floodsub-protocol candidates and to min(10, n) of its n
    randomsub-protocol ones when n > 6 (all of them otherwise); a floodsub
    holder sends to every candidate.  Candidates exclude ReceivedFrom and the
    author."""
    e, hops = scenarios.mixed_randomsub(oracle_path)
    e.step(hops)
    routers = e.routers_h
    c = e.counters()
    want = 0
    for m in range(e.n_published):
        hop, frm = e.deliveries(m)
        author = int(np.flatnonzero((hop >= 0) & (frm < 0))[0])
        for h in np.flatnonzero(hop >= 0):
            nb = e.col[e.rowptr[h]:e.rowptr[h + 1]]
            cand = [int(p) for p in nb if p != frm[h] and p != author]
            if routers[h] == GS_ROUTER_FLOODSUB:
                want += len(cand)
                continue
            fs = [p for p in cand if routers[p] == GS_ROUTER_FLOODSUB]
            rs = len(cand) - len(fs)
            want += len(fs) + (min(10, rs) if rs > 6 else rs)
    assert c["transmissions"] == want
    assert c["deliveries"] > 0.99 * e.n_published * (e.N - 1)


def test_enough_peers(oracle_path):
    """EnoughPeers per router: gossipsub (fs + |mesh| >= suggested or |mesh| >=
    Dhi, suggested 0 = Dlo), randomsub (fs + rs >= suggested or rs >= 6,
    suggested 0 = 6), floodsub (|topic peers| >= suggested, 0 = 5)."""
    gp = GossipSubParams()
    for build in (scenarios.mixed_gossip_flood, scenarios.mixed_randomsub):
        e, hops = build(oracle_path)
        e.step(hops)
        routers = getattr(e, "routers_h", np.array([GS_ROUTER_GOSSIPSUB] * 20 + [GS_ROUTER_FLOODSUB] * 10))
        mesh = e.mesh()
        for sug in (0, 3, 5, 8, 13):
            got = e.enough_peers(0, sug)
            for u in range(e.N):
                nb = e.col[e.rowptr[u]:e.rowptr[u + 1]]
                r = routers[u]
                if r == GS_ROUTER_GOSSIPSUB:
                    fs = int(sum(routers[p] in (GS_ROUTER_FLOODSUB, GS_ROUTER_RANDOMSUB) for p in nb))
                    gs = int(sum((mesh[e.rowptr[u]:e.rowptr[u + 1]] & 1) != 0))
                    want = fs + gs >= (sug or gp.Dlo) or gs >= gp.Dhi
                elif r == GS_ROUTER_RANDOMSUB:
                    fs = int(sum(routers[p] == GS_ROUTER_FLOODSUB for p in nb))
                    rs = int(sum(routers[p] == GS_ROUTER_RANDOMSUB for p in nb))
                    want = fs + rs >= (sug or 6) or rs >= 6
                else:
                    want = len(nb) >= (sug or 5)
                assert got[u] == want, (build.__name__, sug, u)
    with pytest.raises(GossipEngineError):
        e.enough_peers(0, -1)


def test_protocol_validation(oracle_path):
    """proto[e] must be spoken by both hosts and equal on both directions;
    gossipsub hosts need a gossipsub engine; attackers must run gossipsub."""
    g = graphs.dense_connect(10, 1)
    rowptr, col, ob = g
    routers = np.array([GS_ROUTER_GOSSIPSUB] * 5 + [GS_ROUTER_FLOODSUB] * 5, np.uint8)
    good = negotiated(routers, rowptr, col)
    e = NewGossipSub(10, 1, g, graphs.all_subscribed(10, 1), WithRouters(routers), WithProtocols(good),
                     lib=oracle_path)
    e.step(2)
    bad = good.copy()
    src = np.repeat(np.arange(10), np.diff(rowptr))
    k = int(np.flatnonzero((src < 5) & (col >= 5))[0])
    bad[k] = GS_PROTO_GOSSIPSUB_V11  # a floodsub host cannot speak gossipsub
    e = NewGossipSub(10, 1, g, graphs.all_subscribed(10, 1), WithRouters(routers), WithProtocols(bad),
                     lib=oracle_path)
    with pytest.raises(GossipEngineError):
        e.step(1)
    # v1.0 on one direction of a gossipsub-gossipsub connection only
    bad = good.copy()
    k = int(np.flatnonzero((src < 5) & (col < 5))[0])
    bad[k] = GS_PROTO_GOSSIPSUB_V10
    e = NewGossipSub(10, 1, g, graphs.all_subscribed(10, 1), WithRouters(routers), WithProtocols(bad),
                     lib=oracle_path)
    with pytest.raises(GossipEngineError):
        e.step(1)
    # ... on both directions it is a valid choice (a v1.0 stream on a v1.1 pair)
    k2 = int(np.flatnonzero((src == col[k]) & (col == src[k]))[0])
    bad[k2] = GS_PROTO_GOSSIPSUB_V10
    e = NewGossipSub(10, 1, g, graphs.all_subscribed(10, 1), WithRouters(routers), WithProtocols(bad),
                     lib=oracle_path)
    e.step(2)
    e = NewRandomSub(10, 1, g, graphs.all_subscribed(10, 1), 10, WithRouters(routers), lib=oracle_path)
    with pytest.raises(GossipEngineError):
        e.step(1)


def test_add_peer_trace_carries_the_protocol(oracle_path):
    """tracer.AddPeer(p, proto) (gossipsub.go:507, randomsub.go:49,
    floodsub.go:45): on a mixed network each AddPeer event names the
    connection's protocol, and the encoders write its protocol.ID."""
    from pubsub_amd import _abi, encode_trace
    e, hops = scenarios.mixed_scored(oracle_path, extra=(WithEventTracer(list(range(40))),))
    e.step(3)
    ev = e.trace_events()
    add = ev[ev["type"] == _abi.GS_TRACE_ADD_PEER] if hasattr(_abi, "GS_TRACE_ADD_PEER") else ev[ev["type"] == 4]
    assert len(add) > 0
    proto = negotiated(e.routers_h, e.rowptr, e.col)
    for x in add:
        k = int(np.searchsorted(e.col[e.rowptr[x["node"]]:e.rowptr[x["node"] + 1]], x["peer"])) + int(e.rowptr[x["node"]])
        assert int(x["reason"]) == int(proto[k])
    assert set(int(r) for r in add["reason"]) >= {GS_PROTO_FLOODSUB, GS_PROTO_GOSSIPSUB_V10, GS_PROTO_GOSSIPSUB_V11}
