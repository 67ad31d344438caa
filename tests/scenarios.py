"""Seeded simulation scenarios shared by the oracle tests (CPU) and the GPU
parity tests.  Each builder takes the ABI library path so the same calls
drive the oracle and the HIP engine; `compare()` checks every readback
bit-exactly (float64 compared on their bit patterns)."""
import numpy as np

from pubsub_amd import (NewFloodSub, NewGossipSub, NewRandomSub, PeerScoreParams, Second,
                        TopicScoreParams, WithDirectPeers, WithFloodPublish, WithGossipSubParams, WithHop,
                        WithMessageWindow, WithPeerScore, WithRecordDeliveries, WithSeed,
                        eth2_peer_score_params, eth2_thresholds, eth2_topic_score_params)
from pubsub_amd import graphs
from pubsub_amd.params import GossipSubParams, Millisecond, PeerScoreThresholds  # noqa: F401

HOP = 100 * Millisecond


def _publish_schedule(n, topics, count, start, every, seed, srcs=None):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, count) if srcs is None else rng.choice(srcs, count)
    top = rng.integers(0, topics, count)
    hops = start + np.arange(count) * every if every else np.full(count, start)
    return src.astype(np.int32), top.astype(np.int32), np.asarray(hops, dtype=np.int64)


def floodsub_dense(lib, seed=1, extra=()):
    """TestFloodsubDense-like: 20 hosts, denseConnect, 100 messages."""
    n = 20
    g = graphs.dense_connect(n, seed)
    e = NewFloodSub(n, 1, g, graphs.all_subscribed(n, 1), WithRecordDeliveries(), WithSeed(seed),
                    WithMessageWindow(128), *extra, lib=lib)
    src, top, hops = _publish_schedule(n, 1, 100, 1, 2, seed)
    e.publish(src, top, hops)
    return e, int(hops[-1]) + 20


def floodsub_multitopic(lib, n=300, k=12, topics=3, seed=4, msgs=240, extra=()):
    """floodsub.go:76-100 with several topics and partial subscriptions: hosts
    forward only their own topics' messages, to the peers subscribed to them,
    and publish to topics they may not be subscribed to (floodsub's Publish
    needs no subscription).  A dense-frontier engine (k_flood_a) on one GPU."""
    g = graphs.random_regular(n, k, seed)
    rng = np.random.default_rng(seed)
    subs = np.zeros(n, dtype=np.uint64)
    for t in range(topics):
        subs |= (rng.random(n) < 0.6).astype(np.uint64) << np.uint64(t)
    e = NewFloodSub(n, topics, g, subs, WithRecordDeliveries(), WithSeed(seed), WithMessageWindow(128), *extra,
                    lib=lib)
    src, top, hops = _publish_schedule(n, topics, msgs, 1, 1, seed + 1)
    e.publish(src, top, hops)
    return e, int(hops[-1]) + 20


def randomsub(lib, size, n=200, k=16, seed=2, msgs=60, extra=()):
    g = graphs.random_regular(n, k, seed)
    e = NewRandomSub(n, 1, g, graphs.all_subscribed(n, 1), size, WithRecordDeliveries(), WithSeed(seed),
                     WithMessageWindow(128), *extra, lib=lib)
    src, top, hops = _publish_schedule(n, 1, msgs, 0, 1, seed)
    e.publish(src, top, hops)
    return e, int(hops[-1]) + 20


def gossipsub_dense(lib, seed=1, msgs=100, extra=()):
    """TestDenseGossipsub (gossipsub_test.go:84-123): 20 hosts, denseConnect,
    2 s of heartbeats, then 100 messages from random owners."""
    n = 20
    g = graphs.dense_connect(n, seed)
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithRecordDeliveries(), WithSeed(seed),
                     WithHop(HOP), WithMessageWindow(256), *extra, lib=lib)
    src, top, hops = _publish_schedule(n, 1, msgs, 20, 1, seed)
    e.publish(src, top, hops)
    return e, int(hops[-1]) + 40


def gossipsub_scored(lib, n=300, k=20, topics=1, seed=3, msgs=300, hb=12, flood=False, sub_frac=1.0,
                     app_neg_frac=0.0, ip_groups=0, params=None, window=1024, extra=(), app_neg=-150.0,
                     direct_frac=0.0, topic0_frac=0.0, burst=None):
    """gossipsub v1.1 with Eth2-derived scoring over a random regular graph.
    window = slots_per_topic; direct_frac: fraction of the undirected edges
    made direct peers on both ends (WithDirectPeers); topic0_frac: fraction of
    the messages forced onto topic 0; burst = (node, count, hop): `count` more
    messages by `node` at `hop`, on random topics."""
    rng = np.random.default_rng(seed)
    g = graphs.random_regular(n, k, seed)
    if direct_frac:
        rowptr, col, _ = g
        src = np.repeat(np.arange(n), np.diff(rowptr))
        pick = np.random.default_rng(seed + 55).random(len(col)) < direct_frac
        und = set()
        for u, v in zip(src[pick], col[pick]):
            und.add((min(u, v), max(u, v)))
        direct = np.zeros(len(col), dtype=np.uint8)
        for e in range(len(col)):
            if (min(src[e], col[e]), max(src[e], col[e])) in und:
                direct[e] = 1
        extra = tuple(extra) + (WithDirectPeers(direct),)
    if sub_frac >= 1.0:
        subs = graphs.all_subscribed(n, topics)
    else:
        subs = np.zeros(n, dtype=np.uint64)
        for t in range(topics):
            subs |= (rng.random(n) < sub_frac).astype(np.uint64) << np.uint64(t)
    sp = eth2_peer_score_params(topics)
    thr = eth2_thresholds()
    app = np.zeros(n)
    if app_neg_frac:
        app[rng.random(n) < app_neg_frac] = app_neg
    ipv4 = None
    if ip_groups:
        ipv4 = (rng.integers(0, ip_groups, n) + (10 << 24)).astype(np.uint32)
    opts = [WithPeerScore(sp, thr), WithRecordDeliveries(), WithSeed(seed), WithHop(HOP),
            WithMessageWindow(window)]
    if params is not None:
        opts.append(WithGossipSubParams(params))
    if flood:
        opts.append(WithFloodPublish(True))
    e = NewGossipSub(n, topics, g, subs, *opts, *extra, app_score=app, ipv4=ipv4, lib=lib)
    rng2 = np.random.default_rng(seed + 100)
    src = rng2.integers(0, n, msgs).astype(np.int32)
    top = rng2.integers(0, topics, msgs).astype(np.int32)
    if topic0_frac:
        top[rng2.random(msgs) < topic0_frac] = 0
    hops = (5 + (np.arange(msgs) * (hb * 10 - 20)) // msgs).astype(np.int64)
    if burst is not None:
        bn, bc, bh = burst
        src = np.concatenate([src, np.full(bc, bn, np.int32)])
        top = np.concatenate([top, rng2.integers(0, topics, bc).astype(np.int32)])
        hops = np.concatenate([hops, np.full(bc, bh, np.int64)])
        order = np.argsort(hops, kind="stable")
        src, top, hops = src[order], top[order], hops[order]
        msgs += bc
    e.publish(src, top, hops)
    e.sched_top, e.sched_hops = top, hops
    st = window
    if msgs > st:
        # the engine reads back only messages whose slot is not recycled yet:
        # each topic's last `st` messages (slots are a ring per topic)
        keep = []
        for t in range(topics):
            keep += list(np.flatnonzero(top == t)[-st:])
        e.snapshot_ids = sorted(int(i) for i in keep)
    return e, hb * 10 + 5


SCENARIOS = {
    "floodsub_dense": lambda lib, x=(): floodsub_dense(lib, extra=x),
    "floodsub_multitopic": lambda lib, x=(): floodsub_multitopic(lib, extra=x),
    "randomsub_100": lambda lib, x=(): randomsub(lib, 100, extra=x),
    "randomsub_N": lambda lib, x=(): randomsub(lib, 200, extra=x),
    "gossipsub_dense": lambda lib, x=(): gossipsub_dense(lib, extra=x),
    "gossipsub_scored": lambda lib, x=(): gossipsub_scored(lib, extra=x),
    "gossipsub_flood_publish": lambda lib, x=(): gossipsub_scored(lib, n=200, flood=True, seed=5, extra=x),
    "gossipsub_multitopic": lambda lib, x=(): gossipsub_scored(lib, n=200, topics=3, sub_frac=0.7, seed=7, msgs=240, extra=x),
    "gossipsub_negative_app": lambda lib, x=(): gossipsub_scored(lib, n=200, app_neg_frac=0.2, ip_groups=40, seed=9, extra=x),
    "gossipsub_dense_dhi": lambda lib, x=(): gossipsub_scored(lib, n=120, k=40, seed=11, hb=20, msgs=200, extra=x),
    # message windows smaller than the message count: slots are recycled, and
    # every active word mixes young slots with older or retired ones (phase A's
    # young-slot tables)
    "gossipsub_slot_reuse": lambda lib, x=(): gossipsub_scored(lib, n=200, seed=13, msgs=400, hb=16, window=320,
                                                               extra=x),
    "gossipsub_slot_reuse_4t": lambda lib, x=(): gossipsub_scored(lib, n=200, topics=4, seed=17, msgs=600, hb=16,
                                                                  window=128, extra=x),
    # graylisting (score < GraylistThreshold -> AcceptNone, gossipsub.go:584) and
    # direct peers (AcceptAll, always forwarded, GRAFT answered with PRUNE)
    "gossipsub_graylist_direct": lambda lib, x=(): gossipsub_scored(lib, n=300, k=20, seed=23, app_neg_frac=0.15,
                                                                    app_neg=-400.0, direct_frac=0.03, extra=x),
}

# The benchmarked shapes (bench.py), at a size the oracle finishes in seconds:
# the same kernel instantiations as the 1M-peer runs.
HEAVY = {
    # config4: 64 topics x 256 slots -> W = 256 words (4 per lane), degree 32 ->
    # 2048 (edge, topic) pairs per node (batches of 32), 8-bit phase-A counters
    "c4shape": lambda lib, x=(): gossipsub_scored(lib, n=1000, k=32, topics=64, window=256, msgs=1200, hb=8,
                                                  seed=21, extra=x),
    # W = 256 with more than 255 live messages in topic 0: 32-bit counters
    "c4shape_wide": lambda lib, x=(): gossipsub_scored(lib, n=1000, k=32, topics=16, window=1024, msgs=1200, hb=8,
                                                       seed=22, topic0_frac=0.4, extra=x),
    # config3: 1 topic x 10048 slots -> W = 157 words (3 per lane)
    "c3shape": lambda lib, x=(): gossipsub_scored(lib, n=2000, k=32, topics=1, window=10048, msgs=2000, hb=8,
                                                  seed=23, extra=x),
    # config4's steady-state phase B: an honest engine with
    # T = 4 whose gossip bound holds more than MaxIHaveLength ids over all
    # topics but fewer in any one, so from hop ~90 on phase B runs the honest
    # sender-cut instantiation (cutMode == 2: handleIHave's iasked cut,
    # gossipsub.go:625-667) with push active (T >= 4); 1536 slots per topic are
    # recycled once (phase A pass 2b's seen retirement, mcache.go:94-104)
    "cut_honest_4t": lambda lib, x=(): gossipsub_scored(lib, n=200, k=16, topics=4, window=1536, msgs=9000, hb=18,
                                                        seed=25, extra=x),
    # k_push's region overflow (more than GS_PUSHR = 2048 copies from one sender
    # in one hop: record -1, its receivers walk its frontier list): flood
    # publish of a 150-message burst by node 0 to its 24 peers, T = 4
    "push_overflow": lambda lib, x=(): gossipsub_scored(lib, n=200, k=24, topics=4, flood=True, window=512,
                                                        msgs=400, hb=10, seed=27, burst=(0, 150, 40), extra=x),
    # emitGossip's MaxIHaveLength truncation (gossipsub.go:1700-1710) on more
    # (sender, topic) items per node and hop than phase B keeps in LDS (GS_CUTS
    # = 64): 16 topics, MaxIHaveLength 3, gossip to every non-mesh peer, so a
    # heartbeat's IHAVE hop brings ~250 over-length items to each node and the
    # thresholds past the 64th spill into the rank's cut table
    "cut_spill_16t": lambda lib, x=(): gossipsub_scored(lib, n=200, k=24, topics=16, window=128, msgs=600, hb=12,
                                                        seed=29, params=_cut_spill_params(), extra=x),
}


def _cut_spill_params():
    p = GossipSubParams()
    p.MaxIHaveLength = 3
    p.GossipFactor = 1.0
    return p
SCENARIOS.update(HEAVY)




def snapshot(e, msg_ids):
    out = dict(counters=e.counters(), mesh=e.mesh(), fanout=e.fanout(), backoff=e.backoff(),
               scores=e.scores(), bp=e.behaviour_penalty())
    out.update({"ts_" + k: v for k, v in e.topic_stats().items()})
    out["deliv"] = [e.deliveries(i) for i in msg_ids]
    if getattr(e, "rpc_acct", False):
        out["rpc_bytes"], out["rpc_count"] = e.rpc_bytes()
    return out


def run(lib, name, extra_hops=0, extra=()):
    e, hops = SCENARIOS[name](lib, extra)
    e.step(hops + extra_hops)
    snap = snapshot(e, getattr(e, "snapshot_ids", range(e.n_published)))
    snap["node_range"], snap["edge_range"] = e.node_range, e.edge_range
    return snap


def restrict(s, T):
    """The part of a snapshot a partitioned rank owns (its nodes and their
    edges); counters are left out (they are per rank, compared summed)."""
    n0, n1 = s["node_range"]
    e0, e1 = s["edge_range"]
    out = {}
    for k, v in s.items():
        if k in ("counters", "node_range", "edge_range"):
            continue
        if k == "deliv":
            out[k] = [(h[n0:n1], f[n0:n1]) for h, f in v]
        elif k in ("backoff",) or k.startswith("ts_"):
            out[k] = np.asarray(v).reshape(T, -1)[:, e0:e1]
        else:
            out[k] = np.asarray(v)[e0:e1]
    return out


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint64) if a.dtype == np.float64 else a


def compare(a, b):
    """Returns a list of human-readable mismatches (empty = bit-exact)."""
    bad = []
    for k in a:
        if k in ("node_range", "edge_range"):
            continue
        if k == "counters":
            if a[k] != b[k]:
                bad.append(f"counters: {a[k]} != {b[k]}")
        elif k == "deliv":
            for i, ((h1, f1), (h2, f2)) in enumerate(zip(a[k], b[k])):
                if not (np.array_equal(h1, h2) and np.array_equal(f1, f2)):
                    bad.append(f"deliveries of message {i} differ")
                    break
        else:
            x, y = _bits(a[k]), _bits(b[k])
            if not np.array_equal(x, y):
                idx = np.argwhere(x != y)[:5]
                bad.append(f"{k}: {int((x != y).sum())} mismatches, first at {idx.tolist()}")
    return bad


# ---------------------------------------------------------------- adversarial
# The reference's attack tests restated on the simulator (gossipsub_spam_test.go,
# gossipsub_test.go:1388-1469, 1665-1815) and a config-5-like mix.  Each builder
# returns (engine, hops); tests/test_oracle_spam.py checks the reference's own
# assertions on the oracle, the GPU parity tests compare the engine with it.
from pubsub_amd import (GS_BEHAVE_GRAFT_SPAM, GS_BEHAVE_IHAVE_SPAM, GS_BEHAVE_IWANT_SPAM, GS_BEHAVE_NO_FORWARD,  # noqa: E402
                        GS_MSG_PHANTOM, GS_MSG_REJECT, DefaultPeerGaterParams, ScoreParameterDecay,
                        WithBehaviour, WithPeerGater, WithValidation)
from pubsub_amd.params import Minute  # noqa: E402


def _pair():
    """Two connected hosts (connect(t, hosts[0], hosts[1])): host 0 dialed."""
    return (np.array([0, 1, 2], dtype=np.int64), np.array([1, 0], dtype=np.int32),
            np.array([1, 0], dtype=np.uint8))


def _spam_score(bpw=-1.0):
    """The legit host's score params in gossipsub_spam_test.go:151-166 / 365-380."""
    return (PeerScoreParams(AppSpecificScore=True, BehaviourPenaltyWeight=bpw,
                            BehaviourPenaltyDecay=ScoreParameterDecay(Minute), DecayInterval=Second,
                            DecayToZero=0.01),
            PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-500, GraylistThreshold=-1000))


def spam_iwant(lib, extra=()):
    """TestGossipsubAttackSpamIWANT (gossipsub_spam_test.go:24-132): host 1
    re-requests every message it gets; host 0 publishes one message."""
    e = NewGossipSub(2, 1, _pair(), graphs.all_subscribed(2, 1), WithRecordDeliveries(), WithHop(HOP),
                     WithMessageWindow(64), WithBehaviour(np.array([0, GS_BEHAVE_IWANT_SPAM], np.uint8)),
                     *extra, lib=lib)
    e.publish([0], [0], [5])
    return e, 80


def spam_ihave(lib, topics=1, per_topic=3 * 5000, extra=()):
    """TestGossipsubAttackSpamIHAVE (gossipsub_spam_test.go:135-270): host 1
    advertises ids it never sends (3 x MaxIHaveLength of them)."""
    sp, thr = _spam_score()
    n_ph = topics * per_topic
    e = NewGossipSub(2, topics, _pair(), graphs.all_subscribed(2, topics), WithPeerScore(sp, thr),
                     WithHop(HOP), WithMessageWindow(((per_topic + 63) // 64) * 64),
                     WithBehaviour(np.array([0, GS_BEHAVE_IHAVE_SPAM], np.uint8)), *extra, lib=lib)
    e.publish(np.ones(n_ph, np.int32), np.repeat(np.arange(topics), per_topic).astype(np.int32),
              np.full(n_ph, 2, np.int64), kind=np.full(n_ph, GS_MSG_PHANTOM, np.uint8))
    e.snapshot_ids = []  # phantom ids are never delivered
    return e, 70


def spam_graft(lib, extra=()):
    """TestGossipsubAttackGRAFTDuringBackoff (gossipsub_spam_test.go:349-548):
    host 1 leaves host 0's mesh with a PRUNE, then GRAFTs during the backoff."""
    sp, thr = _spam_score(-100.0)
    e = NewGossipSub(2, 1, _pair(), graphs.all_subscribed(2, 1), WithPeerScore(sp, thr), WithHop(HOP),
                     WithMessageWindow(64), WithBehaviour(np.array([0, GS_BEHAVE_GRAFT_SPAM], np.uint8)),
                     *extra, lib=lib)
    e.snapshot_ids = []
    return e, 80


def spam_invalid(lib, extra=()):
    """TestGossipsubAttackInvalidMessageSpam (gossipsub_spam_test.go:563-703):
    host 1 sends 100 messages host 0's validator rejects (Eth2 scoring)."""
    sp = eth2_peer_score_params(1)
    thr = eth2_thresholds()
    e = NewGossipSub(2, 1, _pair(), graphs.all_subscribed(2, 1), WithPeerScore(sp, thr), WithHop(HOP),
                     WithMessageWindow(128), WithValidation([1]), WithRecordDeliveries(), *extra, lib=lib)
    e.publish(np.ones(100, np.int32), np.zeros(100, np.int32), 5 + np.arange(100, dtype=np.int64) // 10,
              kind=np.full(100, GS_MSG_REJECT, np.uint8))
    return e, 40


def squatters(lib, extra=()):
    """TestGossipsubOpportunisticGrafting (gossipsub_test.go:1665-1779): 10
    honest hosts (connectSome degree 5) and 40 sybilSquatters connected to every
    honest host; 1000 messages from the honest hosts."""
    n, honest = 50, 10
    r, c, o = graphs.connect_some(honest, 5, 31)
    pairs = [(int(u), int(v)) for u in range(honest) for v in c[r[u]:r[u + 1]] if o[r[u] + list(c[r[u]:r[u + 1]]).index(v)] and u < n]
    und = {(min(a, b), max(a, b)): a for a, b in pairs}
    for s in range(honest, n):
        for h in range(honest):
            und[(h, s)] = s  # connect(t, squatter, real): the squatter dials
    g = graphs._to_csr(n, np.array([[d, b if d == a else a] for (a, b), d in und.items()], dtype=np.int64))
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshWeight=0.0002777, TimeInMeshQuantum=Second,
                          TimeInMeshCap=3600, FirstMessageDeliveriesWeight=1,
                          FirstMessageDeliveriesDecay=0.9997, FirstMessageDeliveriesCap=100,
                          InvalidMessageDeliveriesDecay=0.99997)
    sp = PeerScoreParams(Topics={0: tp}, AppSpecificScore=True, AppSpecificWeight=0, DecayInterval=Second,
                         DecayToZero=0.01)
    thr = PeerScoreThresholds(GossipThreshold=-10, PublishThreshold=-100, GraylistThreshold=-10000,
                              OpportunisticGraftThreshold=1)
    gp = GossipSubParams(PruneBackoff=500 * Millisecond, GraftFloodThreshold=100 * Millisecond,
                         OpportunisticGraftTicks=2)
    beh = np.zeros(n, np.uint8)
    beh[honest:] = GS_BEHAVE_NO_FORWARD
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithPeerScore(sp, thr), WithGossipSubParams(gp),
                     WithFloodPublish(True), WithHop(HOP), WithMessageWindow(1024), WithBehaviour(beh),
                     WithRecordDeliveries(), *extra, lib=lib)
    # 1000 messages 20 ms apart = 5 per 100 ms hop, from hosts i % 10, after 1 s
    e.publish((np.arange(1000) % honest).astype(np.int32), np.zeros(1000, np.int32),
              10 + np.arange(1000, dtype=np.int64) // 5)
    e.honest = honest
    return e, 10 + 200 + 70


def sinkhole(lib, extra=()):
    """TestGossipsubNegativeScore (gossipsub_test.go:1388-1469): host 0 has app
    score -1000; 20 messages, one from every host."""
    n = 20
    sp = PeerScoreParams(AppSpecificScore=True, AppSpecificWeight=1, DecayInterval=Second, DecayToZero=0.01)
    thr = PeerScoreThresholds(GossipThreshold=-10, PublishThreshold=-100, GraylistThreshold=-10000)
    app = np.zeros(n)
    app[0] = -1000
    e = NewGossipSub(n, 1, graphs.dense_connect(n, 41), graphs.all_subscribed(n, 1), WithPeerScore(sp, thr),
                     WithRecordDeliveries(), WithHop(HOP), WithMessageWindow(64), *extra, app_score=app,
                     lib=lib)
    e.publish(np.arange(n, dtype=np.int32), np.zeros(n, np.int32), 30 + np.arange(n, dtype=np.int64) // 5)
    return e, 30 + 4 + 20


def adversarial_mix(lib, n=400, k=16, seed=51, sybil_frac=0.2, queue=6, msgs=600, hb=10, gater=True,
                    window=2048, churn=0, retain=None, px=0.0, extra=()):
    """A config-5-like mix: 20% Sybils split over IWANT spam,
    GRAFT spam, phantom-IHAVE spam and invalid-message publishing, 20 Sybils
    per shared IP (P6), the peer gater, topic validator with a bounded queue,
    Eth2 scoring.  churn: connections going down per 3 hops (each back after
    5-40 hops); retain: the gater's RetainStats; px: peer exchange on, with
    this fraction of the connections starting down (PX dials bring them up;
    pxConnect's PrunePeers truncation, gossipsub.go:856-905)."""
    rng = np.random.default_rng(seed)
    g = graphs.random_regular(n, k, seed)
    sybil = rng.random(n) < sybil_frac
    ids = np.flatnonzero(sybil)
    beh = np.zeros(n, np.uint8)
    kind_of = rng.integers(0, 4, len(ids))        # 0 IWANT spam, 1 GRAFT spam, 2 phantom IHAVE, 3 invalid
    beh[ids[kind_of == 0]] = GS_BEHAVE_IWANT_SPAM
    beh[ids[kind_of == 1]] = GS_BEHAVE_GRAFT_SPAM
    beh[ids[kind_of == 2]] = GS_BEHAVE_IHAVE_SPAM
    ipv4 = (np.arange(n) + (10 << 24)).astype(np.uint32)
    ipv4[ids] = (192 << 24) + (np.arange(len(ids)) // 20).astype(np.uint32)
    sp = eth2_peer_score_params(1)
    thr = eth2_thresholds()
    opts = [WithPeerScore(sp, thr), WithHop(HOP), WithMessageWindow(window), WithSeed(seed), WithBehaviour(beh),
            WithValidation([1], queue), WithRecordDeliveries()]
    if gater:
        gpar = DefaultPeerGaterParams()
        if retain is not None:
            gpar.RetainStats = retain
        opts.append(WithPeerGater(gpar))
    if px:
        rowptr, col, _ = g
        pairs = [(u, int(v)) for u in range(n) for v in col[rowptr[u]:rowptr[u + 1]] if u < v]
        prng = np.random.default_rng(seed + 91)
        dormant = [pairs[i] for i in np.flatnonzero(prng.random(len(pairs)) < px)]
        opts += [WithPeerExchange(True), WithDormant(dormant)]
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), *opts, *extra, ipv4=ipv4, lib=lib)
    if churn:
        crng = np.random.default_rng(seed + 77)
        pairs = _pairs_of(g, range(n))
        ev = []
        for h in range(12, hb * 10 - 10, 3):
            for i in crng.choice(len(pairs), churn, replace=False):
                a, b = pairs[i]
                ev.append((h, GS_EV_DISCONNECT, a, b))
                ev.append((h + int(crng.integers(5, 40)), GS_EV_CONNECT, a, b))
        ev.sort(key=lambda x: x[0])
        e.schedule_events([x[1] for x in ev], [x[2] for x in ev], [x[3] for x in ev], [x[0] for x in ev])
    honest_ids = np.flatnonzero(~sybil)
    hops = (5 + (np.arange(msgs) * (hb * 10 - 20)) // msgs).astype(np.int64)
    src = rng.choice(honest_ids, msgs).astype(np.int32)
    kind = np.zeros(msgs, np.uint8)
    inv = ids[kind_of == 3]
    ph = ids[kind_of == 2]
    # a third of the slots go to invalid messages, a sixth to phantom ids
    r = rng.random(msgs)
    if len(inv):
        sel = r < 1 / 3
        src[sel] = rng.choice(inv, int(sel.sum()))
        kind[sel] = GS_MSG_REJECT
    if len(ph):
        sel = (r >= 1 / 3) & (r < 0.5)
        src[sel] = rng.choice(ph, int(sel.sum()))
        kind[sel] = GS_MSG_PHANTOM
    e.publish(src, np.zeros(msgs, np.int32), hops, kind=kind)
    e.sybil = sybil
    return e, hb * 10 + 5


def promise_flood(lib, leaves=60, seed=53, follow_s=None, beats=9, extra=()):
    """More live IWANT promises per node than one wave's 64-entry bank: host 0
    at the centre of a star of 60 IHAVE spammers, each advertising a phantom id
    every heartbeat (gossipsub_spam_test.go:135-270).  Host 0 asks each one,
    promises (gossip_tracer.go:48-77), and every promise breaks 3 s later; with
    no P7 weight the spammers stay above GossipThreshold, so about 4 x 60
    promises are alive at once (the table holds degree x (IWantFollowupTime /
    HeartbeatInterval + 2) = 300 entries).  follow_s: IWantFollowupTime in
    seconds (with 12, about 13 x 60 promises live at once: the table's liveness
    bound is 840 entries); beats: phantom rounds."""
    n = leaves + 1
    rowptr = np.concatenate([[0, leaves], leaves + np.arange(1, leaves + 1)]).astype(np.int64)
    col = np.concatenate([np.arange(1, n), np.zeros(leaves)]).astype(np.int32)
    outbound = np.concatenate([np.ones(leaves), np.zeros(leaves)]).astype(np.uint8)
    sp = eth2_peer_score_params(1)
    sp.BehaviourPenaltyWeight = 0.0
    beh = np.zeros(n, np.uint8)
    beh[1:] = GS_BEHAVE_IHAVE_SPAM
    e = NewGossipSub(n, 1, (rowptr, col, outbound), graphs.all_subscribed(n, 1), WithPeerScore(sp, eth2_thresholds()),
                     WithBehaviour(beh), WithRecordDeliveries(), WithSeed(seed), WithHop(HOP),
                     WithMessageWindow(4096),
                     *(() if follow_s is None else (WithGossipSubParams(GossipSubParams(IWantFollowupTime=follow_s * Second)),)),
                     *extra, lib=lib)
    hops = np.repeat(np.arange(5, 10 * beats + 5, 10), leaves).astype(np.int64)
    src = np.tile(np.arange(1, n), beats).astype(np.int32)
    e.publish(src, np.zeros(len(src), np.int32), hops, kind=np.full(len(src), GS_MSG_PHANTOM, np.uint8))
    return e, 10 * beats + 10


ADVERSARIAL = {
    "promise_flood": lambda lib, x=(): promise_flood(lib, extra=x),
    # a promise table past 512 entries per node (its liveness bound, 840)
    "promise_flood_long": lambda lib, x=(): promise_flood(lib, follow_s=12, beats=24, extra=x),
    "spam_iwant": lambda lib, x=(): spam_iwant(lib, extra=x),
    "spam_ihave": lambda lib, x=(): spam_ihave(lib, extra=x),
    "spam_ihave_2t": lambda lib, x=(): spam_ihave(lib, topics=2, per_topic=4000, extra=x),
    "spam_graft": lambda lib, x=(): spam_graft(lib, extra=x),
    "spam_invalid": lambda lib, x=(): spam_invalid(lib, extra=x),
    "squatters": lambda lib, x=(): squatters(lib, extra=x),
    "sinkhole": lambda lib, x=(): sinkhole(lib, extra=x),
    "adversarial_mix": lambda lib, x=(): adversarial_mix(lib, extra=x),
    "adversarial_mix_nogater": lambda lib, x=(): adversarial_mix(lib, gater=False, queue=0, seed=52, extra=x),
}
SCENARIOS.update(ADVERSARIAL)
# bench.py config5 at a size the oracle finishes in seconds: degree 32, one
# topic x 10240 slots (W = 160, 3 words per lane), validation queue 32, ~60
# messages per hop, the ADV instantiations of phase A / phase B
HEAVY["c5shape"] = lambda lib, x=(): adversarial_mix(lib, n=2000, k=32, seed=53, queue=32, msgs=4000, hb=10,
                                                     window=10240, extra=x)
SCENARIOS["c5shape"] = HEAVY["c5shape"]


# ---------------------------------------------------------------- churn
# Connection churn and subscription changes (gs_schedule_events): the
# reference's RemovePeer / Prune / Graft tests restated, and a scored mix.
from pubsub_amd import GS_EV_CONNECT, GS_EV_DISCONNECT, GS_EV_JOIN, GS_EV_LEAVE  # noqa: E402


def _pairs_of(g, nodes):
    """Every connection (a < b) touching one of `nodes`."""
    rowptr, col, _ = g
    out = set()
    for u in nodes:
        for v in col[rowptr[u]:rowptr[u + 1]]:
            out.add((min(u, int(v)), max(u, int(v))))
    return sorted(out)


def churn_remove_peer(lib, extra=()):
    """TestGossipsubRemovePeer (gossipsub_test.go:629-676): 20 hosts, denseConnect,
    2 s of heartbeats, hosts 0-4 close (every connection down), a heartbeat, then
    10 messages from hosts 5-19 that hosts 5-19 must all receive."""
    n, seed = 20, 61
    g = graphs.dense_connect(n, seed)
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithRecordDeliveries(), WithSeed(seed),
                     WithHop(HOP), WithMessageWindow(64), *extra, lib=lib)
    pairs = _pairs_of(g, range(5))
    e.schedule_events([GS_EV_DISCONNECT] * len(pairs), [a for a, _ in pairs], [b for _, b in pairs],
                      [20] * len(pairs))
    rng = np.random.default_rng(seed)
    e.publish(5 + rng.integers(0, n - 5, 10), np.zeros(10, np.int32), 30 + np.arange(10))
    return e, 60


def churn_prune(lib, extra=()):
    """TestGossipsubPrune (gossipsub_test.go:535-582): hosts 0-4 cancel their
    subscription after the mesh formed (Leave -> PRUNE), 10 messages that
    hosts 5-19 must all receive."""
    n, seed = 20, 62
    g = graphs.dense_connect(n, seed)
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithRecordDeliveries(), WithSeed(seed),
                     WithHop(HOP), WithMessageWindow(64), *extra, lib=lib)
    e.schedule_events([GS_EV_LEAVE] * 5, list(range(5)), [0] * 5, [20] * 5)
    rng = np.random.default_rng(seed)
    e.publish(rng.integers(0, n, 10), np.zeros(10, np.int32), 21 + np.arange(10))
    return e, 50


def churn_graft(lib, extra=()):
    """TestGossipsubGraft (gossipsub_test.go:584-627): a sparse graph whose hosts
    subscribe one after another (Join -> GRAFT, announcements), then 100
    messages that every host must receive."""
    n, seed = 20, 63
    g = graphs.sparse_connect(n, seed)
    subs = np.zeros(n, dtype=np.uint64)
    e = NewGossipSub(n, 1, g, subs, WithRecordDeliveries(), WithSeed(seed), WithHop(HOP), WithMessageWindow(256),
                     *extra, lib=lib)
    e.schedule_events([GS_EV_JOIN] * n, list(range(n)), [0] * n, list(range(10, 10 + n)))
    rng = np.random.default_rng(seed)
    e.publish(rng.integers(0, n, 100), np.zeros(100, np.int32), 45 + np.arange(100))
    return e, 170


def churn_scored(lib, n=240, k=16, topics=2, seed=65, msgs=400, hb=14, extra=()):
    """A scored mix: 15% negative app scores and shared IPs (retained vs dropped
    records, P6 recounted), random connections going down and coming back,
    topics left and re-joined, Eth2 scoring with a RetainScore of 2 s."""
    rng = np.random.default_rng(seed)
    g = graphs.random_regular(n, k, seed)
    subs = graphs.all_subscribed(n, topics)
    sp = eth2_peer_score_params(topics)
    sp.RetainScore = 2 * Second
    thr = eth2_thresholds()
    app = np.zeros(n)
    app[rng.random(n) < 0.15] = -150.0
    ipv4 = (rng.integers(0, 60, n) + (10 << 24)).astype(np.uint32)
    e = NewGossipSub(n, topics, g, subs, WithPeerScore(sp, thr), WithRecordDeliveries(), WithSeed(seed),
                     WithHop(HOP), WithMessageWindow(512), *extra, app_score=app, ipv4=ipv4, lib=lib)
    pairs = _pairs_of(g, range(n))
    ev = []
    for h in range(12, hb * 10 - 10, 3):
        for i in rng.choice(len(pairs), 4, replace=False):
            a, b = pairs[i]
            ev.append((h, GS_EV_DISCONNECT, a, b))
            ev.append((h + int(rng.integers(5, 40)), GS_EV_CONNECT, a, b))
        for _ in range(2):
            a, t = int(rng.integers(0, n)), int(rng.integers(0, topics))
            ev.append((h, GS_EV_LEAVE, a, t))
            ev.append((h + int(rng.integers(3, 30)), GS_EV_JOIN, a, t))
    ev.sort(key=lambda x: x[0])
    e.schedule_events([x[1] for x in ev], [x[2] for x in ev], [x[3] for x in ev], [x[0] for x in ev])
    src = rng.integers(0, n, msgs).astype(np.int32)
    top = rng.integers(0, topics, msgs).astype(np.int32)
    hops = (5 + (np.arange(msgs) * (hb * 10 - 20)) // msgs).astype(np.int64)
    e.publish(src, top, hops)
    return e, hb * 10 + 5


CHURN = {
    # the peer gater under churn: peerGater.AddPeer / RemovePeer with a 2 s
    # RetainStats, so stats objects of disconnected IPs freeze, expire and
    # restart from zero (peer_gater.go:219-259, 366-383)
    "churn_gater": lambda lib, x=(): adversarial_mix(lib, n=300, seed=66, churn=6, retain=2 * Second, hb=12, extra=x),
    "churn_remove_peer": lambda lib, x=(): churn_remove_peer(lib, extra=x),
    "churn_prune": lambda lib, x=(): churn_prune(lib, extra=x),
    "churn_graft": lambda lib, x=(): churn_graft(lib, extra=x),
    "churn_scored": lambda lib, x=(): churn_scored(lib, extra=x),
}
SCENARIOS.update(CHURN)


# ---------------------------------------------------------------- RPC bytes
# Per-edge RPC byte accounting (gs_set_rpc_accounting)
# on top of scenarios that send every RPC kind: forwarded / published messages
# (floodsub, randomsub, gossipsub, fanout), GRAFT / PRUNE / IHAVE / IWANT,
# served replies, IWANT spam, squatters, hellos and announcements under churn.
# Message sizes straddle the one-byte varint boundary per topic.
from pubsub_amd import WithRPCAccounting  # noqa: E402


def _acct(T):
    return WithRPCAccounting(np.array([120 + 5 * t for t in range(T)], np.int32), id_len=30)


ACCT = {
    "acct_floodsub": lambda lib, x=(): floodsub_dense(lib, extra=(_acct(1),) + tuple(x)),
    "acct_randomsub": lambda lib, x=(): randomsub(lib, 100, extra=(_acct(1),) + tuple(x)),
    "acct_multitopic": lambda lib, x=(): gossipsub_scored(lib, n=200, topics=3, sub_frac=0.7, seed=7, msgs=240,
                                                          extra=(_acct(3),) + tuple(x)),
    "acct_graylist_direct": lambda lib, x=(): gossipsub_scored(lib, n=300, k=20, seed=23, app_neg_frac=0.15,
                                                               app_neg=-400.0, direct_frac=0.03,
                                                               extra=(_acct(1),) + tuple(x)),
    "acct_adversarial": lambda lib, x=(): adversarial_mix(lib, extra=(_acct(1),) + tuple(x)),
    "acct_churn": lambda lib, x=(): churn_scored(lib, extra=(_acct(2),) + tuple(x)),
}
SCENARIOS.update(ACCT)


# ---------------------------------------------------------------- peer exchange
# PRUNE peer exchange (WithPeerExchange, gossipsub.go:806-937, 1803-1839).
from pubsub_amd import WithDormant, WithPeerExchange  # noqa: E402


def px_star(lib, n=20, seed=71, extra=()):
    """TestGossipsubStarTopology (gossipsub_test.go:945-1024) restated: host 0
    dials hosts 1..n-1 (a star); every other pair is a connection slot that
    starts down.  D = 4, Dlo = 3, Dhi = 5, Dscore = 3, flood publish, PX on.
    The leaves' GRAFTs fill the centre's mesh (it dialled them: outbound peers
    pass the Dhi check), its heartbeat prunes the excess with PX, the pruned
    leaves dial the suggested peers and graft each other; then every host
    publishes a message that every host must receive."""
    rowptr = np.arange(0, n * (n - 1) + 1, n - 1, dtype=np.int64)
    col = np.array([v for u in range(n) for v in range(n) if v != u], dtype=np.int32)
    # the centre dials the leaves; a leaf pair is dialled by its lower index
    src = np.repeat(np.arange(n), n - 1)
    outbound = ((src == 0) | ((col != 0) & (src < col) & (src != 0))).astype(np.uint8)
    dormant = [(a, b) for a in range(1, n) for b in range(a + 1, n)]
    gp = GossipSubParams(D=4, Dlo=3, Dhi=5, Dscore=3)
    e = NewGossipSub(n, 1, (rowptr, col, outbound), graphs.all_subscribed(n, 1), WithGossipSubParams(gp),
                     WithPeerExchange(True), WithFloodPublish(True), WithDormant(dormant), WithRecordDeliveries(),
                     WithSeed(seed), WithHop(HOP), WithMessageWindow(64), *extra, lib=lib)
    e.publish(np.arange(n, dtype=np.int32), np.zeros(n, np.int32), 100 + np.arange(n))
    return e, 100 + n + 30


def px_scored(lib, extra=(), gater=False):
    """PX in a scored random graph with connection slots: 15% of every node's
    connections start down, negative app scores (noPX for negative-score
    prunes, AcceptPXThreshold), Dhi pruning of degree-24 nodes.  gater: the
    peer gater with a 2-entry validation queue, so PX dials (AddPeer) reach
    throttling gaters (peer_gater.go:366-372)."""
    n, k, seed = 200, 24, 72
    g = graphs.random_regular(n, k, seed)
    rowptr, col, _ = g
    rng = np.random.default_rng(seed)
    pairs = [(u, int(v)) for u in range(n) for v in col[rowptr[u]:rowptr[u + 1]] if u < v]
    dormant = [pairs[i] for i in np.flatnonzero(rng.random(len(pairs)) < 0.15)]
    sp = eth2_peer_score_params(1)
    app = np.where(rng.random(n) < 0.15, -150.0, 0.0)
    thr = eth2_thresholds()
    thr.AcceptPXThreshold = 0.0
    if gater:
        gpar = DefaultPeerGaterParams()
        gpar.RetainStats = 2 * Second
        extra = (WithPeerGater(gpar), WithValidation([1], 2)) + tuple(extra)
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithPeerScore(sp, thr), WithPeerExchange(True),
                     WithDormant(dormant), WithRecordDeliveries(), WithSeed(seed), WithHop(HOP),
                     WithMessageWindow(2048 if gater else 512), *extra, app_score=app, lib=lib)
    e.app_score = app  # for the test's checks
    src, top, hops = _publish_schedule(n, 1, 200, 20, 1, seed)
    e.publish(src, top, hops)
    return e, int(hops[-1]) + 40


def direct_peers(lib, seed=73, extra=()):
    """TestGossipsubDirectPeers (gossipsub_test.go:1122-1184) restated: hosts 1
    and 2 are direct peers, DirectConnectTicks = 2; host 0 connects to both, the
    1-2 connection starts down and the initial direct dial brings it up; the
    hosts subscribe, publish 3 messages; 1-2 closes, the heartbeat's
    directConnect redials it, 3 more messages reach everyone."""
    n = 3
    rowptr = np.array([0, 2, 4, 6], np.int64)
    col = np.array([1, 2, 0, 2, 0, 1], np.int32)
    outbound = np.array([1, 1, 0, 1, 0, 0], np.uint8)
    direct = np.array([0, 0, 0, 1, 0, 1], np.uint8)
    gp = GossipSubParams(DirectConnectTicks=2)
    e = NewGossipSub(n, 1, (rowptr, col, outbound), np.zeros(n, np.uint64), WithGossipSubParams(gp),
                     WithDirectPeers(direct), WithDormant([(1, 2)]), WithRecordDeliveries(), WithSeed(seed),
                     WithHop(HOP), WithMessageWindow(64), *extra, lib=lib)
    e.schedule_events([GS_EV_JOIN] * 3 + [GS_EV_DISCONNECT], [0, 1, 2, 1], [0, 0, 0, 2], [20, 20, 20, 40])
    e.publish(np.array([0, 1, 2, 0, 1, 2], np.int32), np.zeros(6, np.int32),
              np.array([30, 31, 32, 90, 91, 92], np.int64))
    return e, 110


def direct_churn(lib, extra=()):
    """Scored random graph with 5% direct connections: half of them start
    down (dialled after DirectConnectInitialDelay), the rest close at random
    hops and are redialled by directConnect every 3 heartbeats; ordinary
    connections churn beside them."""
    n, k, seed = 200, 16, 74
    g = graphs.random_regular(n, k, seed)
    rowptr, col, _ = g
    src = np.repeat(np.arange(n), np.diff(rowptr))
    rng = np.random.default_rng(seed)
    pairs = sorted({(min(int(a), int(b)), max(int(a), int(b))) for a, b in zip(src, col)})
    dpairs = [pairs[i] for i in np.flatnonzero(rng.random(len(pairs)) < 0.05)]
    dset = set(dpairs)
    direct = np.array([(min(a, b), max(a, b)) in dset for a, b in zip(src, col)], np.uint8)
    dormant = dpairs[::2]
    ev = []
    for h in range(15, 120, 7):
        a, b = dpairs[1::2][int(rng.integers(0, len(dpairs[1::2])))]
        ev.append((h, GS_EV_DISCONNECT, a, b))
        a, b = pairs[int(rng.integers(0, len(pairs)))]
        ev.append((h, GS_EV_DISCONNECT, a, b))
        ev.append((h + int(rng.integers(3, 20)), GS_EV_CONNECT, a, b))
    ev.sort(key=lambda x: x[0])
    gp = GossipSubParams(DirectConnectTicks=3, DirectConnectInitialDelay=500 * Millisecond)
    sp = eth2_peer_score_params(1)
    thr = eth2_thresholds()
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithGossipSubParams(gp), WithPeerScore(sp, thr),
                     WithDirectPeers(direct), WithDormant(dormant), WithRecordDeliveries(), WithSeed(seed),
                     WithHop(HOP), WithMessageWindow(512), *extra, lib=lib)
    e.schedule_events([x[1] for x in ev], [x[2] for x in ev], [x[3] for x in ev], [x[0] for x in ev])
    src_ = rng.integers(0, n, 240).astype(np.int32)
    e.publish(src_, np.zeros(240, np.int32), (5 + np.arange(240) // 2).astype(np.int64))
    e.direct_pairs, e.dormant_pairs = dpairs, dormant
    return e, 150


PX = {
    "px_star": lambda lib, x=(): px_star(lib, extra=x),
    "direct_peers": lambda lib, x=(): direct_peers(lib, extra=x),
    "direct_churn": lambda lib, x=(): direct_churn(lib, extra=x),
    "px_scored": lambda lib, x=(): px_scored(lib, extra=x),
    "px_gater": lambda lib, x=(): px_scored(lib, extra=x, gater=True),
    # PX beside the attackers: GRAFT spammers' PRUNE replies
    # and the honest hosts' heartbeat prunes of negative-score peers, dials into
    # slots that start down, IWANT spam on the new connections
    "px_adversarial": lambda lib, x=(): adversarial_mix(lib, n=300, seed=67, hb=12, px=0.15, extra=x),
    # PX under RPC byte accounting: every PRUNE carries its PeerInfo entries
    # (makePrune, gossipsub.go:1811-1836; 38-byte peer ids, no signed records)
    "acct_px_scored": lambda lib, x=(): px_scored(lib, extra=(_acct(1),) + tuple(x)),
    "acct_px_adversarial": lambda lib, x=(): adversarial_mix(lib, n=300, seed=67, hb=12, px=0.15,
                                                             extra=(_acct(1),) + tuple(x)),
    "acct_px_star_records": lambda lib, x=(): px_star(lib, extra=(WithRPCAccounting(130, id_len=30, peer_id_len=39,
                                                                                    record_len=200),) + tuple(x)),
}
SCENARIOS.update(PX)


# ---------------------------------------------------------------- mixed networks
# Hosts running different routers and connections running different protocols
# (gs_set_routers / gs_set_graph_ex; PubSubRouter.AddPeer(peer.ID, protocol.ID),
# pubsub.go:165; gossipsub_feat.go:18-56).
from pubsub_amd import (GS_ROUTER_FLOODSUB, GS_ROUTER_GOSSIPSUB, GS_ROUTER_GOSSIPSUB_V10,  # noqa: E402
                        GS_ROUTER_RANDOMSUB, WithRouters)


def mixed_gossip_flood(lib, seed=81, extra=()):
    """TestMixedGossipsub (gossipsub_test.go:810-851): 30 hosts, 20 run
    gossipsub and 10 floodsub, sparseConnect, one topic, 2 s of heartbeats, then
    100 messages from random owners; every host must get every message."""
    n = 30
    g = graphs.sparse_connect(n, seed)
    routers = np.array([GS_ROUTER_GOSSIPSUB] * 20 + [GS_ROUTER_FLOODSUB] * 10, np.uint8)
    e = NewGossipSub(n, 1, g, graphs.all_subscribed(n, 1), WithRouters(routers), WithRecordDeliveries(),
                     WithSeed(seed), WithHop(HOP), WithMessageWindow(256), *extra, lib=lib)
    src, top, hops = _publish_schedule(n, 1, 100, 20, 1, seed)
    e.publish(src, top, hops)
    return e, int(hops[-1]) + 40


def mixed_routers(n, seed, flood=0.15, v10=0.15, rs=0.10):
    """Per-host routers: the given fractions run floodsub, gossipsub v1.0 and
    randomsub, the rest gossipsub v1.1."""
    r = np.random.default_rng(seed + 31).random(n)
    routers = np.full(n, GS_ROUTER_GOSSIPSUB, np.uint8)
    routers[r < flood + v10 + rs] = GS_ROUTER_RANDOMSUB
    routers[r < flood + v10] = GS_ROUTER_GOSSIPSUB_V10
    routers[r < flood] = GS_ROUTER_FLOODSUB
    return routers


def mixed_scored(lib, n=300, k=20, topics=3, seed=82, msgs=300, hb=12, px=True, extra=()):
    """A scored mixed network: 15% floodsub, 15% gossipsub-v1.0-only and 10%
    randomsub (size 50) hosts among gossipsub v1.1 ones, 3 topics with 70%
    subscription (publishes to unjoined topics use fanout), negative app
    scores around PublishThreshold (-200): a gossipsub host forwards to its
    non-mesh peers only at score >= PublishThreshold (gossipsub.go:969-975).
    PX on with 10% of the connections starting down: v1.0 peers get PRUNEs
    without PX and backoff (gossipsub.go:1804-1807), PX lists hold
    mesh-capable peers only (getPeers, :1849)."""
    rng = np.random.default_rng(seed)
    g = graphs.random_regular(n, k, seed)
    rowptr, col, _ = g
    routers = mixed_routers(n, seed)
    subs = np.zeros(n, dtype=np.uint64)
    for t in range(topics):
        subs |= (rng.random(n) < 0.7).astype(np.uint64) << np.uint64(t)
    sp = eth2_peer_score_params(topics)
    thr = eth2_thresholds()
    thr.AcceptPXThreshold = 0.0
    app = np.zeros(n)
    neg = rng.random(n)
    app[neg < 0.08] = -250.0   # below PublishThreshold, above GraylistThreshold
    app[(neg >= 0.08) & (neg < 0.15)] = -150.0
    opts = [WithPeerScore(sp, thr), WithRouters(routers), WithRecordDeliveries(), WithSeed(seed), WithHop(HOP),
            WithMessageWindow(512)]
    if px:
        pairs = [(u, int(v)) for u in range(n) for v in col[rowptr[u]:rowptr[u + 1]] if u < v]
        dormant = [pairs[i] for i in np.flatnonzero(rng.random(len(pairs)) < 0.10)]
        opts += [WithPeerExchange(True), WithDormant(dormant)]
    e = NewGossipSub(n, topics, g, subs, *opts, *extra, app_score=app, randomsub_size=50, lib=lib)
    rng2 = np.random.default_rng(seed + 100)
    src = rng2.integers(0, n, msgs).astype(np.int32)
    top = rng2.integers(0, topics, msgs).astype(np.int32)
    hops = (5 + (np.arange(msgs) * (hb * 10 - 20)) // msgs).astype(np.int64)
    e.publish(src, top, hops)
    e.routers_h = routers
    return e, hb * 10 + 5


def mixed_randomsub(lib, n=200, k=16, seed=83, msgs=60, extra=()):
    """randomsub.go:99-160 in a network where 30% of the hosts run floodsub:
    a randomsub host always forwards to its floodsub-protocol topic peers and
    samples max(6, ceil(sqrt(100))) = 10 of its randomsub-protocol ones."""
    g = graphs.random_regular(n, k, seed)
    routers = np.where(np.random.default_rng(seed).random(n) < 0.3, GS_ROUTER_FLOODSUB,
                       GS_ROUTER_RANDOMSUB).astype(np.uint8)
    e = NewRandomSub(n, 1, g, graphs.all_subscribed(n, 1), 100, WithRouters(routers), WithRecordDeliveries(),
                     WithSeed(seed), WithMessageWindow(128), *extra, lib=lib)
    src, top, hops = _publish_schedule(n, 1, msgs, 0, 1, seed)
    e.publish(src, top, hops)
    e.routers_h = routers
    return e, int(hops[-1]) + 20


MIXED = {
    "mixed_gossip_flood": lambda lib, x=(): mixed_gossip_flood(lib, extra=x),
    "mixed_scored": lambda lib, x=(): mixed_scored(lib, extra=x),
    "mixed_randomsub": lambda lib, x=(): mixed_randomsub(lib, extra=x),
    "acct_mixed": lambda lib, x=(): mixed_scored(lib, px=False, seed=84, extra=(_acct(3),) + tuple(x)),
    # with PX: v1.1 peers' PRUNEs carry PeerInfo entries, v1.0 peers' none
    "acct_mixed_px": lambda lib, x=(): mixed_scored(lib, seed=86, extra=(_acct(3),) + tuple(x)),
    # T >= 4: k_push is on, so its randomsub filter (rs_host && sel) and the
    # floodsub-peer publish filter run in the pushed segments
    "mixed_scored_4t": lambda lib, x=(): mixed_scored(lib, topics=4, seed=85, msgs=400, extra=x),
}
SCENARIOS.update(MIXED)
