"""The benchmarked configurations at their BASELINE.json sizes, on the GPU.

The oracle cannot simulate 1M peers in a test's time, so these runs are checked
by what holds at any size, plus a true oracle check of score():
  * every subscriber gets every message exactly once (deliveries =
    published x (N - 1) once the schedule has drained; the seen set makes a
    second first delivery impossible);
  * every copy on the wire is a delivery or a duplicate (deliveries +
    duplicates = transmissions, nothing graylisted in these honest runs);
  * no device error (a capacity or model error raises in step());
  * score() of a few thousand sampled edges, recomputed by the oracle's own
    PeerScore from the engine's counters (tests/score_check.py, pinned on
    the oracle by tests/test_score_check.py), equals gs_read_scores bit for
    bit: a21 at E x T = 2.05e9 (edge, topic) pairs;
  * router-specific closed forms (floodsub / randomsub transmissions).
The engines are built by bench.build_engine, i.e. exactly the benchmarked
workload (graph, schedule, params), with the schedule cut to a few rounds."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import bench  # noqa: E402
from replay import HostReplay, compare_events, compare_state, engine_state  # noqa: E402
from score_check import oracle_scores, sample_edges  # noqa: E402

pytestmark = pytest.mark.gpu

H = bench.HOPS_PER_ROUND


def _drain_and_check(e, rounds, extra_hops):
    """Join + `rounds` rounds of publishes + extra hops; the common properties."""
    e.step(1 + rounds * H + extra_hops)
    c = e.counters()
    published = rounds * bench.MSGS_PER_ROUND
    assert c["published"] == published
    assert c["deliveries"] == published * (e.N - 1), c
    assert c["graylisted"] == 0, c
    assert c["deliveries"] + c["duplicates"] == c["transmissions"], c
    return c


def _score_check(olib, e, n=3000, seed=7):
    edges = sample_edges(e.E, n, seed, must=[0, e.E - 1])
    got, st = oracle_scores(olib, e.score_params, e, edges)
    want = e.scores()[edges]
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert len(bad) == 0, f"{len(bad)} of {len(edges)} scores differ, first edge {edges[bad[0]]}: " \
                          f"engine {want[bad[0]]!r} oracle {got[bad[0]]!r}"
    # the sample is not trivial: mesh members with time in mesh and deliveries
    assert (st["flags"] & 1).mean() > 0.05, (st["flags"] & 1).mean()
    assert (st["fmd"] > 0).mean() > 0.05 and (st["mesh_time"] > 0).any()
    return got


def test_config4_full_size(olib):
    """BASELINE configs[3] on one GPU: 1M peers, k = 32, 64 topics, Eth2
    scoring, 1000 msgs/round, at the benchmarked steady state: 16 rounds of
    publishes after Join (hop 161), drained.  From about hop 50 the gossip
    bound holds more than MaxIHaveLength ids, so phase B runs its sender-cut
    instantiation on every later hop, and every one of the 192 slots per topic
    is recycled once (phase A pass 2b's seen retirement, k_publish re-setting the author's bit) -- the hops bench.py times."""
    wl = bench.WORKLOADS["config4"]
    rounds = 16
    e, g = bench.build_engine(wl, rounds, 3, 0)
    assert rounds * bench.MSGS_PER_ROUND / wl["topics"] > wl["slots"]  # slots recycled
    _drain_and_check(e, rounds, 3 * H)
    scores = _score_check(olib, e)
    assert np.isfinite(scores).all()
    mesh = e.mesh()
    sizes = np.add.reduceat(np.bitwise_count(mesh).astype(np.int64), g[0][:-1]) / wl["topics"]
    from pubsub_amd.params import GossipSubParams
    gp = GossipSubParams()
    assert gp.Dlo <= np.median(sizes) <= gp.Dhi, np.median(sizes)  # meshes maintained per (node, topic)


def _replay_check(oracle_path, name, rounds, nhosts, seed=3):
    """Sampled hosts of the full-size run replayed on the oracle (tests/replay.py):
    the engine traces `nhosts` random hosts (plus hosts 0 and N-1) with RPC
    events; after every round each host's RecvRPC blocks drive its oracle
    replay (the per-host phase bodies of the oracle simulation), and the
    replay's events -- every DeliverMessage with its first deliverer, every
    DuplicateMessage, Graft / Prune / Join, every SendRPC with its forwarded
    messages, IHAVE ids, IWANT lists, GRAFTs and PRUNEs -- must equal the
    engine's, byte for byte.  At the end the hosts' mesh / fanout masks,
    backoff expiries, fmd / mmd / mfp / imd, meshTime / graftTime / flags,
    behaviour penalties and scores must equal the engine's bit for bit.  So
    every state transition of the sampled hosts is checked, at the
    benchmarked size, against the reference's restated router and score
    code (gossipsub.go:591-1552, score.go:256-964, pubsub.go:902-1022)."""
    from pubsub_amd import WithEventTracer
    wl = bench.WORKLOADS[name]
    rng = np.random.default_rng(17)
    hosts = np.unique(np.concatenate([[0, wl["n"] - 1], rng.choice(wl["n"], nhosts, replace=False)]))
    e, g = bench.build_engine(wl, rounds, seed, 0, extra=(WithEventTracer(hosts, capacity=1 << 25, rpc=True),))
    # one never-stepped oracle engine with the run's exact inputs hosts every replay
    oe, _ = bench.build_engine(wl, rounds, seed, 0, lib=oracle_path, graph=g)
    reps = {int(u): HostReplay(oe, int(u)) for u in hosts}
    chunks = [1 + H] + [H] * (rounds + 2)  # (drained every round: the device trace buffer's size)
    bad, checked = [], 0
    for k in chunks:
        e.step(k)
        ev = e.trace_events()
        order = np.argsort(ev["node"], kind="stable")
        nodes_sorted = ev["node"][order]
        for u in hosts:
            lo, hi = np.searchsorted(nodes_sorted, [u, u + 1])
            mine = ev[np.sort(order[lo:hi])]
            r = reps[int(u)]
            r.run(k, mine)
            bad += compare_events(r.events(), mine, int(u))
            checked += len(mine)
        print(f"{name} replay: hop {e.hop}, {len(ev)} events, {checked} host events checked", flush=True)
        assert not bad, "\n".join(bad[:12])
    want = engine_state(e, hosts)
    for u in hosts:
        bad += compare_state(reps[int(u)].state(), want[int(u)], int(u))
    assert not bad, "\n".join(bad[:12])
    for r in reps.values():
        r.close()
    oe.close()
    return e, checked


def test_config4_replay_sampled_hosts(oracle_path):
    """N1 at the headline size: config4 (1M peers x 64 topics, Eth2 scoring,
    1000 msgs/round) for 16 rounds of publishes plus the drain -- joins, the
    steady state with recycled slots and every heartbeat -- with 96 sampled
    hosts replayed bit-exactly on the oracle from their own RPC streams."""
    e, checked = _replay_check(oracle_path, "config4", 16, 128)
    assert checked > 1e7, checked
    c = e.counters()
    assert c["deliveries"] == 16 * bench.MSGS_PER_ROUND * (e.N - 1), c


def test_config3_replay_sampled_hosts(oracle_path):
    """The same at config3 (1M peers, 1 topic) into the MaxIHaveLength cut
    steady state: the sampled hosts' IHAVE subsets, IWANT cuts and promises."""
    e, checked = _replay_check(oracle_path, "config3", 9, 48)
    assert e.counters()["ihave_sent"] > 0 and checked > 1e6


def test_config5_replay_sampled_hosts(oracle_path):
    """The same at config5's adversarial mix (1M peers, 20% Sybils, gater,
    validation queue): the sampled hosts' AcceptFrom / gater draws,
    validation verdicts, P4 / P7 penalties and broken promises."""
    e, checked = _replay_check(oracle_path, "config5", 7, 48)
    c = e.counters()
    assert c["promises_broken"] > 0 and c["gated"] > 0 and checked > 1e6, c


def test_config3_full_size_with_ihave_cuts(olib):
    """BASELINE configs[2]: 1M peers, one topic x 10048 slots, 1000 msgs per
    heartbeat.  Nine rounds of publishes reach the steady state in which a
    gossip window holds more ids than MaxIHaveLength (5000): phase B runs
    its cut instantiation and the receivers take the senders' keyed subsets
    (gossipsub.go:650-653, 1702-1709)."""
    wl = bench.WORKLOADS["config3"]
    rounds = 9
    e, _ = bench.build_engine(wl, rounds, 3, 0)
    # the engine's cut-mode bound (gs_engine.hip stepOne): messages published
    # within HistoryGossip + 1 heartbeats plus the delivery age bound
    per_hop = bench.MSGS_PER_ROUND // H
    window = (5 + 1) * H + 3 * H + 2
    assert per_hop * window > 5000
    # the gossip windows (5 heartbeats of mcache) hold ~5000 ids plus the late
    # ones: real cuts from round ~7
    c = _drain_and_check(e, rounds, 3 * H)
    assert c["ihave_sent"] > 0 and c["iwant_sent"] > 0
    _score_check(olib, e)


def test_config5_full_size_steady_state(olib):
    """BASELINE configs[4]'s adversarial mix on one GPU at 1M peers (bench.py
    --workload config5), past its broken-promise regime: the first IWANT
    promise can break at hop 50 (IWantFollowupTime = 3 s after the hop-11
    IWANTs), so 7 rounds (hop 71) reach P7 penalties, graylisting, validation
    rejections, queue-full throttling and gater drops all at once
    (gossip_tracer.go:79-117, gossipsub.go:1566-1571, peer_gater.go:320-363).
    Checked: no device error (step raises on one), every adversarial counter
    active after round 5, the copy accounting (every copy on the wire is a
    delivery, a duplicate, a rejection, a queue drop, or inside a graylisted or
    gated RPC), and 3,000 sampled scores -- P4 invalid deliveries, P6 shared
    IPs and the P7 behaviour penalty included -- recomputed bit for bit by the
    oracle's score() from the engine's counters."""
    from pubsub_amd import GS_MSG_VALID
    wl = bench.WORKLOADS["config5"]
    rounds = 7
    e, g = bench.build_engine(wl, rounds, 3, 0)
    e.step(1 + 5 * H)
    c5 = e.counters()
    for k in ("promises_broken", "graylisted", "rejected", "throttled", "gated"):
        assert c5[k] > 0, (k, c5)
    e.step(2 * H + 1)
    c = e.counters()
    assert c["promises_broken"] > c5["promises_broken"], c
    handled = c["deliveries"] + c["duplicates"] + c["rejected"] + c["throttled"]
    # graylisted / gated count RPCs, each carrying at least one copy
    assert handled + c["graylisted"] + c["gated"] <= c["transmissions"], c
    valid = int((e.kinds == GS_MSG_VALID).sum())
    assert c["deliveries"] <= valid * (e.N - 1)
    assert c["deliveries"] > 0.9 * valid * (e.N - 1), (c["deliveries"], valid)
    bp = e.behaviour_penalty()
    rng = np.random.default_rng(5)
    pen = np.flatnonzero(bp > 0)
    assert len(pen) > 0
    # edges towards invalid-message authors carry P4 (imd)
    from pubsub_amd import GS_MSG_REJECT
    inv = np.unique(e.srcs[e.kinds == GS_MSG_REJECT])
    to_inv = np.flatnonzero(np.isin(e.col, inv))
    edges = np.unique(np.concatenate([sample_edges(e.E, 2000, 7, must=[0, e.E - 1]),
                                      rng.choice(pen, min(1000, len(pen)), replace=False),
                                      rng.choice(to_inv, min(500, len(to_inv)), replace=False)]))
    got, st = oracle_scores(olib, e.score_params, e, edges, ipv4=e.ipv4)
    want = e.scores()[edges]
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert len(bad) == 0, f"{len(bad)} of {len(edges)} scores differ, first edge {edges[bad[0]]}: " \
                          f"engine {want[bad[0]]!r} oracle {got[bad[0]]!r}"
    assert (st["imd"] > 0).any() and (bp[edges] > 0).sum() >= min(1000, len(pen))
    assert (want < 0).any()  # penalised peers are in the sample


@pytest.mark.parametrize("size", ["100", "N"])
def test_config2_randomsub_100k(size):
    """BASELINE configs[1], the randomsub leg: 100k peers, random 32-regular
    graph, 1 topic, 10,000 messages at hop 0.  size = 100 samples
    max(6, ceil(sqrt(100))) = 10 targets per forward (randomsub.go:115-149);
    size = N degenerates to floodsub (every candidate)."""
    from pubsub_amd import NewRandomSub, WithMessageWindow, WithSeed, graphs
    n, k, m = 100_000, 32, 10_000
    rowptr, col, outbound = graphs.random_regular_fast(n, k, 2)
    deg = np.diff(rowptr)
    assert deg.min() >= 12  # every holder has more than 10 candidates
    rs = 100 if size == "100" else n
    e = NewRandomSub(n, 1, (rowptr, col, outbound), graphs.all_subscribed(n, 1), rs, WithSeed(2),
                     WithMessageWindow(10_048))
    rng = np.random.default_rng(2)
    e.publish(rng.integers(0, n, m).astype(np.int32), np.zeros(m, np.int32), np.zeros(m, np.int64))
    e.step(40)
    c = e.counters()
    assert c["published"] == m
    assert c["duplicates"] == c["transmissions"] - c["deliveries"]
    if size == "N":
        # floodsub's closed form (tests/test_scale_gpu.py)
        assert c["deliveries"] == m * (n - 1)
        assert c["transmissions"] == m * (int(deg.sum()) - (n - 1))
    else:
        # every holder (the author, then every first receiver) sends exactly
        # 10 copies: its candidates (all but the sender and the author) number
        # at least deg - 2 > 10, and the keyed shuffle takes 10 of them
        assert c["transmissions"] == 10 * (m + c["deliveries"])
        # a node is missed only if none of its ~32 holders picked it
        assert c["deliveries"] > 0.999 * m * (n - 1)
        assert c["deliveries"] <= m * (n - 1)
