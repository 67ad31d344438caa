"""Direct peers' connector (gossipsub.go:492-502 initial dial after
DirectConnectInitialDelay, directConnect :1594-1616 every DirectConnectTicks
heartbeats).

CPU, the oracle:
  * TestGossipsubDirectPeers (gossipsub_test.go:1122-1184) restated: the
    direct pair's connection, down at the start, comes up after the initial
    delay; closed, it comes back at the next directConnect tick; every message
    reaches every host both times;
  * a scored random graph with churn: every direct connection that is down is
    back within DirectConnectTicks heartbeats, ordinary connections are never
    dialled by the connector, and the run ends with every direct pair up.
GPU: both scenarios equal the oracle (readbacks in test_parity_gpu, the event
trace here)."""
import numpy as np
import pytest

import scenarios
from pubsub_amd import PRODUCT_LIB, GossipSubParams, NewGossipSub, GossipEngineError, WithEventTracer, \
    WithGossipSubParams, _abi, graphs

T = _abi.TRACE_TYPES.index


def _run(lib, name, nodes):
    e, hops = scenarios.SCENARIOS[name](lib, (WithEventTracer(nodes),))
    e.step(hops)
    return e, hops, e.trace_events()


def _conn(ev, a, b):
    """(hop, up) of node a's AddPeer / RemovePeer events for peer b."""
    m = (ev["node"] == a) & (ev["peer"] == b) & ((ev["type"] == T("ADD_PEER")) | (ev["type"] == T("REMOVE_PEER")))
    return [(int(r["hop"]), int(r["type"]) == T("ADD_PEER")) for r in ev[m]]


def test_oracle_direct_peers(oracle_path):
    e, hops, ev = _run(oracle_path, "direct_peers", [0, 1, 2])
    # the initial dial (DirectConnectInitialDelay = 1 s = hop 10) connects at
    # hop 11; the close at hop 40 is redialled at the heartbeat of tick 6
    # (hop 51: heartbeats at 1, 11, 21, ...; DirectConnectTicks = 2) -> hop 52
    assert _conn(ev, 1, 2) == [(11, True), (40, False), (52, True)]
    assert _conn(ev, 2, 1) == [(11, True), (40, False), (52, True)]
    assert _conn(ev, 0, 1) == [(0, True)]
    for m in range(e.n_published):
        hop, _ = e.deliveries(m)
        assert (hop >= 0).all(), m


def test_oracle_direct_churn(oracle_path):
    e, hops, ev = _run(oracle_path, "direct_churn", list(range(200)))
    dset = set(e.direct_pairs)
    ticks_hops = 3 * 10  # DirectConnectTicks heartbeats of 10 hops
    late_adds = 0
    for a, b in e.direct_pairs:
        c = _conn(ev, a, b)
        assert c and c[-1][1], (a, b, c)                # up at the end
        for (h0, up0), (h1, up1) in zip(c, c[1:]):
            if not up0:
                assert up1 and h1 - h0 <= ticks_hops + 1, (a, b, c)
        if (a, b) in set(e.dormant_pairs):
            assert c[0] == (6, True), c                  # InitialDelay 500 ms -> dial at hop 5
        late_adds += sum(1 for h, up in c if up and h > 0)
    assert late_adds > len(e.dormant_pairs)              # redials after closes happened
    # the connector dials nothing but direct peers: every other late AddPeer is
    # a scheduled GS_EV_CONNECT
    adds = ev[(ev["type"] == T("ADD_PEER")) & (ev["hop"] > 0)]
    for r in adds:
        p = (min(int(r["node"]), int(r["peer"])), max(int(r["node"]), int(r["peer"])))
        if p not in dset:
            assert int(r["hop"]) >= 15
    for m in range(e.n_published):
        hop, _ = e.deliveries(m)
        assert (hop >= 0).mean() > 0.99, m


@pytest.mark.parametrize("lib", ["oracle", pytest.param("product", marks=pytest.mark.gpu)])
def test_direct_connect_ticks_zero_is_rejected(lib, oracle_path):
    path = oracle_path if lib == "oracle" else PRODUCT_LIB
    g = graphs.dense_connect(4, 1)
    with pytest.raises(GossipEngineError) as ei:
        NewGossipSub(4, 1, g, graphs.all_subscribed(4, 1), WithGossipSubParams(GossipSubParams(DirectConnectTicks=0)),
                     lib=path)
    assert ei.value.code == _abi.GS_EINVAL


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["direct_peers", "direct_churn"])
def test_gpu_direct_trace_equals_oracle(name, oracle_path):
    nodes = [0, 1, 2] if name == "direct_peers" else list(range(200))
    _, _, ew = _run(oracle_path, name, nodes)
    _, _, eg = _run(PRODUCT_LIB, name, nodes)
    assert len(eg) == len(ew) and np.array_equal(eg, ew)
