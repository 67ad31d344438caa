"""Peer exchange (WithPeerExchange: makePrune's peer list gossipsub.go:1803-1839,
handlePrune's PX acceptance :827-836, pxConnect :856-905) over connection slots
that start down (gs_set_dormant).

CPU, the oracle:
  * TestGossipsubStarTopology (gossipsub_test.go:945-1024) restated: a star
    whose centre prunes its overfull mesh with PX; every leaf ends with more
    than one connection, and a message from every host reaches every host;
  * the RPC trace carries the PX lists: at most PrunePeers peers, never the
    pruned peer itself, each a connected topic peer of the pruner; a
    scored mix: no PX on the PRUNEs of negative-score peers (noPX,
    gossipsub.go:1350-1356), and PX from a pruner below AcceptPXThreshold is
    not dialled;
  * the encoders write ControlPruneMeta.peers.
GPU: the engine equals the oracle bit for bit on both scenarios (readbacks in
test_parity_gpu, the RPC trace with the PX lists here); PX with RPC
accounting is refused (the accounting does not size PX records)."""
import base64
import json

import numpy as np
import pytest

import scenarios
from pubsub_amd import PRODUCT_LIB, GossipEngineError, WithEventTracer, _abi, encode_trace
from test_trace import _fields, _varint
from test_trace_rpc import blocks

T = _abi.TRACE_TYPES.index
SEND, RECV, ITEM = T("SEND_RPC"), T("RECV_RPC"), _abi.GS_TRACE_RPC_ITEM


def _run(lib, name, nodes):
    e, hops = scenarios.SCENARIOS[name](lib, (WithEventTracer(nodes, rpc=True),))
    # read the trace every few hops: a 300-node adversarial run records more
    # events than the default capacity holds between two reads
    parts = []
    for h0 in range(0, hops, 8):
        e.step(min(8, hops - h0))
        parts.append(e.trace_events())
    return e, hops, np.concatenate(parts)


def test_oracle_star_topology_bootstraps_through_px(oracle_path):
    n = 20
    e, hops, ev = _run(oracle_path, "px_star", list(range(n)))
    adds = ev[ev["type"] == T("ADD_PEER")]
    conns = np.bincount(adds["node"], minlength=n)
    assert conns[0] == n - 1
    assert (conns[1:] > 1).all(), conns          # "peer %d has ony a single connection"
    assert conns[1:].sum() > n - 1                # the leaves dialled each other
    # a message from every host reached every host (assertReceive for all subs)
    for m in range(e.n_published):
        hop, _ = e.deliveries(m)
        assert (hop >= 0).all(), m
    # the centre's PRUNEs carried peers; every PX list is short and sound
    npx = 0
    for hd, items in blocks(ev):
        if hd["type"] != SEND:
            continue
        px = items[items["reason"] == _abi.GS_RPC_ITEM_PX]
        for t in set(px["topic"].tolist()):
            peers = px["msg"][px["topic"] == t]
            assert len(peers) <= 16 and int(hd["peer"]) not in peers.tolist()
            npx += len(peers)
    assert npx > 0


def test_oracle_px_scored_rules(oracle_path):
    nodes = list(range(200))
    e, hops, ev = _run(oracle_path, "px_scored", nodes)
    app = e.app_score
    n_px = 0
    offered = set()   # (receiver, suggested peer) of PX from a pruner at or above AcceptPXThreshold (0)
    for hd, items in blocks(ev):
        if hd["type"] != SEND:
            continue
        pr = items[items["reason"] == _abi.GS_RPC_ITEM_PRUNE]
        px = items[items["reason"] == _abi.GS_RPC_ITEM_PX]
        assert set(px["topic"].tolist()) <= set(pr["topic"].tolist())
        n_px += len(px)
        # the heartbeat's PRUNEs to a negative-score peer carry no PX
        if (hd["msg"] >> 40) == 4 and app[int(hd["peer"])] < 0:
            assert len(px) == 0
        if app[int(hd["node"])] >= 0:
            offered |= {(int(hd["peer"]), int(x)) for x in px["msg"]}
    assert n_px > 0
    # PX dials happened (connections came up after the start), each one
    # suggested by a pruner whose score passed AcceptPXThreshold: a PX from a
    # negative-app-score host is never dialled
    late = ev[(ev["type"] == T("ADD_PEER")) & (ev["hop"] > 0)]
    assert len(late) > 0
    for r in late:
        a, b = int(r["node"]), int(r["peer"])
        assert (a, b) in offered or (b, a) in offered, (a, b)


def test_oracle_px_adversarial_dials(oracle_path):
    """PX beside the attackers: PRUNEs carry peer lists, the pruned hosts dial
    connection slots that start down, and every list pxConnect sees holds at
    most PrunePeers suggestions (gossipsub.go:856-905)."""
    nodes = list(range(300))
    e, hops, ev = _run(oracle_path, "px_adversarial", nodes)
    n_px = 0
    for hd, items in blocks(ev):
        if hd["type"] != SEND:
            continue
        px = items[items["reason"] == _abi.GS_RPC_ITEM_PX]
        for t in set(px["topic"].tolist()):
            assert (px["topic"] == t).sum() <= 16  # PrunePeers
        n_px += len(px)
    assert n_px > 0
    late = ev[(ev["type"] == T("ADD_PEER")) & (ev["hop"] > 0)]
    assert len(late) > 0


def _rows():
    rows = [dict(hop=3, msg=(4 << 40), type=SEND, node=1, peer=2, topic=-1, phase=4, reason=0),
            dict(hop=3, msg=-1, type=ITEM, node=1, peer=2, topic=-1, phase=4, reason=_abi.GS_RPC_ITEM_CTL),
            dict(hop=3, msg=-1, type=ITEM, node=1, peer=2, topic=0, phase=4, reason=_abi.GS_RPC_ITEM_PRUNE),
            dict(hop=3, msg=5, type=ITEM, node=1, peer=2, topic=0, phase=4, reason=_abi.GS_RPC_ITEM_PX),
            dict(hop=3, msg=9, type=ITEM, node=1, peer=2, topic=0, phase=4, reason=_abi.GS_RPC_ITEM_PX)]
    a = np.zeros(len(rows), dtype=_abi.TRACE_EVENT_DTYPE)
    for k, r in enumerate(rows):
        for f, v in r.items():
            a[k][f] = v
    return a


def test_encode_prune_peers():
    import os
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    buf = encode_trace(_rows(), _abi.GS_TRACE_FORMAT_PB, topic_names=["t"])
    n, i = _varint(buf, 0)
    ev = _fields(buf[i:i + n])
    meta = _fields(_fields(ev[3][1])[1][1])
    ctl = _fields(meta[0][1])
    assert ctl[0][0] == 4 and _fields(ctl[0][1]) == [(1, b"t"), (2, b"n5"), (2, b"n9")]
    js = json.loads(encode_trace(_rows(), _abi.GS_TRACE_FORMAT_JSON, topic_names=["t"]).decode())
    b = lambda s: base64.b64encode(s).decode()  # noqa: E731
    assert js["sendRPC"]["meta"]["control"]["prune"] == [{"topic": "t", "peers": [b(b"n5"), b(b"n9")]}]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["px_star", "px_scored", "px_adversarial"])
def test_gpu_px_trace_equals_oracle(name, oracle_path):
    nodes = list(range(20)) if name == "px_star" else list(range(300 if name == "px_adversarial" else 200))
    _, _, ew = _run(oracle_path, name, nodes)
    _, _, eg = _run(PRODUCT_LIB, name, nodes)
    assert len(eg) == len(ew) and np.array_equal(eg, ew)
