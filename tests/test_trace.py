"""Trace events (EventTracer, trace.go:61-499 + pb/trace.proto).

CPU: the oracle's events of traced hosts against the readbacks they must agree
with (every DeliverMessage is the recorded first delivery, the Graft/Prune
sequence replays to the final mesh, AddPeer/Join at time 0, every recorded
type present — trace_test.go:159-193 for the recorded subset), and the
product library's encoder against the pb/trace.proto wire format and the
JSONTracer's encoding/json layout.
GPU: the HIP engine's event sequence equals the oracle's, field for field.
"""
import base64
import json

import numpy as np
import pytest

import scenarios
from pubsub_amd import PRODUCT_LIB, WithEventTracer, _abi, encode_trace

TRACED = [0, 3, 17, 42, 99, 150]
T = _abi.TRACE_TYPES.index


def traced_run(lib, name, nodes=TRACED, extra=()):
    e, hops = scenarios.SCENARIOS[name](lib, (WithEventTracer(nodes),) + tuple(extra))
    evs = []
    for _ in range(4):  # drain between steps too
        e.step(hops // 4)
        evs.append(e.trace_events())
    e.step(hops - 4 * (hops // 4))
    evs.append(e.trace_events())
    return e, np.concatenate(evs)


def check_invariants(e, ev, nodes):
    assert len(ev)
    key = [(r["hop"], r["node"], r["phase"]) for r in ev]
    assert key == sorted(key), "events out of canonical order"
    types = set(ev["type"].tolist())
    want = {T("ADD_PEER"), T("JOIN"), T("PUBLISH_MESSAGE"), T("DELIVER_MESSAGE"), T("DUPLICATE_MESSAGE")}
    if e.router == _abi.GS_ROUTER_GOSSIPSUB:
        # a mixed network's few traced gossipsub hosts may never prune
        want |= {T("GRAFT")} if getattr(e, "routers", None) is not None else {T("GRAFT"), T("PRUNE")}
    assert want <= types, f"missing event types {want - types}"
    deg = np.diff(e.rowptr)
    mesh = e.mesh()
    for u in nodes:
        mine = ev[ev["node"] == u]
        assert (mine["type"] == T("ADD_PEER")).sum() == deg[u]
        assert sorted(mine[mine["type"] == T("ADD_PEER")]["peer"].tolist()) == \
            e.col[e.rowptr[u]:e.rowptr[u + 1]].tolist()
        # DeliverMessage <-> the first delivery readback (hop, ReceivedFrom)
        dl = mine[mine["type"] == T("DELIVER_MESSAGE")]
        for r in dl:
            hop, frm = e.deliveries(int(r["msg"]))
            assert hop[u] == r["hop"]
            assert (frm[u] if frm[u] >= 0 else u) == r["peer"]
        seen = sum(1 for m in range(e.n_published) if e.deliveries(m)[0][u] >= 0)
        assert len(dl) == seen
        assert len(set(dl["msg"].tolist())) == len(dl)
        # Graft/Prune replay (tracer.Prune also for non-members: a no-op erase)
        members = {}
        for r in mine:
            if r["type"] == T("GRAFT"):
                members.setdefault(int(r["topic"]), set()).add(int(r["peer"]))
            elif r["type"] == T("PRUNE"):
                members.setdefault(int(r["topic"]), set()).discard(int(r["peer"]))
        for i, v in enumerate(e.col[e.rowptr[u]:e.rowptr[u + 1]]):
            m = int(mesh[e.rowptr[u] + i])
            for t in range(e.T):
                assert ((m >> t) & 1) == (int(v) in members.get(t, set())), (u, int(v), t)


@pytest.mark.parametrize("name", ["gossipsub_scored", "gossipsub_multitopic", "floodsub_dense",
                                  "gossipsub_dense_dhi", "acct_mixed"])
def test_oracle_trace_invariants(oracle_path, name):
    nodes = [u for u in TRACED if u < 20] if name == "floodsub_dense" else [u for u in TRACED if u < 120]
    e, ev = traced_run(oracle_path, name, nodes)
    check_invariants(e, ev, nodes)


# ---------------------------------------------------------------- encoder
def _varint(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def _fields(b):
    """protobuf message -> [(field, value)]: wire types 0 and 2 only."""
    i, out = 0, []
    while i < len(b):
        tag, i = _varint(b, i)
        if tag & 7 == 0:
            v, i = _varint(b, i)
        else:
            assert tag & 7 == 2
            n, i = _varint(b, i)
            v, i = b[i:i + n], i + n
        out.append((tag >> 3, v))
    return out


def _events(rows):
    a = np.zeros(len(rows), dtype=_abi.TRACE_EVENT_DTYPE)
    for k, r in enumerate(rows):
        for f, v in r.items():
            a[k][f] = v
    return a


SAMPLE = [dict(hop=0, msg=-1, type=T("ADD_PEER"), node=7, peer=9, topic=-1, phase=0),
          dict(hop=0, msg=-1, type=T("JOIN"), node=7, peer=-1, topic=2, phase=0),
          dict(hop=3, msg=12, type=T("PUBLISH_MESSAGE"), node=7, peer=-1, topic=2, phase=1),
          dict(hop=4, msg=13, type=T("DELIVER_MESSAGE"), node=7, peer=9, topic=1, phase=2),
          dict(hop=4, msg=11, type=T("DUPLICATE_MESSAGE"), node=7, peer=300, topic=0, phase=2),
          dict(hop=5, msg=-1, type=T("GRAFT"), node=7, peer=9, topic=1, phase=3),
          dict(hop=20, msg=-1, type=T("PRUNE"), node=7, peer=9, topic=1, phase=4)]


def _need_product():
    import os
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")


def test_encode_pb_wire_format():
    """Delimited TraceEvent (PBTracer): field numbers of pb/trace.proto."""
    _need_product()
    names = ["beacon_block", "aggregate", "attestation"]
    buf = encode_trace(_events(SAMPLE), _abi.GS_TRACE_FORMAT_PB, hop_ns=100_000_000, topic_names=names)
    i, evs = 0, []
    while i < len(buf):
        n, i = _varint(buf, i)
        evs.append(_fields(buf[i:i + n]))
        i += n
    assert len(evs) == len(SAMPLE)
    sub = {0: 4, 2: 6, 3: 7, 4: 8, 9: 13, 11: 15, 12: 16}  # TraceEvent sub-message field per type
    for f, s in zip(evs, SAMPLE):
        assert [x[0] for x in f] == [1, 2, 3, sub[s["type"]]]  # ascending field numbers (gogo)
        assert f[0][1] == s["type"] and f[1][1] == b"n7" and f[2][1] == s["hop"] * 100_000_000
        body = dict(_fields(f[3][1]))
        t = s["type"]
        if t == T("ADD_PEER"):
            assert body == {1: b"n9", 2: b"/meshsub/1.1.0"}
        elif t == T("JOIN"):
            assert body == {1: b"attestation"}
        elif t == T("PUBLISH_MESSAGE"):
            assert body == {1: b"12", 2: b"attestation"}
        elif t == T("DELIVER_MESSAGE"):   # messageID=1, topic=2, receivedFrom=3
            assert body == {1: b"13", 2: b"aggregate", 3: b"n9"}
        elif t == T("DUPLICATE_MESSAGE"):  # messageID=1, receivedFrom=2, topic=3
            assert body == {1: b"11", 2: b"n300", 3: b"beacon_block"}
        else:
            assert body == {1: b"n9", 2: b"aggregate"}
    # an exact vector: the second record, JOIN of topic "attestation" by n7 at t=0
    j = 1 + buf[0]
    assert buf[j:j + 24] == bytes([23, 0x08, 9, 0x12, 2]) + b"n7" + bytes([0x18, 0, 0x6A, 13, 0x0A, 11]) + \
        b"attestation"


def test_encode_json_lines():
    """JSONTracer: encoding/json of pb.TraceEvent ([]byte base64, enum as number)."""
    _need_product()
    out = encode_trace(_events(SAMPLE), _abi.GS_TRACE_FORMAT_JSON, hop_ns=100_000_000)
    lines = out.decode().splitlines()
    assert len(lines) == len(SAMPLE) and out.endswith(b"\n")
    d = [json.loads(x) for x in lines]
    assert list(d[3]) == ["type", "peerID", "timestamp", "deliverMessage"]
    assert d[3]["type"] == 3 and base64.b64decode(d[3]["peerID"]) == b"n7"
    assert d[3]["timestamp"] == 400_000_000
    assert list(d[3]["deliverMessage"]) == ["messageID", "topic", "receivedFrom"]
    assert base64.b64decode(d[3]["deliverMessage"]["messageID"]) == b"13"
    assert d[3]["deliverMessage"]["topic"] == "1"
    assert base64.b64decode(d[4]["duplicateMessage"]["receivedFrom"]) == b"n300"
    assert d[1] == {"type": 9, "peerID": base64.b64encode(b"n7").decode(), "timestamp": 0,
                    "join": {"topic": "2"}}
    assert list(d[6]["prune"]) == ["peerID", "topic"]


def test_encode_json_string_escapes():
    """encoding/json's string encoder (Go 1.13-1.15 encodeState.string, HTML-safe):
    short escapes for \\n \\r \\t, \\u00XX for other control bytes and < > &,
    U+2028 / U+2029 escaped, one \\ufffd per invalid UTF-8 byte."""
    _need_product()
    name = b'x\n\r\t"\\<>&\x01\xe2\x80\xa8\xe2\x80\xa9\xff\xc3(z\xc3\xa9'
    out = encode_trace(_events(SAMPLE)[1:2], _abi.GS_TRACE_FORMAT_JSON, topic_names=[b"a", b"b", name])
    want = (b'"topic":"x\\n\\r\\t\\"\\\\\\u003c\\u003e\\u0026\\u0001\\u2028\\u2029'
            b'\\ufffd\\ufffd(z\xc3\xa9"')
    assert want in out, out
    assert json.loads(out)["join"]["topic"] == 'x\n\r\t"\\<>&\x01\u2028\u2029\ufffd\ufffd(z\u00e9'


def test_encode_round_trip_sizes(oracle_path):
    """A real event stream encodes to one record per event in both formats."""
    _need_product()
    e, ev = traced_run(oracle_path, "gossipsub_scored", [0, 3])
    pb = encode_trace(ev, _abi.GS_TRACE_FORMAT_PB)
    i = k = 0
    while i < len(pb):
        n, i = _varint(pb, i)
        i += n
        k += 1
    assert k == len(ev)
    js = encode_trace(ev, _abi.GS_TRACE_FORMAT_JSON).decode().splitlines()
    assert len(js) == len(ev) and all(json.loads(x)["type"] == int(t) for x, t in zip(js, ev["type"]))


# ---------------------------------------------------------------- GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gossipsub_scored", "gossipsub_multitopic", "floodsub_dense",
                                  "gossipsub_dense_dhi", "gossipsub_negative_app", "gossipsub_flood_publish", "acct_mixed"])
def test_gpu_trace_equals_oracle(oracle_path, name):
    nodes = [u for u in TRACED if u < 20] if name == "floodsub_dense" else [u for u in TRACED if u < 120]
    _, ref = traced_run(oracle_path, name, nodes)
    e, got = traced_run(PRODUCT_LIB, name, nodes)
    assert len(got) == len(ref), (len(got), len(ref))
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, f"{len(bad)} events differ, first {got[bad[0]]} vs {ref[bad[0]]}"
    check_invariants(e, got, nodes)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gossipsub_scored", "churn_scored"])
def test_gpu_trace_repeatable(oracle_path, name):
    """traced_run drains between steps: the device's event counter is reset on
    the engine's stream before the next hop appends (gs_engine.hip drainTrace).
    Three more runs must each reproduce the oracle's stream."""
    nodes = TRACED
    _, ref = traced_run(oracle_path, name, nodes)
    for _ in range(3):
        _, got = traced_run(PRODUCT_LIB, name, nodes)
        assert len(got) == len(ref) and not np.any(got != ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["churn_scored", "churn_prune", "churn_graft"])
def test_gpu_trace_equals_oracle_churn(oracle_path, name):
    """RemovePeer / AddPeer / Leave / Join events of the churn scenarios
    (trace.go:199-233, 399-414): the GPU stream equals the oracle's."""
    nodes = [u for u in TRACED if u < 20] if name != "churn_scored" else TRACED
    _, ref = traced_run(oracle_path, name, nodes)
    _, got = traced_run(PRODUCT_LIB, name, nodes)
    assert len(got) == len(ref), (len(got), len(ref))
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, f"{len(bad)} events differ, first {got[bad[0]]} vs {ref[bad[0]]}"


@pytest.mark.parametrize("name", ["churn_scored", "churn_prune"])
def test_oracle_churn_trace_types(oracle_path, name):
    """The churn events appear in the trace: RemovePeer / AddPeer for every
    connection change of a traced host, Leave / Join for its topic changes."""
    nodes = [u for u in TRACED if u < 20] if name != "churn_scored" else TRACED
    _, ev = traced_run(oracle_path, name, nodes)
    types = set(ev["type"].tolist())
    assert T("LEAVE") in types
    if name == "churn_scored":
        assert {T("REMOVE_PEER"), T("ADD_PEER"), T("JOIN")} <= types
        rm = ev[ev["type"] == T("REMOVE_PEER")]
        add = ev[(ev["type"] == T("ADD_PEER")) & (ev["hop"] > 0)]
        assert len(rm) >= len(add) > 0  # every reconnect follows a disconnect
