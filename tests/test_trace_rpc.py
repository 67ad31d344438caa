"""RPC trace events (RecvRPC / SendRPC with traceRPCMeta, trace.go:241-383;
the reference's trace_test.go:159-193 wants every event type present).

CPU, the oracle against what its traced hosts must agree with:
  * every RPC a traced host sends is a SEND_RPC block, and its items are the
    RPC: summed with the RPC size model (include/gs_rpcsize.h) they give the
    per-edge RPC.Size() totals of the byte accounting (gs_read_rpc_bytes,
    which also counts the untraced hello packets, pubsub.go:494), RPC for RPC;
  * every SEND from a traced host to a traced peer is that peer's RECV in the
    next hop with the same items (unless its connection closed first);
  * the canonical block order of include/gs_trace.h;
  * the encoders: pb.TraceEvent RecvRPC/SendRPC{peer, RPCMeta} in gogo field
    order, and the JSONTracer's struct layout.
GPU: the HIP engine's event stream, RPC blocks included, equals the oracle's.
DROP_RPC never occurs: outbound queues never drop in this model."""
import base64
import json
from collections import Counter, defaultdict

import numpy as np
import pytest

import scenarios
from pubsub_amd import PRODUCT_LIB, WithEventTracer, _abi, encode_trace
from test_trace import _fields, _varint

T = _abi.TRACE_TYPES.index
RECV, SEND, ITEM = T("RECV_RPC"), T("SEND_RPC"), _abi.GS_TRACE_RPC_ITEM
TRACED = [0, 3, 17, 42, 99, 150]


def run(lib, name, nodes, chunks=4):
    e, hops = scenarios.SCENARIOS[name](lib, (WithEventTracer(nodes, rpc=True),))
    evs = []
    for _ in range(chunks):  # drain between steps too
        e.step(hops // chunks)
        evs.append(e.trace_events())
    e.step(hops - chunks * (hops // chunks))
    evs.append(e.trace_events())
    return e, hops, np.concatenate(evs)


def blocks(ev):
    """[(head row, [item rows])] of the RPC events, in stream order."""
    out, i = [], 0
    while i < len(ev):
        j = i + 1
        if ev[i]["type"] in (RECV, SEND):
            while j < len(ev) and ev[j]["type"] == ITEM:
                j += 1
            out.append((ev[i], ev[i + 1:j]))
        else:
            assert ev[i]["type"] != ITEM, "an RPC item without its RPC event"
        i = j
    return out


def _pbf(n):  # gs_pb_field
    v, k = n, 1
    while v >= 0x80:
        v >>= 7
        k += 1
    return 1 + k + n


def rpc_size(items, msg_size, id_len, tl, backoff_s=60):
    """RPC.Size() of the RPC an item list describes (include/gs_rpcsize.h)."""
    k = items["reason"]
    s = sum(_pbf(msg_size[t]) for t in items["topic"][k == _abi.GS_RPC_ITEM_MSG])
    s += sum(_pbf(2 + _pbf(tl[t])) for t in items["topic"][k == _abi.GS_RPC_ITEM_SUB])
    if (k == _abi.GS_RPC_ITEM_CTL).any():
        c = 0
        ih = items[k == _abi.GS_RPC_ITEM_IHAVE]
        for t, n in Counter(ih["topic"].tolist()).items():
            c += _pbf(_pbf(tl[t]) + n * _pbf(id_len))
        nw = int((k == _abi.GS_RPC_ITEM_IWANT).sum())
        if nw:
            c += _pbf(nw * _pbf(id_len))
        c += sum(_pbf(_pbf(tl[t])) for t in items["topic"][k == _abi.GS_RPC_ITEM_GRAFT])
        bl = 1 if backoff_s < 0x80 else 2
        c += sum(_pbf(_pbf(tl[t]) + 1 + bl) for t in items["topic"][k == _abi.GS_RPC_ITEM_PRUNE])
        s += _pbf(c)
    return s


ACCT = ["acct_multitopic", "acct_graylist_direct", "acct_adversarial", "acct_floodsub", "acct_randomsub"]


@pytest.mark.parametrize("name", ACCT)
def test_oracle_sends_are_the_accounted_rpcs(oracle_path, name):
    """Per directed edge of a traced host: the SEND_RPC blocks count and size
    exactly the RPCs the byte accounting saw, minus the hello packet."""
    nodes = [u for u in TRACED if u < 20] if name == "acct_floodsub" else [0, 3, 17, 42]
    e, _, ev = run(oracle_path, name, nodes)
    T_ = e.T
    msg_size = [120 + 5 * t for t in range(T_)]  # scenarios._acct
    tl = [len(str(t)) for t in range(T_)]
    nbytes, ncount = e.rpc_bytes()
    sent_n, sent_b = defaultdict(int), defaultdict(int)
    for hd, items in blocks(ev):
        if hd["type"] == SEND:
            sent_n[(int(hd["node"]), int(hd["peer"]))] += 1
            sent_b[(int(hd["node"]), int(hd["peer"]))] += rpc_size(items, msg_size, 30, tl)
    subs = e.subs
    for u in nodes:
        hello = sum(_pbf(2 + _pbf(tl[t])) for t in range(T_) if (int(subs[u]) >> t) & 1)
        for k in range(e.rowptr[u], e.rowptr[u + 1]):
            p = int(e.col[k])
            assert sent_n[(u, p)] == ncount[k] - 1, (u, p)
            assert sent_b[(u, p)] == nbytes[k] - hello, (u, p)
    assert sum(sent_n.values()) > 0


@pytest.mark.parametrize("name", ["gossipsub_scored", "adversarial_mix", "churn_scored", "gossipsub_multitopic"])
def test_oracle_send_is_received_next_hop(oracle_path, name):
    nodes = list(range(0, 40, 3))
    e, hops, ev = run(oracle_path, name, nodes)
    traced = set(nodes)
    recv = {}
    types = Counter()
    for hd, items in blocks(ev):
        key = (int(hd["hop"]), int(hd["node"]), int(hd["peer"]), int(hd["msg"]))
        types[int(hd["type"])] += 1
        if hd["type"] == RECV:
            assert key not in recv
            recv[key] = items[["reason", "topic", "msg"]].tolist()
            assert hd["phase"] in ((2,) if (items["reason"] == _abi.GS_RPC_ITEM_MSG).any() else (0, 3))
    assert types[SEND] and types[RECV]
    lost = 0
    for hd, items in blocks(ev):
        if hd["type"] != SEND or int(hd["peer"]) not in traced or hd["hop"] + 1 >= hops:
            continue
        key = (int(hd["hop"]) + 1, int(hd["peer"]), int(hd["node"]), int(hd["msg"]))
        if key not in recv:
            lost += 1  # only a connection closed at the start of the next hop loses it
            assert name.startswith("churn"), key
            continue
        assert recv[key] == items[["reason", "topic", "msg"]].tolist(), key
    if not name.startswith("churn"):
        assert lost == 0


def test_oracle_rpc_blocks_in_canonical_order(oracle_path):
    e, _, ev = run(oracle_path, "gossipsub_scored", [0, 3, 17])
    key = [(r["hop"], r["node"], r["phase"]) for r in ev]
    assert key == sorted(key)
    # inside a phase: RECV_RPCs first (sender, ordinal), SEND_RPCs last (receiver, ordinal)
    last = None
    for hd, items in blocks(ev):
        k = (int(hd["hop"]), int(hd["node"]), int(hd["phase"]), 0 if hd["type"] == RECV else 1, int(hd["peer"]),
             int(hd["msg"]))
        if last is not None and k[:3] == last[:3]:
            assert k[3:] >= last[3:] or k[3] > last[3]
        last = k
        kinds = items["reason"].tolist()
        assert kinds == sorted(kinds)
        # IHAVE ids of one topic ascending (every RPC of this scenario is below MaxIHaveLength)
        ih = items[items["reason"] == _abi.GS_RPC_ITEM_IHAVE]
        for t in set(ih["topic"].tolist()):
            ids = ih["msg"][ih["topic"] == t]
            assert (np.diff(ids) > 0).all()


def test_oracle_every_event_type_but_drop(oracle_path):
    """trace_test.go:159-193 wants all 13 types; DROP_RPC is unreachable here."""
    _, _, ev = run(oracle_path, "churn_scored", list(range(0, 240, 7)))
    have = set(ev["type"].tolist())
    want = set(range(13)) - {T("DROP_RPC"), T("REJECT_MESSAGE")}  # no validator in this scenario
    assert want <= have, sorted(want - have)


# ---------------------------------------------------------------- encoder
def _rpc_rows():
    rows = [dict(hop=5, msg=(3 << 40) | 98, type=SEND, node=7, peer=9, topic=-1, phase=3, reason=0)]
    for k, t, m in [(_abi.GS_RPC_ITEM_MSG, 1, 13), (_abi.GS_RPC_ITEM_CTL, -1, -1), (_abi.GS_RPC_ITEM_IHAVE, 0, 4),
                    (_abi.GS_RPC_ITEM_IHAVE, 0, 6), (_abi.GS_RPC_ITEM_IHAVE, 2, 5), (_abi.GS_RPC_ITEM_IWANT, -1, 21),
                    (_abi.GS_RPC_ITEM_IWANT, -1, 20), (_abi.GS_RPC_ITEM_GRAFT, 1, -1),
                    (_abi.GS_RPC_ITEM_PRUNE, 2, -1)]:
        rows.append(dict(hop=5, msg=m, type=ITEM, node=7, peer=9, topic=t, phase=3, reason=k))
    rows.append(dict(hop=6, msg=0, type=RECV, node=7, peer=11, topic=-1, phase=0, reason=0))
    rows.append(dict(hop=6, msg=1, type=ITEM, node=7, peer=11, topic=2, phase=0, reason=_abi.GS_RPC_ITEM_SUB))
    rows.append(dict(hop=6, msg=0, type=ITEM, node=7, peer=11, topic=0, phase=0, reason=_abi.GS_RPC_ITEM_SUB))
    a = np.zeros(len(rows), dtype=_abi.TRACE_EVENT_DTYPE)
    for k, r in enumerate(rows):
        for f, v in r.items():
            a[k][f] = v
    return a


def _need_product():
    import os
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")


def test_encode_rpc_meta_pb():
    """SendRPC{sendTo=1, meta=2}; RPCMeta{messages=1, subscription=2,
    control=3{ihave=1, iwant=2, graft=3, prune=4}} (pb/trace.proto:73-145)."""
    _need_product()
    names = ["a", "bb", "ccc"]
    buf = encode_trace(_rpc_rows(), _abi.GS_TRACE_FORMAT_PB, hop_ns=1000, topic_names=names)
    evs, i = [], 0
    while i < len(buf):
        n, i = _varint(buf, i)
        evs.append(_fields(buf[i:i + n]))
        i += n
    assert len(evs) == 2
    send, recv = evs
    assert [f for f, _ in send] == [1, 2, 3, 11] and send[0][1] == SEND and send[2][1] == 5000
    body = _fields(send[3][1])
    assert body[0] == (1, b"n9") and body[1][0] == 2
    meta = _fields(body[1][1])
    assert [f for f, _ in meta] == [1, 3]
    assert dict(_fields(meta[0][1])) == {1: b"13", 2: b"bb"}
    ctl = _fields(meta[1][1])
    assert [f for f, _ in ctl] == [1, 1, 2, 3, 4]
    assert _fields(ctl[0][1]) == [(1, b"a"), (2, b"4"), (2, b"6")]
    assert _fields(ctl[1][1]) == [(1, b"ccc"), (2, b"5")]
    assert _fields(ctl[2][1]) == [(1, b"21"), (1, b"20")]
    assert _fields(ctl[3][1]) == [(1, b"bb")] and _fields(ctl[4][1]) == [(1, b"ccc")]
    assert [f for f, _ in recv] == [1, 2, 3, 10]
    rb = _fields(recv[3][1])
    assert rb[0] == (1, b"n11")
    subs = _fields(rb[1][1])
    assert [dict(_fields(v)) for f, v in subs] == [{1: 1, 2: b"ccc"}, {1: 0, 2: b"a"}]


def test_encode_rpc_meta_json():
    _need_product()
    lines = encode_trace(_rpc_rows(), _abi.GS_TRACE_FORMAT_JSON, hop_ns=1000, topic_names=["a", "bb", "ccc"])
    d = [json.loads(x) for x in lines.decode().splitlines()]
    b = lambda s: base64.b64encode(s).decode()  # noqa: E731
    assert d[0] == {"type": SEND, "peerID": b(b"n7"), "timestamp": 5000, "sendRPC": {
        "sendTo": b(b"n9"), "meta": {
            "messages": [{"messageID": b(b"13"), "topic": "bb"}],
            "control": {"ihave": [{"topic": "a", "messageIDs": [b(b"4"), b(b"6")]},
                                  {"topic": "ccc", "messageIDs": [b(b"5")]}],
                        "iwant": [{"messageIDs": [b(b"21"), b(b"20")]}],
                        "graft": [{"topic": "bb"}], "prune": [{"topic": "ccc"}]}}}}
    assert d[1]["recvRPC"] == {"receivedFrom": b(b"n11"), "meta": {"subscription": [
        {"subscribe": True, "topic": "ccc"}, {"subscribe": False, "topic": "a"}]}}


# ---------------------------------------------------------------- GPU
GPU_CASES = ["gossipsub_scored", "gossipsub_multitopic", "floodsub_dense", "randomsub_100", "adversarial_mix",
             "churn_scored", "spam_ihave", "c3shape", "mixed_scored", "mixed_randomsub"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_CASES)
def test_gpu_rpc_trace_equals_oracle(oracle_path, name):
    nodes = [u for u in TRACED if u < 20] if name in ("floodsub_dense", "spam_ihave") else TRACED
    if name.startswith("spam_"):
        nodes = [0, 1]
    _, _, want = run(oracle_path, name, nodes)
    _, _, got = run(PRODUCT_LIB, name, nodes)
    assert (got["type"] == SEND).any() and (got["type"] == RECV).any()
    if len(got) != len(want) or not np.array_equal(got, want):
        n = min(len(got), len(want))
        bad = np.flatnonzero(got[:n] != want[:n])
        i = int(bad[0]) if len(bad) else n
        raise AssertionError(f"{name}: {len(got)} vs {len(want)} events; first difference at {i}: "
                             f"gpu {got[max(0, i - 2):i + 3]} oracle {want[max(0, i - 2):i + 3]}")
