"""Per-edge RPC byte accounting (gs_set_rpc_accounting, SURVEY.md §8(f) rank 3:
sendRPC measures out.Size(), gossipsub.go:1121-1137).

The size model (include/gs_rpcsize.h) is pinned against real protobuf
encodings of the same RPCs (oracle/oracle_rpc.py, whose encoder is pinned by
TestFragmentRPCFunction and hand-derived gogo Size() values, test_rpc_fragment
.py); the oracle's per-edge sums are pinned by closed forms on the routers that
only send messages and hellos; the GPU equals the oracle on the acct_*
scenarios (test_parity_gpu.py, test_golden.py)."""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import oracle_rpc as pb  # noqa: E402
import scenarios  # noqa: E402


# ---- include/gs_rpcsize.h restated
def vlen(v):
    n = 1
    while v >= 0x80:
        v >>= 7
        n += 1
    return n


def field(n):
    return 1 + vlen(n) + n


def subopts(tl):
    return 2 + field(tl)


def ihave(tl, n, L):
    return field(tl) + n * field(L)


def iwant(n, L):
    return n * field(L)


def graft(tl):
    return field(tl)


def prune(tl, bo):
    return field(tl) + 1 + vlen(bo)


def peerinfo(pid, rec):
    return field(pid) + (field(rec) if rec else 0)


def prune_px(tl, bo, npx, pi):
    return prune(tl, bo) + npx * field(pi)


def test_px_prune_size_matches_protobuf_encoder():
    """makePrune with PX (gossipsub.go:1811-1836): PeerInfo{peerID,
    signedPeerRecord} entries, the record absent when nil (gs_pb_peerinfo /
    gs_pb_prune_px of include/gs_rpcsize.h)."""
    rng = random.Random(11)
    for _ in range(200):
        tl = rng.choice([1, 5, 126, 200])
        bo = rng.choice([0, 60, 128, 70000])
        pid = rng.choice([34, 38, 39, 130])
        rec = rng.choice([0, 0, 120, 300])
        k = rng.choice([0, 1, 16, 40])
        pr = pb.Prune("x" * tl, peers=[b"p" * pid] * k, backoff=bo, records=[b"r" * rec] * k if rec else None)
        assert pb.size(pb.RPC(control=pb.Control(prune=[pr]))) == field(field(prune_px(tl, bo, k, peerinfo(pid, rec))))


def _msg(ms, rng):
    """A pb.Message whose Size() is ms (from / seqno / topic set, data fills)."""
    base = pb.Message(from_=b"p" * 38, seqno=b"s" * 8, topic="t")
    fixed = pb.size(base)
    pad = ms - fixed - 2
    while pad > 0 and field(pad) + fixed != ms:
        pad -= 1
    m = pb.Message(from_=b"p" * 38, seqno=b"s" * 8, topic="t", data=bytes(rng.randrange(256) for _ in range(pad)))
    assert pb.size(m) == ms
    return m


def test_size_model_matches_protobuf_encoder():
    rng = random.Random(7)
    for _ in range(300):
        L = rng.choice([1, 20, 46, 127, 130])
        tls = [rng.choice([1, 5, 40, 126, 200]) for _ in range(4)]
        topics = ["x" * tl for tl in tls]
        ids = lambda n: [bytes([rng.randrange(256)]) * L for _ in range(n)]  # noqa: E731
        bo = rng.choice([0, 60, 127, 128, 70000])
        # heartbeat RPC: IHAVE per topic, GRAFTs, PRUNEs with backoff
        ih = [(t, rng.choice([0, 1, 7, 300])) for t in range(4) if rng.random() < 0.6]
        gr = [t for t in range(4) if rng.random() < 0.4]
        pr = [t for t in range(4) if rng.random() < 0.4]
        r = pb.RPC(control=pb.Control(ihave=[pb.IHave(topics[t], ids(n)) for t, n in ih],
                                      graft=[pb.Graft(topics[t]) for t in gr],
                                      prune=[pb.Prune(topics[t], backoff=bo) for t in pr]))
        body = (sum(field(ihave(tls[t], n, L)) for t, n in ih) + sum(field(graft(tls[t])) for t in gr)
                + sum(field(prune(tls[t], bo)) for t in pr))
        assert pb.size(r) == field(body)
        # HandleRPC reply: served messages + IWANT + PRUNEs (rpcWithControl)
        ms = [rng.choice([60, 120, 125, 130, 300, 20000]) for _ in range(rng.randrange(4))]
        nw = rng.choice([0, 1, 50])
        r = pb.RPC(publish=[_msg(m, rng) for m in ms],
                   control=pb.Control(iwant=[pb.IWant(ids(nw))] if nw else [],
                                      prune=[pb.Prune(topics[t], backoff=bo) for t in pr]))
        body = (field(iwant(nw, L)) if nw else 0) + sum(field(prune(tls[t], bo)) for t in pr)
        assert pb.size(r) == sum(field(m) for m in ms) + field(body)
        # a forwarded message (rpcWithMessages: no control)
        m = rng.choice([60, 125, 127, 129, 5000])
        assert pb.size(pb.RPC(publish=[_msg(m, rng)])) == field(m)
        # hello / announcement (rpcWithSubs)
        sub = [t for t in range(4) if rng.random() < 0.5]
        r = pb.RPC(subscriptions=[pb.SubOpts(subscribe=bool(rng.random() < 0.5), topicid=topics[t]) for t in sub])
        assert pb.size(r) == sum(field(subopts(tls[t])) for t in sub)


def test_oracle_floodsub_bytes_closed_form(oracle_path):
    """floodsub sends only forwarded messages (one 120-byte message each, an RPC of
    field(120) bytes) and, per connection, one hello with one SubOpts."""
    s = scenarios.run(oracle_path, "acct_floodsub")
    b, n = s["rpc_bytes"], s["rpc_count"]
    E = len(b)
    tx = s["counters"]["transmissions"]
    assert int(n.sum()) == tx + E
    assert int(b.sum()) == tx * field(120) + E * field(subopts(1))


def test_oracle_randomsub_bytes_closed_form(oracle_path):
    s = scenarios.run(oracle_path, "acct_randomsub")
    b, n = s["rpc_bytes"], s["rpc_count"]
    E = len(b)
    tx = s["counters"]["transmissions"]
    assert int(n.sum()) == tx + E
    assert int(b.sum()) == tx * field(120) + E * field(subopts(1))


def test_oracle_gossipsub_bytes_cover_every_rpc(oracle_path):
    """Every RPC kind shows up: more RPCs than payload copies plus hellos, and
    bytes beyond the payload (control, replies)."""
    s = scenarios.run(oracle_path, "acct_multitopic")
    b, n = s["rpc_bytes"], s["rpc_count"]
    c = s["counters"]
    assert int(n.sum()) > len(b) + c["grafts_sent"]
    assert (n > 0).all()  # a hello on every connection (empty for a host with no topic)
    assert int(b.sum()) > c["transmissions"] * field(120)
