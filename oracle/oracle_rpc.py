"""ORACLE (test infrastructure only: imported by tests/, never by the product path).

CPU restatement of fragmentRPC / fragmentMessageIds (gossipsub.go:1158-1272) over
real RPC objects.  Unlike the product (go-libp2p-pubsub_amd/csrc/gs_rpc.cpp), which
works on a size shape, this module builds the messages and measures them by
encoding them: Size() is len(marshal()) with a minimal proto2 encoder following
pb/rpc.proto field order (gogo marshals fields in ascending field number).

Pinned by the reference's known-answer test TestFragmentRPCFunction
(gossipsub_test.go:2085-2250), restated in tests/test_rpc_fragment.py.
"""
from dataclasses import dataclass, field
from typing import List, Optional


def _uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(num: int, body: bytes) -> bytes:
    """A length-delimited field (wire type 2)."""
    return _uvarint(num << 3 | 2) + _uvarint(len(body)) + body


@dataclass
class Message:  # pb/rpc.proto Message
    from_: Optional[bytes] = None
    data: Optional[bytes] = None
    seqno: Optional[bytes] = None
    topic: Optional[str] = None
    signature: Optional[bytes] = None
    key: Optional[bytes] = None

    def marshal(self) -> bytes:
        out = b""
        for num, v in ((1, self.from_), (2, self.data), (3, self.seqno),
                       (4, None if self.topic is None else self.topic.encode()),
                       (5, self.signature), (6, self.key)):
            if v is not None:
                out += _ld(num, v)
        return out


@dataclass
class SubOpts:  # RPC.SubOpts
    subscribe: Optional[bool] = None
    topicid: Optional[str] = None

    def marshal(self) -> bytes:
        out = b""
        if self.subscribe is not None:
            out += _uvarint(1 << 3 | 0) + _uvarint(int(self.subscribe))
        if self.topicid is not None:
            out += _ld(2, self.topicid.encode())
        return out


@dataclass
class IHave:  # ControlIHave
    topic: Optional[str] = None
    ids: List[bytes] = field(default_factory=list)

    def marshal(self) -> bytes:
        out = _ld(1, self.topic.encode()) if self.topic is not None else b""
        return out + b"".join(_ld(2, m) for m in self.ids)


@dataclass
class IWant:  # ControlIWant
    ids: List[bytes] = field(default_factory=list)

    def marshal(self) -> bytes:
        return b"".join(_ld(1, m) for m in self.ids)


@dataclass
class Graft:  # ControlGraft
    topic: Optional[str] = None

    def marshal(self) -> bytes:
        return _ld(1, self.topic.encode()) if self.topic is not None else b""


@dataclass
class Prune:  # ControlPrune
    topic: Optional[str] = None
    peers: List[bytes] = field(default_factory=list)  # PeerInfo{peerID} each
    backoff: Optional[int] = None
    records: Optional[List[bytes]] = None  # PeerInfo.signedPeerRecord per peer (None: nil)

    def marshal(self) -> bytes:
        out = _ld(1, self.topic.encode()) if self.topic is not None else b""
        recs = self.records or [b""] * len(self.peers)
        out += b"".join(_ld(2, _ld(1, p) + (_ld(2, r) if r else b"")) for p, r in zip(self.peers, recs))
        if self.backoff is not None:
            out += _uvarint(3 << 3 | 0) + _uvarint(self.backoff)
        return out


@dataclass
class Control:  # ControlMessage
    ihave: list = field(default_factory=list)
    iwant: list = field(default_factory=list)
    graft: list = field(default_factory=list)
    prune: list = field(default_factory=list)

    def marshal(self) -> bytes:
        return (b"".join(_ld(1, x.marshal()) for x in self.ihave)
                + b"".join(_ld(2, x.marshal()) for x in self.iwant)
                + b"".join(_ld(3, x.marshal()) for x in self.graft)
                + b"".join(_ld(4, x.marshal()) for x in self.prune))


@dataclass
class RPC:
    subscriptions: list = field(default_factory=list)
    publish: list = field(default_factory=list)
    control: Optional[Control] = None

    def marshal(self) -> bytes:
        out = b"".join(_ld(1, s.marshal()) for s in self.subscriptions)
        out += b"".join(_ld(2, m.marshal()) for m in self.publish)
        if self.control is not None:
            out += _ld(3, self.control.marshal())
        return out


def size(x) -> int:
    return len(x.marshal())


def fragment_message_ids(ids, limit):
    """fragmentMessageIds, gossipsub.go:1249-1272 (2 bytes of overhead per id)."""
    out = [[]]
    cur = 0
    blen = 0
    for m in ids:
        sz = len(m) + 2
        if sz > limit:
            continue  # gossipsub.go:1258-1262: dropped from the outgoing gossip
        blen += sz
        if blen > limit:
            out.append([])
            cur += 1
            blen = sz
        out[cur].append(m)
    return out


def fragment_rpc(rpc: RPC, limit: int):
    """fragmentRPC, gossipsub.go:1158-1247.  Returns the list of RPCs; raises
    ValueError like the reference's error return (gossipsub.go:1191-1193)."""
    if size(rpc) < limit:
        return [rpc]
    rpcs = [RPC()]

    def out_rpc(add, with_ctl):  # gossipsub.go:1170-1186
        cur = rpcs[-1]
        if size(cur) + add + 1 < limit:
            if with_ctl and cur.control is None:
                cur.control = Control()
            return cur
        nxt = RPC(control=Control() if with_ctl else None)
        rpcs.append(nxt)
        return nxt

    for m in rpc.publish:
        s = size(m)
        if s > limit:
            raise ValueError(f"message with len={s} exceeds limit {limit}")
        out_rpc(s, False).publish.append(m)
    for s in rpc.subscriptions:
        out_rpc(size(s), False).subscriptions.append(s)
    ctl = rpc.control
    if ctl is None:
        return rpcs
    whole = RPC(control=ctl)
    if size(whole) < limit:  # gossipsub.go:1209-1213
        rpcs.append(whole)
        return rpcs
    for g in ctl.graft:
        out_rpc(size(g), True).control.graft.append(g)
    for p in ctl.prune:
        out_rpc(size(p), True).control.prune.append(p)
    for w in ctl.iwant:  # gossipsub.go:1228-1236
        for ids in fragment_message_ids(w.ids, limit - 6):
            nw = IWant(ids=ids)
            out_rpc(size(nw), True).control.iwant.append(nw)
    for h in ctl.ihave:  # gossipsub.go:1237-1245 (the fragment drops TopicID)
        for ids in fragment_message_ids(h.ids, limit - 6):
            nh = IHave(ids=ids)
            out_rpc(size(nh), True).control.ihave.append(nh)
    return rpcs
