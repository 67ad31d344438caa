"""RPC fragmentation: fragmentRPC / fragmentMessageIds,
gossipsub.go:1158-1272.

* The oracle (oracle/oracle_rpc.py, real protobuf encodings) is pinned by the
  reference's TestFragmentRPCFunction (gossipsub_test.go:2085-2250), restated here.
* The product (libgossip_engine.so, gs_fragment_rpc over a size shape) must put
  every part in the same fragment as the oracle and report the same fragment
  sizes, on the reference test's cases and on seeded random RPCs.
Host code only (no device), so these run without a GPU.
"""
import os
import random
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle_rpc as O  # noqa: E402

from pubsub_amd import PRODUCT_LIB  # noqa: E402
from pubsub_amd.engine import GossipEngineError  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(PRODUCT_LIB),
                                reason="product library not built (run __graft_entry__.build())")

LIMIT = 1024


def mk_msg(rng, size):
    # gossipsub_test.go:2091-2096: Data of size-4 bytes
    return O.Message(data=bytes(rng.getrandbits(8) for _ in range(size - 4)))


def mk_id(rng, n, tag):
    b = tag.to_bytes(4, "big")
    return (b + bytes(rng.getrandbits(8) for _ in range(max(0, n - 4))))[:max(n, 4)] if n >= 4 else b[:n]


def reference_case_rpcs():
    """The RPCs TestFragmentRPCFunction feeds to fragmentRPC, in order, with the
    test's expectation for each (gossipsub_test.go:2107-2249)."""
    rng = random.Random(2085)
    topic = "test"
    cases = []
    cases.append(("fits", O.RPC(publish=[mk_msg(rng, 10), mk_msg(rng, 10)])))
    cases.append(("too_big", O.RPC(publish=[mk_msg(rng, 10), mk_msg(rng, LIMIT * 2)])))
    subs = [O.SubOpts(subscribe=True, topicid=topic)]
    pubs = [mk_msg(rng, 200) for _ in range(100)]
    cases.append(("publish", O.RPC(subscriptions=subs, publish=pubs)))
    ctl = O.Control(graft=[O.Graft(topic)], prune=[O.Prune(topic)],
                    ihave=[O.IHave(ids=[b"foo"])], iwant=[O.IWant(ids=[b"bar"])])
    cases.append(("control_whole", O.RPC(subscriptions=subs, publish=pubs, control=ctl)))
    tag = 0
    ihave, iwant = [], []
    for _ in range(5):
        ids = []
        for _ in range(100):
            tag += 1
            ids.append(mk_id(rng, 32, tag))
        ihave.append(O.IHave(ids=ids))
        iwant.append(O.IWant(ids=ids))
    ctl2 = O.Control(graft=ctl.graft, prune=ctl.prune, ihave=ihave, iwant=iwant)
    cases.append(("control_split", O.RPC(subscriptions=subs, publish=pubs, control=ctl2)))
    giant = bytes(rng.getrandbits(8) for _ in range(LIMIT * 2))
    cases.append(("giant_id", O.RPC(control=O.Control(iwant=[O.IWant(ids=[b"hello", giant])]))))
    return cases


# ---- the oracle against the reference's own assertions ---------------------

def test_oracle_pinned_by_reference_test():
    cases = dict(reference_case_rpcs())
    below = lambda rs: all(O.size(r) <= LIMIT for r in rs)  # noqa: E731
    assert len(O.fragment_rpc(cases["fits"], LIMIT)) == 1
    with pytest.raises(ValueError):
        O.fragment_rpc(cases["too_big"], LIMIT)
    msgs_per_rpc = LIMIT // 200
    r = O.fragment_rpc(cases["publish"], LIMIT)
    assert below(r) and len(r) == 100 // msgs_per_rpc
    assert sum(len(x.publish) for x in r) == 100 and sum(len(x.subscriptions) for x in r) == 1
    rpc = cases["control_whole"]
    r = O.fragment_rpc(rpc, LIMIT)
    assert below(r) and len(r) == 100 // msgs_per_rpc + 1
    assert r[-1].control is not None and r[-1].control.marshal() == rpc.control.marshal()
    rpc = cases["control_split"]
    r = O.fragment_rpc(rpc, LIMIT)
    assert below(r)
    assert len(r) >= 100 // msgs_per_rpc + O.size(rpc.control) // LIMIT
    r = O.fragment_rpc(cases["giant_id"], LIMIT)
    assert len(r) == 1 and len(r[0].control.iwant) == 1
    assert r[0].control.iwant[0].ids[0] == b"hello"


def test_oracle_encoder_sizes():
    # msg.Size() of mkMsg(n): 1 + uvarint(n-4) + (n-4)
    assert O.size(O.Message(data=b"x" * 6)) == 8
    assert O.size(O.Message(data=b"x" * 196)) == 199
    assert O.size(O.SubOpts(subscribe=True, topicid="test")) == 8
    assert O.size(O.Prune("t", peers=[b"p1"], backoff=300)) == 3 + 6 + 3
    # hand-derived from the gogo Size() methods of pb/rpc.pb.go (tag 1 byte,
    # uvarint length, body): ControlPrune with two PX peers and a backoff ...
    #   topicID "topic" 1+1+5; peers PeerInfo{peerID "peer-a"} 1+1+(1+1+6),
    #   PeerInfo{peerID "p"} 1+1+(1+1+1); backoff 60: 1+1
    assert O.size(O.Prune("topic", peers=[b"peer-a", b"p"], backoff=60)) == 7 + 10 + 5 + 2
    # ... inside ControlMessage (field 4) inside RPC (field 3)
    assert O.size(O.RPC(control=O.Control(prune=[O.Prune("topic", peers=[b"peer-a", b"p"], backoff=60)]))) == \
        1 + 1 + (1 + 1 + 24)
    # ControlIHave with a TopicID: topicID "blocks" 1+1+6; ids "m1", "msg22": 1+1+2, 1+1+5
    assert O.size(O.IHave("blocks", [b"m1", b"msg22"])) == 8 + 4 + 7
    assert O.size(O.IHave(None, [b"m1"])) == 4   # a nil TopicID is not written


# ---- product against the oracle --------------------------------------------

def shape_of(rpc):
    from pubsub_amd.rpc import RpcShape
    c = rpc.control
    return RpcShape(
        sub_size=[O.size(s) for s in rpc.subscriptions],
        pub_size=[O.size(m) for m in rpc.publish],
        has_control=c is not None,
        ihave_topic_len=[None if h.topic is None else len(h.topic.encode()) for h in (c.ihave if c else [])],
        ihave_ids=[[len(m) for m in h.ids] for h in (c.ihave if c else [])],
        iwant_ids=[[len(m) for m in w.ids] for w in (c.iwant if c else [])],
        graft_size=[O.size(g) for g in (c.graft if c else [])],
        prune_size=[O.size(p) for p in (c.prune if c else [])])


def check_against_oracle(rpc, limit):
    from pubsub_amd.rpc import GS_RPC_IHAVE, GS_RPC_IWANT, fragment_rpc, rpc_size
    assert rpc_size(shape_of(rpc)) == O.size(rpc)
    try:
        want = O.fragment_rpc(rpc, limit)
    except ValueError as e:
        with pytest.raises(GossipEngineError, match=str(e)):
            fragment_rpc(shape_of(rpc), limit)
        return None
    got = fragment_rpc(shape_of(rpc), limit)
    assert got.n_frag == len(want)
    assert list(got.frag_size) == [O.size(r) for r in want]

    def where(parts, pick):
        pos = {id(x): k for k, r in enumerate(want) for x in pick(r)}
        return [pos[id(x)] for x in parts]

    c = rpc.control
    assert list(got.sub_frag) == where(rpc.subscriptions, lambda r: r.subscriptions)
    assert list(got.pub_frag) == where(rpc.publish, lambda r: r.publish)
    if c is None:
        return got
    ctl_of = lambda r: r.control if r.control is not None else O.Control()  # noqa: E731
    whole = ctl_of(want[-1]) is c
    if whole:
        assert got.control_whole or got.n_frag == 1
        assert list(got.graft_frag) == [len(want) - 1] * len(c.graft)
        assert list(got.prune_frag) == [len(want) - 1] * len(c.prune)
    else:
        assert not got.control_whole
        assert list(got.graft_frag) == where(c.graft, lambda r: ctl_of(r).graft)
        assert list(got.prune_frag) == where(c.prune, lambda r: ctl_of(r).prune)
    # buckets: ids by their position in the shape's id order (ihave ids, then iwant ids)
    all_ids = [m for h in c.ihave for m in h.ids] + [m for w in c.iwant for m in w.ids]
    got_buckets = []
    for b in range(len(got.bucket_frag)):
        ids = [all_ids[i] for i in range(len(all_ids)) if got.id_bucket[i] == b]
        got_buckets.append((int(got.bucket_frag[b]), int(got.bucket_kind[b]), ids))
    if whole:
        exp = ([(len(want) - 1, GS_RPC_IHAVE, h.ids) for h in c.ihave]
               + [(len(want) - 1, GS_RPC_IWANT, w.ids) for w in c.iwant])
    else:
        exp = ([(k, GS_RPC_IWANT, w.ids) for k, r in enumerate(want) for w in ctl_of(r).iwant]
               + [(k, GS_RPC_IHAVE, h.ids) for k, r in enumerate(want) for h in ctl_of(r).ihave])
    assert got_buckets == exp
    # every bucket's ids come from the entry bucket_src names
    n_ih = sum(len(h.ids) for h in c.ihave)
    owner = ([(GS_RPC_IHAVE, j) for j, h in enumerate(c.ihave) for _ in h.ids]
             + [(GS_RPC_IWANT, j) for j, w in enumerate(c.iwant) for _ in w.ids])
    assert len(owner) == len(all_ids) >= n_ih
    for i, b in enumerate(got.id_bucket):
        if b >= 0:
            assert owner[i] == (int(got.bucket_kind[b]), int(got.bucket_src[b]))
    kept = {id(m) for _, _, ids in exp for m in ids}
    for i, m in enumerate(all_ids):
        assert (got.id_bucket[i] >= 0) == (id(m) in kept)
    return got


@pytest.mark.parametrize("name", [n for n, _ in reference_case_rpcs()])
def test_product_matches_oracle_on_reference_cases(name):
    rpc = dict(reference_case_rpcs())[name]
    got = check_against_oracle(rpc, LIMIT)
    if name == "too_big":
        assert got is None
    if name == "control_split":
        assert not got.control_whole and got.n_frag > 20
    if name == "giant_id":
        assert list(got.id_bucket) == [0, -1]


def random_rpc(rng, tag0=0):
    tag = [tag0]

    def mid(n):
        tag[0] += 1
        return mk_id(rng, n, tag[0])

    topics = ["t%d" % i for i in range(rng.randint(1, 6))]
    subs = [O.SubOpts(subscribe=rng.random() < 0.5, topicid=rng.choice(topics))
            for _ in range(rng.randint(0, 6))]
    pubs = [O.Message(from_=b"peer" * rng.randint(0, 3), data=bytes(rng.randint(0, 400)),
                      seqno=bytes(8), topic=rng.choice(topics)) for _ in range(rng.randint(0, 40))]
    ctl = None
    if rng.random() < 0.8:
        ids_len = lambda: rng.choice([4, 8, 20, 32, 40, 120, 600, 1100])  # noqa: E731
        ctl = O.Control(
            ihave=[O.IHave(topic=rng.choice(topics + [None]),
                           ids=[mid(ids_len()) for _ in range(rng.randint(0, 120))])
                   for _ in range(rng.randint(0, 5))],
            iwant=[O.IWant(ids=[mid(ids_len()) for _ in range(rng.randint(0, 120))])
                   for _ in range(rng.randint(0, 5))],
            graft=[O.Graft(rng.choice(topics)) for _ in range(rng.randint(0, 8))],
            prune=[O.Prune(rng.choice(topics), peers=[bytes(38)] * rng.randint(0, 16),
                           backoff=rng.choice([None, 60, 100000])) for _ in range(rng.randint(0, 8))])
    return O.RPC(subscriptions=subs, publish=pubs, control=ctl)


@pytest.mark.parametrize("seed", range(40))
def test_product_matches_oracle_random(seed):
    rng = random.Random(seed)
    rpc = random_rpc(rng)
    for limit in (64, 300, 1024, 4096, 1 << 20):
        check_against_oracle(rpc, limit)


def test_empty_rpc_and_bad_arguments():
    from pubsub_amd.rpc import RpcShape, fragment_rpc
    got = fragment_rpc(RpcShape(), LIMIT)
    assert got.n_frag == 1 and list(got.frag_size) == [0]
    with pytest.raises(GossipEngineError):
        fragment_rpc(RpcShape(), 0)
    with pytest.raises(GossipEngineError):  # control entries without a control message
        fragment_rpc(RpcShape(graft_size=[6]), LIMIT)


def _raw_call(pub=(10,), sub=(), topic_len=None, frag_cap=4, bucket_cap=4, null=()):
    """gs_fragment_rpc through ctypes with hand-built arguments."""
    import ctypes as C
    from pubsub_amd import rpc as R
    lib = R._library()
    keep = []

    def arr(vals, ct):
        a = (ct * max(1, len(vals)))(*vals)
        keep.append(a)
        return C.cast(a, C.POINTER(ct))

    sh = R._Shape()
    sh.n_pub, sh.pub_size = len(pub), arr(pub, C.c_int64)
    sh.n_sub, sh.sub_size = len(sub), arr(sub, C.c_int64)
    if topic_len is not None:
        sh.has_control, sh.n_ihave = 1, 1
        sh.ihave_topic_len, sh.ihave_nids = arr([topic_len], C.c_int64), arr([0], C.c_int32)
    fr = R._Frags()
    fr.sub_frag, fr.pub_frag = arr([0] * 4, C.c_int32), arr([0] * 4, C.c_int32)
    fr.frag_cap, fr.bucket_cap = frag_cap, bucket_cap
    for name, ct in (("frag_size", C.c_int64), ("bucket_frag", C.c_int32), ("bucket_kind", C.c_int32),
                     ("bucket_src", C.c_int32)):
        if name not in null:
            setattr(fr, name, arr([0] * 4, ct))
    return lib.gs_fragment_rpc(C.byref(sh), 1 << 20, C.byref(fr))


@pytest.mark.parametrize("case", [dict(pub=(-1,)), dict(sub=(-3,)), dict(topic_len=-2),
                                  dict(null=("frag_size",)), dict(null=("bucket_frag",)),
                                  dict(null=("bucket_kind",)), dict(null=("bucket_src",))])
def test_fragment_rpc_rejects_bad_arguments(case):
    """Negative part sizes, a TopicID length below -1 (nil) and NULL output
    arrays with a non-zero capacity are GS_EINVAL, not a silently wrong split."""
    assert _raw_call(**case) == -1  # GS_EINVAL


def test_fragment_rpc_accepts_null_outputs_without_capacity():
    assert _raw_call(topic_len=-1) == 0
    assert _raw_call(frag_cap=0, bucket_cap=0, null=("frag_size", "bucket_frag", "bucket_kind", "bucket_src")) \
        == -5  # GS_ECAPACITY: one fragment needed, none room for


def test_product_matches_golden_fixture():
    """tests/golden/rpc_fragment.json (tests/golden/make_rpc_golden.py): the oracle's
    fragment sizes on the reference test's RPCs and on seeded random RPCs."""
    import json
    from pubsub_amd.rpc import RpcShape, fragment_rpc
    cases = json.load(open(os.path.join(REPO, "tests", "golden", "rpc_fragment.json")))
    assert len(cases) == 36
    for c in cases:
        shape = RpcShape(**c["shape"])
        if "error" in c:
            with pytest.raises(GossipEngineError, match=c["error"]):
                fragment_rpc(shape, c["limit"])
        else:
            assert list(fragment_rpc(shape, c["limit"]).frag_size) == c["frag_size"], c["name"]
