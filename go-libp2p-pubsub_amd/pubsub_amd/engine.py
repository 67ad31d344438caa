"""Host-side mirror of the reference's router selection over the C-ABI.

The reference builds one PubSub per host with NewFloodSub / NewRandomSub /
NewGossipSub plus Options (pubsub.go:221, floodsub.go:25, randomsub.go:21,
gossipsub.go:198-391).  This engine is one batched instance for N simulated
hosts; the constructors below take the same parameter structs and options:

    eng = NewGossipSub(n, topics, graph, WithGossipSubParams(p),
                       WithPeerScore(score_params, thresholds), WithFloodPublish(True))

The product path loads ONLY the HIP library (libgossip_engine.so, built for
gfx950) and raises if it is missing: there is no CPU fallback.  Tests pass an
explicit `lib=` to drive the CPU oracle through the identical ABI.
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from .params import GossipSubParams, Millisecond

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(os.path.dirname(_HERE), "build", "libgossip_engine.so")

_lib_cache = {}


def load(path=None):
    """Bind the ABI on `path` (default: the HIP product library)."""
    path = os.path.abspath(path or PRODUCT_LIB)
    if path not in _lib_cache:
        _lib_cache[path] = _abi.bind(path)
    return _lib_cache[path]


class GossipEngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gossip engine error {code}: {msg}")
        self.code = code


def _check(lib, rc):
    if rc != _abi.GS_OK:
        raise GossipEngineError(rc, lib.gs_last_error().decode(errors="replace"))
    return rc


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None


# ---------------------------------------------------------------- options
def WithGossipSubParams(cfg):
    return ("gossipsub_params", cfg)


def WithPeerScore(params, thresholds):
    return ("peer_score", (params, thresholds))


def WithFloodPublish(flood):
    return ("flood_publish", bool(flood))


def WithPeerExchange(do_px=True):
    """WithPeerExchange (gossipsub.go:320): PRUNEs carry peer suggestions and a
    pruned host dials them (needs connection slots: WithDormant)."""
    return ("px", bool(do_px))


def WithDormant(pairs):
    """Connections (a, b) of the graph that start down (gs_set_dormant): slots
    a peer-exchange dial or a GS_EV_CONNECT event can bring up."""
    return ("dormant", [(int(a), int(b)) for a, b in pairs])


def WithDirectPeers(direct_edges):
    """direct_edges: uint8[E] flags in CSR order (WithDirectPeers, gossipsub.go:338)."""
    return ("direct", direct_edges)


def WithSeed(seed):
    return ("seed", int(seed))


def WithHop(hop_ns):
    return ("hop_ns", int(hop_ns))


def WithMessageWindow(slots_per_topic):
    return ("slots_per_topic", int(slots_per_topic))


def WithRecordDeliveries(on=True):
    return ("record", bool(on))


def WithDevice(dev):
    return ("device", int(dev))


def WithRPCAccounting(msg_size, id_len=40, topic_len=None, peer_id_len=38, record_len=0):
    """Per-edge RPC byte accounting (gs_set_rpc_accounting, SURVEY.md §8(f)
    rank 3): every RPC a host sends is measured as RPC.Size() (gossipsub.go:
    1121-1137) with messages of topic t msg_size[t] bytes (a scalar: all
    topics), ids id_len bytes, topic names topic_len[t] bytes (default: the
    decimal index's length, as the trace encoder names topics), PX entries of
    a PRUNE PeerInfo{peer id of peer_id_len bytes, signed record of record_len
    bytes or none} (makePrune, gossipsub.go:1811-1836; gs_set_rpc_px_sizes).
    Read with Engine.rpc_bytes()."""
    return ("rpc_acct", (msg_size, int(id_len), topic_len, int(peer_id_len), int(record_len)))


def WithEventTracer(nodes, capacity=1 << 22, rpc=False):
    """EventTracer (pubsub.go:418, trace.go) for the hosts in `nodes` (indices
    or a bool mask): their PublishMessage / DeliverMessage / DuplicateMessage /
    AddPeer / Join / Graft / Prune events, and with rpc=True every RPC they
    send or receive (SendRPC / RecvRPC with the RPCMeta items), read with
    Engine.trace_events()."""
    return ("trace", (nodes, int(capacity), bool(rpc)))


def WithPeerGater(params):
    """WithPeerGater (peer_gater.go:164-191): random early drop of payload from
    peers with poor goodput while the validation queue is throttling."""
    return ("gater", params)


def WithValidation(topic_validators, queue_per_hop=0):
    """RegisterTopicValidator for the topics with topic_validators[t] true (the
    verdict is each message's `kind`, see Engine.publish), and the validation
    queue: at most queue_per_hop received messages enter validation per node
    per hop (0 = unlimited; WithValidateQueueSize, validation.go:236-241)."""
    return ("validation", (topic_validators, int(queue_per_hop)))


def WithBehaviour(bits):
    """Per-node attacker behaviours (uint8[N] of GS_BEHAVE_* bits)."""
    return ("behaviour", bits)


def WithRouters(routers):
    """The router each host runs (gs_set_routers): GS_ROUTER_FLOODSUB /
    RANDOMSUB / GOSSIPSUB / GOSSIPSUB_V10 per node -- a mixed network
    (TestMixedGossipsub, gossipsub_test.go:810-851)."""
    return ("routers", np.ascontiguousarray(routers, dtype=np.uint8))


def WithProtocols(proto):
    """The protocol.ID of every connection (GS_PROTO_* per CSR edge, the
    `proto` of PubSubRouter.AddPeer, pubsub.go:165); default: negotiated from
    the hosts' routers."""
    return ("protocols", np.ascontiguousarray(proto, dtype=np.uint8))


def WithPeertxCapacity(home_bits, overflow_bits):
    """mcache.peertx capacity (gs_set_peertx_capacity): 2^home_bits slots per
    node, and a per-rank overflow table of 2^overflow_bits entries for nodes
    whose own table is full."""
    return ("peertx", (int(home_bits), int(overflow_bits)))


def WithFrontierLists():
    """Phase A reads the senders' per-copy frontier lists even where the engine
    would OR their frontier bitmaps (gs_set_frontier_mode GS_FRONTIER_LISTS):
    same results, the other kernel path (A/B runs and parity tests)."""
    return ("frontier_mode", 1)


def WithFrontierBitmaps():
    """Phase A ORs the senders' frontier bitmaps wherever the engine supports
    them (GS_FRONTIER_BITMAPS), also where the lists measured faster."""
    return ("frontier_mode", 2)


def WithPartition(rank, world, transport):
    """Simulate only this rank's node range; exchange RPCs with the other
    ranks through `transport` (a pubsub_amd.transport.TorchTransport) once per
    hop.  Every rank makes the same calls (graph, subscriptions, publishes)."""
    return ("partition", (int(rank), int(world), transport))


class Engine:
    """One batched simulation of N routers (see module docstring)."""

    def __init__(self, router, num_nodes, num_topics, graph, subscriptions, *options,
                 randomsub_size=0, app_score=None, ipv4=None, lib=None):
        self.lib = load(lib)
        opts = dict(options)
        gsp = opts.get("gossipsub_params") or GossipSubParams()
        score = opts.get("peer_score")
        cfg = _abi.ConfigC()
        cfg.router = router
        cfg.randomsub_size = randomsub_size
        cfg.num_nodes = num_nodes
        cfg.num_topics = num_topics
        cfg.slots_per_topic = opts.get("slots_per_topic", 1024)
        cfg.seed = opts.get("seed", 1)
        cfg.hop_ns = opts.get("hop_ns", 100 * Millisecond)
        flags = 0
        if score is not None:
            flags |= _abi.GS_FLAG_SCORING
        if opts.get("flood_publish"):
            flags |= _abi.GS_FLAG_FLOOD_PUBLISH
        if opts.get("px"):
            flags |= _abi.GS_FLAG_PEER_EXCHANGE
        if opts.get("record"):
            flags |= _abi.GS_FLAG_RECORD_DELIVERIES
        cfg.flags = flags
        cfg.device = opts.get("device", 0)
        self.N, self.T = num_nodes, num_topics
        self.score_params = score[0] if score is not None else None
        gsp_c = gsp.to_c()
        psp_c = topics_c = scored_c = thr_c = None
        if score is not None:
            params, thresholds = score
            psp_c = params.to_c()
            topics_c, scored_c = params.topics_c(num_topics)
            thr_c = thresholds.to_c()
        h = C.c_void_p()
        _check(self.lib, self.lib.gs_engine_create(
            C.byref(cfg), C.byref(gsp_c),
            C.byref(psp_c) if psp_c is not None else None,
            topics_c, scored_c,
            C.byref(thr_c) if thr_c is not None else None,
            C.byref(opts["gater"].to_c()) if opts.get("gater") is not None else None, C.byref(h)))
        self.h = h
        rowptr, col, outbound = graph
        self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        self.E = int(self.rowptr[-1])
        ob = np.ascontiguousarray(outbound, dtype=np.uint8) if outbound is not None else None
        direct = opts.get("direct")
        direct = np.ascontiguousarray(direct, dtype=np.uint8) if direct is not None else None
        proto = opts.get("protocols")
        if proto is None:
            _check(self.lib, self.lib.gs_set_graph(h, _ptr(self.rowptr, C.c_int64), _ptr(self.col, C.c_int32),
                                                   _ptr(ob, C.c_uint8), _ptr(direct, C.c_uint8)))
        else:
            _check(self.lib, self.lib.gs_set_graph_ex(h, _ptr(self.rowptr, C.c_int64), _ptr(self.col, C.c_int32),
                                                      _ptr(ob, C.c_uint8), _ptr(direct, C.c_uint8),
                                                      _ptr(proto, C.c_uint8)))
        routers = opts.get("routers")
        if routers is not None:
            _check(self.lib, self.lib.gs_set_routers(h, _ptr(routers, C.c_uint8)))
        self.routers = routers
        dormant = opts.get("dormant")
        if dormant:
            da = np.array([a for a, _ in dormant], dtype=np.int32)
            db = np.array([b for _, b in dormant], dtype=np.int32)
            _check(self.lib, self.lib.gs_set_dormant(h, len(da), _ptr(da, C.c_int32), _ptr(db, C.c_int32)))
        tr = opts.get("trace")
        if tr is not None:
            nodes, cap, rpc = tr
            mask = np.zeros(num_nodes, dtype=np.uint8)
            nodes = np.asarray(nodes)
            mask[np.nonzero(nodes)[0] if nodes.dtype == bool else nodes] = 1
            _check(self.lib, self.lib.gs_set_trace(h, _ptr(mask, C.c_uint8), cap))
            if rpc:
                _check(self.lib, self.lib.gs_set_trace_rpc(h, 1))
        ptx = opts.get("peertx")
        if ptx is not None:
            _check(self.lib, self.lib.gs_set_peertx_capacity(h, *ptx))
        if opts.get("frontier_mode"):
            _check(self.lib, self.lib.gs_set_frontier_mode(h, opts["frontier_mode"]))
        acct = opts.get("rpc_acct")
        if acct is not None:
            ms, idl, tl, pid, rec = acct
            ms = np.ascontiguousarray(np.broadcast_to(np.asarray(ms, dtype=np.int32), (num_topics,)))
            tl = (np.array([len(str(t)) for t in range(num_topics)], dtype=np.int32) if tl is None
                  else np.ascontiguousarray(np.broadcast_to(np.asarray(tl, dtype=np.int32), (num_topics,))))
            _check(self.lib, self.lib.gs_set_rpc_accounting(h, _ptr(ms, C.c_int32), idl, _ptr(tl, C.c_int32)))
            _check(self.lib, self.lib.gs_set_rpc_px_sizes(h, pid, rec))
        self.rpc_acct = acct is not None
        self.router = router
        self.hop_ns = cfg.hop_ns
        self.rank, self.world, self.transport = opts.get("partition", (0, 1, None))
        if self.world > 1:
            _check(self.lib, self.lib.gs_set_partition(h, self.rank, self.world, C.byref(self.transport.c)))
        b, e = C.c_int32(), C.c_int32()
        _check(self.lib, self.lib.gs_partition_range(h, C.byref(b), C.byref(e)))
        self.node_range = (b.value, e.value)
        self.n_published = 0  # messages scheduled by publish() (all ranks)
        self.edge_range = (int(self.rowptr[b.value]), int(self.rowptr[e.value]))
        subs = np.ascontiguousarray(subscriptions, dtype=np.uint64)
        _check(self.lib, self.lib.gs_set_subscriptions(h, _ptr(subs, C.c_uint64)))
        self.subs = subs  # the initial subscriptions (topic bit masks per node)
        val = opts.get("validation")
        if val is not None:
            tv = np.zeros(num_topics, dtype=np.uint8)
            tv[:] = np.asarray(val[0], dtype=bool)[:num_topics] if np.ndim(val[0]) else bool(val[0])
            _check(self.lib, self.lib.gs_set_validation(h, _ptr(tv, C.c_uint8), val[1]))
        beh = opts.get("behaviour")
        if beh is not None:
            beh = np.ascontiguousarray(beh, dtype=np.uint8)
            _check(self.lib, self.lib.gs_set_behaviour(h, _ptr(beh, C.c_uint8)))
        app = np.ascontiguousarray(app_score, dtype=np.float64) if app_score is not None else None
        ips = np.ascontiguousarray(ipv4, dtype=np.uint32) if ipv4 is not None else None
        self.app_attr, self.ipv4_attr = app, ips  # gs_set_peer_attrs inputs (None: zeros)
        if app is not None or ips is not None:
            _check(self.lib, self.lib.gs_set_peer_attrs(h, _ptr(app, C.c_double), _ptr(ips, C.c_uint32)))

    def close(self):
        if getattr(self, "h", None):
            self.lib.gs_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- driving
    def publish(self, src, topic, hop, kind=None):
        """Topic.Publish at node src[i] at hop hop[i]; kind[i] (GS_MSG_*) is the
        verdict of the receivers' topic validator, or PHANTOM (advertised only)."""
        src = np.ascontiguousarray(src, dtype=np.int32)
        topic = np.ascontiguousarray(topic, dtype=np.int32)
        hop = np.ascontiguousarray(hop, dtype=np.int64)
        ids = np.empty(len(src), dtype=np.int64)
        kd = np.ascontiguousarray(kind, dtype=np.uint8) if kind is not None else None
        _check(self.lib, self.lib.gs_publish_ex(self.h, len(src), _ptr(src, C.c_int32), _ptr(topic, C.c_int32),
                                                _ptr(hop, C.c_int64), _ptr(kd, C.c_uint8), _ptr(ids, C.c_int64)))
        self.n_published += len(src)
        return ids

    def schedule_events(self, kind, a, b, hop):
        """Connection churn and subscription changes at the start of hop[i]
        (gs_schedule_events): GS_EV_DISCONNECT / GS_EV_CONNECT of the connection
        a[i] - b[i], GS_EV_LEAVE / GS_EV_JOIN of topic b[i] by node a[i]."""
        kind = np.ascontiguousarray(kind, dtype=np.int32)
        a = np.ascontiguousarray(a, dtype=np.int32)
        b = np.ascontiguousarray(b, dtype=np.int32)
        hop = np.ascontiguousarray(hop, dtype=np.int64)
        _check(self.lib, self.lib.gs_schedule_events(self.h, len(kind), _ptr(kind, C.c_int32), _ptr(a, C.c_int32),
                                                     _ptr(b, C.c_int32), _ptr(hop, C.c_int64)))

    def exchange_stats(self):
        """(host ms spent in the transport, bytes received from other ranks)."""
        ms, nb = C.c_double(), C.c_int64()
        _check(self.lib, self.lib.gs_read_exchange_stats(self.h, C.byref(ms), C.byref(nb)))
        return ms.value, nb.value

    @property
    def frontier_dense(self):
        """True once started if phase A ORs frontier bitmaps (gs_frontier_dense)."""
        return bool(self.lib.gs_frontier_dense(self.h))

    def step(self, hops=1):
        _check(self.lib, self.lib.gs_step(self.h, int(hops)))

    def sync(self):
        _check(self.lib, self.lib.gs_sync(self.h))

    def set_topic_score_params(self, topic, p):
        c = p.to_c()
        _check(self.lib, self.lib.gs_set_topic_score_params(self.h, topic, C.byref(c)))

    @property
    def hop(self):
        return int(self.lib.gs_current_hop(self.h))

    # ---------------------------------------------------------------- readbacks
    def counters(self):
        c = _abi.CountersC()
        _check(self.lib, self.lib.gs_read_counters(self.h, C.byref(c)))
        return c.as_dict()

    def scores(self):
        a = np.empty(self.E, dtype=np.float64)
        _check(self.lib, self.lib.gs_read_scores(self.h, _ptr(a, C.c_double)))
        return a

    def mesh(self):
        a = np.empty(self.E, dtype=np.uint64)
        _check(self.lib, self.lib.gs_read_mesh(self.h, _ptr(a, C.c_uint64)))
        return a

    def fanout(self):
        a = np.empty(self.E, dtype=np.uint64)
        _check(self.lib, self.lib.gs_read_fanout(self.h, _ptr(a, C.c_uint64)))
        return a

    def backoff(self):
        a = np.empty(self.E * self.T, dtype=np.int64)
        _check(self.lib, self.lib.gs_read_backoff(self.h, _ptr(a, C.c_int64)))
        return a.reshape(self.T, self.E)

    def topic_stats(self):
        n = self.E * self.T
        fmd, mmd, mfp, imd = (np.empty(n, dtype=np.float64) for _ in range(4))
        mt, gt = np.empty(n, dtype=np.int64), np.empty(n, dtype=np.int64)
        fl = np.empty(n, dtype=np.uint8)
        _check(self.lib, self.lib.gs_read_topic_stats(
            self.h, _ptr(fmd, C.c_double), _ptr(mmd, C.c_double), _ptr(mfp, C.c_double),
            _ptr(imd, C.c_double), _ptr(mt, C.c_int64), _ptr(gt, C.c_int64), _ptr(fl, C.c_uint8)))
        sh = (self.T, self.E)
        return dict(fmd=fmd.reshape(sh), mmd=mmd.reshape(sh), mfp=mfp.reshape(sh), imd=imd.reshape(sh),
                    mesh_time=mt.reshape(sh), graft_time=gt.reshape(sh), flags=fl.reshape(sh))

    def topic_stats_at(self, edges):
        """topic_stats() of the given edges only, shape (len(edges), T) per field
        (gs_read_topic_stats_edges): spot checks at full size."""
        edges = np.ascontiguousarray(edges, dtype=np.int64)
        n = len(edges) * self.T
        fmd, mmd, mfp, imd = (np.empty(n, dtype=np.float64) for _ in range(4))
        mt, gt = np.empty(n, dtype=np.int64), np.empty(n, dtype=np.int64)
        fl = np.empty(n, dtype=np.uint8)
        _check(self.lib, self.lib.gs_read_topic_stats_edges(
            self.h, len(edges), _ptr(edges, C.c_int64), _ptr(fmd, C.c_double), _ptr(mmd, C.c_double),
            _ptr(mfp, C.c_double), _ptr(imd, C.c_double), _ptr(mt, C.c_int64), _ptr(gt, C.c_int64),
            _ptr(fl, C.c_uint8)))
        sh = (len(edges), self.T)
        return dict(fmd=fmd.reshape(sh), mmd=mmd.reshape(sh), mfp=mfp.reshape(sh), imd=imd.reshape(sh),
                    mesh_time=mt.reshape(sh), graft_time=gt.reshape(sh), flags=fl.reshape(sh))

    def backoff_at(self, edges):
        """backoff() of the given edges only, shape (len(edges), T) (gs_read_backoff_edges)."""
        edges = np.ascontiguousarray(edges, dtype=np.int64)
        out = np.empty(len(edges) * self.T, dtype=np.int64)
        _check(self.lib, self.lib.gs_read_backoff_edges(self.h, len(edges), _ptr(edges, C.c_int64),
                                                        _ptr(out, C.c_int64)))
        return out.reshape(len(edges), self.T)

    def enough_peers(self, topic, suggested=0):
        """PubSubRouter.EnoughPeers(topic, suggested) of every host (bool [N])."""
        out = np.zeros(self.N, dtype=np.uint8)
        _check(self.lib, self.lib.gs_enough_peers(self.h, int(topic), int(suggested), _ptr(out, C.c_uint8)))
        return out.astype(bool)

    def behaviour_penalty(self):
        a = np.empty(self.E, dtype=np.float64)
        _check(self.lib, self.lib.gs_read_behaviour_penalty(self.h, _ptr(a, C.c_double)))
        return a

    def set_profiling(self, on=True):
        _check(self.lib, self.lib.gs_set_profiling(self.h, 1 if on else 0))

    def kernel_stats(self):
        """{kernel: (total_ms, launches)} accumulated since set_profiling(True)."""
        n = len(_abi.KERNEL_NAMES)
        ms = np.zeros(n, dtype=np.float64)
        cnt = np.zeros(n, dtype=np.int64)
        _check(self.lib, self.lib.gs_read_kernel_stats(self.h, _ptr(ms, C.c_double), _ptr(cnt, C.c_int64)))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(_abi.KERNEL_NAMES)}

    def rpc_bytes(self):
        """(bytes[E], rpcs[E]) sent over every directed edge since the start."""
        b = np.empty(self.E, dtype=np.int64)
        n = np.empty(self.E, dtype=np.int64)
        _check(self.lib, self.lib.gs_read_rpc_bytes(self.h, _ptr(b, C.c_int64), _ptr(n, C.c_int64)))
        return b, n

    def trace_events(self, chunk=1 << 16):
        """Every recorded event since the last call, in canonical order
        (include/gs_trace.h), as a structured array (_abi.TRACE_EVENT_DTYPE)."""
        parts = []
        n = C.c_int64()
        while True:
            buf = np.empty(chunk, dtype=_abi.TRACE_EVENT_DTYPE)
            _check(self.lib, self.lib.gs_trace_read(self.h, buf.ctypes.data, chunk, C.byref(n)))
            parts.append(buf[:n.value])
            if n.value < chunk:
                return np.concatenate(parts)

    def deliveries(self, msg_id):
        hop = np.empty(self.N, dtype=np.int32)
        frm = np.empty(self.N, dtype=np.int32)
        _check(self.lib, self.lib.gs_read_deliveries(self.h, int(msg_id), _ptr(hop, C.c_int32),
                                                     _ptr(frm, C.c_int32)))
        return hop, frm


PROTOCOLS = {_abi.GS_ROUTER_FLOODSUB: "/floodsub/1.0.0", _abi.GS_ROUTER_RANDOMSUB: "/randomsub/1.0.0",
             _abi.GS_ROUTER_GOSSIPSUB: "/meshsub/1.1.0"}  # floodsub.go:15, randomsub.go:16, gossipsub.go:25


def encode_trace(events, fmt=_abi.GS_TRACE_FORMAT_PB, hop_ns=100 * Millisecond, topic_names=None,
                 proto="/meshsub/1.1.0", lib=None):
    """The reference tracers' output for `events` (Engine.trace_events()):
    uvarint-delimited pb.TraceEvent (PBTracer) or JSON lines (JSONTracer)."""
    lib = load(lib)
    ev = np.ascontiguousarray(events, dtype=_abi.TRACE_EVENT_DTYPE)
    names = None
    if topic_names is not None:
        names = (C.c_char_p * len(topic_names))(*[t if isinstance(t, bytes) else t.encode() for t in topic_names])
    need = C.c_int64()
    rc = lib.gs_trace_encode(ev.ctypes.data, len(ev), fmt, hop_ns, names, proto.encode(), None, 0, C.byref(need))
    if rc not in (_abi.GS_OK, _abi.GS_ECAPACITY):
        _check(lib, rc)
    buf = (C.c_uint8 * max(1, need.value))()
    _check(lib, lib.gs_trace_encode(ev.ctypes.data, len(ev), fmt, hop_ns, names, proto.encode(),
                                    C.cast(buf, C.c_void_p), need.value, C.byref(need)))
    return bytes(buf[:need.value])


def NewFloodSub(num_nodes, num_topics, graph, subscriptions, *options, **kw):
    """floodsub.go:25-27 (batched)."""
    return Engine(_abi.GS_ROUTER_FLOODSUB, num_nodes, num_topics, graph, subscriptions, *options, **kw)


def NewRandomSub(num_nodes, num_topics, graph, subscriptions, size, *options, **kw):
    """randomsub.go:21-27 (batched)."""
    return Engine(_abi.GS_ROUTER_RANDOMSUB, num_nodes, num_topics, graph, subscriptions, *options,
                  randomsub_size=size, **kw)


def NewGossipSub(num_nodes, num_topics, graph, subscriptions, *options, **kw):
    """gossipsub.go:198-222 (batched)."""
    return Engine(_abi.GS_ROUTER_GOSSIPSUB, num_nodes, num_topics, graph, subscriptions, *options, **kw)
