"""ctypes mirror of include/gossip_engine.h.

Struct layouts and function signatures are declared once here and bound to
whichever library exports the ABI: the product (libgossip_engine.so, HIP) or,
in tests only, the CPU oracle (oracle/_build/libgossip_oracle.so).
"""
import ctypes as C

import numpy as np
import os

GS_OK = 0
GS_EINVAL = -1
GS_ESTATE = -2
GS_ENOMEM = -3
GS_EDEVICE = -4
GS_ECAPACITY = -5
GS_EUNSUPPORTED = -6

GS_ROUTER_FLOODSUB = 0
GS_ROUTER_RANDOMSUB = 1
GS_ROUTER_GOSSIPSUB = 2
GS_ROUTER_GOSSIPSUB_V10 = 3  # gs_set_routers only: a gossipsub host speaking v1.0 + floodsub

# protocol.ID of a connection (gs_set_graph_ex)
GS_PROTO_DEFAULT, GS_PROTO_FLOODSUB, GS_PROTO_RANDOMSUB, GS_PROTO_GOSSIPSUB_V10, GS_PROTO_GOSSIPSUB_V11 = 0, 1, 2, 3, 4

GS_FLAG_SCORING = 1 << 0
GS_FLAG_FLOOD_PUBLISH = 1 << 1
GS_FLAG_RECORD_DELIVERIES = 1 << 2
GS_FLAG_PEER_EXCHANGE = 1 << 3

GS_MSG_VALID, GS_MSG_REJECT, GS_MSG_IGNORE, GS_MSG_PHANTOM = 0, 1, 2, 3
GS_BEHAVE_NO_FORWARD, GS_BEHAVE_IWANT_SPAM, GS_BEHAVE_GRAFT_SPAM, GS_BEHAVE_IHAVE_SPAM = 1, 2, 4, 8
GS_EV_DISCONNECT, GS_EV_CONNECT, GS_EV_LEAVE, GS_EV_JOIN = 0, 1, 2, 3
REJECT_REASONS = ["blacklisted peer", "blacklisted source", "missing signature", "unexpected signature",
                  "unexpected auth info", "invalid signature", "validation queue full", "validation throttled",
                  "validation failed", "validation ignored", "self originated message"]  # tracer.go:27-38

i32, i64, u32, u64, f64, u8 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double, C.c_uint8


class GossipSubParamsC(C.Structure):
    _fields_ = [
        ("D", i32), ("Dlo", i32), ("Dhi", i32), ("Dscore", i32), ("Dout", i32),
        ("HistoryLength", i32), ("HistoryGossip", i32), ("Dlazy", i32),
        ("GossipFactor", f64), ("GossipRetransmission", i32),
        ("HeartbeatInitialDelay", i64), ("HeartbeatInterval", i64), ("FanoutTTL", i64),
        ("PrunePeers", i32), ("PruneBackoff", i64), ("Connectors", i32),
        ("MaxPendingConnections", i32), ("ConnectionTimeout", i64),
        ("DirectConnectTicks", u64), ("DirectConnectInitialDelay", i64),
        ("OpportunisticGraftTicks", u64), ("OpportunisticGraftPeers", i32),
        ("GraftFloodThreshold", i64), ("MaxIHaveLength", i32), ("MaxIHaveMessages", i32),
        ("IWantFollowupTime", i64),
    ]


class PeerScoreParamsC(C.Structure):
    _fields_ = [
        ("TopicScoreCap", f64), ("AppSpecificScorePresent", i32), ("AppSpecificWeight", f64),
        ("IPColocationFactorWeight", f64), ("IPColocationFactorThreshold", i32),
        ("BehaviourPenaltyWeight", f64), ("BehaviourPenaltyThreshold", f64),
        ("BehaviourPenaltyDecay", f64), ("DecayInterval", i64), ("DecayToZero", f64),
        ("RetainScore", i64),
    ]


class TopicScoreParamsC(C.Structure):
    _fields_ = [
        ("TopicWeight", f64), ("TimeInMeshWeight", f64), ("TimeInMeshQuantum", i64),
        ("TimeInMeshCap", f64), ("FirstMessageDeliveriesWeight", f64),
        ("FirstMessageDeliveriesDecay", f64), ("FirstMessageDeliveriesCap", f64),
        ("MeshMessageDeliveriesWeight", f64), ("MeshMessageDeliveriesDecay", f64),
        ("MeshMessageDeliveriesCap", f64), ("MeshMessageDeliveriesThreshold", f64),
        ("MeshMessageDeliveriesWindow", i64), ("MeshMessageDeliveriesActivation", i64),
        ("MeshFailurePenaltyWeight", f64), ("MeshFailurePenaltyDecay", f64),
        ("InvalidMessageDeliveriesWeight", f64), ("InvalidMessageDeliveriesDecay", f64),
    ]


class PeerScoreThresholdsC(C.Structure):
    _fields_ = [
        ("GossipThreshold", f64), ("PublishThreshold", f64), ("GraylistThreshold", f64),
        ("AcceptPXThreshold", f64), ("OpportunisticGraftThreshold", f64),
    ]


class PeerGaterParamsC(C.Structure):
    _fields_ = [
        ("Threshold", f64), ("GlobalDecay", f64), ("SourceDecay", f64), ("DecayInterval", i64),
        ("DecayToZero", f64), ("RetainStats", i64), ("Quiet", i64), ("DuplicateWeight", f64),
        ("IgnoreWeight", f64), ("RejectWeight", f64),
    ]


class ConfigC(C.Structure):
    _fields_ = [
        ("router", i32), ("randomsub_size", i32), ("num_nodes", i32), ("num_topics", i32),
        ("slots_per_topic", i32), ("seed", u32), ("hop_ns", i64), ("flags", u32), ("device", i32),
    ]


# gs_trace_event (gossip_engine.h): 32 bytes
TRACE_EVENT_DTYPE = np.dtype([("hop", "<i8"), ("msg", "<i8"), ("type", "<i4"), ("node", "<i4"),
                              ("peer", "<i4"), ("topic", "<i2"), ("phase", "u1"), ("reason", "u1")])
TRACE_TYPES = ["PUBLISH_MESSAGE", "REJECT_MESSAGE", "DUPLICATE_MESSAGE", "DELIVER_MESSAGE", "ADD_PEER",
               "REMOVE_PEER", "RECV_RPC", "SEND_RPC", "DROP_RPC", "JOIN", "LEAVE", "GRAFT", "PRUNE"]
GS_TRACE_FORMAT_PB, GS_TRACE_FORMAT_JSON = 0, 1
# not a pb.TraceEvent type: one RPCMeta entry of the RPC event before it (gossip_engine.h)
GS_TRACE_RPC_ITEM = 32
(GS_RPC_ITEM_MSG, GS_RPC_ITEM_SUB, GS_RPC_ITEM_CTL, GS_RPC_ITEM_IHAVE, GS_RPC_ITEM_IWANT, GS_RPC_ITEM_GRAFT,
 GS_RPC_ITEM_PRUNE, GS_RPC_ITEM_PX) = range(8)


class CountersC(C.Structure):
    _fields_ = [
        ("hops", i64), ("heartbeats", i64), ("published", i64), ("deliveries", i64),
        ("duplicates", i64), ("transmissions", i64), ("grafts_sent", i64), ("prunes_sent", i64),
        ("ihave_sent", i64), ("iwant_sent", i64), ("iwant_served", i64),
        ("promises_broken", i64), ("graylisted", i64), ("rejected", i64), ("throttled", i64),
        ("gated", i64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


P = C.c_void_p

# gs_transport callbacks (gossip_engine.h)
ALLGATHER_I64 = C.CFUNCTYPE(C.c_int, P, C.POINTER(i64), i32, C.POINTER(i64))
ALLGATHER = C.CFUNCTYPE(C.c_int, P, P, P, i64)
ALLTOALLV = C.CFUNCTYPE(C.c_int, P, P, C.POINTER(i64), P, C.POINTER(i64))


class TransportC(C.Structure):
    _fields_ = [("user", P), ("allgather_i64", ALLGATHER_I64), ("allgather", ALLGATHER),
                ("alltoallv", ALLTOALLV)]


# (name, restype, argtypes) for every function declared in gossip_engine.h
ABI_FUNCTIONS = [
    ("gs_abi_version", C.c_int, []),
    ("gs_last_error", C.c_char_p, []),
    ("gs_default_gossipsub_params", None, [C.POINTER(GossipSubParamsC)]),
    ("gs_default_peer_gater_params", None, [C.POINTER(PeerGaterParamsC)]),
    ("gs_score_parameter_decay_with_base", f64, [i64, i64, f64]),
    ("gs_score_parameter_decay", f64, [i64]),
    ("gs_validate_thresholds", C.c_int, [C.POINTER(PeerScoreThresholdsC)]),
    ("gs_validate_peer_score_params", C.c_int,
     [C.POINTER(PeerScoreParamsC), C.POINTER(TopicScoreParamsC), C.POINTER(u8), i32]),
    ("gs_validate_topic_score_params", C.c_int, [C.POINTER(TopicScoreParamsC)]),
    ("gs_validate_peer_gater_params", C.c_int, [C.POINTER(PeerGaterParamsC)]),
    ("gs_engine_create", C.c_int,
     [C.POINTER(ConfigC), C.POINTER(GossipSubParamsC), C.POINTER(PeerScoreParamsC),
      C.POINTER(TopicScoreParamsC), C.POINTER(u8), C.POINTER(PeerScoreThresholdsC),
      C.POINTER(PeerGaterParamsC), C.POINTER(P)]),
    ("gs_engine_destroy", C.c_int, [P]),
    ("gs_set_graph", C.c_int, [P, C.POINTER(i64), C.POINTER(i32), C.POINTER(u8), C.POINTER(u8)]),
    ("gs_set_graph_ex", C.c_int, [P, C.POINTER(i64), C.POINTER(i32), C.POINTER(u8), C.POINTER(u8), C.POINTER(u8)]),
    ("gs_set_routers", C.c_int, [P, C.POINTER(u8)]),
    ("gs_enough_peers", C.c_int, [P, i32, i32, C.POINTER(u8)]),
    ("gs_set_subscriptions", C.c_int, [P, C.POINTER(u64)]),
    ("gs_set_peer_attrs", C.c_int, [P, C.POINTER(f64), C.POINTER(u32)]),
    ("gs_set_ip_whitelist", C.c_int, [P, i32, C.POINTER(u32), C.POINTER(u32)]),
    ("gs_publish", C.c_int, [P, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i64), C.POINTER(i64)]),
    ("gs_publish_ex", C.c_int, [P, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i64), C.POINTER(u8),
                                C.POINTER(i64)]),
    ("gs_set_validation", C.c_int, [P, C.POINTER(u8), i32]),
    ("gs_set_behaviour", C.c_int, [P, C.POINTER(u8)]),
    ("gs_schedule_events", C.c_int, [P, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i64)]),
    ("gs_step", C.c_int, [P, i64]),
    ("gs_sync", C.c_int, [P]),
    ("gs_set_topic_score_params", C.c_int, [P, i32, C.POINTER(TopicScoreParamsC)]),
    ("gs_set_partition", C.c_int, [P, i32, i32, C.POINTER(TransportC)]),
    ("gs_partition_range", C.c_int, [P, C.POINTER(i32), C.POINTER(i32)]),
    ("gs_read_exchange_stats", C.c_int, [P, C.POINTER(f64), C.POINTER(i64)]),
    ("gs_num_edges", i64, [P]),
    ("gs_current_hop", i64, [P]),
    ("gs_read_counters", C.c_int, [P, C.POINTER(CountersC)]),
    ("gs_read_scores", C.c_int, [P, C.POINTER(f64)]),
    ("gs_read_mesh", C.c_int, [P, C.POINTER(u64)]),
    ("gs_read_fanout", C.c_int, [P, C.POINTER(u64)]),
    ("gs_read_backoff", C.c_int, [P, C.POINTER(i64)]),
    ("gs_read_topic_stats", C.c_int,
     [P, C.POINTER(f64), C.POINTER(f64), C.POINTER(f64), C.POINTER(f64), C.POINTER(i64),
      C.POINTER(i64), C.POINTER(u8)]),
    ("gs_read_behaviour_penalty", C.c_int, [P, C.POINTER(f64)]),
    ("gs_read_backoff_edges", C.c_int, [P, i64, C.POINTER(i64), C.POINTER(i64)]),
    ("gs_read_topic_stats_edges", C.c_int,
     [P, i64, C.POINTER(i64), C.POINTER(f64), C.POINTER(f64), C.POINTER(f64), C.POINTER(f64), C.POINTER(i64),
      C.POINTER(i64), C.POINTER(u8)]),
    ("gs_read_deliveries", C.c_int, [P, i64, C.POINTER(i32), C.POINTER(i32)]),
    ("gs_set_rpc_accounting", C.c_int, [P, C.POINTER(i32), i32, C.POINTER(i32)]),
    ("gs_set_rpc_px_sizes", C.c_int, [P, i32, i32]),
    ("gs_read_rpc_bytes", C.c_int, [P, C.POINTER(i64), C.POINTER(i64)]),
    ("gs_set_trace", C.c_int, [P, C.POINTER(u8), i64]),
    ("gs_set_trace_rpc", C.c_int, [P, i32]),
    ("gs_set_peertx_capacity", C.c_int, [P, i32, i32]),
    ("gs_set_frontier_mode", C.c_int, [P, i32]),
    ("gs_frontier_dense", C.c_int, [P]),
    ("gs_set_dormant", C.c_int, [P, i32, C.POINTER(i32), C.POINTER(i32)]),
    ("gs_trace_read", C.c_int, [P, P, i64, C.POINTER(i64)]),
    ("gs_trace_encode", C.c_int, [P, i64, i32, i64, C.POINTER(C.c_char_p), C.c_char_p, P, i64, C.POINTER(i64)]),
    ("gs_set_profiling", C.c_int, [P, C.c_int]),
    ("gs_read_kernel_stats", C.c_int, [P, C.POINTER(f64), C.POINTER(i64)]),
]

# include/gs_transport.h (product library only; bound by transport.RcclTransport)
GS_RCCL_ID_BYTES = 128
RCCL_FUNCTIONS = [
    ("gs_rccl_get_unique_id", C.c_int, [C.POINTER(u8)]),
    ("gs_rccl_create", C.c_int, [i32, i32, C.POINTER(u8), i32, C.POINTER(P)]),
    ("gs_rccl_transport", C.c_int, [P, C.POINTER(TransportC)]),
    ("gs_rccl_stats", C.c_int, [P, C.POINTER(i64), C.POINTER(i64)]),
    ("gs_rccl_destroy", C.c_int, [P]),
]

KERNEL_NAMES = ["score", "refresh", "join", "fanout", "fwd", "phase_a", "publish", "phase_b",
                "hb_pre", "heartbeat", "push"]


def bind(path):
    """dlopen `path` and declare every gossip_engine.h function on it."""
    if not os.path.exists(path):
        raise OSError(f"gossip engine library not found: {path}")
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    for name, res, args in ABI_FUNCTIONS:
        fn = getattr(lib, name)  # AttributeError = missing export: fail loudly
        fn.restype = res
        fn.argtypes = args
    return lib
