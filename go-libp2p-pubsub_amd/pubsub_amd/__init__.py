"""pubsub_amd — MI355X batched gossip engine (host side).

Mirrors the router-selection / parameter API of go-libp2p-pubsub over the
C-ABI in include/gossip_engine.h; the compute runs in the HIP library
build/libgossip_engine.so (gfx950).
"""
from ._abi import (GS_BEHAVE_GRAFT_SPAM, GS_BEHAVE_IHAVE_SPAM, GS_BEHAVE_IWANT_SPAM, GS_BEHAVE_NO_FORWARD, GS_MSG_IGNORE,  # noqa: F401
                   GS_EV_CONNECT, GS_EV_DISCONNECT, GS_EV_JOIN, GS_EV_LEAVE, GS_MSG_PHANTOM, GS_MSG_REJECT, GS_MSG_VALID, GS_ROUTER_FLOODSUB, GS_ROUTER_GOSSIPSUB,
                   GS_ROUTER_RANDOMSUB, GS_ROUTER_GOSSIPSUB_V10, GS_PROTO_DEFAULT, GS_PROTO_FLOODSUB,
                   GS_PROTO_RANDOMSUB, GS_PROTO_GOSSIPSUB_V10, GS_PROTO_GOSSIPSUB_V11)
from .params import (DefaultGossipSubParams, DefaultPeerGaterParams, GossipSubParams,  # noqa: F401
                     Hour, Microsecond, Millisecond, Minute, NewPeerGaterParams, PeerGaterParams,
                     PeerScoreParams, PeerScoreThresholds, ScoreParameterDecay,
                     ScoreParameterDecayWithBase, Second, TopicScoreParams, eth2_peer_score_params,
                     eth2_thresholds, eth2_topic_score_params)
from .engine import (PRODUCT_LIB, Engine, GossipEngineError, NewFloodSub, NewGossipSub,  # noqa: F401
                     NewRandomSub, PROTOCOLS, WithDevice, WithEventTracer, encode_trace, WithDirectPeers, WithFloodPublish, WithGossipSubParams,
                     WithHop, WithMessageWindow, WithPartition, WithPeerScore, WithPeertxCapacity, WithFrontierLists, WithFrontierBitmaps, WithRecordDeliveries, WithSeed,
                     WithBehaviour, WithPeerGater, WithRPCAccounting, WithValidation, WithPeerExchange, WithDormant,
                     WithRouters, WithProtocols,
                     load)
