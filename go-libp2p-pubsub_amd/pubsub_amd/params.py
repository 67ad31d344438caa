"""Parameter structs with the reference's Go names and defaults.

GossipSubParams      gossipsub.go:62-195, DefaultGossipSubParams gossipsub.go:226-255
PeerScoreParams      score_params.go:53-96
TopicScoreParams     score_params.go:98-148
PeerScoreThresholds  score_params.go:12-32
PeerGaterParams      peer_gater.go:31-55, DefaultPeerGaterParams peer_gater.go:114-116

Durations are int nanoseconds (Go time.Duration).  Validation lives in the
native library (gs_validate_*), mirroring score_params.go:34-268 and
peer_gater.go:57-88, so the Python layer and a Go/cgo caller see the same
error behaviour.
"""
import math
from dataclasses import dataclass, field, fields

from . import _abi

Nanosecond = 1
Microsecond = 1000
Millisecond = 1000 * Microsecond
Second = 1000 * Millisecond
Minute = 60 * Second
Hour = 60 * Minute

DefaultDecayInterval = Second  # score_params.go:271
DefaultDecayToZero = 0.01      # score_params.go:272


def ScoreParameterDecayWithBase(decay, base, decayToZero):
    """score_params.go:282-287 (pure arithmetic; equals the native export)."""
    ticks = float(decay // base)
    return math.pow(decayToZero, 1 / ticks)


def ScoreParameterDecay(decay):
    """score_params.go:277-279."""
    return ScoreParameterDecayWithBase(decay, DefaultDecayInterval, DefaultDecayToZero)


def _to_c(obj, cls):
    c = cls()
    for f in cls._fields_:
        setattr(c, f[0], getattr(obj, f[0]))
    return c


@dataclass
class GossipSubParams:
    D: int = 6
    Dlo: int = 5
    Dhi: int = 12
    Dscore: int = 4
    Dout: int = 2
    HistoryLength: int = 5
    HistoryGossip: int = 5  # fork quirk: = GossipSubHistoryLength (gossipsub.go:234)
    Dlazy: int = 6
    GossipFactor: float = 0.25
    GossipRetransmission: int = 3
    HeartbeatInitialDelay: int = 100 * Millisecond
    HeartbeatInterval: int = 1 * Second
    FanoutTTL: int = 60 * Second
    PrunePeers: int = 16
    PruneBackoff: int = Minute
    Connectors: int = 8
    MaxPendingConnections: int = 128
    ConnectionTimeout: int = 30 * Second
    DirectConnectTicks: int = 300
    DirectConnectInitialDelay: int = Second
    OpportunisticGraftTicks: int = 60
    OpportunisticGraftPeers: int = 2
    GraftFloodThreshold: int = 10 * Second
    MaxIHaveLength: int = 5000
    MaxIHaveMessages: int = 10
    IWantFollowupTime: int = 3 * Second

    def to_c(self):
        return _to_c(self, _abi.GossipSubParamsC)


def DefaultGossipSubParams():
    return GossipSubParams()


@dataclass
class TopicScoreParams:
    TopicWeight: float = 0.0
    TimeInMeshWeight: float = 0.0
    TimeInMeshQuantum: int = 0
    TimeInMeshCap: float = 0.0
    FirstMessageDeliveriesWeight: float = 0.0
    FirstMessageDeliveriesDecay: float = 0.0
    FirstMessageDeliveriesCap: float = 0.0
    MeshMessageDeliveriesWeight: float = 0.0
    MeshMessageDeliveriesDecay: float = 0.0
    MeshMessageDeliveriesCap: float = 0.0
    MeshMessageDeliveriesThreshold: float = 0.0
    MeshMessageDeliveriesWindow: int = 0
    MeshMessageDeliveriesActivation: int = 0
    MeshFailurePenaltyWeight: float = 0.0
    MeshFailurePenaltyDecay: float = 0.0
    InvalidMessageDeliveriesWeight: float = 0.0
    InvalidMessageDeliveriesDecay: float = 0.0

    def to_c(self):
        return _to_c(self, _abi.TopicScoreParamsC)


@dataclass
class PeerScoreParams:
    """Topics maps topic index -> TopicScoreParams (the Go map's key set).
    AppSpecificScore is a per-node array (or None = function not set)."""
    Topics: dict = field(default_factory=dict)
    TopicScoreCap: float = 0.0
    AppSpecificScore: object = None
    AppSpecificWeight: float = 0.0
    IPColocationFactorWeight: float = 0.0
    IPColocationFactorThreshold: int = 0
    BehaviourPenaltyWeight: float = 0.0
    BehaviourPenaltyThreshold: float = 0.0
    BehaviourPenaltyDecay: float = 0.0
    DecayInterval: int = 0
    DecayToZero: float = 0.0
    RetainScore: int = 0

    def to_c(self):
        c = _abi.PeerScoreParamsC()
        for name, _ in _abi.PeerScoreParamsC._fields_:
            if name == "AppSpecificScorePresent":
                c.AppSpecificScorePresent = 0 if self.AppSpecificScore is None else 1
            else:
                setattr(c, name, getattr(self, name))
        return c

    def topics_c(self, num_topics):
        import ctypes as C
        arr = (_abi.TopicScoreParamsC * num_topics)()
        scored = (C.c_uint8 * num_topics)()
        for t, tp in self.Topics.items():
            if not 0 <= t < num_topics:
                raise ValueError(f"topic index {t} outside [0, {num_topics})")
            arr[t] = tp.to_c()
            scored[t] = 1
        return arr, scored


@dataclass
class PeerScoreThresholds:
    GossipThreshold: float = 0.0
    PublishThreshold: float = 0.0
    GraylistThreshold: float = 0.0
    AcceptPXThreshold: float = 0.0
    OpportunisticGraftThreshold: float = 0.0

    def to_c(self):
        return _to_c(self, _abi.PeerScoreThresholdsC)


@dataclass
class PeerGaterParams:
    Threshold: float = 0.33
    GlobalDecay: float = 0.0
    SourceDecay: float = 0.0
    DecayInterval: int = DefaultDecayInterval
    DecayToZero: float = DefaultDecayToZero
    RetainStats: int = 6 * Hour
    Quiet: int = Minute
    DuplicateWeight: float = 0.125
    IgnoreWeight: float = 1.0
    RejectWeight: float = 16.0

    def to_c(self):
        return _to_c(self, _abi.PeerGaterParamsC)


def NewPeerGaterParams(threshold, globalDecay, sourceDecay):
    """peer_gater.go:97-111."""
    return PeerGaterParams(Threshold=threshold, GlobalDecay=globalDecay, SourceDecay=sourceDecay)


def DefaultPeerGaterParams():
    """peer_gater.go:114-116."""
    return NewPeerGaterParams(0.33, ScoreParameterDecay(2 * Minute), ScoreParameterDecay(Hour))


def eth2_topic_score_params():
    """The Eth2-derived topic parameters the reference's spam test uses
    (gossipsub_spam_test.go:584-602); SURVEY.md §8(d) config 3."""
    return TopicScoreParams(
        TopicWeight=0.25, TimeInMeshWeight=0.0027, TimeInMeshQuantum=Second, TimeInMeshCap=3600,
        FirstMessageDeliveriesWeight=0.664, FirstMessageDeliveriesDecay=0.9916,
        FirstMessageDeliveriesCap=1500, MeshMessageDeliveriesWeight=-0.25,
        MeshMessageDeliveriesDecay=0.97, MeshMessageDeliveriesCap=400,
        MeshMessageDeliveriesThreshold=100, MeshMessageDeliveriesActivation=30 * Second,
        MeshMessageDeliveriesWindow=5 * Minute, MeshFailurePenaltyWeight=-0.25,
        MeshFailurePenaltyDecay=0.997, InvalidMessageDeliveriesWeight=-99,
        InvalidMessageDeliveriesDecay=0.9994)


def eth2_peer_score_params(num_topics=1):
    """Global params of gossipsub_spam_test.go:575-583 with DecayInterval 1 s
     and builder-chosen Eth2-style P6/P7 (no reference
    values exist): P6 weight -35.11 threshold 10, P7 weight -15.92 with decay
    ScoreParameterDecay(10 s)."""
    return PeerScoreParams(
        Topics={t: eth2_topic_score_params() for t in range(num_topics)},
        AppSpecificScore=True, AppSpecificWeight=1.0,
        IPColocationFactorWeight=-35.11, IPColocationFactorThreshold=10,
        BehaviourPenaltyWeight=-15.92, BehaviourPenaltyThreshold=0.0,
        BehaviourPenaltyDecay=ScoreParameterDecay(10 * Second),
        DecayInterval=Second, DecayToZero=0.01, RetainScore=10 * Second)


def eth2_thresholds():
    """gossipsub_spam_test.go:603-608 + opportunistic graft 1 (gossipsub_test.go:1708)."""
    return PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-200,
                               GraylistThreshold=-300, AcceptPXThreshold=0,
                               OpportunisticGraftThreshold=1)
