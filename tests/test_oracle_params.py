"""Restates score_params_test.go (validation tables + ScoreParameterDecay) on
the native validate() mirrors.  Runs against the oracle library and — via
test_abi.py — the product library exports the same functions."""
import ctypes as C
import math

import pytest

from pubsub_amd import _abi
from pubsub_amd.params import (Hour, Millisecond, PeerScoreParams, PeerScoreThresholds, Second,
                               ScoreParameterDecay, TopicScoreParams)

INF, NAN = math.inf, math.nan


@pytest.fixture(scope="module")
def lib(oracle_path):
    return _abi.bind(oracle_path)


def thr_ok(lib, **kw):
    return lib.gs_validate_thresholds(C.byref(PeerScoreThresholds(**kw).to_c())) == 0


def topic_ok(lib, **kw):
    return lib.gs_validate_topic_score_params(C.byref(TopicScoreParams(**kw).to_c())) == 0


def peer_ok(lib, p):
    arr, scored = p.topics_c(max(1, len(p.Topics)))
    return lib.gs_validate_peer_score_params(C.byref(p.to_c()), arr, scored, max(1, len(p.Topics))) == 0


def test_thresholds_validation(lib):  # score_params_test.go:11-46
    assert not thr_ok(lib, GossipThreshold=1)
    assert not thr_ok(lib, PublishThreshold=1)
    assert not thr_ok(lib, GossipThreshold=-1, PublishThreshold=0)
    assert not thr_ok(lib, GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=0)
    assert not thr_ok(lib, AcceptPXThreshold=-1)
    assert not thr_ok(lib, OpportunisticGraftThreshold=-1)
    assert thr_ok(lib, GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=-3, AcceptPXThreshold=1,
                  OpportunisticGraftThreshold=2)
    base = dict(GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=-3, AcceptPXThreshold=1,
                OpportunisticGraftThreshold=2)
    for k, v in [("GossipThreshold", -INF), ("PublishThreshold", -INF), ("GraylistThreshold", -INF),
                 ("AcceptPXThreshold", NAN), ("OpportunisticGraftThreshold", INF)]:
        assert not thr_ok(lib, **{**base, k: v})


GOOD_TOPIC = dict(TopicWeight=1, TimeInMeshWeight=0.01, TimeInMeshQuantum=Second, TimeInMeshCap=10,
                  FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=0.5, FirstMessageDeliveriesCap=10,
                  MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=0.5, MeshMessageDeliveriesCap=10,
                  MeshMessageDeliveriesThreshold=5, MeshMessageDeliveriesWindow=Millisecond,
                  MeshMessageDeliveriesActivation=Second, MeshFailurePenaltyWeight=-1,
                  MeshFailurePenaltyDecay=0.5, InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=0.5)


def test_topic_score_params_validation(lib):  # score_params_test.go:48-155
    Q = dict(TimeInMeshQuantum=Second)
    bad = [
        {}, dict(TopicWeight=-1), dict(TimeInMeshWeight=-1, TimeInMeshQuantum=Second),
        dict(TimeInMeshWeight=1, TimeInMeshQuantum=-1),
        dict(TimeInMeshWeight=1, TimeInMeshQuantum=Second, TimeInMeshCap=-1),
        dict(Q, FirstMessageDeliveriesWeight=-1),
        dict(Q, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=-1),
        dict(Q, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=2),
        dict(Q, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=.5, FirstMessageDeliveriesCap=-1),
        dict(Q, MeshMessageDeliveriesWeight=1),
        dict(Q, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=-1),
        dict(Q, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=2),
        dict(Q, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5, MeshMessageDeliveriesCap=-1),
        dict(Q, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5, MeshMessageDeliveriesCap=5,
             MeshMessageDeliveriesThreshold=-3),
        dict(Q, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5, MeshMessageDeliveriesCap=5,
             MeshMessageDeliveriesThreshold=3, MeshMessageDeliveriesWindow=-1),
        dict(Q, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5, MeshMessageDeliveriesCap=5,
             MeshMessageDeliveriesThreshold=3, MeshMessageDeliveriesWindow=Millisecond,
             MeshMessageDeliveriesActivation=Millisecond),
        dict(Q, MeshFailurePenaltyWeight=1),
        dict(Q, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=-1),
        dict(Q, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=2),
        dict(Q, InvalidMessageDeliveriesWeight=1),
        dict(Q, InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=-1),
        dict(Q, InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=2),
    ]
    for kw in bad:
        assert not topic_ok(lib, **kw), kw
    assert topic_ok(lib, **GOOD_TOPIC)


def test_peer_score_params_validation(lib):  # score_params_test.go:157-320
    app = True
    bad = [
        PeerScoreParams(TopicScoreCap=-1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01),
        PeerScoreParams(TopicScoreCap=1, DecayInterval=Second, DecayToZero=0.01),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01,
                        IPColocationFactorWeight=1),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=-1),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Millisecond, DecayToZero=0.01,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=-1,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=2,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1),
        PeerScoreParams(AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01, BehaviourPenaltyWeight=1),
        PeerScoreParams(AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01, BehaviourPenaltyWeight=-1),
        PeerScoreParams(AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01, BehaviourPenaltyWeight=-1,
                        BehaviourPenaltyDecay=2),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1,
                        Topics={0: TopicScoreParams(**{**GOOD_TOPIC, "TopicWeight": -1})}),
        PeerScoreParams(AppSpecificScore=app, DecayInterval=Second, DecayToZero=INF,
                        IPColocationFactorWeight=-INF, IPColocationFactorThreshold=1,
                        BehaviourPenaltyWeight=INF, BehaviourPenaltyDecay=NAN),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1,
                        Topics={0: TopicScoreParams(
                            TopicWeight=INF, TimeInMeshWeight=NAN, TimeInMeshQuantum=Second, TimeInMeshCap=10,
                            FirstMessageDeliveriesWeight=INF, FirstMessageDeliveriesDecay=0.5,
                            FirstMessageDeliveriesCap=10, MeshMessageDeliveriesWeight=-INF,
                            MeshMessageDeliveriesDecay=NAN, MeshMessageDeliveriesCap=INF,
                            MeshMessageDeliveriesThreshold=5, MeshMessageDeliveriesWindow=Millisecond,
                            MeshMessageDeliveriesActivation=Second, MeshFailurePenaltyWeight=-1,
                            MeshFailurePenaltyDecay=NAN, InvalidMessageDeliveriesWeight=INF,
                            InvalidMessageDeliveriesDecay=NAN)}),
    ]
    for p in bad:
        assert not peer_ok(lib, p), p
    good = [
        PeerScoreParams(AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01, IPColocationFactorWeight=-1,
                        IPColocationFactorThreshold=1, BehaviourPenaltyWeight=-1, BehaviourPenaltyDecay=0.999),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1, BehaviourPenaltyWeight=-1,
                        BehaviourPenaltyDecay=0.999),
        PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Second, DecayToZero=0.01,
                        IPColocationFactorWeight=-1, IPColocationFactorThreshold=1,
                        Topics={0: TopicScoreParams(**GOOD_TOPIC)}),
    ]
    for p in good:
        assert peer_ok(lib, p), p


def test_score_parameter_decay(lib):  # score_params_test.go:322-328
    assert ScoreParameterDecay(Hour) == .9987216039048303
    assert lib.gs_score_parameter_decay(Hour) == .9987216039048303
