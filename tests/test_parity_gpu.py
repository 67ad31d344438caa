"""GPU parity: the HIP engine (product library) against the CPU oracle on the
same seeded scenarios, through the identical C-ABI calls.  Everything is
compared bit-exactly: counters, per-(node, message) first-delivery hop and
sender, mesh/fanout masks, backoff expiries, every float64 score counter and
score (on their bit patterns, tolerance 0)."""
import pytest

import scenarios
from pubsub_amd import PRODUCT_LIB

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(scenarios.SCENARIOS))
def test_gpu_matches_oracle(oracle_path, name):
    ref = scenarios.run(oracle_path, name)
    got = scenarios.run(PRODUCT_LIB, name)
    bad = scenarios.compare(ref, got)
    assert bad == [], "\n".join(bad)


def test_gpu_stepwise_equals_one_call(oracle_path):
    """gs_step(1) x K and gs_step(K) produce identical state."""
    e1, hops = scenarios.SCENARIOS["gossipsub_scored"](PRODUCT_LIB)
    for _ in range(hops):
        e1.step(1)
    e2, _ = scenarios.SCENARIOS["gossipsub_scored"](PRODUCT_LIB)
    e2.step(hops)
    ids = range(e1.counters()["published"])
    assert scenarios.compare(scenarios.snapshot(e1, ids), scenarios.snapshot(e2, ids)) == []


def _retuned(lib):
    """Topic.SetScoreParams mid-run (score.go:192-232): topic 1 gets lower
    first/mesh delivery caps (the recap clamps existing counters) and new
    weights; topic 2, unscored so far, becomes scored."""
    from pubsub_amd import eth2_topic_score_params
    e, hops = scenarios.SCENARIOS["gossipsub_multitopic"](lib)
    e.step(hops // 2)
    p = eth2_topic_score_params()
    p.FirstMessageDeliveriesCap = 3.0
    p.MeshMessageDeliveriesCap = 4.0
    p.MeshMessageDeliveriesThreshold = 2.0
    p.TopicWeight = 0.5
    e.set_topic_score_params(1, p)
    e.step(3)
    q = eth2_topic_score_params()
    q.TimeInMeshWeight = 0.01
    e.set_topic_score_params(2, q)
    e.step(hops - hops // 2)
    return scenarios.snapshot(e, range(e.n_published))


def test_gpu_set_topic_score_params_matches_oracle(oracle_path):
    bad = scenarios.compare(_retuned(oracle_path), _retuned(PRODUCT_LIB))
    assert bad == [], "\n".join(bad)


def _scored_with_pool_cap(lib, cap, monkeypatch):
    monkeypatch.setenv("GS_DEBUG_POOL_SUB_CAP", str(cap))
    try:
        e, hops = scenarios.SCENARIOS["gossipsub_scored"](lib)
        e.step(hops)
        return scenarios.snapshot(e, range(e.n_published))
    finally:
        monkeypatch.delenv("GS_DEBUG_POOL_SUB_CAP")


def test_gpu_pool_sub_arena_spill(oracle_path, monkeypatch):
    """pool_take (gs_device.h): when a node's sub-arena of the IWANT arena is
    full the allocation spills into the next sub-arena before E_POOL (ADVICE
    r4).  GS_DEBUG_POOL_SUB_CAP caps the 16 sub-arenas of an unpartitioned
    engine and makes every node try sub-arena 0 first: at 256 ids each (4096
    per hop; gossipsub_scored peaks at about 700 request and served ids per
    hop) every busy hop fills sub-arena 0 and spills, and the run still equals
    the oracle; at 4 ids each the hop's ids do not fit at all and the engine
    reports the arena overflow."""
    from pubsub_amd import GossipEngineError, _abi
    ref = scenarios.run(oracle_path, "gossipsub_scored")
    got = _scored_with_pool_cap(PRODUCT_LIB, 256, monkeypatch)
    bad = scenarios.compare(ref, got)
    assert bad == [], "\n".join(bad)
    with pytest.raises(GossipEngineError) as ei:
        _scored_with_pool_cap(PRODUCT_LIB, 4, monkeypatch)
    assert ei.value.code == _abi.GS_ECAPACITY and "arena" in str(ei.value)
