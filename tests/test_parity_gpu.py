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
