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
