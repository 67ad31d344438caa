"""Golden vectors (tests/golden/scenarios.json, made by make_golden.py): the
oracle on CPU and the HIP engine on the GPU must both reproduce every counter
and every readback digest of every parity scenario."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import scenarios  # noqa: E402
from make_golden import digest  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "golden", "scenarios.json")))


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_oracle_reproduces_golden(oracle_path, name):
    assert digest(scenarios.run(oracle_path, name)) == GOLDEN[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_gpu_reproduces_golden(name):
    from pubsub_amd import PRODUCT_LIB
    assert digest(scenarios.run(PRODUCT_LIB, name)) == GOLDEN[name]


# Races show up as run-to-run differences before they show up as a wrong
# digest: the scenarios with the most cross-lane LDS and global atomics in
# phase B (IWANT serving, IHAVE handling, spam, cuts) run three more times.
RACE_PRONE = ["gossipsub_dense_dhi", "c5shape", "adversarial_mix", "spam_ihave_2t", "churn_graft"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in RACE_PRONE if n in GOLDEN])
def test_gpu_golden_repeatable(name):
    from pubsub_amd import PRODUCT_LIB
    for _ in range(3):
        assert digest(scenarios.run(PRODUCT_LIB, name)) == GOLDEN[name]


# mcache.peertx spills (mcache.go:66-80 keeps an unbounded map): with 4 slots
# per node, every node that serves more than 4 (message, requester) IWANT
# entries within its cache window takes the rest in the rank's overflow table
# (gs_set_peertx_capacity); the heartbeat's rebuild moves survivors back when
# a node's own table has room.  The goldens must not move.
PEERTX_SPILL = ["c3shape", "adversarial_mix", "gossipsub_slot_reuse", "churn_scored", "c4shape", "px_adversarial"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in PEERTX_SPILL if n in GOLDEN])
def test_gpu_peertx_overflow_reproduces_golden(name):
    from pubsub_amd import PRODUCT_LIB, WithPeertxCapacity
    # (2^20 overflow entries: c3shape alone spills more than the default 2^16)
    assert digest(scenarios.run(PRODUCT_LIB, name, extra=(WithPeertxCapacity(2, 20),))) == GOLDEN[name]


@pytest.mark.gpu
def test_gpu_peertx_overflow_full_is_capacity_error():
    """An overflow table too small for the live entries is GS_ECAPACITY, not a
    silent miscount."""
    from pubsub_amd import PRODUCT_LIB, GossipEngineError, WithPeertxCapacity, _abi
    with pytest.raises(GossipEngineError) as ei:
        scenarios.run(PRODUCT_LIB, "c3shape", extra=(WithPeertxCapacity(2, 8),))
    assert ei.value.code == _abi.GS_ECAPACITY and "overflow table" in str(ei.value)
