"""Phase A's two ways of reading what the senders forwarded give the same
simulation (gs_set_frontier_mode): the frontier bitmaps (k_flood_a for
floodsub, k_phase_a's dense pass 1 for one-topic gossipsub)
and the per-copy lists.  Each scenario runs both ways on the GPU; both must
reproduce the oracle-made golden digest (tests/golden/scenarios.json), and the
bitmap run must have taken the bitmap path where the engine supports it.

Reference: FloodSubRouter.Publish floodsub.go:76-100, GossipSubRouter.Publish
gossipsub.go:939-1009 (mesh peers, flood publish, ReceivedFrom and author
exclusion), pushMsg pubsub.go:978-1022."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import scenarios  # noqa: E402
from make_golden import digest  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "golden", "scenarios.json")))

# one-topic gossipsub shapes the dense pass 1 covers (scored, flood publish,
# graylisting + direct peers, Dhi pruning, slot recycling, config3's shape) and
# floodsub; the adversarial / churn / PX / multi-topic ones use the lists
DENSE = ["gossipsub_dense", "gossipsub_scored", "gossipsub_flood_publish", "gossipsub_negative_app",
         "gossipsub_dense_dhi", "gossipsub_slot_reuse", "gossipsub_graylist_direct", "c3shape", "floodsub_dense"]
LISTS_ONLY = ["gossipsub_multitopic", "adversarial_mix", "churn_scored"]


def _run(name, extra=()):
    from pubsub_amd import PRODUCT_LIB
    e, hops = scenarios.SCENARIOS[name](PRODUCT_LIB, extra)
    e.step(hops)
    snap = scenarios.snapshot(e, getattr(e, "snapshot_ids", range(e.n_published)))
    snap["node_range"], snap["edge_range"] = e.node_range, e.edge_range
    return e.frontier_dense, snap


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in DENSE if n in GOLDEN])
def test_gpu_dense_and_lists_reproduce_golden(name):
    from pubsub_amd import WithFrontierBitmaps, WithFrontierLists
    dense, snap = _run(name, (WithFrontierBitmaps(),))
    assert dense, f"{name}: expected the frontier-bitmap path"
    assert digest(snap) == GOLDEN[name]
    dense, snap = _run(name, (WithFrontierLists(),))
    assert not dense
    assert digest(snap) == GOLDEN[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in LISTS_ONLY if n in GOLDEN])
def test_gpu_lists_where_bitmaps_do_not_apply(name):
    from pubsub_amd import WithFrontierBitmaps
    dense, snap = _run(name, (WithFrontierBitmaps(),))
    assert not dense
    assert digest(snap) == GOLDEN[name]
