"""The full-size score check (tests/score_check.py) pinned on the oracle
itself: the oracle's counters of sampled edges, read with
gs_read_topic_stats_edges and injected into a fresh oracle peerScore, give back
exactly the oracle simulator's own scores (score.go:256-333), and the sampled
readback equals the full one."""
import numpy as np
import pytest

import scenarios
from score_check import oracle_scores, sample_edges


@pytest.mark.parametrize("name", ["gossipsub_scored", "gossipsub_multitopic", "c4shape"])
def test_injected_state_reproduces_oracle_scores(oracle_path, olib, name):
    e, hops = scenarios.SCENARIOS[name](oracle_path)
    e.step(hops)
    edges = sample_edges(e.E, 300, 1, must=[0, e.E - 1])
    sp = e.score_params
    got, st = oracle_scores(olib, sp, e, edges)
    want = e.scores()[edges]
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    full = e.topic_stats()
    for k in ("fmd", "mmd", "mfp", "imd", "mesh_time", "graft_time", "flags"):
        assert np.array_equal(np.asarray(st[k]).T, np.asarray(full[k])[:, edges]), k
    assert (st["flags"] & 1).any()  # the sample holds mesh members


def test_topic_stats_edges_bad_edge(oracle_path):
    from pubsub_amd import GossipEngineError
    e, _ = scenarios.SCENARIOS["gossipsub_dense"](oracle_path)
    e.step(3)
    with pytest.raises(GossipEngineError):
        e.topic_stats_at([e.E])
