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


def test_injected_state_with_ips_reproduces_oracle_scores(oracle_path, olib):
    """The config-5 variant (shared Sybil IPs: P6, invalid messages: P4,
    broken promises and GRAFT spam: P7) on bench.build_engine's own workload at
    1,500 peers past hop 50: the per-edge record sets of the IP-aware check give
    back the simulator's scores bit for bit."""
    import bench
    wl = dict(bench.WORKLOADS["config5"], n=1500)
    e, _ = bench.build_engine(wl, 6, 3, 0, lib=oracle_path)
    e.step(1 + 6 * bench.HOPS_PER_ROUND)
    bp = e.behaviour_penalty()
    pen = np.flatnonzero(bp > 0)
    assert len(pen) > 0
    edges = np.unique(np.concatenate([sample_edges(e.E, 300, 1, must=[0, e.E - 1]), pen[:200]]))
    got, st = oracle_scores(olib, e.score_params, e, edges, ipv4=e.ipv4)
    want = e.scores()[edges]
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    assert (st["imd"] > 0).any()


def test_injected_state_with_dense_ips(oracle_path, olib):
    """P6 itself: 200 peers of degree 20 over 2 IPs, so most observers see more
    than IPColocationFactorThreshold (10) peers of one IP; without the IPs the
    recomputed scores differ, with them they are the simulator's bit for bit."""
    e, _ = scenarios.gossipsub_scored(oracle_path, n=200, ip_groups=2, seed=9, app_neg_frac=0.1)
    e.step(60)
    edges = sample_edges(e.E, 300, 1, must=[0, e.E - 1])
    got, _ = oracle_scores(olib, e.score_params, e, edges, app=e.app_attr, ipv4=e.ipv4_attr)
    want = e.scores()[edges]
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    plain, _ = oracle_scores(olib, e.score_params, e, edges, app=e.app_attr)
    assert not np.array_equal(plain.view(np.uint64), want.view(np.uint64))
