"""The per-host replay (tests/replay.py, gs_oracle_replay_*) pinned on the
oracle itself: a full simulation with every host traced (RPC events on), then
sampled hosts replayed alone from their own RecvRPC streams.  Every replayed
host's event stream and final router / score state must equal the full run's.
This is what makes the replay a valid checker for the 1M-peer GPU runs, where
only the sampled hosts can be simulated on the CPU."""
import numpy as np
import pytest

import scenarios
from replay import HostReplay, compare_events, compare_state, engine_state, host_events
from pubsub_amd import WithEventTracer, _abi

CASES = {
    # name: (builder, hosts)
    "gossipsub_scored": (lambda lib, x: scenarios.gossipsub_scored(lib, n=120, msgs=200, hb=10, extra=x), 6),
    "gossipsub_multitopic": (lambda lib, x: scenarios.SCENARIOS["gossipsub_multitopic"](lib, x), 6),
    "gossipsub_negative_app": (lambda lib, x: scenarios.SCENARIOS["gossipsub_negative_app"](lib, x), 6),
    "gossipsub_dense_dhi": (lambda lib, x: scenarios.SCENARIOS["gossipsub_dense_dhi"](lib, x), 6),
    "cut_8t": (lambda lib, x: scenarios.gossipsub_scored(lib, n=120, k=16, topics=8, window=1024, msgs=4000,
                                                          hb=12, seed=71, extra=x), 5),
    "adversarial_mix": (lambda lib, x: scenarios.adversarial_mix(lib, n=200, msgs=300, extra=x), 8),
    "spam_ihave": (lambda lib, x: scenarios.SCENARIOS["spam_ihave"](lib, x), 2),
    "floodsub_dense": (lambda lib, x: scenarios.SCENARIOS["floodsub_dense"](lib, x), 4),
    "randomsub_100": (lambda lib, x: scenarios.SCENARIOS["randomsub_100"](lib, x), 4),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_replay_equals_full_run(oracle_path, name):
    build, nh = CASES[name]
    probe, _ = build(oracle_path, ())
    n = probe.N
    probe.close()
    tr = (WithEventTracer(np.ones(n, bool), capacity=1 << 30, rpc=True),)
    full, hops = build(oracle_path, tr)
    full.step(hops)
    ev = full.trace_events()
    assert (ev["type"] == _abi.TRACE_TYPES.index("RECV_RPC")).any()  # the run recorded its RPCs
    rng = np.random.default_rng(5)
    nodes = np.unique(np.concatenate([[0, n - 1], rng.choice(n, min(n, nh), replace=False)]))
    want_state = engine_state(full, nodes, scored=full.score_params is not None)
    # one never-stepped oracle engine with the same inputs hosts every replay,
    # fed in two parts as the GPU tests feed it round by round
    oeng, _ = build(oracle_path, ())
    reps = {int(u): HostReplay(oeng, int(u)) for u in nodes}
    half = hops // 2
    bad = []
    for part, k in ((ev["hop"] < half, half), (ev["hop"] >= half, hops - half)):
        for u in nodes:
            r = reps[int(u)]
            r.run(k, host_events(ev[part], u))
            bad += compare_events(r.events(), host_events(ev[part], u), u)
    for u in nodes:
        bad += compare_state(reps[int(u)].state(), want_state[int(u)], u)
        reps[int(u)].close()
    oeng.close()
    assert not bad, "\n".join(bad[:20])
