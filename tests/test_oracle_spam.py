"""The reference's attack tests restated on the oracle simulator
(gossipsub_spam_test.go, gossipsub_test.go:1388-1469 and 1665-1779).  Each
test keeps the reference test's own assertions; the scenarios live in
tests/scenarios.py (ADVERSARIAL) and are also GPU parity cases."""
import numpy as np

import scenarios
from pubsub_amd import _abi

GR = 3                  # GossipSubGossipRetransmission (gossipsub.go:37)
MAX_IHAVE_LENGTH = 5000  # GossipSubMaxIHaveLength (gossipsub.go:51)
HB = 10                 # hops per heartbeat (100 ms hops, 1 s heartbeat)


def test_iwant_spam_gets_one_plus_retransmissions(oracle_path):
    """gossipsub_spam_test.go:63-71: after the original message the attacker
    keeps sending IWANT; it gets exactly 1 + GossipRetransmission copies."""
    e, hops = scenarios.spam_iwant(oracle_path)
    e.step(hops)
    c = e.counters()
    assert c["transmissions"] == 1 + GR
    assert c["iwant_served"] == GR
    assert c["deliveries"] == 1 and c["duplicates"] == GR


def _per_heartbeat(e, hops, key):
    out, last = [], e.counters()[key]
    for h in range(hops):
        e.step(1)
        if (h - 1) % HB == 0:  # heartbeats at hops 1, 11, 21, ...
            cur = e.counters()[key]
            out.append(cur - last)
            last = cur
    return out


def test_ihave_spam_iwant_bound_and_broken_promises(oracle_path):
    """gossipsub_spam_test.go:207-258: at most MaxIHaveLength IWANT ids per
    heartbeat, more after the next heartbeat, score 0 until the promises
    expire (IWantFollowupTime), negative after."""
    e, hops = scenarios.spam_ihave(oracle_path)
    first = None
    scores = []
    iw = []
    last = 0
    for h in range(hops):
        e.step(1)
        c = e.counters()
        if c["iwant_sent"] > last and first is None:
            first = h
        iw.append(c["iwant_sent"] - last)
        last = c["iwant_sent"]
        scores.append(e.scores()[0])  # host 0's score of the attacker
    per_hb = [sum(iw[i:i + HB]) for i in range(0, len(iw), HB)]
    assert max(per_hb) <= MAX_IHAVE_LENGTH and max(per_hb) == MAX_IHAVE_LENGTH
    assert sum(1 for x in per_hb if x) >= 2           # more IWANTs after the next heartbeat
    follow = 30                                       # IWantFollowupTime = 3 s = 30 hops
    assert all(s == 0 for s in scores[:first + follow])
    assert scores[-1] < 0
    assert e.counters()["promises_broken"] >= 1


def test_ihave_spam_iwant_cut_across_topics(oracle_path):
    """handleIHave's cut (gossipsub.go:650-653): one IHAVE with two 4000-id
    topics asks for MaxIHaveLength ids, not 8000."""
    e, hops = scenarios.SCENARIOS["spam_ihave_2t"](oracle_path)
    per_hb = _per_heartbeat(e, hops, "iwant_sent")
    assert max(per_hb) == MAX_IHAVE_LENGTH


def test_graft_during_backoff(oracle_path):
    """gossipsub_spam_test.go:424-535: a GRAFT during the backoff is penalised
    (P7) and answered with a PRUNE, the score drops with every such GRAFT, and
    once below GraylistThreshold the GRAFTs are ignored; the attacker never
    gets back into the mesh."""
    e, hops = scenarios.spam_graft(oracle_path)
    prunes, scores, gray = [], [], []
    for h in range(hops):
        e.step(1)
        c = e.counters()
        prunes.append(c["prunes_sent"])
        gray.append(c["graylisted"])
        scores.append(e.scores()[0])
        if h >= 2:
            assert e.mesh()[0] == 0  # host 0's mesh never holds the attacker again
    assert prunes[2] == 1 and scores[2] == 0          # the attacker's own PRUNE; no penalty yet
    # every answered GRAFT lowers the score; the first one already makes it negative
    answered = [h for h in range(3, hops) if prunes[h] > prunes[h - 1]]
    assert len(answered) >= 2
    s_after = [scores[h] for h in answered]
    assert s_after[0] < 0 and s_after[1] < s_after[0]
    assert min(scores) < -1000                        # below the graylist threshold
    # while graylisted, GRAFTs are dropped and not answered
    for h in range(1, hops):
        if scores[h - 1] < -1000 and gray[h] > gray[h - 1]:
            assert prunes[h] == prunes[h - 1]
    assert gray[-1] > 0


def test_invalid_message_spam(oracle_path):
    """gossipsub_spam_test.go:656-690: invalid messages give the attacker a
    negative score (P4), every one is traced as REJECT_MESSAGE, and the
    attacker is pruned."""
    from pubsub_amd import WithEventTracer
    e, hops = scenarios.spam_invalid(oracle_path, extra=(WithEventTracer([0]),))
    e.step(hops)
    c = e.counters()
    ev = e.trace_events()
    rej = ev[ev["type"] == _abi.TRACE_TYPES.index("REJECT_MESSAGE")]
    assert c["rejected"] > 0 and len(rej) == c["rejected"]
    assert all(_abi.REJECT_REASONS[r] == "validation failed" for r in rej["reason"])
    assert e.scores()[0] < 0
    assert e.mesh()[0] == 0
    st = e.topic_stats()
    assert st["imd"][0, 0] > 0


def test_opportunistic_grafting_with_squatters(oracle_path):
    """gossipsub_test.go:1759-1778: with 40 sybil squatters connected to every
    honest host, opportunistic grafting leaves >= 3 honest peers in every
    honest host's mesh."""
    e, hops = scenarios.squatters(oracle_path)
    e.step(hops)
    m = e.mesh()
    for u in range(e.honest):
        nb = e.col[e.rowptr[u]:e.rowptr[u + 1]]
        mm = m[e.rowptr[u]:e.rowptr[u + 1]] & np.uint64(1)
        assert int(((nb < e.honest) & (mm != 0)).sum()) >= 3, u


def test_negative_score_sinkhole(oracle_path):
    """gossipsub_test.go:1436-1468: the sinkholed host receives only its own
    message and nobody receives a message from it."""
    e, hops = scenarios.sinkhole(oracle_path)
    e.step(hops)
    for i in range(20):
        hop, frm = e.deliveries(i)
        assert (frm != 0).all()                         # no first delivery from host 0
        assert (hop[0] >= 0) == (i == 0)               # host 0 only has its own message


def test_gater_throttles_under_validation_overload(oracle_path):
    """peer_gater.go:320-363: a validation queue that overflows (RejectValidation-
    QueueFull) turns the gater on, which then drops payload RPCs (AcceptControl)
    and throttles promises; without the gater nothing is gated."""
    e, hops = scenarios.adversarial_mix(oracle_path)
    e.step(hops)
    c = e.counters()
    assert c["throttled"] > 0 and c["gated"] > 0 and c["rejected"] > 0
    assert c["promises_broken"] > 0 and c["graylisted"] > 0
    e2, hops2 = scenarios.SCENARIOS["adversarial_mix_nogater"](oracle_path)
    e2.step(hops2)
    assert e2.counters()["gated"] == 0 and e2.counters()["throttled"] == 0
