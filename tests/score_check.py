"""score() of sampled edges recomputed by the oracle's own PeerScore object
from an engine's state (SURVEY.md §8 a21 at sizes the oracle cannot simulate).

The engine's per-(edge, topic) counters of each sampled edge are injected
into one oracle peerScore record (ops_set_stats, ops_set_behaviour_penalty,
ops_set_app_score), and PeerScore::score (oracle_core.hpp, restating
score.go:256-333) recomputes the score.  With peer IPs (`ipv4`, per node),
each sampled edge gets its own record set: every connected peer of the
observer is added with its IP (setIPs, score.go:1011-1049), so P6
(ipColocationFactor, score.go:335-379) counts the observer's peers per IP as
the reference does; without IPs P6 is 0 on both sides."""
import ctypes as C

import numpy as np


def oracle_scores(olib, sp, eng, edges, app=None, ipv4=None):
    """(recomputed, stats): the oracle's score() of every edge in `edges` from
    eng's topic counters (gs_read_topic_stats_edges) and behaviour penalties."""
    edges = np.asarray(edges, dtype=np.int64)
    st = eng.topic_stats_at(edges)
    bp = eng.behaviour_penalty()[edges]
    col = eng.col[edges]
    if ipv4 is not None:
        return _oracle_scores_ip(olib, sp, eng, edges, st, bp, app, np.asarray(ipv4, dtype=np.uint32)), st
    ps = olib.ops_new(C.byref(sp.to_c()))
    try:
        for t, tp in sp.Topics.items():
            olib.ops_set_topic(ps, int(t), C.byref(tp.to_c()))
        out = np.empty(len(edges))
        for i in range(len(edges)):
            olib.ops_add_peer(ps, i)
            olib.ops_set_app_score(ps, i, 0.0 if app is None else float(app[col[i]]))
            for t in sp.Topics:
                olib.ops_set_stats(ps, i, int(t), int(st["flags"][i, t]), int(st["graft_time"][i, t]),
                                   int(st["mesh_time"][i, t]), float(st["fmd"][i, t]), float(st["mmd"][i, t]),
                                   float(st["mfp"][i, t]), float(st["imd"][i, t]))
            olib.ops_set_behaviour_penalty(ps, i, float(bp[i]))
            out[i] = olib.ops_score(ps, i)
    finally:
        olib.ops_free(ps)
    return out, st


def sample_edges(E, n, seed, must=()):
    rng = np.random.default_rng(seed)
    pick = np.unique(np.concatenate([rng.integers(0, E, n), np.asarray(must, dtype=np.int64)]))
    return pick.astype(np.int64)


def _oracle_scores_ip(olib, sp, eng, edges, st, bp, app, ipv4):
    """One oracle record set per sampled edge e (observer u = the CSR row of e):
    u's peers as records 0..deg-1 with their IPs, e's counters on its own."""
    out = np.empty(len(edges))
    rows = np.searchsorted(eng.rowptr, edges, side="right") - 1
    for i, e in enumerate(edges):
        u = int(rows[i])
        b, f = int(eng.rowptr[u]), int(eng.rowptr[u + 1])
        ps = olib.ops_new(C.byref(sp.to_c()))
        try:
            for t, tp in sp.Topics.items():
                olib.ops_set_topic(ps, int(t), C.byref(tp.to_c()))
            for j in range(f - b):
                olib.ops_add_peer(ps, j)
                ip = int(ipv4[eng.col[b + j]])
                if ip:
                    a = (C.c_uint32 * 1)(ip)
                    olib.ops_set_ips(ps, j, 1, a)
            k = int(e) - b
            olib.ops_set_app_score(ps, k, 0.0 if app is None else float(app[eng.col[e]]))
            for t in sp.Topics:
                olib.ops_set_stats(ps, k, int(t), int(st["flags"][i, t]), int(st["graft_time"][i, t]),
                                   int(st["mesh_time"][i, t]), float(st["fmd"][i, t]), float(st["mmd"][i, t]),
                                   float(st["mfp"][i, t]), float(st["imd"][i, t]))
            olib.ops_set_behaviour_penalty(ps, k, float(bp[i]))
            out[i] = olib.ops_score(ps, k)
        finally:
            olib.ops_free(ps)
    return out
