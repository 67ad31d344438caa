"""Per-host replay of a simulation run (test infrastructure only).

A host's router and score state is a function of what it receives, what it
publishes and the static inputs every host shares (graph, subscriptions,
peer attributes, the publish schedule).  Its EventTracer stream with RPC
tracing (trace.go:241-383: RecvRPC / SendRPC with their RPCMeta) holds
everything it receives.  The oracle's gs_oracle_replay_* entry points
(oracle/oracle_sim.cpp, struct Replay) rebuild one host from that stream:
they parse its RecvRPC blocks back into RPCs and run, hop by hop, the same
per-host phase bodies the full oracle simulation runs (memo, payload,
control, refreshScores, heartbeat).  The replayed host's own events
(Deliver / Duplicate / Graft / Prune / Join / Publish, every SendRPC with its
items) and its final mesh, fanout, backoff, peer-score counters and scores
must equal what the run under test recorded for that host.

The full-size GPU tests (tests/test_fullsize_gpu.py) replay sampled hosts of
the 1M-peer runs from the engine's own trace; tests/test_oracle_replay.py pins
the replay itself against full oracle runs on CPU."""
import ctypes as C

import numpy as np

from pubsub_amd import _abi

_BOUND = set()


def _bind(lib):
    if id(lib) in _BOUND:
        return
    P, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    lib.gs_oracle_replay_new.argtypes = [P, i32, C.POINTER(P)]
    lib.gs_oracle_replay_new.restype = C.c_int
    lib.gs_oracle_replay_run.argtypes = [P, i64, P, i64]
    lib.gs_oracle_replay_run.restype = C.c_int
    lib.gs_oracle_replay_events.argtypes = [P, P, i64, C.POINTER(i64)]
    lib.gs_oracle_replay_events.restype = C.c_int
    lib.gs_oracle_replay_state.argtypes = [P] * 13
    lib.gs_oracle_replay_state.restype = C.c_int
    lib.gs_oracle_replay_free.argtypes = [P]
    lib.gs_oracle_replay_free.restype = None
    _BOUND.add(id(lib))


def _ck(lib, rc):
    if rc != 0:
        raise RuntimeError(f"oracle replay error {rc}: {lib.gs_last_error().decode()}")


class HostReplay:
    """One host of `oeng` (an oracle Engine built with the run's exact inputs
    and never stepped) replayed from its trace, hop by hop."""

    def __init__(self, oeng, node):
        self.lib, self.node, self.T = oeng.lib, int(node), oeng.T
        _bind(self.lib)
        self.deg = int(oeng.rowptr[node + 1] - oeng.rowptr[node])
        self.h = C.c_void_p()
        _ck(self.lib, self.lib.gs_oracle_replay_new(oeng.h, self.node, C.byref(self.h)))

    def run(self, hops, events):
        """Replays `hops` hops; `events` holds (at least) the host's RecvRPC
        blocks for them (any other host's events are ignored)."""
        ev = np.ascontiguousarray(events, dtype=_abi.TRACE_EVENT_DTYPE)
        _ck(self.lib, self.lib.gs_oracle_replay_run(self.h, int(hops), ev.ctypes.data, len(ev)))

    def events(self, chunk=1 << 18):
        parts = []
        n = C.c_int64()
        while True:
            buf = np.empty(chunk, dtype=_abi.TRACE_EVENT_DTYPE)
            _ck(self.lib, self.lib.gs_oracle_replay_events(self.h, buf.ctypes.data, chunk, C.byref(n)))
            parts.append(buf[:n.value])
            if n.value < chunk:
                return np.concatenate(parts)

    def state(self):
        d, T = self.deg, self.T
        s = dict(mesh=np.empty(d, np.uint64), fanout=np.empty(d, np.uint64), backoff=np.empty(d * T, np.int64),
                 score=np.empty(d, np.float64), bp=np.empty(d, np.float64), fmd=np.empty(d * T, np.float64),
                 mmd=np.empty(d * T, np.float64), mfp=np.empty(d * T, np.float64), imd=np.empty(d * T, np.float64),
                 mesh_time=np.empty(d * T, np.int64), graft_time=np.empty(d * T, np.int64),
                 flags=np.empty(d * T, np.uint8))
        keys = ["mesh", "fanout", "backoff", "score", "bp", "fmd", "mmd", "mfp", "imd", "mesh_time", "graft_time",
                "flags"]
        _ck(self.lib, self.lib.gs_oracle_replay_state(self.h, *[s[k].ctypes.data for k in keys]))
        for k in ("backoff", "fmd", "mmd", "mfp", "imd", "mesh_time", "graft_time", "flags"):
            s[k] = s[k].reshape(d, T)
        return s

    def close(self):
        if self.h:
            self.lib.gs_oracle_replay_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_events(events, node):
    """The events of one host (an RPC's items carry its host, so blocks stay whole)."""
    return events[events["node"] == node]


def engine_state(e, nodes, scored=True):
    """The run's state for the out-edges of `nodes`, per node, in the layout
    of HostReplay.state() (readbacks through the ABI under test)."""
    rows = [np.arange(e.rowptr[u], e.rowptr[u + 1]) for u in nodes]
    edges = np.concatenate(rows)
    mesh, fanout, bp = e.mesh()[edges], e.fanout()[edges], e.behaviour_penalty()[edges]
    score = e.scores()[edges] if scored else np.zeros(len(edges))
    bo = e.backoff_at(edges)
    st = e.topic_stats_at(edges)
    out, k = {}, 0
    for u, r in zip(nodes, rows):
        sl = slice(k, k + len(r))
        out[int(u)] = dict(mesh=mesh[sl], fanout=fanout[sl], backoff=bo[sl], score=score[sl], bp=bp[sl],
                           **{f: st[f][sl] for f in ("fmd", "mmd", "mfp", "imd", "mesh_time", "graft_time",
                                                     "flags")})
        k += len(r)
    return out


def _fmt(ev):
    return {n: (int(ev[n]) if n != "msg" else int(ev[n])) for n in ev.dtype.names}


def compare_events(got, want, node, limit=3):
    """Mismatch descriptions between two canonical event streams of one host."""
    if len(got) == len(want) and (len(got) == 0 or np.array_equal(got.view(np.uint8), want.view(np.uint8))):
        return []
    n = min(len(got), len(want))
    gb = got[:n].view(np.uint8).reshape(n, -1)
    wb = want[:n].view(np.uint8).reshape(n, -1)
    diff = np.flatnonzero((gb != wb).any(axis=1))
    out = [f"host {node}: {len(got)} replayed events vs {len(want)} recorded"]
    for i in diff[:limit]:
        out.append(f"  event {i}: replay {_fmt(got[i])} recorded {_fmt(want[i])}")
    if not len(diff):
        i = n
        extra = got[i] if len(got) > n else want[i]
        out.append(f"  first extra event {i}: {_fmt(extra)} ({'replay' if len(got) > n else 'recorded'})")
    return out


def compare_state(got, want, node):
    out = []
    for k, w in want.items():
        g = got[k]
        same = np.array_equal(g.view(np.uint64) if g.dtype == np.float64 else g,
                              w.view(np.uint64) if w.dtype == np.float64 else w)
        if not same:
            bad = np.argwhere(np.asarray(g != w) if g.dtype != np.float64 else
                              (g.view(np.uint64) != w.view(np.uint64)))
            out.append(f"host {node} {k}: {len(bad)} entries differ, first {tuple(bad[0])}: "
                       f"replay {g[tuple(bad[0])]!r} run {w[tuple(bad[0])]!r}")
    return out
