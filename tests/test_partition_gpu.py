"""Partitioned engine (one rank per node range) against the
oracle.  `world` processes share the one GPU of the test box and exchange their
per-hop RPCs through the gloo transport (host-staged); every rank checks the
part of the state it owns — its nodes' first-delivery hops and first senders,
its edges' mesh / fanout / backoff / score counters / scores — bit-exactly
against the unpartitioned oracle, and the summed event counters against the
oracle's.  On the 8-GPU node the same engine code runs with the RCCL ("nccl")
transport (bench.py --gpus N)."""
import multiprocessing as mp
import os
import socket
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


TRACED = [0, 3, 17, 42, 99, 150]


def _worker(rank, world, port, name, oracle, q):
    try:
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
        import numpy as np
        import torch
        import torch.distributed as dist

        import scenarios
        from pubsub_amd import PRODUCT_LIB, WithPartition
        from pubsub_amd.transport import TorchTransport
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from pubsub_amd import WithEventTracer
        tr = TorchTransport(memory="device")
        traced = [0, 1] if name.startswith("spam_") else [u for u in TRACED if u < 20]  # spam pairs: 2 nodes
        e, hops = scenarios.SCENARIOS[name](PRODUCT_LIB, (WithPartition(rank, world, tr), WithEventTracer(traced)))
        e.step(hops)
        ids = getattr(e, "snapshot_ids", range(e.n_published))  # (slots not recycled yet)
        got = scenarios.snapshot(e, ids)
        got["node_range"], got["edge_range"] = e.node_range, e.edge_range
        ev = e.trace_events()
        eo, _ = scenarios.SCENARIOS[name](oracle, (WithEventTracer(traced),))
        eo.step(hops)
        ref = scenarios.snapshot(eo, ids)
        evo = eo.trace_events()
        T = got["ts_fmd"].shape[0]
        ref_part = dict(ref, node_range=got["node_range"], edge_range=got["edge_range"])
        bad = scenarios.compare(scenarios.restrict(ref_part, T), scenarios.restrict(got, T))
        keys = sorted(k for k in ref["counters"] if k not in ("hops", "heartbeats"))
        mine = torch.tensor([got["counters"][k] for k in keys], dtype=torch.int64)
        dist.all_reduce(mine)
        summed = dict(zip(keys, mine.tolist()))
        want = {k: ref["counters"][k] for k in keys}
        if summed != want:
            bad.append(f"summed counters {summed} != oracle {want}")
        # trace events: this rank records its own traced hosts only
        n0, n1 = got["node_range"]
        want_ev = evo[(evo["node"] >= n0) & (evo["node"] < n1)]
        if len(ev) != len(want_ev) or (len(ev) and not np.array_equal(ev, want_ev)):
            bad.append(f"trace events differ: {len(ev)} vs {len(want_ev)}")
        if tr.calls == 0:
            bad.append("the transport was never called")
        q.put((rank, bad, got["node_range"]))
        dist.destroy_process_group()
    except Exception as ex:  # report instead of hanging the parent
        import traceback
        q.put((rank, [f"worker raised: {ex!r}\n{traceback.format_exc()}"], None))


def run_partitioned(world, name, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, oracle, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=240))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return sorted(res, key=lambda r: r[0])


@pytest.mark.gpu
@pytest.mark.parametrize("world,name", [
    (2, "gossipsub_scored"),
    (2, "floodsub_dense"),
    (2, "gossipsub_dense"),
    (3, "gossipsub_multitopic"),
    (2, "gossipsub_negative_app"),
    (3, "gossipsub_dense_dhi"),
    (2, "gossipsub_flood_publish"),
    # the adversarial model across ranks: IWANT-spam re-request lists, served
    # replies, GRAFT / IHAVE spam, the gater and the validation queue
    (2, "spam_iwant"),
    (2, "adversarial_mix"),
    (3, "adversarial_mix_nogater"),
    # per-edge RPC byte accounting, counted by the sender's rank
    (2, "acct_floodsub"),
    (3, "acct_multitopic"),
    (2, "acct_adversarial"),
    # connection churn and subscription changes: each rank takes its side of
    # every connection event and its own nodes' leaves / joins
    (2, "churn_remove_peer"),
    (2, "churn_prune"),
    (3, "churn_graft"),
    (2, "churn_scored"),
    (3, "acct_churn"),
    # a mixed network (TestMixedGossipsub): floodsub hosts beside gossipsub ones
    (2, "mixed_gossip_flood"),
    # the peer gater's AddPeer / RemovePeer / RetainStats under churn
    (2, "churn_gater"),
    # peer exchange and the direct-peer connector: PX lists travel in the edge
    # records and arena, dials are gathered from every rank
    (2, "px_scored"),
    (3, "px_star"),
    (2, "direct_churn"),
    (2, "px_gater"),
    # PX under RPC byte accounting: PRUNE sizes with their PeerInfo entries
    (2, "acct_px_scored"),
    (3, "acct_px_adversarial"),
    # T >= 4: k_push's segments of cross-rank edges travel in the exchange and
    # the receivers read them as local ones (gs_exchange.h k_xp_*); a sender
    # whose region overflows sends -1 records (its receivers walk its list)
    (2, "c4shape"),
    (3, "cut_honest_4t"),
    (2, "push_overflow"),
    # MaxIHaveLength cuts past GS_CUTS per node: each rank's own cut table
    (2, "cut_spill_16t"),
    # the promise table past 512 entries on the rank owning the star's centre
    (2, "promise_flood_long"),
    # randomsub: a sender's per-message target masks (d.sel) travel with its
    # frontier list entries (gs_exchange.h k_x_sel); at T >= 4 k_push applies
    # them on the sender's rank
    (3, "randomsub_100"),
    (2, "randomsub_N"),
    (2, "mixed_randomsub"),
    (3, "mixed_scored_4t"),
])
def test_partitioned_engine_matches_oracle(world, name, oracle_path):
    res = run_partitioned(world, name, oracle_path)
    ranges = [r[2] for r in res]
    assert all(r is not None for r in ranges), res
    assert ranges[0][0] == 0 and all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    bad = [f"rank {r}: {m}" for r, ms, _ in res for m in ms]
    assert not bad, "\n".join(bad)


def _err_worker(rank, world, port, q):
    """Rank 0 traces node 0 with a 16-event buffer, so its device error word
    gets E_TRACE within a few hops; rank 1 has no device error of its own."""
    try:
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
        import torch
        import torch.distributed as dist

        import scenarios
        from pubsub_amd import PRODUCT_LIB, GossipEngineError, WithEventTracer, WithPartition, _abi
        from pubsub_amd.transport import TorchTransport
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tr = TorchTransport(memory="device")
        e, hops = scenarios.SCENARIOS["gossipsub_scored"](
            PRODUCT_LIB, (WithPartition(rank, world, tr), WithEventTracer([0], capacity=16)))
        try:
            e.step(hops)
            q.put((rank, None, e.hop))
        except GossipEngineError as ex:
            q.put((rank, (ex.code, str(ex)), e.hop))
        dist.destroy_process_group()
        del _abi
    except Exception as ex:  # report instead of hanging the parent
        import traceback
        q.put((rank, ("raised", f"{ex!r}\n{traceback.format_exc()}"), -1))


@pytest.mark.gpu
def test_partitioned_device_error_stops_every_rank():
    """A device error on one rank: every rank returns it at the
    same hop instead of the healthy ranks waiting in the next exchange."""
    from pubsub_amd import _abi
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_err_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(r[1] is not None for r in res), res
    assert all(r[1][0] == _abi.GS_ECAPACITY for r in res), res
    assert res[0][2] == res[1][2], res            # both stopped at the same hop
    assert "rank 0" in res[1][1][1], res          # rank 1 names the failing rank


def _rpc_worker(rank, world, port, name, q):
    """RPC trace events on a partitioned engine: this rank's stream."""
    try:
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
        import torch
        import torch.distributed as dist

        import scenarios
        from pubsub_amd import PRODUCT_LIB, WithEventTracer, WithPartition
        from pubsub_amd.transport import TorchTransport
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tr = TorchTransport(memory="device")
        e, hops = scenarios.SCENARIOS[name](PRODUCT_LIB, (WithPartition(rank, world, tr),
                                                          WithEventTracer(TRACED, rpc=True)))
        e.step(hops)
        q.put((rank, e.trace_events().tobytes(), e.node_range))
        dist.destroy_process_group()
    except Exception as ex:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, f"worker raised: {ex!r}\n{traceback.format_exc()}"))


@pytest.mark.gpu
@pytest.mark.parametrize("world,name", [(2, "gossipsub_scored"), (3, "churn_scored"), (2, "adversarial_mix")])
def test_partitioned_rpc_trace_union_equals_oracle(world, name, oracle_path):
    """gs_set_trace_rpc on a partitioned engine: each rank records the RPCs its
    hosts send (SEND_RPC of its traced hosts, RECV_RPC of any traced receiver)
    and its hosts' own events; the union of the ranks' streams is the oracle's
    stream event for event (compared as multisets: one canonical order per
    rank), and every non-RPC event sits on the rank owning its host."""
    import numpy as np

    import scenarios
    from pubsub_amd import WithEventTracer, _abi
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rpc_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(r[1] is not None for r in res), [r[2] for r in res]
    eo, hops = scenarios.SCENARIOS[name](oracle_path, (WithEventTracer(TRACED, rpc=True),))
    eo.step(hops)
    want = eo.trace_events()
    streams = [np.frombuffer(r[1], dtype=_abi.TRACE_EVENT_DTYPE) for r in res]
    for (rank, _, (n0, n1)), ev in zip(res, streams):
        plain = ev[(ev["type"] != _abi.TRACE_TYPES.index("RECV_RPC")) & (ev["type"] != 32)]
        assert ((plain["node"] >= n0) & (plain["node"] < n1)).all(), rank
    got = np.concatenate(streams)
    assert (got["type"] == _abi.TRACE_TYPES.index("RECV_RPC")).any() and len(got) == len(want)
    key = lambda a: np.sort(a.view(np.dtype((np.void, a.dtype.itemsize))))  # noqa: E731
    assert np.array_equal(key(got), key(want))
