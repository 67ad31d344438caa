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
        tr = TorchTransport(memory="device")
        got = scenarios.run(PRODUCT_LIB, name, extra=(WithPartition(rank, world, tr),))
        ref = scenarios.run(oracle, name)
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
])
def test_partitioned_engine_matches_oracle(world, name, oracle_path):
    res = run_partitioned(world, name, oracle_path)
    ranges = [r[2] for r in res]
    assert all(r is not None for r in ranges), res
    assert ranges[0][0] == 0 and all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    bad = [f"rank {r}: {m}" for r, ms, _ in res for m in ms]
    assert not bad, "\n".join(bad)
