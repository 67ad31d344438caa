"""The gs_transport implementation of a partitioned engine (pubsub_amd.
transport) on CPU: world-size 2 and 3 gloo groups drive the three callbacks
through their C function pointers exactly as the engine's exchange does
(gossip_engine.h), on host buffers, and check the collective semantics:
all-gather of sizes, equal-chunk all-gather, and all-to-all-v with uneven and
empty blocks."""
import ctypes as C
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _blk(src, dst, n):
    """Bytes rank `src` sends to rank `dst` (n of them)."""
    return (np.arange(n, dtype=np.int64) * 7 + 31 * src + 5 * dst).astype(np.uint8)


def _splits(src, world):
    return [(3 * src + 2 * d + 1) % 5 * 8 for d in range(world)]  # uneven, some empty


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "go-libp2p-pubsub_amd"))
        import torch.distributed as dist

        from pubsub_amd import _abi
        from pubsub_amd.transport import TorchTransport
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        tr = TorchTransport(memory="host")
        c = tr.c
        bad = []
        # allgather_i64
        mine = np.array([rank * 10 + i for i in range(4)], dtype=np.int64)
        out = np.zeros(4 * world, dtype=np.int64)
        rc = c.allgather_i64(None, mine.ctypes.data_as(C.POINTER(C.c_int64)), 4,
                             out.ctypes.data_as(C.POINTER(C.c_int64)))
        want = np.array([r * 10 + i for r in range(world) for i in range(4)], dtype=np.int64)
        if rc != 0 or not np.array_equal(out, want):
            bad.append(f"allgather_i64 {rc} {out}")
        # allgather of equal chunks
        chunk = 24
        send = (np.arange(chunk) + 100 * rank).astype(np.uint8)
        recv = np.zeros(chunk * world, dtype=np.uint8)
        rc = c.allgather(None, send.ctypes.data, recv.ctypes.data, chunk)
        want = np.concatenate([(np.arange(chunk) + 100 * r).astype(np.uint8) for r in range(world)])
        if rc != 0 or not np.array_equal(recv, want):
            bad.append("allgather")
        # alltoallv with uneven / empty blocks
        sb = np.array(_splits(rank, world), dtype=np.int64)
        rb = np.array([_splits(s, world)[rank] for s in range(world)], dtype=np.int64)
        send = np.concatenate([_blk(rank, d, int(sb[d])) for d in range(world)] + [np.zeros(0, np.uint8)])
        recv = np.zeros(max(int(rb.sum()), 1), dtype=np.uint8)
        rc = c.alltoallv(None, send.ctypes.data if send.size else None, sb.ctypes.data_as(C.POINTER(C.c_int64)),
                         recv.ctypes.data, rb.ctypes.data_as(C.POINTER(C.c_int64)))
        want = np.concatenate([_blk(s, rank, int(rb[s])) for s in range(world)] + [np.zeros(0, np.uint8)])
        if rc != 0 or not np.array_equal(recv[:int(rb.sum())], want):
            bad.append(f"alltoallv {rc}")
        # a failing collective returns nonzero instead of unwinding into C
        rc = c.allgather(None, send.ctypes.data, None, -1)
        if rc == 0:
            bad.append("bad arguments did not report failure")
        if tr.calls != 3:
            bad.append(f"calls {tr.calls}")
        q.put((rank, bad))
        dist.destroy_process_group()
    except Exception as ex:
        import traceback
        q.put((rank, [f"{ex!r}\n{traceback.format_exc()}"]))


@pytest.mark.parametrize("world", [2, 3])
def test_transport_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=120) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    bad = [f"rank {r}: {m}" for r, ms in res for m in ms]
    assert not bad, "\n".join(bad)


def test_partition_entry_points_on_oracle(oracle_path):
    """The oracle simulates the whole graph: world 1 only, full range."""
    from pubsub_amd import NewFloodSub, graphs
    from pubsub_amd import _abi
    g = graphs.dense_connect(10, 1)
    e = NewFloodSub(10, 1, g, graphs.all_subscribed(10, 1), lib=oracle_path)
    assert e.node_range == (0, 10) and e.edge_range == (0, e.E)
    assert e.lib.gs_set_partition(e.h, 0, 2, None) == _abi.GS_EUNSUPPORTED
    assert e.exchange_stats() == (0.0, 0)
