"""Per-rank device footprint of a partitioned engine, measured on ONE GPU.

A partitioned rank allocates its owned nodes' and owned edges' state, the
full-graph CSR and the mirrors it reads across ranks.  This
probe builds rank RANK of WORLD for a bench.py workload at --peers, with a
transport that plays the other ranks as silent (every size they report is 0,
their device chunks are zero: no lists, no arena, no records), steps the warm-up
and prints the device memory the engine holds.  Buffers sized by traffic from
other ranks (the XRec receive buffer, pushed segments behind ibx) are not
exercised; the script prints the matching send-side sizes as their estimate.

    python scripts/mem_probe.py --workload config5 --peers 10000000 --world 8
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-libp2p-pubsub_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from pubsub_amd import WithPartition, _abi  # noqa: E402


class SoloTransport:
    """gs_transport for one rank whose peers never send anything."""

    def __init__(self, rank, world):
        self.rank, self.world, self.calls = rank, world, 0
        self.c = _abi.TransportC()
        self.c.user = None
        self._cb = (_abi.ALLGATHER_I64(self._ag64), _abi.ALLGATHER(self._ag), _abi.ALLTOALLV(self._a2a))
        self.c.allgather_i64, self.c.allgather, self.c.alltoallv = self._cb

    def _ag64(self, _u, mine, n, out):
        o = np.ctypeslib.as_array(out, shape=(self.world * n,))
        o[:] = 0
        o[self.rank * n:(self.rank + 1) * n] = np.ctypeslib.as_array(mine, shape=(n,))
        self.calls += 1
        return 0

    def _dev(self, ptr, nbytes):
        return torch.as_tensor(_Ptr(ptr, nbytes), device="cuda")

    def _ag(self, _u, send, recv, nbytes):
        if nbytes:
            r = self._dev(recv, nbytes * self.world)
            r.zero_()
            r[self.rank * nbytes:(self.rank + 1) * nbytes].copy_(self._dev(send, nbytes))
            torch.cuda.synchronize()
        self.calls += 1
        return 0

    def _a2a(self, _u, send, send_bytes, recv, recv_bytes):
        sb = np.ctypeslib.as_array(send_bytes, shape=(self.world,)).copy()
        rb = np.ctypeslib.as_array(recv_bytes, shape=(self.world,)).copy()
        self.sent = getattr(self, "sent", 0) + int(sb.sum() - sb[self.rank])
        assert rb.sum() == rb[self.rank] == sb[self.rank]
        if rb[self.rank]:
            so = int(sb[:self.rank].sum())
            self._dev(recv, int(rb[self.rank])).copy_(self._dev(send + so, int(sb[self.rank])))
            torch.cuda.synchronize()
        self.calls += 1
        return 0


class _Ptr:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1",
                                         "data": (int(ptr), False), "version": 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config5", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--peers", type=int, default=0)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=3, help="warm-up rounds stepped before the reading")
    args = ap.parse_args()
    wl = dict(bench.WORKLOADS[args.workload])
    if args.peers:
        wl["n"] = args.peers
    tr = SoloTransport(args.rank, args.world)
    t_start = time.perf_counter()

    def tick():  # a progress line while the host builds the graph
        while True:
            time.sleep(30)
            print(f"mem_probe: {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=tick, daemon=True).start()
    free0 = torch.cuda.mem_get_info(0)[0]
    t0 = time.perf_counter()
    eng, g = bench.build_engine(wl, args.rounds + 2, 3, 0, extra=(WithPartition(args.rank, args.world, tr),))
    eng.step(1 + args.rounds * bench.hops_per_step(wl))
    eng.sync()
    free1 = torch.cuda.mem_get_info(0)[0]
    n0, n1 = eng.node_range
    e0, e1 = eng.edge_range
    print(json.dumps({
        "workload": args.workload, "peers": wl["n"], "world": args.world, "rank": args.rank,
        "owned_nodes": int(n1 - n0), "edges": int(eng.rowptr[-1]), "owned_edges": int(e1 - e0),
        "device_gib": round((free0 - free1) / 2**30, 2), "device_gb": round((free0 - free1) / 1e9, 2),
        "bytes_sent_to_silent_ranks": tr.sent if hasattr(tr, "sent") else 0,
        "transport_calls": tr.calls, "setup_s": round(time.perf_counter() - t0, 1),
        "note": "other ranks silent: receive-side buffers (XRec records, pushed segments) not exercised"}),
        flush=True)


if __name__ == "__main__":
    main()
