"""Debug: distribution of per-node mcache.peertx entries (GS_STAMPS build) over
a workload's hops: python3 scripts/ptx_occupancy.py config5 60"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

LIB = os.path.join(REPO, "go-libp2p-pubsub_amd", "build", os.environ.get("GS_STAMPS_LIB", "libgossip_engine_var_pb2.so"))


def main():
    wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "config5"]
    hops = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    eng, _ = bench.build_engine(wl, hops // bench.HOPS_PER_ROUND + 2, 3, 0, lib=LIB)
    raw = C.CDLL(LIB)
    raw.gs_debug_ptxn.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int]
    buf = np.zeros(eng.N, dtype=np.int32)
    for h in range(0, hops, 5):
        eng.step(5)
        assert raw.gs_debug_ptxn(eng.h, buf.ctypes.data_as(C.POINTER(C.c_int32)), eng.N) == 0
        print(f"hop {h + 5}: mean {buf.mean():.1f} p50 {np.median(buf):.0f} p99 {np.percentile(buf, 99):.0f} "
              f"p99.99 {np.percentile(buf, 99.99):.0f} max {buf.max()}", flush=True)


if __name__ == "__main__":
    main()
