"""Debug: per-pass cycle stamps of phase A (GS_STAMPS build) at config4."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

LIB = os.path.join(REPO, "go-libp2p-pubsub_amd", "build", os.environ.get("GS_STAMPS_LIB", "libgossip_engine_stamps.so"))


def main():
    wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "config4"]
    eng, _ = bench.build_engine(wl, 4, 3, 0, lib=LIB)
    eng.step(1 + 2 * bench.HOPS_PER_ROUND + 3)
    raw = C.CDLL(LIB)
    n = (eng.N // 1024 + 1) * 8
    buf = np.zeros(n, dtype=np.uint64)
    raw.gs_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    rc = raw.gs_debug_stamps(eng.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n)
    assert rc == 0
    s = buf.reshape(-1, 8)[:, :5].astype(np.int64)
    s = s[(s[:, 0] > 0) & (s[:, 4] > 0)]
    d = np.diff(s, axis=1)
    names = ["setup", "pass1", "pass2", "pass3"]
    print("samples", len(d))
    for i, nm in enumerate(names):
        print(f"{nm}: mean {d[:, i].mean():.0f} cycles  p50 {np.median(d[:, i]):.0f}  p99 {np.percentile(d[:, i], 99):.0f}")
    print("total mean", d.sum(1).mean())
    c = buf.reshape(-1, 8)[:, 5:8].astype(np.int64)
    print("copies/node mean", c[:, 0].mean(), "pass-1 list-load cycles mean", c[:, 1].mean(), "pass-1 delivery-drain cycles mean",
          c[:, 2].mean())


if __name__ == "__main__":
    main()
