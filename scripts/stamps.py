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
    # publish schedule of `rounds` rounds (bench.py: warm-up + steps + 1)
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    extra = ()
    fm = os.environ.get("GS_STAMPS_FRONTIER")  # phase A's frontier mode: lists / bitmaps (default: auto)
    if fm in ("lists", "bitmaps"):
        from pubsub_amd import WithFrontierBitmaps, WithFrontierLists
        extra = ((WithFrontierLists if fm == "lists" else WithFrontierBitmaps)(),)
    eng, _ = bench.build_engine(wl, rounds, 3, 0, lib=LIB, extra=extra)
    hops = int(sys.argv[2]) if len(sys.argv) > 2 else 1 + 2 * bench.HOPS_PER_ROUND + 3
    eng.step(hops)
    raw = C.CDLL(LIB)
    n = (eng.N // 1024 + 1) * 24
    buf = np.zeros(n, dtype=np.uint64)
    raw.gs_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    rc = raw.gs_debug_stamps(eng.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), n)
    assert rc == 0
    K = eng.N // 1024 + 1
    hbbuf = buf[16 * K:]
    buf = buf[:16 * K]
    s = buf.reshape(-1, 8)[: len(buf) // 16, :5].astype(np.int64)
    s = s[(s[:, 0] > 0) & (s[:, 4] > 0)]
    d = np.diff(s, axis=1)
    names = ["setup", "pass1", "pass2", "pass3"]
    print("samples", len(d))
    for i, nm in enumerate(names):
        print(f"{nm}: mean {d[:, i].mean():.0f} cycles  p50 {np.median(d[:, i]):.0f}  p99 {np.percentile(d[:, i], 99):.0f}")
    print("total mean", d.sum(1).mean())
    s5 = buf.reshape(-1, 8)[: len(buf) // 16, :6].astype(np.int64)
    s5 = s5[(s5[:, 0] > 0) & (s5[:, 4] > 0) & (s5[:, 5] > 0)]
    if len(s5):
        print(f"  pass3 rmw only: mean {(s5[:, 5] - s5[:, 3]).mean():.0f}, pass2b stores: mean {(s5[:, 4] - s5[:, 5]).mean():.0f}")
    s8 = buf.reshape(-1, 8)[: len(buf) // 16, :8].astype(np.int64)
    s8 = s8[(s8[:, 3] > 0) & (s8[:, 5] > 0) & (s8[:, 6] > 0) & (s8[:, 7] > 0) & (s8[:, 4] > 0)]
    if len(s8):
        print(f"  pass3 split: rmw {(s8[:, 5] - s8[:, 3]).mean():.0f}, P4 + gater {(s8[:, 6] - s8[:, 5]).mean():.0f}, "
              f"IWANT spam {(s8[:, 7] - s8[:, 6]).mean():.0f} (p99 {np.percentile(s8[:, 7] - s8[:, 6], 99):.0f}), "
              f"pass2b {(s8[:, 4] - s8[:, 7]).mean():.0f} (p99 {np.percentile(s8[:, 4] - s8[:, 7], 99):.0f})")
    hb = hbbuf.reshape(-1, 8).astype(np.int64)
    hb = hb[(hb[:, 0] > 0) & (hb[:, 5] > 0)]
    if len(hb):
        cols = [0, 1, 2, 3, 5]
        dh = np.diff(hb[:, cols], axis=1)
        print("heartbeat samples", len(hb))
        for i, nm in enumerate(["gw windows", "exact scores", "topic loop", "fanout + outbox + shift"]):
            print(f"  {nm}: mean {dh[:, i].mean():.0f} cycles  p50 {np.median(dh[:, i]):.0f}  p99 {np.percentile(dh[:, i], 99):.0f}")
        print(f"  topic loop split: mesh maintenance {hb[:, 6].mean():.0f}, emitGossip {hb[:, 7].mean():.0f}"
              f" (paired: stats + live scores {hb[:, 7].mean():.0f}, peer selection {hb[:, 4].mean():.0f})")
    bb = buf.reshape(-1, 8)[len(buf) // 16:].astype(np.int64)
    bb = bb[(bb[:, 0] > 0) & (bb[:, 4] > 0)]
    b = bb[:, :5]
    if len(b):
        db = np.diff(b, axis=1)
        print("phase B samples", len(b))
        for i, nm in enumerate(["step1", "step2 iwant", "step3 ihave", "step4"]):
            print(f"  {nm}: mean {db[:, i].mean():.0f} cycles  p50 {np.median(db[:, i]):.0f}  p99 {np.percentile(db[:, i], 99):.0f}")
        sub = bb[(bb[:, 5] > 0) & (bb[:, 7] > 0)]
        if len(sub) and os.environ.get("GS_STAMPS_PB2"):
            print("  step2 (nodes serving, %d): setup %.0f, table load + windows %.0f, passes a/b %.0f, write-back %.0f" % (
                len(sub), (sub[:, 5] - sub[:, 1]).mean(), (sub[:, 6] - sub[:, 5]).mean(), (sub[:, 7] - sub[:, 6]).mean(),
                (sub[:, 2] - sub[:, 7]).mean()))
        elif len(sub):
            print("  step3 (nodes with IHAVE work, %d): setup %.0f, pass a %.0f, pass a2 %.0f, pass b + arena %.0f" % (
                len(sub), (sub[:, 5] - sub[:, 2]).mean() - (sub[:, 5] - sub[:, 5]).mean(), 0, 0, 0)
                  if False else "  step3 (nodes with IHAVE work, %d): to pass a end %.0f, pass a2 %.0f, pass b + arena %.0f, promises + rest %.0f" % (
                len(sub), (sub[:, 5] - sub[:, 2]).mean(), (sub[:, 6] - sub[:, 5]).mean(), (sub[:, 7] - sub[:, 6]).mean(),
                (sub[:, 3] - sub[:, 7]).mean()))


if __name__ == "__main__":
    main()
