"""Headline benchmark: peer-message deliveries/s + gossipsub rounds/s.

Workload (BASELINE.json configs[3], the metric's "1M peers, 64 topics"): a
1,000,000-peer random 32-regular graph, 64 topics, every peer subscribed to
every topic, gossipsub v1.1 with the Eth2-derived peer scoring (P1-P7), 1,000
messages published per heartbeat round (100 per 100 ms hop, topics round-robin,
sources uniform).  One step = one gossipsub round = 10 hops of propagation +
control handling, one refreshScores and one heartbeat (mesh maintenance,
IHAVE emission, mcache shift).  `--workload config3` runs BASELINE configs[2]
(1M peers, 1 topic) instead.

Contract: python bench.py --gpus N --steps K --warmup W; with N > 1 it is
launched by torch.distributed.run and every rank runs its own replica of the
workload on its GPU ("replicas", weak scaling: the partitioned multi-GPU
exchange over RCCL is not built yet).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

from pubsub_amd import (Millisecond, NewGossipSub, WithDevice, WithHop, WithMessageWindow,  # noqa: E402
                        WithPeerScore, WithSeed, eth2_peer_score_params, eth2_thresholds)
from pubsub_amd import graphs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
HOPS_PER_ROUND = 10
MSGS_PER_ROUND = 1000

WORKLOADS = {
    "config4": dict(n=1_000_000, k=32, topics=64, slots=256),
    "config3": dict(n=1_000_000, k=32, topics=1, slots=10048),
}


def build_engine(wl, rounds, seed, device, lib=None, n=None, msgs_per_round=MSGS_PER_ROUND):
    n = n or wl["n"]
    T = wl["topics"]
    g = graphs.random_regular_fast(n, wl["k"], seed)
    subs = graphs.all_subscribed(n, T)
    opts = [WithPeerScore(eth2_peer_score_params(T), eth2_thresholds()), WithHop(100 * Millisecond),
            WithMessageWindow(wl["slots"]), WithSeed(seed)]
    if lib is None:
        opts.append(WithDevice(device))
    eng = NewGossipSub(n, T, g, subs, *opts, lib=lib)
    per_hop = msgs_per_round // HOPS_PER_ROUND
    hops = np.repeat(np.arange(1, rounds * HOPS_PER_ROUND + 1, dtype=np.int64), per_hop)
    rng = np.random.default_rng(seed + 7)
    src = rng.integers(0, n, len(hops)).astype(np.int32)
    top = (np.arange(len(hops)) % T).astype(np.int32)
    eng.publish(src, top, hops)
    return eng, g


def algorithmic_bytes(kernel, eng, wl, launches_per_round):
    """Algorithmic HBM bytes of ONE launch (DESIGN.md §5 lists the formulas)."""
    N, E, T = eng.N, eng.E, wl["topics"]
    W = T * wl["slots"] // 64
    Wt = wl["slots"] // 64
    if kernel == "phase_a":
        # read the forwarded topics' frontier words of every forwarding edge,
        # read+write seen, write the next frontier: (E_fwd_words + 3 N W) * 8
        mesh = eng.mesh()
        fwd_topic_edges = int(np.unpackbits(mesh.view(np.uint8)).sum())
        return (fwd_topic_edges * Wt + 3 * N * W) * 8, dict(fwd_topic_edges=fwd_topic_edges, W=W)
    if kernel == "score":
        # per (edge, topic): flags 1 + fmd/mmd/mfp/imd 32 + meshTime 8; per edge:
        # col 4 + app[col] 8 + p6 8 + bp 8 + score write 8
        return E * (41 * T + 36), dict(E=E, T=T)
    if kernel == "refresh":
        # per (edge, topic): 4 counters r+w 64 + flags r+w 2 + graftTime r 8 + meshTime w 8; per edge bp r+w 16
        return E * (82 * T + 16), dict(E=E, T=T)
    if kernel == "heartbeat":
        # per (edge, topic): backoff 8 + flags 1 (+ stats touched on graft/prune);
        # per edge: mesh r+w 16, fanout r+w 16, score 8, col 4, sub[col] 8, direct+outbound 2,
        # control outbox writes 25; per node: mcache windows of all topics (HG*W*8) + clear W*8
        return E * (9 * T + 79) + N * W * 8 * 6, dict(E=E, T=T)
    return None, {}


def cpu_baseline(wl):
    """The CPU oracle (a faithful single-threaded C++ restatement of the
    reference's routers + peerScore) on a bounded sample of the workload."""
    lib = os.path.join(REPO, "oracle", "_build", "libgossip_oracle.so")
    if not os.path.exists(lib):
        return None
    n = 2000
    T = min(wl["topics"], 8)
    swl = dict(wl, n=n, topics=T, slots=max(256, wl["slots"] if T == 1 else 256))
    rounds = 3
    eng, _ = build_engine(swl, rounds + 1, 11, 0, lib=lib, n=n, msgs_per_round=100)
    eng.step(HOPS_PER_ROUND + 1)
    c0 = eng.counters()
    t0 = time.perf_counter()
    eng.step(rounds * HOPS_PER_ROUND - 1)
    dt = time.perf_counter() - t0
    c1 = eng.counters()
    dlv = c1["deliveries"] - c0["deliveries"]
    return {"value": dlv / dt, "unit": "deliveries/s", "cores": 1, "kind": "port",
            "rounds_per_sec": (rounds * HOPS_PER_ROUND - 1) / HOPS_PER_ROUND / dt,
            "sample": f"oracle/ (C++ restatement), {n} peers k=32, {T} topics, Eth2 scoring, "
                      f"100 msgs/round, {rounds} rounds after warm-up, 1 thread, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="config4", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    wl = WORKLOADS[args.workload]
    rounds = args.warmup + args.steps + 1
    t_setup = time.perf_counter()
    eng, g = build_engine(wl, rounds, 3 + rank, local)
    # hop 0 (Join) + warm-up rounds: meshes form, the message window fills
    eng.step(1 + args.warmup * HOPS_PER_ROUND)
    setup_s = time.perf_counter() - t_setup

    def barrier():
        if dist is not None:
            dist.barrier()
        eng.sync()

    c0 = eng.counters()
    eng.set_profiling(True)
    barrier()
    t0 = time.perf_counter()
    eng.step(args.steps * HOPS_PER_ROUND)
    eng.sync()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    c1 = eng.counters()
    kstats = eng.kernel_stats()
    eng.set_profiling(False)
    deliveries = c1["deliveries"] - c0["deliveries"]
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dv = torch.tensor([deliveries], dtype=torch.float64, device="cuda")
        dist.all_reduce(dv, op=dist.ReduceOp.SUM)
        deliveries = int(dv.item())
    if rank != 0:
        dist.destroy_process_group()
        return

    dom = max(kstats, key=lambda k: kstats[k][0])
    total_ms, launches = kstats[dom]
    avg_ms = total_ms / max(1, launches)
    bytes_per_launch, bytes_info = algorithmic_bytes(dom, eng, wl, launches / args.steps)
    roofline = None
    if bytes_per_launch:
        achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": dom,
                    "avg_launch_ms": round(avg_ms, 4), "bytes_per_launch": int(bytes_per_launch),
                    **{k: v for k, v in bytes_info.items()}}
    rounds_per_s = args.steps / elapsed
    out = {
        "metric": "peer-message deliveries/sec + gossipsub rounds/sec (node), 1M peers 64 topics",
        "value": deliveries / elapsed,
        "unit": "deliveries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64+u64",
        "data": "synthetic (seeded random 32-regular graph, seeded publish schedule)",
        "config": {"workload": args.workload + ": " + ("1M peers, 64 topics" if wl["topics"] == 64
                                                        else "1M peers, 1 topic") +
                   ", k=32, gossipsub v1.1 + Eth2 scoring, 1000 msgs/round, 10 hops/round",
                   "peers": wl["n"], "topics": wl["topics"], "degree": wl["k"],
                   "msgs_per_round": MSGS_PER_ROUND, "hops_per_round": HOPS_PER_ROUND,
                   "parallelism": f"replicas{world}"},
        "rounds_per_sec": rounds_per_s * world,
        "hops_per_sec": rounds_per_s * HOPS_PER_ROUND,
        "kernel_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in kstats.items() if v[1]},
        "roofline": roofline,
        "setup_s": round(setup_s, 1),
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl)
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
