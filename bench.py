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
launched by torch.distributed.run, one rank per GPU.  By default the ranks
PARTITION the one 1M-peer graph: rank r simulates a contiguous
node range and exchanges its nodes' RPCs with the other ranks once per hop over
RCCL (all-gather of frontier lists / IWANT arena / IHAVE rows, all-to-all-v of
per-edge forwarding + control records; pubsub_amd.transport).  The total work
is fixed, so scaling is "strong".  `--mode replicas` runs N independent copies
instead (weak scaling).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))

from pubsub_amd import (GS_BEHAVE_GRAFT_SPAM, GS_BEHAVE_IHAVE_SPAM, GS_BEHAVE_IWANT_SPAM,  # noqa: E402
                        GS_MSG_PHANTOM, GS_MSG_REJECT, DefaultPeerGaterParams, Millisecond, NewGossipSub,
                        WithBehaviour, WithDevice, WithHop, WithMessageWindow, WithPartition, WithPeerGater,
                        WithPeerScore, WithSeed, WithValidation, eth2_peer_score_params, eth2_thresholds)
from pubsub_amd import graphs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
HOPS_PER_ROUND = 10
MSGS_PER_ROUND = 1000

WORKLOADS = {
    # slots per topic: a message holds its slot for retireHops = 100 hops (3
    # heartbeats of delivery horizon + HistoryLength + 2 heartbeats), i.e. 10
    # rounds x 1000 / 64 = 157 messages per topic; 192 (3 words) is the least
    # multiple of 64 that covers it (W = 192 words: phase A's 3-word variant)
    "config4": dict(n=1_000_000, k=32, topics=64, slots=192),
    "config3": dict(n=1_000_000, k=32, topics=1, slots=10048),
    # BASELINE configs[4] (the adversarial run) on ONE GPU: 1M peers (the
    # 10M-peer figure is the 8-GPU node's; --peers raises it), 20% Sybils split
    # over IWANT spam, GRAFT spam, phantom-IHAVE spam and invalid publishing,
    # 20 Sybils per shared IP, the peer gater, a topic validator with a
    # 32-entry queue per hop.  500 msgs/round: the adversarial delivery
    # window keeps 200 hops of messages alive (10240 slots).
    "config5": dict(n=1_000_000, k=32, topics=1, slots=10240, msgs=500, adversarial=True),
    # BASELINE configs[1]: floodsub, and randomsub with size 100 (size = N
    # degenerates to floodsub), on a 100k-peer random 32-regular
    # graph, one topic, 10,000 messages published at one hop from uniform random
    # sources.  One step = that batch published and propagated: 50 hops (a
    # floodsub / randomsub engine has a nominal 16-hop heartbeat, so its message
    # window recycles a slot after maxAge + 2 = 3 x 16 + 2 = 50 hops; the copies
    # stop after ~6 of them, the rest are cheap empty hops).
    "config2": dict(n=100_000, k=32, topics=1, slots=10048, msgs=10_000, router="floodsub", hops=50),
    "config2_rs100": dict(n=100_000, k=32, topics=1, slots=10048, msgs=10_000, router="randomsub", size=100,
                          hops=50),
}


def hops_per_step(wl):
    return wl.get("hops", HOPS_PER_ROUND)


def build_engine(wl, rounds, seed, device, lib=None, n=None, msgs_per_round=None, extra=(), graph=None):
    """The workload's engine (graph, subscriptions, params, publish schedule);
    `graph` reuses a graph this function built before with the same seed."""
    n = n or wl["n"]
    T = wl["topics"]
    msgs_per_round = msgs_per_round or wl.get("msgs", MSGS_PER_ROUND)
    g = graph if graph is not None else graphs.random_regular_fast(n, wl["k"], seed)
    subs = graphs.all_subscribed(n, T)
    if wl.get("router") in ("floodsub", "randomsub"):
        # config2: the batch of each step published at its first hop
        from pubsub_amd import NewFloodSub, NewRandomSub
        opts = [WithMessageWindow(wl["slots"]), WithSeed(seed)]
        if lib is None or "libgossip_engine" in os.path.basename(lib):
            opts.append(WithDevice(device))
        if wl["router"] == "floodsub":
            eng = NewFloodSub(n, T, g, subs, *opts, *extra, lib=lib)
        else:
            eng = NewRandomSub(n, T, g, subs, wl["size"], *opts, *extra, lib=lib)
        rng = np.random.default_rng(seed + 7)
        hps = hops_per_step(wl)
        hops = np.repeat(1 + hps * np.arange(rounds, dtype=np.int64), msgs_per_round)
        src = rng.integers(0, n, len(hops)).astype(np.int32)
        top = np.zeros(len(hops), np.int32)
        eng.publish(src, top, hops)
        eng.schedule = (top, hops)
        eng.kinds, eng.srcs, eng.ipv4 = None, src, None
        return eng, g
    opts = [WithPeerScore(eth2_peer_score_params(T), eth2_thresholds()), WithHop(100 * Millisecond),
            WithMessageWindow(wl["slots"]), WithSeed(seed)]
    if lib is None or "libgossip_engine" in os.path.basename(lib):
        opts.append(WithDevice(device))
    kw = {}
    rng = np.random.default_rng(seed + 7)
    per_hop = msgs_per_round // HOPS_PER_ROUND
    hops = np.repeat(np.arange(1, rounds * HOPS_PER_ROUND + 1, dtype=np.int64), per_hop)
    src = rng.integers(0, n, len(hops)).astype(np.int32)
    top = (np.arange(len(hops)) % T).astype(np.int32)
    kind = None
    if wl.get("adversarial"):
        # the config-5 mix (tests/scenarios.py adversarial_mix, at scale)
        arng = np.random.default_rng(seed + 11)
        sybil = arng.random(n) < 0.2
        ids = np.flatnonzero(sybil)
        kind_of = arng.integers(0, 4, len(ids))  # 0 IWANT spam, 1 GRAFT spam, 2 phantom IHAVE, 3 invalid
        beh = np.zeros(n, np.uint8)
        beh[ids[kind_of == 0]] = GS_BEHAVE_IWANT_SPAM
        beh[ids[kind_of == 1]] = GS_BEHAVE_GRAFT_SPAM
        beh[ids[kind_of == 2]] = GS_BEHAVE_IHAVE_SPAM
        ipv4 = (np.arange(n) + (10 << 24)).astype(np.uint32)
        ipv4[ids] = (192 << 24) + (np.arange(len(ids)) // 20).astype(np.uint32)  # 20 Sybils per IP
        kw["ipv4"] = ipv4
        opts += [WithBehaviour(beh), WithValidation([1] * T, 32), WithPeerGater(DefaultPeerGaterParams())]
        honest = np.flatnonzero(~sybil)
        src = honest[rng.integers(0, len(honest), len(hops))].astype(np.int32)
        kind = np.zeros(len(hops), np.uint8)
        r = rng.random(len(hops))
        inv, ph = ids[kind_of == 3], ids[kind_of == 2]
        sel = r < 1 / 3  # a third invalid messages, a sixth phantom ids
        src[sel] = inv[rng.integers(0, len(inv), int(sel.sum()))]
        kind[sel] = GS_MSG_REJECT
        sel = (r >= 1 / 3) & (r < 0.5)
        src[sel] = ph[rng.integers(0, len(ph), int(sel.sum()))]
        kind[sel] = GS_MSG_PHANTOM
    eng = NewGossipSub(n, T, g, subs, *opts, *extra, lib=lib, **kw)
    eng.publish(src, top, hops, kind=kind)
    eng.schedule = (top, hops)
    eng.kinds = kind  # GS_MSG_* per published message (None: all valid)
    eng.srcs = src
    eng.ipv4 = kw.get("ipv4")
    return eng, g


def active_words(eng, wl, hop):
    """Words of the message window phase A touches at `hop` (the engine's amR:
    words holding a message published within the last 3 heartbeats + 1 hop,
    slots assigned round-robin per topic as gs_publish does)."""
    top, hops = eng.schedule
    if not hasattr(eng, "sched_slots"):
        St = wl["slots"]
        slots = np.empty(len(top), dtype=np.int64)
        for t in range(wl["topics"]):
            idx = np.nonzero(top == t)[0]  # publish order (hops are non-decreasing)
            slots[idx] = t * St + np.arange(len(idx)) % St
        eng.sched_slots = slots
    slots = eng.sched_slots
    max_age = (13 if wl.get("adversarial") else 3) * HOPS_PER_ROUND  # gs_engine setWindow
    live = (hops >= hop - 1 - max_age) & (hops <= hop - 1)
    return len(np.unique(slots[live] // 64))


def algorithmic_bytes(kernel, eng, wl, per_hop):
    """Algorithmic HBM bytes of ONE launch of `kernel`: the data
    the algorithm must move with the engine's representation, not what the
    caches end up fetching.  per_hop: measured averages over the timed hops."""
    # a partitioned rank's kernels cover its own nodes [n0, n1) and edges [e0, e1)
    (n0, n1), (e0, e1) = eng.node_range, eng.edge_range
    N, E, T = n1 - n0, e1 - e0, wl["topics"]
    if kernel == "phase_a":
        scored = not wl.get("router") in ("floodsub", "randomsub")
        if scored:
            mesh = eng.mesh()[e0:e1]
            fwd_edges = int((mesh != 0).sum())      # edges with a forwarding topic
        else:
            fwd_edges = E                           # floodsub / randomsub: every edge may forward
        W = per_hop["active_words"]
        # SURVEY.md §8(d) "Propagation hop": B_hop = (E_fwd + 3N) * W * 8 --
        # one sender frontier word per forwarding edge, and per node its seen
        # words read and written and its next frontier written, over the active
        # message window (the words phase A touches: messages younger than the
        # delivery horizon).  This is the line's `achieved` model.
        b = (fwd_edges + 3.0 * N) * W * 8.0
        if per_hop.get("prop_hops_per_step") is not None:
            # config2: only the hops with copies on the wire propagate; the
            # per-launch average spreads them over the step's launches
            b *= per_hop["prop_hops_per_step"] / hops_per_step(wl)
        # the engine's own representation, for comparison with the PMC traffic:
        # each copy sent is one 16-bit slot of the sender's pushed segment for
        # that edge (k_push), read once by its receiver, plus the segment's
        # 8-byte record; the receiver writes its own frontier list (4 B per
        # entry), read-modify-writes the pending counts per (edge, topic), its
        # seen words, and per-edge metadata
        items = per_hop["deliveries"] + per_hop["published"]   # frontier-list entries written per hop
        copies = per_hop["transmissions"] - per_hop["iwant_served"]  # served ids: 4 B each from the pool
        list_reads = 2.0 * copies + 8.0 * fwd_edges + 4.0 * per_hop["iwant_served"]
        list_writes = 4.0 * items
        # pending-delivery counts, read + write per (edge, topic): 16-bit words
        # when a topic's slots fit a byte count (gs_engine.hip narrowDlt)
        pend_b = 0.0 if not scored else (4.0 if wl["slots"] <= 254 and T % 2 == 0 else 8.0)
        pending = pend_b * T * E
        seen = 16.0 * N * W                          # seen words of the active window, read + write
        meta = 49.0 * E                              # rev, col, fwd masks, IWANT ref, S0 memo, direct, mesh
        eb = list_reads + list_writes + pending + seen + meta
        return b, dict(model="SURVEY 8(d): (E_fwd + 3N) * W * 8", fwd_edges=fwd_edges, active_words=W,
                       engine_model_bytes=int(eb), list_entries_per_hop=items, copies_per_hop=copies,
                       engine_bytes_lists=int(list_reads + list_writes), engine_bytes_pending=int(pending),
                       engine_bytes_seen=int(seen), engine_bytes_meta=int(meta))
    if kernel == "refresh":
        # 80 B per (edge, topic) (the four f64 counters read
        # and written 64, meshTime written 8, graft time read, flags r+w,
        # padded to 80) + 16 B per edge (P7 read and written).  The engine
        # moves less (PMC `traffic`): unchanged counters (zeros staying zero)
        # are not written back and its pending word is 4 B.
        return E * (80.0 * T + 16), dict(E=E, T=T, per_pair=80, per_edge=16)
    if kernel == "heartbeat":
        # 14 B per candidate edge per (node, topic) (score 8,
        # backoff 4, outbound and mesh bits 2) over the joined topics, plus the
        # gossip windows (HistoryGossip mcache windows of W words read per
        # node, the node's gw row written) and the per-edge masks (mesh and
        # fanout read and written, backoff mask read: 40 B)
        deg = np.diff(eng.rowptr)[n0:n1].astype(np.int64)
        subs = np.asarray(eng.subs, dtype=np.uint64)[n0:n1]
        joined = np.array([bin(int(x)).count("1") for x in subs], dtype=np.int64) if len(subs) < 4096 else \
            np.unpackbits(subs.view(np.uint8).reshape(-1, 8), axis=1).sum(axis=1).astype(np.int64)
        cand = int((deg * joined).sum())
        W = T * wl["slots"] // 64
        hg = 5
        b = 14.0 * cand + 8.0 * N * W * (hg + 1) + 40.0 * E
        return b, dict(candidates=cand, W=W)
    if kernel == "phase_b":
        # HandleRPC over one round's control, averaged per launch (10 per
        # round).  Per IHAVE entry (edge, topic): the sender's gossip-window
        # words of the topic and the receiver's seen words of it, 2 * Wt * 8
        # (SURVEY.md §8(d) "Gossip", per topic as the engine reads them); per
        # IWANT id: the id, HistoryLength mcache window words and the peertx
        # entry (4 + 8 * 5 + 8); per served id its response entry (4); per
        # GRAFT / PRUNE the edge's control record (64).  Every hop every in-edge's
        # control-count bytes (cPre, cHb: 2 B per edge).
        ev = per_hop["events_per_round"]
        Wt = wl["slots"] // 64
        b_round = (ev["ihave_sent"] * 2.0 * Wt * 8 + ev["iwant_sent"] * 52.0 + ev["iwant_served"] * 4.0 +
                   (ev["grafts_sent"] + ev["prunes_sent"]) * 64.0)
        b = b_round / HOPS_PER_ROUND + 2.0 * E
        return b, dict(ihave_entries_per_round=ev["ihave_sent"], iwant_ids_per_round=ev["iwant_sent"],
                       served_per_round=ev["iwant_served"], Wt=Wt, per_ihave_entry=2 * Wt * 8, per_iwant_id=52)
    if kernel == "score":
        # full pass: per (edge, topic) flags 1 + fmd/mfp/imd 24 + pending 4 (+ mmd, meshTime when
        # active); per edge col 4 + app 8 + p6 8 + bp 8 + out 8
        return E * (29.0 * T + 36), dict(E=E, T=T)
    return None, {}


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model


def cpu_baseline(wl, seconds=20.0):
    """The CPU oracle (a faithful C++ restatement of the reference's routers +
    peerScore, OpenMP over nodes in every per-node phase) on a bounded sample
    of the SAME workload: same degree, topic count, scoring and per-peer
    message rate (every peer receives all 1000 msgs/round), fewer peers."""
    import ctypes
    lib = os.path.join(REPO, "oracle", "_build", "libgossip_oracle.so")
    if not os.path.exists(lib):
        return None
    olib = ctypes.CDLL(lib)
    threads = olib.gs_oracle_threads()  # OMP_NUM_THREADS: 16 on the GPU box (its CPU share)
    if hasattr(olib, "gs_oracle_set_threads"):
        # one thread and all cores.  The one-thread leg first, on
        # half the time budget; the headline value is the all-cores leg
        olib.gs_oracle_set_threads(1)
        one = cpu_baseline_at(wl, lib, 1, seconds / 2, scale=8)
        olib.gs_oracle_set_threads(threads)
        out = cpu_baseline_at(wl, lib, threads, seconds)
        if one and out:
            out["value_1thread"] = one["value"]
            out["sample_1thread"] = one["sample"]
            out["parallel_speedup"] = out["value"] / one["value"] if one["value"] else None
        return out
    return cpu_baseline_at(wl, lib, threads, seconds)


def cpu_baseline_at(wl, lib, threads, seconds, scale=1):
    """One leg of cpu_baseline: `scale` divides the sample's peer count (the
    one-thread leg runs a smaller graph in a comparable time)."""
    if wl.get("router") in ("floodsub", "randomsub"):
        return cpu_baseline_config2(wl, lib, threads, seconds, scale)
    n = 2000 // scale
    swl = dict(wl, n=n)
    rounds = 8
    eng, _ = build_engine(swl, rounds + 2, 11, 0, lib=lib, n=n)
    eng.step(HOPS_PER_ROUND + 1)  # Join + one warm-up round
    c0 = eng.counters()
    t0 = time.perf_counter()
    hops = 0
    while hops < rounds * HOPS_PER_ROUND and (time.perf_counter() - t0 < seconds or hops < HOPS_PER_ROUND):
        eng.step(1)
        hops += 1
    dt = time.perf_counter() - t0
    c1 = eng.counters()
    dlv = c1["deliveries"] - c0["deliveries"]
    rps = hops / HOPS_PER_ROUND / dt
    return {"value": dlv / dt, "unit": "deliveries/s", "cores": threads, "kind": "port",
            "rounds_per_sec_sample": rps,
            "rounds_per_sec_extrapolated_1M": rps * n / wl["n"],
            "extrapolation": f"per-peer linear: rounds/s x {n}/{wl['n']} (labelled estimate, not measured)",
            "cpu_model": cpu_info(), "nproc": os.cpu_count(),
            "threads_note": "OpenMP threads = OMP_NUM_THREADS, which the GPU box sets to 16 (this job's CPU share "
                            "of the shared host; nproc shows the whole machine)",
            "sample": f"oracle/ (C++ restatement, OpenMP {threads} threads), {n} peers k={wl['k']}, "
                      f"{wl['topics']} topics, Eth2 scoring, {wl.get('msgs', MSGS_PER_ROUND)} msgs/round"
                      f"{' (config-5 adversarial mix)' if wl.get('adversarial') else ''}, {hops} hops "
                      f"after 1 warm-up round, {dt:.1f} s"}


def cpu_baseline_config2(wl, lib, threads, seconds, scale=1):
    """config2 on the oracle: the same router, degree and one-hop batches on a
    20,000-peer graph (divided by `scale`), 200-message batches (each step
    fully propagated), stepped until about `seconds` have passed."""
    n, m = 20_000 // scale, 200
    swl = dict(wl, n=n, msgs=m)
    hps = hops_per_step(wl)
    eng, _ = build_engine(swl, 50, 11, 0, lib=lib, n=n)
    t0 = time.perf_counter()
    steps = 0
    while steps < 50 and (steps == 0 or time.perf_counter() - t0 < seconds):
        eng.step(hps)
        steps += 1
    dt = time.perf_counter() - t0
    dlv = eng.counters()["deliveries"]
    return {"value": dlv / dt, "unit": "deliveries/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_info(), "nproc": os.cpu_count(),
            "sample": f"oracle/ (C++ restatement, OpenMP {threads} threads), {wl['router']}"
                      f"{' size ' + str(wl['size']) if wl.get('size') else ''}, {n} peers k={wl['k']}, "
                      f"{steps} batches of {m} messages each published at one hop and propagated "
                      f"({hps} hops), {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="config4", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default="partition", choices=["partition", "replicas"])
    ap.add_argument("--peers", type=int, default=0, help="override the workload's peer count (rehearsals)")
    ap.add_argument("--slots", type=int, default=0,
                    help="override the engine's message slots per topic (a capacity, not the workload)")
    ap.add_argument("--transport", default="torch", choices=["rccl", "torch"],
                    help="partitioned ranks' exchange: torch.distributed collectives (RCCL under the "
                         "nccl backend; the default, whose multi-rank path the tests run over gloo) or "
                         "the product library's native RCCL transport (include/gs_transport.h), which "
                         "has run at world 1 only")
    ap.add_argument("--rpc-accounting", action="store_true",
                    help="also sum RPC bytes per edge (gs_set_rpc_accounting; 1 KB messages, 40-byte ids)")
    ap.add_argument("--frontier", default="auto", choices=["auto", "lists", "bitmaps"],
                    help="phase A's reading of the senders' frontiers (gs_set_frontier_mode; same results): "
                         "the engine's choice (auto), per-copy lists, or bitmaps wherever supported")
    ap.add_argument("--lib", default=None, help="timing experiments only: another build of the product library "
                    "(results are labelled with it)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not launched by torch.distributed.run: start the N ranks ourselves (a
        # child process, before anything here touches the GPU) and exit with its code
        import socket
        import subprocess
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report a different GPU count")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    extra = ()
    partitioned = world > 1 and args.mode == "partition"
    if world > 1:
        import torch
        import torch.distributed as dist
        # GS_DIST_BACKEND=gloo + several ranks per GPU: a rehearsal of the
        # partitioned path on a 1-GPU box (host-staged exchange)
        backend = os.environ.get("GS_DIST_BACKEND", "nccl")
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if partitioned:
            if backend == "nccl" and args.transport == "rccl":
                from pubsub_amd.transport import RcclTransport
                transport = RcclTransport(rank, world, device=local)
            else:  # gloo rehearsals stage through host memory
                from pubsub_amd.transport import TorchTransport
                transport = TorchTransport(memory="device")
            extra = (WithPartition(rank, world, transport),)

    wl = dict(WORKLOADS[args.workload])
    if args.peers:
        wl["n"] = args.peers
    if args.slots:
        wl["slots"] = args.slots
    hps = hops_per_step(wl)
    gossip = wl.get("router", "gossipsub") == "gossipsub"
    rounds = args.warmup + args.steps + 1
    t_setup = time.perf_counter()
    # partitioned ranks simulate ONE graph and schedule (same seed); replicas differ
    if args.rpc_accounting:
        from pubsub_amd import WithRPCAccounting
        extra = tuple(extra) + (WithRPCAccounting(1000, id_len=40),)
    if args.frontier != "auto":
        from pubsub_amd import WithFrontierBitmaps, WithFrontierLists
        extra = tuple(extra) + ((WithFrontierLists if args.frontier == "lists" else WithFrontierBitmaps)(),)
    def dev_free():
        try:
            import torch
            return torch.cuda.mem_get_info(local)[0]
        except Exception:  # noqa: BLE001 — a report field only
            return None
    free0 = dev_free()
    eng, g = build_engine(wl, rounds, 3 if partitioned else 3 + rank, local, extra=extra, lib=args.lib)
    # hop 0 (Join) + warm-up rounds: meshes form, the message window fills
    eng.step(1)
    prop_hops = None
    if not gossip:
        # config2: the hops of a step in which copies are on the wire (the
        # roofline model's propagation hops), from the first warm-up step
        prop_hops = 0
        for _ in range(hps):
            t0c = eng.counters()["transmissions"]
            eng.step(1)
            prop_hops += eng.counters()["transmissions"] > t0c
        eng.step(max(0, args.warmup - 1) * hps)
    else:
        eng.step(args.warmup * hps)
    eng.sync()
    free1 = dev_free()
    device_gb = round((free0 - free1) / 2**30, 2) if free0 is not None and free1 is not None else None
    setup_s = time.perf_counter() - t_setup

    def barrier():
        if dist is not None:
            dist.barrier()
        eng.sync()

    c0 = eng.counters()
    x0 = eng.exchange_stats()
    hop0 = eng.hop
    eng.set_profiling(True)
    barrier()
    t0 = time.perf_counter()
    eng.step(args.steps * hps)
    eng.sync()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    c1 = eng.counters()
    x1 = eng.exchange_stats()
    kstats = eng.kernel_stats()
    eng.set_profiling(False)
    ev_keys = ("deliveries", "duplicates", "transmissions", "grafts_sent", "prunes_sent",
               "ihave_sent", "iwant_sent", "iwant_served", "promises_broken", "graylisted",
               "rejected", "throttled", "gated")
    events = {k: c1[k] - c0[k] for k in ev_keys}
    if dist is not None:
        import torch
        cdev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dv = torch.tensor([events[k] for k in ev_keys], dtype=torch.int64, device=cdev)
        dist.all_reduce(dv, op=dist.ReduceOp.SUM)
        events = dict(zip(ev_keys, (int(x) for x in dv.tolist())))
    deliveries = events["deliveries"]
    msgs_round = wl.get("msgs", MSGS_PER_ROUND)
    if rank != 0:
        dist.destroy_process_group()
        return

    nh = args.steps * hps
    per_hop = {"events_per_round": {k: v / args.steps for k, v in events.items()},
               "deliveries": (c1["deliveries"] - c0["deliveries"]) / nh,
               "published": (c1["published"] - c0["published"]) / nh,
               "transmissions": (c1["transmissions"] - c0["transmissions"]) / nh,
               "iwant_served": (c1["iwant_served"] - c0["iwant_served"]) / nh,
               "active_words": float(np.mean([active_words(eng, wl, hop0 + i) for i in range(nh)])) if gossip
               else wl["topics"] * wl["slots"] / 64.0,
               "prop_hops_per_step": prop_hops, "steps": args.steps,
               "mesh_pairs": int(np.bitwise_count(eng.mesh()[eng.edge_range[0]:eng.edge_range[1]]).sum(dtype=np.int64))}
    # the roofline is the heaviest kernel with an algorithmic byte model (phase
    # B's control work has none: config3's steady state and config5 can be
    # dominated by it, named in "dominant_kernel")
    top = max(kstats, key=lambda k: kstats[k][0])
    dom, bytes_per_launch, bytes_info = top, None, {}
    for k in sorted(kstats, key=lambda k: -kstats[k][0]):
        if not kstats[k][1]:
            continue
        b_k, info_k = algorithmic_bytes(k, eng, wl, per_hop)
        if b_k:
            dom, bytes_per_launch, bytes_info = k, b_k, info_k
            break
    total_ms, launches = kstats[dom]
    avg_ms = total_ms / max(1, launches)
    roofline = None
    pmc = os.path.join(REPO, "profiles", f"pmc_traffic_{args.workload}.json")
    pmc_recs = json.load(open(pmc)) if os.path.exists(pmc) and not partitioned else {}

    def pmc_traffic(kernel):
        # rocprofv3 PMC passes of this workload (scripts/gpu_pmc.sh + pmc_summary.py):
        # FETCH_SIZE x 2 (gfx950 wide-read correction, MI355X_MICROARCH.md) + WRITE_SIZE,
        # per launch; kernel names carry template arguments ("void k_phase_a<4, true>")
        base = {"refresh": "k_refresh_rows"}.get(kernel, f"k_{kernel}")
        # several instantiations (config3 / config5: the narrow counters of the
        # first hops, then the wide ones): the one dispatched last is the
        # timed window's
        best = None
        for name, rec in pmc_recs.items():
            if name == base or name.startswith(f"void {base}<"):
                if best is None or rec.get("last_dispatch", 0) > best.get("last_dispatch", 0):
                    best = rec
        return (best["traffic_bytes_est"], os.path.relpath(pmc, REPO)) if best else (None, None)

    traffic, traffic_src = pmc_traffic(dom)
    if bytes_per_launch and avg_ms > 0:
        achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    # the same launch priced at its measured DRAM bytes (PMC `traffic`, a
                    # profile of this workload) instead of the algorithmic model: `frac`
                    # uses the model named in `model`, this one what the HBM really moved
                    "frac_traffic": (round(traffic / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                                     if traffic else None),
                    "kernel": dom, "dominant_kernel": top,
                    "avg_launch_ms": round(avg_ms, 4), "bytes_per_launch": int(bytes_per_launch),
                    **{k: v for k, v in bytes_info.items()}}
    # the score kernels' rooflines too (north-star target: >= 50% of HBM on
    # score / propagation): refreshScores streams every (edge, topic) record
    rooflines = {}
    for k in ("refresh", "heartbeat", "phase_b", "phase_a"):
        if k == dom:
            continue
        if k in kstats and kstats[k][1]:
            b_k, _ = algorithmic_bytes(k, eng, wl, per_hop)
            ms_k = kstats[k][0] / kstats[k][1]
            ach = b_k / (ms_k / 1e3) / 1e9
            rooflines[k] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(ms_k, 4),
                            "bytes_per_launch": int(b_k)}
            rooflines[k]["traffic"], rooflines[k]["traffic_source"] = pmc_traffic(k)
            if rooflines[k]["traffic"]:
                rooflines[k]["frac_traffic"] = round(rooflines[k]["traffic"] / (ms_k / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
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
        "scaling": "strong" if partitioned else "weak",
        "vs_baseline": None,
        "dtype": "f64+u64" if gossip else "u64",
        "data": "synthetic (seeded random 32-regular graph, seeded publish schedule)",
        "config": {"workload": f"{args.workload}: {wl['n'] / 1e6:g}M peers, {wl['topics']} topic"
                   f"{'s' if wl['topics'] > 1 else ''}, k=32, " +
                   (f"gossipsub v1.1 + Eth2 scoring, {msgs_round} msgs/round, 10 hops/round" if gossip else
                    f"{wl['router']}{' size ' + str(wl['size']) if wl.get('size') else ''}, {msgs_round} msgs "
                    f"published at one hop per step, {hps} hops/step ({prop_hops} with copies on the wire)") +
                   (", 20% Sybils (IWANT / GRAFT / phantom-IHAVE spam, invalid messages, 20 per IP), "
                    "peer gater, validation queue 32" if wl.get("adversarial") else ""),
                   "peers": wl["n"], "topics": wl["topics"], "degree": wl["k"],
                   "msgs_per_round": msgs_round, "hops_per_round": hps,
                   "parallelism": f"partition{world}" if partitioned else f"replicas{world}"},
        "rounds_per_sec": rounds_per_s * (1 if partitioned else world),
        "hops_per_sec": rounds_per_s * (hps if gossip else prop_hops),
        "kernel_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in kstats.items() if v[1]},
        "events_per_step": {k: v // args.steps for k, v in events.items()},
        # the control counters depend on the canonical schedule: each
        # hop handles every payload RPC before any control RPC; the per-RPC order of
        # the oracle's reference mode roughly doubles iwant_sent on gossipsub_scored
        "schedule": "phase split: payload before control per hop (DESIGN.md 3a; per-RPC order ~2x iwant_sent)",
        "phase_a_reads": "frontier bitmaps" if eng.frontier_dense else "frontier lists",
        "roofline": roofline,
        "rooflines_other": rooflines,
        "device_gib": device_gb,  # device memory the engine holds (free memory before / after its start)
        "setup_s": round(setup_s, 1),
    }
    if args.lib:
        out["experiment_lib"] = os.path.basename(args.lib)
    if args.rpc_accounting:
        rb, rn = eng.rpc_bytes()
        out["rpc_accounting"] = {"bytes_total": int(rb.sum()), "rpcs_total": int(rn.sum()),
                                 "bytes_per_peer_per_round": float(rb.sum()) / wl["n"] / (rounds - 1)}
    if partitioned:
        out["exchange"] = {"transport": type(extra[0][1][2]).__name__,
                           "rank0_host_ms_per_step": round((x1[0] - x0[0]) / args.steps, 3),
                           "rank0_bytes_in_per_step": (x1[1] - x0[1]) // args.steps,
                           "rank0_nodes": eng.node_range[1] - eng.node_range[0]}
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(wl)
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
