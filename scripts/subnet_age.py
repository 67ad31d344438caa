"""Message ages in config4's subnet variant (topic 0 + 2 random subnets per peer) on the
oracle: the largest first-delivery age per message (sparse subscriptions).
    python scripts/subnet_age.py PEERS ROUNDS"""
import sys, time, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/go-libp2p-pubsub_amd")
import bench
wl = dict(n=int(sys.argv[1]), k=32, topics=64, slots=256, subnets=2)
rounds = int(sys.argv[2])
t0 = time.time()
from pubsub_amd import WithRecordDeliveries
eng, g = bench.build_engine(wl, rounds, 3, 0, lib="/root/repo/oracle/_build/libgossip_oracle.so", extra=(WithRecordDeliveries(),))
eng.step(rounds * 10 + 1)
print("stepped", time.time() - t0, flush=True)
top, hops = eng.schedule
ages = []
late = 0
nsub = 0
for m in range(eng.n_published):
    hop, frm = eng.deliveries(m)
    ok = hop >= 0
    if ok.any():
        a = hop[ok] - hops[m]
        ages.append(a.max())
h = np.array(ages)
print("msgs", len(h), "max age", h.max(), "p99", np.percentile(h, 99), "hist", np.bincount(np.minimum(h, 60)))
print(eng.counters())
