"""Seeded peer-graph builders (the simulator's replacement for the reference
test harness's host dialing, floodsub_test.go:57-99).

All graphs are returned as symmetric CSR (rowptr int64[N+1], col int32[E],
outbound uint8[E]) with strictly ascending rows; `outbound[e]` marks the
side that dialed (the lower-index dialer is outbound for
random regular graphs; connectSome marks the dialing host).
"""
import numpy as np


def _to_csr(n, pairs_dialer):
    """pairs_dialer: array (M, 2) of (dialer, target), undirected, no dups."""
    a = pairs_dialer[:, 0].astype(np.int64)
    b = pairs_dialer[:, 1].astype(np.int64)
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    out = np.concatenate([np.ones(len(a), np.uint8), np.zeros(len(a), np.uint8)])
    order = np.lexsort((dst, src))
    src, dst, out = src[order], dst[order], out[order]
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, src + 1, 1)
    rowptr = np.cumsum(rowptr)
    return rowptr, dst.astype(np.int32), out


def random_regular(n, k, seed):
    """Random simple k-regular graph by the pairing model with rejection of
    self-loops / multi-edges (re-pair the rejected stubs a bounded number of
    times, then drop what is left; a few nodes may end with degree < k)."""
    rng = np.random.default_rng(seed)
    stubs = np.repeat(np.arange(n, dtype=np.int64), k)
    edges = set()
    for _ in range(200):
        rng.shuffle(stubs)
        if len(stubs) % 2:
            stubs = stubs[:-1]
        pairs = stubs.reshape(-1, 2)
        lo = np.minimum(pairs[:, 0], pairs[:, 1])
        hi = np.maximum(pairs[:, 0], pairs[:, 1])
        key = lo * n + hi
        ok = lo != hi
        # accept unseen, unique keys
        _, first = np.unique(key, return_index=True)
        uniq = np.zeros(len(key), bool)
        uniq[first] = True
        accept = ok & uniq
        if edges:
            existing = np.fromiter(edges, dtype=np.int64) if len(edges) < 5_000_000 else None
            if existing is not None:
                accept &= ~np.isin(key, existing)
        for kk in key[accept].tolist():
            edges.add(kk)
        rest = pairs[~accept].ravel()
        if len(rest) == 0:
            break
        stubs = rest
    keys = np.fromiter(edges, dtype=np.int64)
    lo, hi = keys // n, keys % n
    return _to_csr(n, np.stack([lo, hi], axis=1))


def random_regular_fast(n, k, seed):
    """Large-N k-regular-ish graph: union of k/2 random perfect matchings over
    a random cyclic ordering (each node gets exactly k distinct neighbours with
    overwhelming probability; duplicate pairs are dropped)."""
    rng = np.random.default_rng(seed)
    pairs = []
    for _ in range(k // 2):
        perm = rng.permutation(n)
        a = perm
        b = np.roll(perm, 1)
        pairs.append(np.stack([a, b], axis=1))
    p = np.concatenate(pairs)
    lo = np.minimum(p[:, 0], p[:, 1]).astype(np.int64)
    hi = np.maximum(p[:, 0], p[:, 1]).astype(np.int64)
    key = np.unique(lo * n + hi)
    lo, hi = key // n, key % n
    return _to_csr(n, np.stack([lo, hi], axis=1))


def connect_some(n, d, seed):
    """connectSome (floodsub_test.go:69-87): every host i dials d random other
    hosts (duplicate dials are no-ops); the dialer is outbound."""
    rng = np.random.default_rng(seed)
    seen = {}
    for i in range(n):
        j = 0
        while j < d:
            m = int(rng.integers(n))
            if m == i:
                continue
            key = (min(i, m), max(i, m))
            if key not in seen:
                seen[key] = i
            j += 1
    arr = np.array([[dialer, b if dialer == a else a] for (a, b), dialer in seen.items()], dtype=np.int64)
    return _to_csr(n, arr)


def dense_connect(n, seed):
    """denseConnect (floodsub_test.go:65-67)."""
    return connect_some(n, 10, seed)


def sparse_connect(n, seed):
    """sparseConnect (floodsub_test.go:61-63)."""
    return connect_some(n, 3, seed)


def all_subscribed(n, topics):
    return np.full(n, (1 << topics) - 1 if topics < 64 else 0xFFFFFFFFFFFFFFFF, dtype=np.uint64)
