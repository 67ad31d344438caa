/*
 * gs_rng.h — the engine's canonical random stream (host + device).
 *
 * The reference draws from Go's global math/rand source (gossipsub.go:1879-
 * 1898 shufflePeers/shuffleStrings, randomsub.go:134, gossip_tracer.go:53,
 * peer_gater.go:357).  That stream is not reproducible across Go versions and
 * its consumption order depends on map iteration order, so every draw is
 * replaced by Philox4x32-10 (Salmon et al., SC'11; Random123 reference
 * constants) keyed by (seed, site) with a 4-word counter naming the draw:
 *
 *   key64(seed, site, a, b, c, d) = hi32:x0 | lo32:x1 of
 *                                   philox4x32_10({a,b,c,d}, {seed, site})
 *
 * "shuffle then take k" (getPeers, emitGossip, handleIHave, Dhi pruning) is
 * canonicalised as "sort ascending by key64, ties by element index, take k";
 * the key counters for each call site are listed with GS_SITE_* below.  The
 * oracle (oracle/) and the HIP kernels include this one header so the stream
 * is identical bit for bit.  Pinned by the Random123 known-answer vectors in
 * tests/test_rng.py.
 */
#ifndef GS_RNG_H
#define GS_RNG_H
#include <stdint.h>

#if defined(__HIPCC__)
#define GS_HD __host__ __device__ __forceinline__
#else
#define GS_HD static inline
#endif

/* call sites (key word 1).  Counter words documented per site. */
enum {
  GS_SITE_RANDOMSUB = 1,       /* {node, msg_id, peer, 0}   randomsub.go:134 */
  GS_SITE_GP_JOIN = 2,         /* {node, hop, peer, topic}  gossipsub.go:1032/1046 */
  GS_SITE_GP_FANOUT_PUB = 3,   /* {node, hop, peer, topic}  gossipsub.go:983 */
  GS_SITE_GP_DLO = 4,          /* {node, hop, peer, topic}  gossipsub.go:1362 */
  GS_SITE_GP_DOUT = 5,         /* {node, hop, peer, topic}  gossipsub.go:1452 */
  GS_SITE_GP_OPPORTUNISTIC = 6,/* {node, hop, peer, topic}  gossipsub.go:1486 */
  GS_SITE_GP_FANOUT_HB = 7,    /* {node, hop, peer, topic}  gossipsub.go:1527 */
  GS_SITE_DHI_SHUFFLE = 8,     /* {node, hop, peer, topic}  gossipsub.go:1380 */
  GS_SITE_DHI_TAIL = 9,        /* {node, hop, peer, topic}  gossipsub.go:1387 */
  GS_SITE_EMIT_PEERS = 10,     /* {node, hop, peer, topic}  gossipsub.go:1695 */
  GS_SITE_EMIT_MIDS = 11,      /* {node, peer, msg_id, hop} gossipsub.go:1707 (gs_key64_mid) */
  GS_SITE_IWANT = 12,          /* {node, peer, msg_id, hop} gossipsub.go:663, gossip_tracer.go:53 (gs_key64_mid) */
  GS_SITE_GATER = 13,          /* {node, peer, hop, 0}      peer_gater.go:357 */
  GS_SITE_PX = 14,             /* {node, hop, peer, pruned << 6 | topic}  gossipsub.go:1813 makePrune's
                                  getPeers (a fresh shuffle per PRUNE: keyed by the pruned peer too) */
  GS_SITE_PX_CONNECT = 15      /* {node, hop, peer, 0}      gossipsub.go:858 pxConnect's shufflePeerInfo */
};

GS_HD void gs_mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

/* Philox4x32 with 10 rounds; ctr/key in, out[4] out. */
GS_HD void gs_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    gs_mulhilo32(0xD2511F53u, c0, &hi0, &lo0);
    gs_mulhilo32(0xCD9E8D57u, c2, &hi1, &lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n1 = lo1;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    uint32_t n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

GS_HD uint64_t gs_key64(uint32_t seed, uint32_t site, uint32_t a, uint32_t b, uint32_t c,
                        uint32_t d) {
  uint32_t ctr[4] = {a, b, c, d};
  uint32_t key[2] = {seed, site};
  uint32_t out[4];
  gs_philox4x32_10(ctr, key, out);
  return ((uint64_t)out[0] << 32) | (uint64_t)out[1];
}

/* Both 64-bit halves of one block: k[0] = hi32:x0 | lo32:x1 (= gs_key64),
 * k[1] = hi32:x2 | lo32:x3. */
GS_HD void gs_key64x2(uint32_t seed, uint32_t site, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                      uint64_t k[2]) {
  uint32_t ctr[4] = {a, b, c, d};
  uint32_t key[2] = {seed, site};
  uint32_t out[4];
  gs_philox4x32_10(ctr, key, out);
  k[0] = ((uint64_t)out[0] << 32) | (uint64_t)out[1];
  k[1] = ((uint64_t)out[2] << 32) | (uint64_t)out[3];
}

/* The message-id sites (GS_SITE_EMIT_MIDS, GS_SITE_IWANT: counter word c is a
 * message id) use the whole block: the key of id m is half (m & 1) of the
 * block for counter word m >> 1, so ids 2j and 2j + 1 share one Philox
 * evaluation (the receiver's IHAVE cut hashes a sender's whole gossip window:
 * gs_kernels_ctl.h, phase B). */
GS_HD uint64_t gs_key64_mid(uint32_t seed, uint32_t site, uint32_t a, uint32_t b, uint32_t mid,
                            uint32_t d) {
  uint64_t k[2];
  gs_key64x2(seed, site, a, b, mid >> 1, d, k);
  return (mid & 1u) ? k[1] : k[0];
}

/* Uniform double in [0,1) from a key (53 high bits), for rand.Float64 sites. */
GS_HD double gs_key_to_unit(uint64_t k) { return (double)(k >> 11) * (1.0 / 9007199254740992.0); }

#endif /* GS_RNG_H */
