// gs_kernels_ctl.h — control-plane kernels: HandleRPC (phase B) and the
// heartbeat.  One wave per node; per-sender / per-topic work is serialised in
// the canonical order (senders ascending, RPCs in send order, topics
// ascending) because GRAFT acceptance depends on the running mesh size.
#pragma once
#include "gs_device.h"

// handleGraft for one topic from sender edge e (gossipsub.go:713-792).
// Scalar (wave-uniform) code; meshcnt is held by lane t.  Returns true when a
// PRUNE for t must be sent back.
// noPX: set when this GRAFT takes the peer exchange off the RPC's PRUNEs
// (unknown topic, direct peer, backoff, negative score: gossipsub.go:716-775).
__device__ __forceinline__ bool graft_one(const Dev& d, int64_t e, int v, int t, double sc, int64_t now,
                                          int& meshcnt_lane, uint64_t& meshE, bool& dirty, bool& dirtyUp,
                                          bool& noPX) {
  if (!((d.sub[v] >> t) & 1)) {  // unknown topic: ignore
    noPX = true;
    return false;
  }
  if ((meshE >> t) & 1) return false;         // already in mesh
  if (d.direct[e]) {
    noPX = true;
    return true;
  }
  const int64_t bi = tix(d, t, e);
  const int64_t be = d.backoff[bi];
  if (be != 0 && now < be) {
    noPX = true;
    if (d.scoring) {
      d.bp[e] += 1.0;
      const int64_t floodCutoff = be + (d.GraftFloodThreshold - d.PruneBackoff);
      if (now < floodCutoff) d.bp[e] += 1.0;
      d.sdirty[e] = 1;
      dirty = true;
    }
    add_backoff(d, e, t, now, d.PruneBackoff);
    return true;
  }
  if (sc < 0) {
    noPX = true;
    add_backoff(d, e, t, now, d.PruneBackoff);
    return true;
  }
  const int mc = lane_get(meshcnt_lane, t);
  if (mc >= d.Dhi && !d.outbound[e]) {
    add_backoff(d, e, t, now, d.PruneBackoff);
    return true;
  }
  stats_graft(d, e, t, now);
  dirtyUp = true;  // a graft never lowers the score (P1 = 0 at meshTime 0, P3 switched off)
  meshE |= 1ull << t;
  if (lane_id() == 0 && is_traced(d, v)) trace_emit(d, now / d.hop_ns, GS_TRACE_GRAFT, v, d.col[e], t, -1, 3);
  if (lane_id() == t) meshcnt_lane++;
  return false;
}

// handlePrune (gossipsub.go:806-838): tracer.Prune even when the peer is not
// in the mesh, removal, and the sender's backoff.
__device__ __forceinline__ void prune_topics(const Dev& d, int64_t e, int v, uint64_t topics, int64_t now,
                                             int& meshcnt_lane, uint64_t& meshE, bool& dirty) {
  while (topics) {
    const int t = __ffsll((long long)topics) - 1;
    topics &= topics - 1;
    if (!((d.sub[v] >> t) & 1)) continue;
    if (lane_id() == 0 && is_traced(d, v))  // gossipsub.go:817, whether or not p is in the mesh
      trace_emit(d, now / d.hop_ns, GS_TRACE_PRUNE, v, d.col[e], t, -1, 3);
    stats_prune(d, e, t);
    if (d.scoring) dirty = true;
    if ((meshE >> t) & 1) {
      meshE &= ~(1ull << t);
      if (lane_id() == t) meshcnt_lane--;
    }
    // a v1.1 PRUNE carries the sender's backoff in whole seconds; a v1.0 one
    // none, so the receiver's own PruneBackoff applies (handlePrune :819-825)
    add_backoff(d, e, t, now, px_peer(d, e) ? d.PruneRecv : d.PruneBackoff);
  }
}

// ---- peer exchange (GS_FLAG_PEER_EXCHANGE)
// makePrune's score filter Score(xp) >= 0 (gossipsub.go:1813) for the lane's
// connected peer: the live score, exact (one wave-wide score per connected
// peer; PX PRUNEs are rare).  Unscored every peer passes.  Wave-uniform.
__device__ __forceinline__ bool px_score_ok(const Dev& d, int64_t base, int deg, double* lds) {
  if (!d.scoring) return true;
  const int lane = lane_id();
  double s = 0.0;
  unsigned long long m = __ballot(lane < deg && edge_up(d, base + lane));
  while (m) {
    const int j = __ffsll((long long)m) - 1;
    m &= m - 1;
    const double sj = edge_score_wave(d, base + j, lds);
    if (lane == j) s = sj;
  }
  return s >= 0.0;
}
// makePrune's peer list (gossipsub.go:1811-1836) for the PRUNE of topic t to
// v's peer on lane p: getPeers(topic, PrunePeers, xp != p && Score(xp) >= 0)
// (ok: the lane passes the score filter, px_score_ok) with its own shuffle
// (GS_SITE_PX keyed by the pruned peer too).  Wave-uniform; returns the lane
// mask of the list.
__device__ __forceinline__ uint64_t px_sel(const Dev& d, int v, int64_t base, int deg, int t, int64_t hop, int p,
                                           bool ok) {
  const int lane = lane_id();
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const int u = valid ? d.col[e] : 0;
  // getPeers: mesh-capable topic peers only (gossipsub.go:1849)
  const bool cand = ok && valid && lane != p && edge_up(d, e) && mesh_peer(d, e) && ((d.subA[u] >> t) & 1);
  const uint32_t pp = (uint32_t)d.col[base + p];
  const uint64_t key = gs_key64(d.seed, GS_SITE_PX, v, (uint32_t)hop, u, (pp << 6) | (uint32_t)t);
  return __ballot(select_k(cand, key, d.PrunePeers));
}
// Appends the list (lane mask of v's edges) of topic t to the PX record of the
// receiver's in-edge re.  One lane; the record is rewritten into a new arena
// segment (the entries of earlier PRUNEs to the same peer in this hop first).
__device__ __forceinline__ void px_append(const Dev& d, int cur, int64_t re, int t, uint64_t list, int64_t base) {
  const int k = __popcll(list);
  if (!k) return;
  const int64_t old = d.cPx[cur][re];
  const int on = old >= 0 ? (int)(old & 0xFFFFFF) : 0;
  const int64_t oo = old >= 0 ? (old >> 24) : 0;
  const unsigned long long off = pool_take(d, cur, (unsigned long long)(on + k));
  if (off == ~0ull) return;
  for (int q = 0; q < on; ++q) d.pool[cur][off + q] = d.pool[cur][oo + q];
  int w = on;
  for (uint64_t m = list; m; m &= m - 1)
    d.pool[cur][off + w++] = (int32_t)(((uint32_t)t << 26) | (uint32_t)d.col[base + __ffsll((long long)m) - 1]);
  d.cPx[cur][re] = ((int64_t)off << 24) | (int64_t)(on + k);
}
// The PX entries of record rec whose topic is in `topics`: fn(topic, peer).
template <class F>
__device__ __forceinline__ void px_each(const Dev& d, int buf, int64_t rec, uint64_t topics, F&& fn) {
  if (rec < 0) return;
  const int64_t off = rec >> 24;
  const int n = (int)(rec & 0xFFFFFF);
  for (int q = 0; q < n; ++q) {
    const uint32_t x = (uint32_t)d.pool[buf][off + q];
    const int t = (int)(x >> 26);
    if ((topics >> t) & 1) fn(t, (int)(x & 0x3FFFFFF));
  }
}
__device__ __forceinline__ int px_count(const Dev& d, int buf, int64_t rec, uint64_t topics) {
  int n = 0;
  px_each(d, buf, rec, topics, [&](int, int) { ++n; });
  return n;
}
// pxConnect (gossipsub.go:856-905) for the PX records of node v's in-edge
// with the pruned topics `topics`: every suggested peer that v has a slot for
// (an edge of the graph) and is not connected to is dialled (a request for the
// host, connected at the next hop's start).  Wave-uniform.
// The record of an edge holds the lists of every PRUNE its sender made this
// hop (reply and heartbeat RPCs); each call filters it by the topics of one
// RPC.  pxConnect's shuffle-and-truncate to PrunePeers (:857-862) is never
// needed: every list comes from makePrune, which takes at most PrunePeers
// peers (an honest sender; PX is refused together with attacker behaviours).
__device__ __forceinline__ void px_connect(const Dev& d, int v, int64_t base, int deg, int buf, int64_t rec,
                                           uint64_t topics) {
  const int lane = lane_id();
  const int myCol = lane < deg ? d.col[base + lane] : -1;
  px_each(d, buf, rec, topics, [&](int, int xp) {
    const unsigned long long f = __ballot(myCol == xp);
    if (!f || xp == v) return;  // no slot for this connection
    const int j = __ffsll((long long)f) - 1;
    if (edge_up(d, base + j)) return;  // connected already
    if (lane == 0) {
      const unsigned long long k = atomicAdd(d.pxqN, 1ull);
      if ((int64_t)k < d.pxqCap) d.pxq[k] = ((unsigned long long)(uint32_t)v << 32) | (uint32_t)xp;
      else set_err(d, E_POOL);
    }
  });
}

// mcache.peertx entries: slot << 14 | in-edge << 8 | count (slot < 2^14,
// in-edge < 64); keys (count bits 0) are passed as u64 slot << 32 | in-edge << 8.
__device__ __forceinline__ uint32_t ptx_key32(uint64_t key) {
  return ((uint32_t)(key >> 32) << 14) | ((uint32_t)((key >> 8) & 0x3F) << 8);
}
__device__ __forceinline__ int ptx_hash(uint32_t key, int hbits) {
  return (int)((key * 0x9E3779B1u) >> (32 - hbits));
}
// the node's peertx table in HBM
__device__ __forceinline__ uint32_t* ptx_row(const Dev& d, int v) { return d.ptxT + ((int64_t)v << d.ptxBits); }

// k-th set bit (0-based) of m
__device__ __forceinline__ int kth_bit(uint64_t m, int k) {
  for (int i = 0; i < k; ++i) m &= m - 1;
  return __ffsll((long long)m) - 1;
}

// The overflow table (Dev::ptxO) for node v: ++count of key, inserting it
// (ins) if absent; 0 with E_PEERTX when this table is full too.
__device__ __forceinline__ uint64_t ptxo_hash(uint64_t x, int bits) {
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 32;
  return x >> (64 - bits);
}
__device__ __forceinline__ int ptxo_settle(const Dev& d, int v, uint32_t key, bool& ins) {
  const unsigned long long tag = ((unsigned long long)(uint32_t)(v + 1) << 32) | key;
  const uint64_t mask = (1ull << d.ptxOBits) - 1;
  uint64_t hs = ptxo_hash(tag, d.ptxOBits);
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long prev = atomicCAS(&d.ptxO[hs], 0ull, tag | 1ull);
    if (prev == 0ull) {
      atomicAdd(&d.ptxOCnt[0], 1u);
      ins = true;
      return 1;
    }
    if ((prev & ~0xFFull) == tag) {
      const int c = (int)(atomicAdd(&d.ptxO[hs], 1ull) & 0xFFull) + 1;
      if (c > d.GR + 1) atomicAdd(&d.ptxO[hs], ~0ull);  // (-1)
      return c;
    }
    hs = (hs + 1) & mask;
  }
  set_err(d, E_PEERTX);
  return 0;
}
__device__ __forceinline__ int ptxo_count(const Dev& d, int v, uint32_t key) {
  const unsigned long long tag = ((unsigned long long)(uint32_t)(v + 1) << 32) | key;
  const uint64_t mask = (1ull << d.ptxOBits) - 1;
  uint64_t hs = ptxo_hash(tag, d.ptxOBits);
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long cur = __hip_atomic_load(&d.ptxO[hs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0ull) return 0;
    if ((cur & ~0xFFull) == tag) return (int)(cur & 0xFFull);
    hs = (hs + 1) & mask;
  }
  return 0;
}

// ++peertx[slot][edge] (mcache.GetForPeer, mcache.go:66-80) in node v's
// HBM hash, given the outcome `prev` of a first CAS(0 -> key | 1) at the key's
// home slot hs; returns the new count and sets ins when the key was inserted.
// A key that finds the node's table full goes to the overflow table: entries
// only leave at the heartbeat, so a full table stays full for the rest of the
// hop and a key's lookup reaches the overflow table exactly when its insert did.  handleIWant only compares the count
// with GossipRetransmission (GR), so a count is held at GR + 1: an increment
// past it is taken back (the byte peaks at GR + 2; one request list names an
// id once and a requester's two lists are counted one after the other, so no
// two increments of one key race).  Entries are never moved during a hop
// (k_ptx_rebuild compacts the table at the heartbeat), so a key found stays.
__device__ __forceinline__ int ptx_settle(const Dev& d, int v, uint32_t* row, uint32_t key, int hs, uint32_t prev,
                                          bool& ins) {
  const int hmask = (1 << d.ptxBits) - 1;
  int hsl = hs;
  for (int probe = 0; probe <= hmask; ++probe) {
    if (probe > 0) prev = atomicCAS(&row[hsl], 0u, key | 1u);
    if (prev == 0u) {
      ins = true;
      return 1;
    }
    if ((prev & ~0xFFu) == key) {
      const int c = (int)(atomicAdd(&row[hsl], 1u) & 0xFFu) + 1;
      if (c > d.GR + 1) atomicSub(&row[hsl], 1u);
      return c;
    }
    hsl = (hsl + 1) & hmask;
  }
  return ptxo_settle(d, v, key, ins);
}

// the count of key in node v's HBM hash (0 = absent)
__device__ __forceinline__ int ptx_count_g(const Dev& d, int v, uint32_t* row, uint32_t key) {
  const int hmask = (1 << d.ptxBits) - 1;
  int hsl = ptx_hash(key, d.ptxBits);
  for (int probe = 0; probe <= hmask; ++probe) {
    const uint32_t cur = __hip_atomic_load(&row[hsl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0u) return 0;
    if ((cur & ~0xFFu) == key) return (int)(cur & 0xFFu);
    hsl = (hsl + 1) & hmask;
  }
  return ptxo_count(d, v, key);  // (the table is full)
}

// Item b of a per-sender item space (sIt = exclusive prefix of item counts
// over the 64 senders): returns the sender; k = item index within it.
__device__ __forceinline__ int item_sender(const int* sIt, int b, int& k) {
  int lo = 0, hi = 63;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sIt[mid] <= b) lo = mid; else hi = mid - 1;
  }
  k = b - sIt[lo];
  return lo;
}

// Exclusive prefix over the 64 lanes; *total gets the sum.
__device__ __forceinline__ int lane_prefix(int x, int* total) {
  const int incl = wave_incl_sum(x);
  *total = wave_last(incl);
  return incl - x;
}

// The served message ids of request record rec (off << 24 | n) for the RPC
// trace: every id, or with flags (IWANT-spam runs) those whose request was
// served.  put(kind, topic, msg) per id.
template <class P>
__device__ __forceinline__ void put_served(const Dev& d, const int32_t* pool, const uint8_t* flags, int64_t rec,
                                           P& put) {
  const int64_t off = rec >> 24;
  const int n = (int)(rec & 0xFFFFFF);
  for (int q = 0; q < n; ++q)
    if (flags == nullptr || flags[off + q]) {
      const int slot = pool[off + q];
      put(GS_RPC_ITEM_MSG, (int)__umulhi((unsigned)slot, d.stMagic), d.slotMid[slot]);
    }
}

// Phase B — HandleRPC for every control RPC sent to node v in the previous
// hop (gossipsub.go:591-838), one wave per node.
//   step 1 (serial, senders ascending, RPCs in send order: join GRAFTs, reply
//          RPCs, heartbeat RPC): everything whose outcome depends on order —
//          GRAFT acceptance against the running mesh size, PRUNEs, backoff,
//          the live score that gates IHAVE / IWANT handling, peerhave;
//   step 2 (lane-parallel): handleIWant of the gated senders — request lists
//          cut into 16-id items spread over the lanes; peertx counts in an LDS
//          hash (every (message, requester) pair is a distinct key, so the
//          order of the increments does not matter);
//   step 3 (lane-parallel): handleIHave of the gated senders — one item per
//          (sender, advertised subscribed topic); wants = IHAVE payload &
//          ~seen; the promised message (gossip_tracer.go:53) is the sender's
//          (key, mid)-smallest want;
//   step 4: per-edge results and reply RPCs written once.
// Id lists (IWANT requests / responses) are sets: their order in the arena is
// irrelevant to every reader.
// ADV (host-selected: attacker behaviours, validators / gater, phantom ids, or
// a possible MaxIHaveLength cut) compiles in the IWANT-spam replies, silent
// squatters, the dynamic peertx hash, phantom ids and the cuts; the honest
// instantiation carries none of them.
template <int WPL, bool ADV>
__device__ __forceinline__ void phase_b_node(const Dev& d, const int v, int64_t h, int64_t now, int cur, int head,
                                             int cutModeArg) {
  const int cutMode = cutModeArg;  // bit 0: a topic's item may be cut; bit 1: a sender's wants may be cut
  if (!gossip_host(d, v)) return;  // FloodSubRouter / RandomSubRouter.HandleRPC: no-ops
  __shared__ uint64_t scache[64 * WPL];  // v's mcache windows (handleIWant, step 2)
  uint64_t* const sseen = scache;        // then v's seen row (handleIHave, step 3)
  __shared__ __attribute__((aligned(16))) unsigned int sH[768];  // step 3's per-sender arrays
  __shared__ double sterm[64];
  __shared__ int sIt[64];                // per-sender exclusive item prefix
  __shared__ int sReqOff[64], sReqN[64]; // step 2: request list of each sender
  __shared__ int sOut[64];               // step 2/3: where each sender's id list starts
  __shared__ int sCnt[64], sCur[64];     // per-sender id counts / write cursors
  __shared__ unsigned long long sBase;
  int* const sNode = (int*)sH;                                  // step 3: sender node
  uint64_t* const sTm = (uint64_t*)(sH + 64);                   // step 3: advertised subscribed topics
  unsigned long long* const sKey = (unsigned long long*)(sH + 192);
  long long* const sMid = (long long*)(sH + 320);
  int* const sSlot = (int*)(sH + 448);
  uint32_t* const sHas = (uint32_t*)(sH + 512);  // step 3: items with a want (<= 64 senders x 64 items)
  uint32_t* const sCand = (uint32_t*)(sH + 640); // step 3: items that held their sender's smallest key
  static_assert(640 + 64 * 64 / 32 <= 768, "step-3 arrays must fit in sH");
  const int lane = lane_id();
  GS_STAMPB_CLEAR();
  const int prv = cur ^ 1;
  const int W = d.W;
  const int Wt = d.Wt;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  // ---- per-sender control words (lane = in-edge), read before any store
  int64_t r = 0;
  int npre = 0, hb = 0;
  if (valid) {
    r = rxi(d, e, d.rev[e]);  // where v's replies to this sender go (its in-edge, or the stage slot)
    npre = d.cPre[prv][e];
    hb = d.cHb[prv][e];
  }
  const bool ctl = npre != 0 || hb != 0;
  const unsigned long long cmask = __ballot(ctl);
  if (!cmask) return;
  uint64_t gJoin = 0, gHb = 0, pRep = 0, pHb = 0, ihaveT = 0, meshE = 0;
  int64_t iwRec = -1, spRec = -1;
  int ph = 0, ia = 0, u = 0;
  double sc = 0.0;
  bool gl = false;
  if (valid) meshE = d.mesh[e];
  if (ctl) {
    gJoin = d.cGraftJoin[prv][e];
    gHb = d.cGraftHb[prv][e];
    pRep = d.cPruneReply[prv][e];
    pHb = d.cPruneHb[prv][e];
    ihaveT = d.cIhave[prv][e];
    iwRec = d.cIwant[prv][e];
    if (ADV && d.cSpam[prv] != nullptr) spRec = d.cSpam[prv][e];  // IWANT spam RPC (an extra reply-group RPC)
    ph = d.peerhave[e];
    ia = d.iasked[e];
    u = d.col[e];
    if (d.scoring) {
      sc = d.score1[e];
      gl = !d.direct[e] && d.score0[e] < d.graylistThr;  // AcceptFrom on the hop-start memo
    }
  }
  GS_STAMPB(0);
  // lane t: current mesh size of topic t
  int meshcnt = 0;
  for (int t = 0; t < d.T; ++t) {
    const int c = __popcll(__ballot((meshE >> t) & 1));
    if (lane == t) meshcnt = c;
  }
  // ---- step 1: order-dependent control, senders ascending.  Only GRAFTs and
  // PRUNEs depend on the order (the running mesh size, backoff, the live
  // score); a sender whose RPCs carry neither is handled in its own lane.
  bool gateIWant = false, gateIHave = false, prunesHb = false, gateSpam = false;
  uint64_t pruneOut = 0;
  uint64_t joinRej = 0, hbPr = 0;  // RPC accounting: the join GRAFTs answered by a PRUNE, the heartbeat RPC's
  int nRep1 = 0;
  long long cPrunes = 0, cGray = 0;
  const bool heavy = ctl && !gl && (gJoin | gHb | pRep | pHb) != 0;
  if (ctl && gl) cGray = npre + hb;  // AcceptNone: the whole RPC is dropped
  if (ctl && !gl && !heavy) {
    // (2) reply RPCs (IWANT requests), (3) heartbeat RPC (IHAVE)
    if (npre > 0) {
      const bool gossipOK = sc >= d.gossipThr;
      if (gossipOK) ph += npre;
      gateIWant = gossipOK && iwRec >= 0;  // handleIWant (gossipsub.go:674-711): step 2
      gateSpam = gossipOK && spRec >= 0;
    }
    if (hb && sc >= d.gossipThr) {
      ph++;
      // handleIHave gates (gossipsub.go:612-628); only topics in our mesh map count (:633)
      gateIHave = ph <= d.MaxIHaveMessages && ia < d.MaxIHaveLength && (ihaveT & sv) != 0;
    }
  }
  {
    unsigned long long m = __ballot(heavy);
    while (m) {
      const int i = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int npre_i = lane_get(npre, i), hb_i = lane_get(hb, i);
      const int64_t ei = base + i;
      const uint64_t gJoin_i = lane_get64(gJoin, i), gHb_i = lane_get64(gHb, i);
      const uint64_t pRep_i = lane_get64(pRep, i), pHb_i = lane_get64(pHb, i), ihaveT_i = lane_get64(ihaveT, i);
      const int64_t iwRec_i = (int64_t)lane_get64((uint64_t)iwRec, i);
      const int64_t spRec_i = (int64_t)lane_get64((uint64_t)spRec, i);
      int ph_i = lane_get(ph, i);
      const int ia_i = lane_get(ia, i);
      double sc_i = lane_getf(sc, i);
      uint64_t mE = lane_get64(meshE, i);
      bool dirty = false;    // the score may have dropped since sc_i
      bool dirtyUp = false;  // the score may have risen since sc_i (grafts)
      // every decision below compares sc_i with 0 or GossipThreshold (<= 0): a
      // stale value >= 0 that can only have risen decides exactly
      auto fresh = [&]() {
        if (dirty || (dirtyUp && !(sc_i >= 0.0))) sc_i = edge_score_wave(d, ei, sterm);
        dirty = dirtyUp = false;
      };
      uint64_t pOut = 0;
      int nR = 0;
      const int64_t reI = d.doPX ? rxi(d, ei, d.rev[ei]) : 0;  // the sender's in-edge: our PX record for it
      // makePrune with PX for the rejected topics of one RPC (live scores)
      auto pxPrunes = [&](uint64_t topics) {
        if (!topics) return;
        const bool ok = px_score_ok(d, base, deg, sterm);
        for (uint64_t mm = topics; mm; mm &= mm - 1) {
          const int t = __ffsll((long long)mm) - 1;
          const uint64_t list = px_sel(d, v, base, deg, t, h, i, ok);
          if (lane == 0) px_append(d, cur, reI, t, list, base);
        }
      };
      // handlePrune's PX acceptance (gossipsub.go:807, 827-836): the sender's
      // live score before the RPC's PRUNEs against AcceptPXThreshold
      auto pxAccept = [&](uint64_t topics) {
        if (!d.doPX || !topics || d.cPx[prv][ei] < 0) return false;
        const double sx = d.scoring ? edge_score_wave(d, ei, sterm) : 0.0;
        return !(sx < d.acceptPX);
      };
      // (1) Join RPCs: one GRAFT each (gossipsub.go:1080-1084)
      uint64_t gj = gJoin_i;
      while (gj) {
        const int t = __ffsll((long long)gj) - 1;
        gj &= gj - 1;
        fresh();
        if (sc_i >= d.gossipThr) ph_i++;  // handleIHave's counter (no IHAVE entries)
        bool pr, noPX = false;
        pr = graft_one(d, ei, v, t, sc_i, now, meshcnt, mE, dirty, dirtyUp, noPX);
        if (pr) {
          pOut |= 1ull << t;
          nR++;
          if (d.doPX && !noPX && px_peer(d, ei)) pxPrunes(1ull << t);  // this RPC's PRUNE reply carries PX
        }
      }
      // (2) reply RPCs: IWANT requests and PRUNEs answering our own control
      bool gIW = false, gSP = false;
      const int nRep = npre_i - __popcll(gJoin_i);
      if (nRep > 0) {
        fresh();
        const bool gossipOK = sc_i >= d.gossipThr;
        if (gossipOK) ph_i += nRep;
        gIW = gossipOK && iwRec_i >= 0;  // handleIWant (gossipsub.go:674-711): step 2
        gSP = gossipOK && spRec_i >= 0;
        const bool acc = pxAccept(pRep_i & d.sub[v]);
        prune_topics(d, ei, v, pRep_i, now, meshcnt, mE, dirty);
        if (acc) px_connect(d, v, base, deg, prv, d.cPx[prv][ei], pRep_i & d.sub[v]);  // the PRUNEs' PX
      }
      // (3) heartbeat RPC: IHAVE (step 3), GRAFT, PRUNE
      bool gIH = false;
      uint64_t prunes = 0;
      if (hb_i) {
        fresh();
        if (sc_i >= d.gossipThr) {
          ph_i++;
          // handleIHave gates (gossipsub.go:612-628); only topics in our mesh map count (:633)
          gIH = ph_i <= d.MaxIHaveMessages && ia_i < d.MaxIHaveLength && (ihaveT_i & sv) != 0;
        }
        uint64_t g = gHb_i;
        bool noPX = false;  // one doPX for the whole heartbeat RPC (gossipsub.go:716)
        while (g) {
          const int t = __ffsll((long long)g) - 1;
          g &= g - 1;
          bool pr;
          pr = graft_one(d, ei, v, t, sc_i, now, meshcnt, mE, dirty, dirtyUp, noPX);
          if (pr) prunes |= 1ull << t;
        }
        if (d.doPX && !noPX && px_peer(d, ei)) pxPrunes(prunes);
        const bool acc = pxAccept(pHb_i & d.sub[v]);
        prune_topics(d, ei, v, pHb_i, now, meshcnt, mE, dirty);
        if (acc) px_connect(d, v, base, deg, prv, d.cPx[prv][ei], pHb_i & d.sub[v]);
      }
      const uint64_t jrej = pOut;
      pOut |= prunes;
      if (lane == i) {
        joinRej = jrej;
        hbPr = prunes;
        meshE = mE;
        ph = ph_i;
        pruneOut = pOut;
        nRep1 = nR;
        gateIWant = gIW;
        gateSpam = gSP;
        gateIHave = gIH;
        prunesHb = prunes != 0;
      }
      cPrunes += __popcll(pOut);
    }
  }

  GS_STAMPB(1);
  const bool silent = ADV && behaves(d, v, GS_BEHAVE_NO_FORWARD);  // a squatter serves nothing, sends nothing
  if (silent) gateIWant = gateSpam = false;
  // ---- step 2: handleIWant — serve cached messages at most GossipRetransmission
  // times per peer; the IHAVE-reply list and the IWANT-spam list of a sender
  // are two RPCs (two replies), served from one peertx table
  int64_t respRec = -1;
  long long cServed = 0;
  int nSrv = 0;  // reply RPCs carrying served messages to this sender
  int srvR = 0, srvS = 0;  // messages served for the sender's IWANT list / its IWANT-spam list
  __shared__ uint32_t sSrvB[64], sSrvBS[64];  // RPC accounting: served message bytes per list
  uint32_t srvB = 0, srvBS = 0;
  if (__ballot(gateIWant || gateSpam)) {
    __shared__ int sSpOff[64], sSpN[64], sItI[64], sCntS[64], sRow[64];
    uint32_t* const prow = ptx_row(d, v);  // v's peertx table (HBM hash)
    const int nI = gateIWant ? (int)(iwRec & 0xFFFFFF) : 0;
    const int nS = gateSpam ? (int)(spRec & 0xFFFFFF) : 0;
    __shared__ uint64_t sNeedW[GS_MAX_WPL];  // the mcache words the requests name (bit per word)
    if (lane < GS_MAX_WPL) sNeedW[lane] = 0ull;
    const int itI = (nI + 15) >> 4, itS = (nS + 15) >> 4;
    int totalItems;
    sIt[lane] = lane_prefix(itI + itS, &totalItems);
    sReqOff[lane] = gateIWant ? (int)(iwRec >> 24) : 0;
    sReqN[lane] = nI;
    sSpOff[lane] = gateSpam ? (int)(spRec >> 24) : 0;
    sSpN[lane] = nS;
    sItI[lane] = itI;
    sSrvB[lane] = 0u;
    sSrvBS[lane] = 0u;
    sRow[lane] = (ADV && d.spamRow != nullptr && valid) ? d.spamRow[e] : -1;  // a spammer's counts: spamCnt
    sCnt[lane] = 0;
    sCntS[lane] = 0;
    sCur[lane] = 0;
    __syncthreads();
#ifdef GS_STAMPS_PB2
    GS_STAMPB(5);
#endif
    // item b: 16 ids of the IHAVE-reply list (k < itI) or of the spam list
    auto item = [&](int b, int& i, int& off, int& cnt, bool& sp) {
      int k;
      i = item_sender(sIt, b, k);
      sp = k >= sItI[i];
      if (sp) {
        k -= sItI[i];
        off = sSpOff[i] + 16 * k;
        cnt = min(16, sSpN[i] - 16 * k);
      } else {
        off = sReqOff[i] + 16 * k;
        cnt = min(16, sReqN[i] - 16 * k);
      }
    };
    // the request ids of an item, four loads in flight: fn(q, slot)
    const int32_t* const req = prv ? d.pool[1] : d.pool[0];
    auto ids = [&](int off, int cnt, auto&& fn) {
      for (int q0 = 0; q0 < cnt; q0 += 4) {
        int sl[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) sl[q] = q0 + q < cnt ? req[off + q0 + q] : -1;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (sl[q] >= 0) fn(q0 + q, sl[q]);
      }
    };
    // mcache.GetForPeer finds the id (mcache.go:66-80); a phantom id is never served
    auto cached = [&](int slot) {
      return ((scache[slot >> 6] >> (slot & 63)) & 1) && !(ADV && d.slotKind[slot] == GS_MSG_PHANTOM);
    };
    // v's mcache windows (HistoryLength windows ORed) for the words the
    // requests name only: a node serves a few dozen ids, not W words' worth
    for (int b = lane; b < totalItems; b += 64) {
      int i, off, cnt;
      bool sp;
      item(b, i, off, cnt, sp);
      ids(off, cnt, [&](int, int slot) {
        const int w = slot >> 6;
        atomicOr((unsigned long long*)&sNeedW[w >> 6], 1ull << (w & 63));
      });
    }
    __syncthreads();
    int nW = 0;  // needed words
#pragma unroll
    for (int j = 0; j < GS_MAX_WPL; ++j) nW += __popcll(sNeedW[j]);
    for (int w = lane; w < W; w += 64)
      if ((sNeedW[w >> 6] >> (w & 63)) & 1) scache[w] = 0ull;
    __syncthreads();
    // one (needed word, window) load per lane: every load in flight at once
    for (int p = lane; p < nW * d.HL; p += 64) {
      const int wi = p / d.HL, k = p - wi * d.HL;
      int j = 0, r = wi;
      while (r >= __popcll(sNeedW[j])) r -= __popcll(sNeedW[j++]);
      const int w = 64 * j + kth_bit(sNeedW[j], r);
      const uint64_t x = d.hist[((int64_t)((head + k) % d.R) * d.nOwnH + (v - d.n0)) * W + w];
      if (x) atomicOr((unsigned long long*)&scache[w], x);
    }
    __syncthreads();
#ifdef GS_STAMPS_PB2
    GS_STAMPB(6);
#endif
    // pass a: increments and per-sender served counts.  A spammer's two lists
    // may name the same message (a copy dropped by the validation queue stays
    // unseen, so it is asked for again after the IHAVE): its re-request RPC was
    // sent first (phase A of the previous hop), so that list is counted first.
    // Each request's verdict is kept for pass b, which walks the same items in
    // the same lanes: 16 bits per item in a register for a lane's first 4
    // items, in pflag (IWANT-spam runs) past them.
    uint64_t vbits = 0;
    int nIns = 0;  // keys inserted into the peertx table
    const bool flags = ADV && d.pflag[0] != nullptr;  // also read by the RPC trace (step 4)
    // (without flags an item past a lane's fourth is looked up again in pass
    // b: an id is asked for at most once per hop, so its count is the verdict)
    auto verdict = [&](int b, int q, int off, bool srv) {
      const int j = (b - lane) >> 6;
      if (flags) d.pflag[prv][off + q] = srv ? 1 : 0;
      if (j < 4 && srv) vbits |= 1ull << (16 * j + q);
    };
    auto passA = [&](int which) {  // 0: IHAVE-reply lists, 1: spam lists
      for (int b = lane; b < totalItems; b += 64) {
        int i, off, cnt;
        bool sp;
        item(b, i, off, cnt, sp);
        if (sp != (which == 1)) continue;
        int c = 0;
        if (ADV && sRow[i] >= 0) {
          // a spammer's counts in HBM: the adds of four requests issued back to
          // back (independent words or nibbles), then their few take-backs
          for (int q0 = 0; q0 < cnt; q0 += 4) {
            int sl[4], cn[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) sl[q] = q0 + q < cnt ? req[off + q0 + q] : -1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              cn[q] = 0;
              if (sl[q] >= 0 && cached(sl[q]))
                cn[q] = (int)((atomicAdd(spam_word(d, sRow[i], sl[q]), 1u << ((sl[q] & 7) * 4)) >> ((sl[q] & 7) * 4)) & 0xF) + 1;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (cn[q] > d.GR + 1) atomicSub(spam_word(d, sRow[i], sl[q]), 1u << ((sl[q] & 7) * 4));
              const bool srv = cn[q] >= 1 && cn[q] <= d.GR;
              if (srv) ++c;
              if (q0 + q < cnt) verdict(b, q0 + q, off, srv);
            }
          }
        } else {
          // v's peertx table: the first CAS(0 -> key | 1) of four requests
          // issued back to back, then each settled (found: +1; taken: probe on)
          for (int q0 = 0; q0 < cnt; q0 += 4) {
            int sl[4];
            uint32_t key[4], pv[4];
            int hs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) sl[q] = q0 + q < cnt ? req[off + q0 + q] : -1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const bool go = sl[q] >= 0 && cached(sl[q]);
              key[q] = ptx_key32(((uint64_t)(uint32_t)(go ? sl[q] : 0) << 32) | ((uint64_t)i << 8));
              hs[q] = ptx_hash(key[q], d.ptxBits);
              pv[q] = go ? atomicCAS(&prow[hs[q]], 0u, key[q] | 1u) : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              bool srv = false;
              if (pv[q] != 0xFFFFFFFFu) {
                bool ins = false;
                const int count = ptx_settle(d, v, prow, key[q], hs[q], pv[q], ins);
                nIns += ins ? 1 : 0;
                srv = count >= 1 && count <= d.GR;
              }
              if (srv) ++c;
              if (q0 + q < cnt) verdict(b, q0 + q, off, srv);
            }
          }
        }
        if (c) atomicAdd(sp ? &sCntS[i] : &sCnt[i], c);
      }
    };
    if (ADV && __ballot(nS > 0)) {
      passA(1);
      __syncthreads();
    }
    passA(0);
    __syncthreads();
    {
      const int ins = wave_sum_int(nIns);
      if (lane == 0 && ins) d.ptxN[v] += ins;
    }
    int totalServed;
    const int myServed = sCnt[lane] + sCntS[lane];
    nSrv = (sCnt[lane] > 0 ? 1 : 0) + (sCntS[lane] > 0 ? 1 : 0);
    srvR = sCnt[lane];
    srvS = sCntS[lane];
    const int myOff = lane_prefix(myServed, &totalServed);
    if (lane == 0 && totalServed) sBase = pool_take(d, cur, (unsigned long long)totalServed);
    __syncthreads();
    if (totalServed) {
      const unsigned long long poolBase = sBase;
      if (poolBase == ~0ull) {  // arena full (E_POOL)
        nSrv = 0;
      } else {
        sOut[lane] = (int)poolBase + myOff;
        if (myServed) respRec = ((int64_t)(poolBase + myOff) << 24) | (int64_t)myServed;
        cServed = totalServed;
        __syncthreads();
        // pass b: write the served ids by each request's verdict
        for (int b = lane; b < totalItems; b += 64) {
          int i, off, cnt;
          bool sp;
          item(b, i, off, cnt, sp);
          const int j = (b - lane) >> 6;
          const uint32_t vb = j < 4 ? (uint32_t)(vbits >> (16 * j)) & 0xFFFFu : 0u;
          if (j < 4 && vb == 0u) continue;
          ids(off, cnt, [&](int q, int slot) {
            bool srv;
            if (j < 4) {
              srv = ((vb >> q) & 1) != 0;
            } else if (flags) {
              srv = d.pflag[prv][off + q] != 0;
            } else {
              const uint32_t key = ptx_key32(((uint64_t)(uint32_t)slot << 32) | ((uint64_t)i << 8));
              const int count = cached(slot) ? ptx_count_g(d, v, prow, key) : 0;
              srv = count >= 1 && count <= d.GR;
            }
            if (srv) {
              d.pool[cur][sOut[i] + atomicAdd(&sCur[i], 1)] = slot;
              if (d.rpcB != nullptr)
                atomicAdd(sp ? &sSrvBS[i] : &sSrvB[i], (uint32_t)d.acc[(int)__umulhi((unsigned)slot, d.stMagic)].msgF);
            }
          });
        }
      }
    }
    __syncthreads();
#ifdef GS_STAMPS_PB2
    GS_STAMPB(7);
#endif
    srvB = sSrvB[lane];
    srvBS = sSrvBS[lane];
    __syncthreads();  // sH is reused by step 3
  }

  GS_STAMPB(2);
  // ---- step 3: handleIHave — IWANT the unseen advertised messages of our topics
  int64_t iwantRec = -1;
  bool iwantAny = false;
  long long cIwantSent = 0;
  const unsigned long long ihMask = __ballot(gateIHave);
  if (ihMask) {
    for (int w = lane; w < W; w += 64) sseen[w] = d.seen[(int64_t)v * W + w];
    const uint64_t tm = gateIHave ? (ihaveT & sv) : 0ull;
    int totalItems;
    // An item is (sender, topic), or with long topic windows (Wt > 16 words,
    // config3's 157) (sender, topic, 16-word chunk), so the lanes share the
    // words of one topic; a cut is decided per (sender, topic) item tb = b / nCh
    // and applied to each of its chunks.  At most 64 items per sender.
    const int nCh = Wt <= 16 ? 1 : (Wt + 15) >> 4;
    sIt[lane] = lane_prefix(__popcll(tm) * nCh, &totalItems);
    sTm[lane] = tm;
    sNode[lane] = u;
    sCnt[lane] = 0;
    sCur[lane] = 0;
    __syncthreads();
    const int nHas = (totalItems + 31) >> 5;
    // ---- MaxIHaveLength cuts (cutMode: the host saw that a topic may hold
    // more gossip ids than that).  Item cut: a sender with more than
    // MaxIHaveLength ids of a topic advertised its own keyed subset to v
    // (emitGossip, gossipsub.go:1702-1709: the MaxIHaveLength smallest
    // (GS_SITE_EMIT_MIDS key, id) of its heartbeat hop h - 1).  Sender cut:
    // more wants than MaxIHaveLength - iasked are cut to the smallest
    // (GS_SITE_IWANT key, id) (handleIHave, :650-653).
    extern __shared__ __attribute__((aligned(16))) uint32_t smemB[];
    uint32_t* const cHist = smemB;                                  // [256] radix histogram
    int* const cPre = (int*)(smemB + 256);                          // [128] cut bits below word j
    unsigned long long* const cK = (unsigned long long*)(smemB + 256 + 128);  // [GS_CUTS] threshold key
    long long* const cM = (long long*)(cK + GS_CUTS);               // [GS_CUTS] threshold id
    unsigned long long* const iK = (unsigned long long*)(cM + GS_CUTS);  // [64] sender cut key
    long long* const iM = (long long*)(iK + 64);                   // [64] sender cut id
    uint32_t* const cBits = (uint32_t*)(iM + 64);                   // [128] item is cut
    int* const cN = (int*)(cBits + 128);
    unsigned long long* const cSp = (unsigned long long*)(cN + 2);  // first spilled entry of this node
    // the item cuts' scratch lives in static LDS that is free until pass a:
    // select_kth_est's kept (key, id) pairs + counter in sH past sTm (sKey ..
    // sCand are initialised after the cuts)
    unsigned long long* const cand = (unsigned long long*)(sH + 192);
    static_assert(192 * 4 + GS_SEL_CAP * 16 + 8 <= 768 * 4, "select_kth_est pairs must fit in sH past sTm");
    // A cut item's index c is its rank among the cut bits (item order); c <
    // GS_CUTS keeps its threshold in LDS, the rest in the rank's spill table
    // from *cSp on (emitGossip truncates every over-length item,
    // gossipsub.go:1700-1710, however many reach one node)
    int nCut = 0;
    unsigned long long spill0 = 0;
    if (cutMode & 1) {
      for (int k = lane; k < 128; k += 64) cBits[k] = 0u;
      if (lane == 0) *cN = 0;
      __syncthreads();
      // cuts are per (sender, topic): topic item tb covers items tb*nCh ..
      const int totalT = totalItems / nCh;
      // an item's id count: long topic windows (config3's 157 words) are
      // summed by the whole wave, item after item; short ones lane per item
      const bool waveSum = Wt > 16;
      for (int tb = waveSum ? 0 : lane; tb < totalT; tb += waveSum ? 1 : 64) {
        int k;
        const int i = item_sender(sIt, tb * nCh, k);
        const int t = kth_bit(sTm[i], k / nCh);
        const int uu = sNode[i];
        int nm = 0;
        if (waveSum) {
          for (int w = t * Wt + lane; w < (t + 1) * Wt; w += 64) nm += __popcll(d.gw[(int64_t)uu * W + w]);
          nm = wave_last(wave_incl_sum(nm));
        } else {
          for (int w = t * Wt; w < (t + 1) * Wt; ++w) nm += __popcll(d.gw[(int64_t)uu * W + w]);
        }
        if (nm > d.MaxIHaveLength && (!waveSum || lane == 0)) {
          atomicAdd(cN, 1);
          atomicOr(&cBits[tb >> 5], 1u << (tb & 31));
        }
      }
      __syncthreads();
      nCut = *cN;
      {
        int tot0, tot1;
        const int p0 = lane_prefix(__popc(cBits[lane]), &tot0);
        const int p1 = lane_prefix(__popc(cBits[lane + 64]), &tot1);
        cPre[lane] = p0;
        cPre[lane + 64] = tot0 + p1;
      }
      if (nCut > GS_CUTS) {
        if (lane == 0) {
          const unsigned long long b = atomicAdd(d.cutSpN, (unsigned long long)(nCut - GS_CUTS));
          *cSp = b;
          if (b + (unsigned long long)(nCut - GS_CUTS) > (unsigned long long)GS_CUTSPILL) set_err(d, E_TRUNCATE);
        }
      }
      __syncthreads();
      if (nCut > GS_CUTS) spill0 = *cSp;
      int cw = 0;
      uint32_t cb = cBits[0];
      for (int c = 0; c < nCut; ++c) {
        while (cb == 0u) cb = cBits[++cw];  // the c-th cut item in item order
        const int tb = cw * 32 + __ffs(cb) - 1;
        cb &= cb - 1u;
        int k;
        const int i = item_sender(sIt, tb * nCh, k);
        const int t = kth_bit(sTm[i], k / nCh);
        const int uu = sNode[i];
        const uint64_t* const g = d.gw + (int64_t)uu * W + t * Wt;  // the sender's words of topic t
        int nm = 0;  // its ids
        for (int w = lane; w < Wt; w += 64) nm += __popcll(g[w]);
        nm = wave_last(wave_incl_sum(nm));
        unsigned long long K;
        long long M;
        // every gossip id of the sender's topic t in word order, by units: a
        // unit is a slot pair (2j, 2j + 1) with at least one of the two in the
        // window.  Lane l takes the units of rank [l n / 64, (l + 1) n / 64), the
        // same count per lane (a word-strided split leaves a third of the lanes
        // with one word more).  A slot pair holds a message-id pair (2m, 2m + 1)
        // whenever a topic's ids fill its slots in order (one topic: slot = id
        // mod St, St even), and then one Philox block keys both ids
        // (gs_key64_mid); an unpaired neighbour takes a block of its own.
        auto units = [](uint64_t x) { return (x | (x >> 1)) & 0x5555555555555555ull; };
        int pre[GS_MAX_WPL];  // units before word 64 j + lane
        int n = 0;
#pragma unroll
        for (int j = 0; j < GS_MAX_WPL; ++j) {
          const int w = 64 * j + lane;
          const int pc = w < Wt ? __popcll(units(g[w])) : 0;
          const int incl = wave_incl_sum(pc);
          pre[j] = n + incl - pc;
          n += wave_last(incl);
        }
        auto preAt = [&](int w) {  // (all lanes: the shuffles read every lane)
          int x = 0;
#pragma unroll
          for (int j = 0; j < GS_MAX_WPL; ++j) {
            const int y = __shfl(pre[j], w & 63);
            if ((w >> 6) == j) x = y;
          }
          return x;
        };
        const int r0 = (int)((int64_t)lane * n / 64), r1 = (int)((int64_t)(lane + 1) * n / 64);
        // the first word holding rank r0: the last w with pre(w) <= r0
        int lo = 0, hi = Wt - 1;
        while (__ballot(lo < hi)) {
          const int mid = (lo + hi + 1) >> 1;
          const int pm = preAt(lo < hi ? mid : lo);
          if (lo < hi) {
            if (pm <= r0) lo = mid; else hi = mid - 1;
          }
        }
        const int wS = lo;
        const uint64_t gS = r0 < r1 ? g[wS] : 0ull;
        uint64_t yS = units(gS);
        for (int sk = r0 - preAt(wS); sk > 0; --sk) yS &= yS - 1;  // the units of lower lanes
#ifndef GS_CUTQ
#define GS_CUTQ 8  // units (one 16-byte message-id load, one key block each) in flight per lane
#endif
        const uint32_t hk = (uint32_t)(h - 1);
        auto each = [&](auto&& fn) {
          int w = wS;
          uint64_t gc = gS, y = yS, ng = (r0 < r1 && wS + 1 < Wt) ? g[wS + 1] : 0ull;
          for (int r = r0; r < r1; r += GS_CUTQ) {
            int bs[GS_CUTQ], ws[GS_CUTQ];
            uint32_t pr[GS_CUTQ];  // the unit's slots in the window: bit 0 slot 2j, bit 1 slot 2j + 1
#pragma unroll
            for (int q = 0; q < GS_CUTQ; ++q) {
              bs[q] = -1;
              ws[q] = w;
              pr[q] = 0;
              if (r + q < r1) {
                while (y == 0) {  // (rank r + q exists: some later word holds it)
                  ++w;
                  gc = ng;
                  y = units(gc);
                  ng = w + 1 < Wt ? g[w + 1] : 0ull;
                }
                bs[q] = __ffsll((long long)y) - 1;
                ws[q] = w;
                pr[q] = (uint32_t)(gc >> bs[q]) & 3u;
                y &= y - 1;
              }
            }
            int64_t m0[GS_CUTQ], m1[GS_CUTQ];
#pragma unroll
            for (int q = 0; q < GS_CUTQ; ++q) {
              m0[q] = m1[q] = 0;
              if (bs[q] >= 0) {  // both ids of the pair (bs even: a 16-byte aligned load)
                const int4 p = *reinterpret_cast<const int4*>(d.slotMid + (int64_t)(t * Wt + ws[q]) * 64 + bs[q]);
                m0[q] = (int64_t)(((uint64_t)(uint32_t)p.y << 32) | (uint32_t)p.x);
                m1[q] = (int64_t)(((uint64_t)(uint32_t)p.w << 32) | (uint32_t)p.z);
              }
            }
#pragma unroll
            for (int q = 0; q < GS_CUTQ; ++q) {
              if (bs[q] < 0) continue;
              const int64_t ma = (pr[q] & 1u) ? m0[q] : m1[q];
              uint64_t kb[2];
              gs_key64x2(d.seed, GS_SITE_EMIT_MIDS, uu, v, (uint32_t)ma >> 1, hk, kb);
              fn((ma & 1) ? kb[1] : kb[0], ma);
              if (pr[q] == 3u) {
                const int64_t mb = m1[q];
                fn(((uint32_t)mb >> 1) == ((uint32_t)ma >> 1) ? ((mb & 1) ? kb[1] : kb[0])
                                                             : gs_key64_mid(d.seed, GS_SITE_EMIT_MIDS, uu, v, (uint32_t)mb, hk),
                   mb);
              }
            }
          }
        };
        select_kth_est(each, d.MaxIHaveLength, nm, cHist, cand, K, M);
        if (lane == 0) {
          if (c < GS_CUTS) {
            cK[c] = K;
            cM[c] = M;
          } else if (spill0 + (unsigned long long)(c - GS_CUTS) < (unsigned long long)GS_CUTSPILL) {
            d.cutSpK[spill0 + (c - GS_CUTS)] = K;
            d.cutSpM[spill0 + (c - GS_CUTS)] = M;
          }
        }
        __syncthreads();
      }
    }
    // item tb's cut threshold (K, M); false: tb is not cut
    auto cutOf = [&](int tb, unsigned long long& K, long long& M) {
      if (!nCut) return false;
      const uint32_t wb = cBits[tb >> 5];
      if (!((wb >> (tb & 31)) & 1u)) return false;
      const int c = cPre[tb >> 5] + __popc(wb & ((1u << (tb & 31)) - 1u));
      if (c < GS_CUTS) {
        K = cK[c];
        M = cM[c];
      } else {
        const unsigned long long s = spill0 + (unsigned long long)(c - GS_CUTS);
        const bool in = s < (unsigned long long)GS_CUTSPILL;  // (else E_TRUNCATE is set)
        K = in ? d.cutSpK[s] : ~0ull;
        M = in ? (long long)d.cutSpM[s] : INT64_MAX;
      }
      return true;
    };
    // (sH past sTm was the cuts' scratch until here)
    sKey[lane] = ~0ull;
    sMid[lane] = INT64_MAX;
    sSlot[lane] = -1;
    for (int k = lane; k < nHas; k += 64) sHas[k] = sCand[k] = 0u;
    __syncthreads();
    // the advertised wants of item b (topic t, chunk ch): fn(w, want) per word
    // with a want
    auto wants = [&](int b, int uu, int t, int ch, auto&& fn) {
      unsigned long long K = 0;
      long long M = 0;
      const bool cut = cutOf(b / nCh, K, M);  // the (sender, topic) item's cut
      const int wBeg = nCh > 1 ? t * Wt + 16 * ch : t * Wt;
      const int wEnd = nCh > 1 ? min(wBeg + 16, (t + 1) * Wt) : (t + 1) * Wt;
      for (int w0 = wBeg; w0 < wEnd; w0 += 4) {
        uint64_t g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = d.gw[(int64_t)uu * W + min(w0 + q, wEnd - 1)];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint64_t want = w0 + q < wEnd ? g[q] & ~sseen[w0 + q] : 0ull;
          if (want && cut) {
            // keep the ids of the sender's subset for v
            uint64_t y = want;
            while (y) {
              const int bb = __ffsll((long long)y) - 1;
              y &= y - 1;
              const int64_t mid = d.slotMid[(int64_t)(w0 + q) * 64 + bb];
              const unsigned long long key = gs_key64_mid(d.seed, GS_SITE_EMIT_MIDS, uu, v, (uint32_t)mid, (uint32_t)(h - 1));
              if (key > K || (key == K && mid > M)) want &= ~(1ull << bb);
            }
          }
          if (want) fn(w0 + q, want);
        }
      }
    };
    __syncthreads();
    // pass a: want counts and the per-sender smallest promise key; items with
    // a want are flagged for passes a2 / b
    for (int b = lane; b < totalItems; b += 64) {
      int k;
      const int i = item_sender(sIt, b, k);
      const int t = kth_bit(sTm[i], k / nCh), ch = k % nCh;
      const int uu = sNode[i];
      int c = 0;
      uint64_t bestKey = ~0ull;
      wants(b, uu, t, ch, [&](int w, uint64_t want) {
        c += __popcll(want);
        uint64_t y = want;
        while (y) {
          const int bb = __ffsll((long long)y) - 1;
          y &= y - 1;
          const int64_t mid = d.slotMid[(int64_t)w * 64 + bb];
          const uint64_t key = gs_key64_mid(d.seed, GS_SITE_IWANT, v, uu, (uint32_t)mid, (uint32_t)h);
          bestKey = key < bestKey ? key : bestKey;
        }
      });
      if (c) {
        atomicAdd(&sCnt[i], c);
        // an item whose key was the sender's smallest when it got there is a
        // candidate for pass a2 (a superset of the items holding the final one)
        if (bestKey <= atomicMin(&sKey[i], bestKey)) atomicOr(&sCand[b >> 5], 1u << (b & 31));
        atomicOr(&sHas[b >> 5], 1u << (b & 31));
      }
    }
    __syncthreads();
#ifndef GS_STAMPS_PB2
    GS_STAMPB(5);
#endif
    // pass a2: the smallest mid among the wants holding the smallest key (only
    // the candidate items can hold it)
    for (int b = lane; b < totalItems; b += 64) {
      if (!((sCand[b >> 5] >> (b & 31)) & 1)) continue;
      int k;
      const int i = item_sender(sIt, b, k);
      const int t = kth_bit(sTm[i], k / nCh), ch = k % nCh;
      const int uu = sNode[i];
      const uint64_t best = sKey[i];
      wants(b, uu, t, ch, [&](int w, uint64_t want) {
        uint64_t y = want;
        while (y) {
          const int bb = __ffsll((long long)y) - 1;
          y &= y - 1;
          const int64_t mid = d.slotMid[(int64_t)w * 64 + bb];
          if (gs_key64_mid(d.seed, GS_SITE_IWANT, v, uu, (uint32_t)mid, (uint32_t)h) == best)
            atomicMin(&sMid[i], (long long)mid);
        }
      });
    }
    __syncthreads();
#ifndef GS_STAMPS_PB2
    GS_STAMPB(6);
#endif
    // the sender cut: iask = MaxIHaveLength - iasked of the smallest keys
    const int myWantAll = sCnt[lane];
    const bool iaCut = gateIHave && myWantAll > 0 && myWantAll + ia > d.MaxIHaveLength;
    const int myWant = iaCut ? d.MaxIHaveLength - ia : myWantAll;
    if (cutMode & 2) {
      unsigned long long cm = __ballot(iaCut);
      while (cm) {
        const int i = __ffsll((long long)cm) - 1;
        cm &= cm - 1;
        const int uu = sNode[i];
        const int kk = lane_get(myWant, i);
        const int b0 = sIt[i] / nCh;  // its first (sender, topic) item
        const int nItems = __popcll(sTm[i]);
        // every want of sender i over its items, lane-strided over words
        auto each = [&](auto&& fn) {
          for (int k = 0; k < nItems; ++k) {
            const int t = kth_bit(sTm[i], k);
            const int b = b0 + k;
            unsigned long long cK0 = 0;
            long long cM0 = 0;
            const bool cut = cutOf(b, cK0, cM0);
            for (int w = t * Wt + lane; w < (t + 1) * Wt; w += 64) {
              uint64_t y = d.gw[(int64_t)uu * W + w] & ~sseen[w];
              while (y) {
                const int bb = __ffsll((long long)y) - 1;
                y &= y - 1;
                const int64_t mid = d.slotMid[(int64_t)w * 64 + bb];
                if (cut) {
                  const unsigned long long ke = gs_key64_mid(d.seed, GS_SITE_EMIT_MIDS, uu, v, (uint32_t)mid, (uint32_t)(h - 1));
                  if (ke > cK0 || (ke == cK0 && mid > cM0)) continue;
                }
                fn(gs_key64_mid(d.seed, GS_SITE_IWANT, v, uu, (uint32_t)mid, (uint32_t)h), mid);
              }
            }
          }
        };
        unsigned long long K;
        long long M;
        select_kth(each, kk, cHist, K, M);  // (sH is live again: the multi-pass select)
        if (lane == 0) {
          iK[i] = K;
          iM[i] = M;
        }
        __syncthreads();
      }
    } else if (__ballot(iaCut)) {
      if (lane == 0) set_err(d, E_TRUNCATE);  // the host ruled the cut out
    }
    const uint64_t cutSenders = __ballot(iaCut);
    int totalWant;
    const int myOff = lane_prefix(myWant, &totalWant);
    if (lane == 0 && totalWant) sBase = pool_take(d, cur, (unsigned long long)totalWant);
    __syncthreads();
    if (totalWant) {
      const unsigned long long poolBase = sBase;
      if (poolBase == ~0ull) {  // arena full (E_POOL)
      } else {
        sOut[lane] = (int)poolBase + myOff;
        __syncthreads();
        // pass b: write the request lists; the promised message's slot
        for (int b = lane; b < totalItems; b += 64) {
          if (!((sHas[b >> 5] >> (b & 31)) & 1)) continue;
          int k;
          const int i = item_sender(sIt, b, k);
          const int t = kth_bit(sTm[i], k / nCh), ch = k % nCh;
          const int uu = sNode[i];
          const long long bestMid = sMid[i];
          const bool cutI = (cutSenders >> i) & 1;
          wants(b, uu, t, ch, [&](int w, uint64_t want) {
            uint64_t y = want;
            while (y) {
              const int bb = __ffsll((long long)y) - 1;
              y &= y - 1;
              const int slot = w * 64 + bb;
              const int64_t mid = d.slotMid[slot];
              if (cutI) {
                const unsigned long long key = gs_key64_mid(d.seed, GS_SITE_IWANT, v, uu, (uint32_t)mid, (uint32_t)h);
                if (key > iK[i] || (key == iK[i] && mid > iM[i])) continue;
              }
              d.pool[cur][sOut[i] + atomicAdd(&sCur[i], 1)] = slot;
              if (mid == bestMid) sSlot[i] = slot;
            }
          });
        }
        if (myWant) {
          iwantRec = ((int64_t)(poolBase + myOff) << 24) | (int64_t)myWant;
          ia += myWant;
          cIwantSent = silent ? 0 : myWant;
          iwantAny = true;
        }
      }
    }
    __syncthreads();
#ifndef GS_STAMPS_PB2
    GS_STAMPB(7);
#endif
  }
  cIwantSent = (long long)wave_sum_ll(cIwantSent);
  cGray = (long long)wave_sum_ll(cGray);  // per-lane (sender) counts

  // ---- gossipTracer.AddPromise (gossip_tracer.go:48-75) for every sender we
  // sent an IWANT, senders ascending; table lane q = entry q
  if (d.scoring) {
    const unsigned long long pm = __ballot(iwantAny);
    if (pm) {
      // the table's first bank of 64 in registers (lane = entry); entries past
      // it (promCap > 64: a node with many peers, each promise alive up to
      // IWantFollowupTime plus a heartbeat) read and appended in memory.  A
      // sender appears once below, so only the entries present before this
      // call can repeat (mid, peer) (AddPromise keeps the first expiry, :66-71).
      const int n0p = d.promN[v];
      int promN = n0p;
      const int64_t row = (int64_t)v * d.promCap;
      int64_t pMid = lane < promN ? d.promMid[row + lane] : -1;
      int64_t pExp = lane < promN ? d.promExp[row + lane] : 0;
      int32_t pSlot = lane < promN ? d.promSlot[row + lane] : 0;
      int pEdge = lane < promN ? d.promEdge[row + lane] : 0;
      unsigned long long m = pm;
      while (m) {
        const int i = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int64_t bm = sMid[i];
        const int bs = sSlot[i];
        unsigned long long ex = __ballot(lane < promN && pMid == bm && pEdge == i);
        for (int b0 = 64; !ex && b0 < n0p; b0 += 64) {
          const bool in = b0 + lane < n0p;
          ex = __ballot(in && d.promMid[row + b0 + lane] == bm && d.promEdge[row + b0 + lane] == i);
        }
        if (ex) continue;
        if (promN >= d.promCap) {
          if (lane == 0) set_err(d, E_PROMISES);
          continue;
        }
        if (promN < 64) {
          if (lane == promN) {
            pMid = bm;
            pSlot = bs;
            pEdge = i;
            pExp = now + d.IWantFollowupTime;
          }
        } else if (lane == 0) {
          d.promMid[row + promN] = bm;
          d.promExp[row + promN] = now + d.IWantFollowupTime;
          d.promSlot[row + promN] = bs;
          d.promEdge[row + promN] = (uint8_t)i;
        }
        promN++;
      }
      if (lane < promN && lane < 64) {
        d.promMid[row + lane] = pMid;
        d.promExp[row + lane] = pExp;
        d.promSlot[row + lane] = pSlot;
        d.promEdge[row + lane] = (uint8_t)pEdge;
      }
      if (lane == 0) d.promN[v] = promN;
    }
  }

  GS_STAMPB(3);
  // ---- step 4: consume the outbox entries, per-edge state, reply RPCs
  if (ctl) {
    d.cPre[prv][e] = 0;
    d.cHb[prv][e] = 0;
    d.cGraftJoin[prv][e] = 0;
    d.cGraftHb[prv][e] = 0;
    d.cPruneReply[prv][e] = 0;
    d.cPruneHb[prv][e] = 0;
    d.cIhave[prv][e] = 0;
    d.cIwant[prv][e] = -1;
    d.cIresp[prv][e] = -1;
    if (d.doPX) d.cPx[prv][e] = -1;
    if (ADV && d.cSpam[prv] != nullptr) {
      d.cSpam[prv][e] = -1;
      d.cNSrv[prv][e] = 0;
    }
    if (!gl) {
      d.mesh[e] = meshE;
      d.peerhave[e] = ph;
      d.iasked[e] = ia;
      // one reply per control RPC that produced one (HandleRPC, gossipsub.go:602-607)
      const int nReplies = nRep1 + nSrv + ((iwantAny || prunesHb) ? 1 : 0);
      if (nReplies && !silent) {
        d.cPre[cur][r] = (uint8_t)(d.cPre[cur][r] + nReplies);
        d.cPruneReply[cur][r] |= pruneOut;
        if (iwantRec >= 0) d.cIwant[cur][r] = iwantRec;
        if (respRec >= 0) d.cIresp[cur][r] = respRec;
        if (nSrv && d.cNSrv[cur] != nullptr) d.cNSrv[cur][r] = (uint8_t)nSrv;
        if (d.rpcB != nullptr) {
          // HandleRPC's replies (gossipsub.go:602-607, rpcWithControl): a PRUNE
          // per rejected join GRAFT; the served messages of each IWANT list
          // with an empty control message (2 bytes); IWANT + PRUNEs for the
          // heartbeat RPC
          int64_t b = 0;
          const int64_t pxA = d.doPX ? d.cPx[cur][r] : -1;  // the PRUNEs' PX lists
          for (uint64_t m = joinRej; m; m &= m - 1) {
            const int t = __ffsll((long long)m) - 1;
            b += gs_pb_field(prune_entry(d, e, t, px_count(d, cur, pxA, 1ull << t)));
          }
          if (srvB) b += (int64_t)srvB + 2;
          if (srvBS) b += (int64_t)srvBS + 2;
          if (iwantAny || prunesHb) {
            int64_t body = iwantAny ? gs_pb_field((int64_t)(iwantRec & 0xFFFFFF) * d.acctIdF) : 0;
            for (uint64_t m = hbPr; m; m &= m - 1) {
              const int t = __ffsll((long long)m) - 1;
              body += prune_entry(d, e, t, px_count(d, cur, pxA, 1ull << t));
            }
            b += gs_pb_field(body);
          }
          acct_send(d, e, b, nReplies);
        }
        if (rpc_traced(d, v, u)) {
          // HandleRPC's replies (gossipsub.go:602-607), each named by the RPC it
          // answers (include/gs_trace.h): a PRUNE per rejected join GRAFT, the
          // served messages of the spam and IWANT lists, IWANT + PRUNEs for
          // the heartbeat RPC
          for (uint64_t m = joinRej; m; m &= m - 1) {
            const int t = __ffsll((long long)m) - 1;
            const int64_t pxr = d.doPX ? d.cPx[cur][r] : -1;
            rpc_trace(d, h, v, u, 3, 3, GS_RPC_ORD(3, t), 2 + px_count(d, cur, pxr, 1ull << t), [&](auto put) {
              put(GS_RPC_ITEM_CTL, -1, -1);
              put(GS_RPC_ITEM_PRUNE, t, -1);
              px_each(d, cur, pxr, 1ull << t, [&](int tt, int q) { put(GS_RPC_ITEM_PX, tt, q); });
            });
          }
          // the served ids of one request list: by each request's verdict
          // (pflag) when spam lists exist, else the whole served record
          const int32_t* const poolPrv = prv ? d.pool[1] : d.pool[0];
          const int32_t* const poolCur = cur ? d.pool[1] : d.pool[0];
          const uint8_t* const flagPrv = (ADV && d.pflag[0] != nullptr) ? (prv ? d.pflag[1] : d.pflag[0]) : nullptr;
          if (srvS > 0 && respRec >= 0)
            rpc_trace(d, h, v, u, 3, 2, GS_RPC_ORD(3, GS_RPC_O_ANS_SPAM), 1 + srvS, [&](auto put) {
              put(GS_RPC_ITEM_CTL, -1, -1);
              put_served(d, poolPrv, flagPrv, spRec, put);
            });
          if (srvR > 0 && respRec >= 0)
            rpc_trace(d, h, v, u, 3, 2, GS_RPC_ORD(3, GS_RPC_O_ANS_REPLY), 1 + srvR, [&](auto put) {
              put(GS_RPC_ITEM_CTL, -1, -1);
              if (flagPrv != nullptr) put_served(d, poolPrv, flagPrv, iwRec, put);
              else put_served(d, poolCur, nullptr, respRec, put);
            });
          if (iwantAny || prunesHb) {
            const int nIw = iwantAny ? (int)(iwantRec & 0xFFFFFF) : 0;
            const int64_t pxr = d.doPX ? d.cPx[cur][r] : -1;
            rpc_trace(d, h, v, u, 3, 3, GS_RPC_ORD(3, GS_RPC_O_ANS_HB), 1 + nIw + __popcll(hbPr) + px_count(d, cur, pxr, hbPr),
                      [&](auto put) {
              put(GS_RPC_ITEM_CTL, -1, -1);
              for (int q = 0; q < nIw; ++q) put(GS_RPC_ITEM_IWANT, -1, d.slotMid[d.pool[cur][(iwantRec >> 24) + q]]);
              for (uint64_t m = hbPr; m; m &= m - 1) put(GS_RPC_ITEM_PRUNE, __ffsll((long long)m) - 1, -1);
              px_each(d, cur, pxr, hbPr, [&](int tt, int q) { put(GS_RPC_ITEM_PX, tt, q); });
            });
          }
        }
      }
    }
  }
  if (silent) cPrunes = 0;  // the PRUNE replies of a squatter are never sent
  if (lane == 0) {
    if (cPrunes) ctr_add(d, C_PRUNES, (unsigned long long)cPrunes);
    if (cIwantSent) ctr_add(d, C_IWANT_SENT, (unsigned long long)cIwantSent);
    if (cServed) ctr_add(d, C_IWANT_SERVED, (unsigned long long)cServed);
    if (cGray) ctr_add(d, C_GRAYLISTED, (unsigned long long)cGray);
  }
  GS_STAMPB(4);
}

template <int WPL, bool ADV>
__global__ __launch_bounds__(64) GS_OCC_PB void k_phase_b(const Dev* __restrict__ dp, int64_t h, int64_t now, int cur,
                                                int head, int cutModeArg) {
  const Dev& d = *dp;  // from device memory, as k_phase_a
  phase_b_node<WPL, ADV>(d, d.n0 + (int)blockIdx.x, h, now, cur, head, cutModeArg);
}

// ---------------------------------------------------------------- heartbeat prelude
// clearBackoff (every 15 ticks, slack 2 * GossipSubHeartbeatInterval = 2 s,
// gossipsub.go:1573-1592), clearIHaveCounters (:1554-1564) and
// applyIwantPenalties (:1566-1571 -> gossip_tracer.go:79-115, score.go:382).
// A promise is fulfilled iff its message has been delivered since (it was
// unseen when promised), so "fulfilled" == "seen now".
// flagDhi: the heartbeat's memo pass (k_score_rows<4>) is exact only where
// a score-lowering change happened or S0 < 0, but the Dhi ranking compares the
// mesh members of an over-full topic by value: those members get sdirty here,
// so the memo pass computes their exact heartbeat-start scores in its
// streaming form (every lane busy, a batch of records in flight) instead of the
// heartbeat wave fetching each 64-topic record on its own.
__global__ __launch_bounds__(64) void k_hb_pre(Dev d, int64_t now, uint64_t ticks, int flagDhi) {
  const int v = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  if (valid) {
    d.peerhave[e] = 0;
    d.iasked[e] = 0;
  }
  if (flagDhi && gossip_host(d, v)) {
    const uint64_t joined = d.sub[v];
    const uint64_t meshl = valid ? d.mesh[e] & joined : 0ull;
    bool needX = false;
    for (uint64_t jm = joined; jm; jm &= jm - 1) {
      const int t = __ffsll((long long)jm) - 1;
      const bool mt = (meshl >> t) & 1;
      if (__popcll(__ballot(mt)) > d.Dhi) needX |= mt;
    }
    if (needX) d.sdirty[e] = 1;
  }
  if (ticks % 15 == 0) {  // v's in-edges own the contiguous pairs [base*T, (base+deg)*T)
    for (int j = 0; j < deg; ++j) {  // one edge's topics per step (lane = topic), its mask rebuilt
      const int64_t i = (base + j) * d.T + lane;
      bool set = false;
      if (lane < d.T) {
        const int64_t be = d.backoff[i];
        if (be != 0 && be + 2000000000LL < now) d.backoff[i] = 0;
        else set = be != 0;
      }
      const uint64_t m = __ballot(set);
      if (lane == 0) d.boMask[base + j] = m;
    }
  }
  if (!d.scoring) return;
  const int n = d.promN[v];
  if (n == 0) return;
  // the table in banks of 64 (lane = entry): broken promises counted per peer
  // over every bank, then one AddPenalty(p, count) per peer (GetBrokenPromises
  // returns a count per peer, gossipsub.go:1566-1571); live entries compacted
  __shared__ int sBroken[64];
  sBroken[lane] = 0;
  __syncthreads();
  int kept = 0, total = 0;
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int64_t ti = (int64_t)v * d.promCap + b0 + lane;
    int64_t mid = -1, exp = 0;
    int slot = 0, edge = 0;
    bool live = b0 + lane < n, broken = false;
    if (live) {
      mid = d.promMid[ti];
      exp = d.promExp[ti];
      slot = d.promSlot[ti];
      edge = d.promEdge[ti];
      const bool seen = (d.seen[(int64_t)v * d.W + (slot >> 6)] >> (slot & 63)) & 1;
      if (seen) live = false;
      else if (exp < now) { live = false; broken = true; }
    }
    if (broken) atomicAdd(&sBroken[edge], 1);
    total += __popcll(__ballot(broken));
    const unsigned long long lm = __ballot(live);
    const int pos = kept + __popcll(lm & ((1ull << lane) - 1));
    if (live) {  // pos <= b0 + lane: never past an entry not yet read
      const int64_t to = (int64_t)v * d.promCap + pos;
      d.promMid[to] = mid;
      d.promExp[to] = exp;
      d.promSlot[to] = slot;
      d.promEdge[to] = (uint8_t)edge;
    }
    kept += __popcll(lm);
  }
  __syncthreads();
  const int nb = sBroken[lane];
  if (nb && has_record(d, base + lane)) {  // AddPenalty needs a record (score.go:681-684)
    d.bp[base + lane] += (double)nb;
    d.sdirty[base + lane] = 1;
  }
  if (lane == 0) {
    d.promN[v] = kept;
    if (total) ctr_add(d, C_PROMISES_BROKEN, (unsigned long long)total);
  }
}

// emitGossip (gossipsub.go:1658-1712) for topic t of node v; lanes = edges.
// The peer filter uses the live Score(p) (:1681): Slive caches it per lane and
// is recomputed (one wave-parallel score per lane) only after the peer's stats
// changed earlier in this heartbeat.
__device__ __forceinline__ uint64_t emit_gossip(const Dev& d, int v, int t, int64_t hop, int head, bool valid,
                                                int vcol, bool inTopic, bool excl, bool dir, double& Slive,
                                                bool& dirty, bool& dirtyUp, int64_t rowBase, double* lds,
                                                int nm) {
  const int lane = lane_id();
  if (nm == 0) return 0;  // nm: message ids of topic t in the gossip windows
  if (behaves(d, v, GS_BEHAVE_NO_FORWARD)) return 0;  // a squatter emits no gossip
  // an IHAVE spammer advertises to every topic peer (mesh, direct, any score)
  if (behaves(d, v, GS_BEHAVE_IHAVE_SPAM)) return valid && inTopic ? (1ull << t) : 0;
  // more than MaxIHaveLength ids: each receiver's own keyed subset
  // (gossipsub.go:1702-1709) is cut by the receiver in k_phase_b
  const bool base = valid && inTopic && !excl && !dir;
  // A graft never lowers a score (P1 is 0 at meshTime 0, the P3 deficit term
  // is switched off; weights validated w1 >= 0, w3 <= 0), so a cached score
  // already at or above the threshold stays a correct decision after one.
  unsigned long long dm = __ballot(base && (dirty || (dirtyUp && !(Slive >= d.gossipThr))));
  while (dm) {  // rare (a peer pruned earlier in this heartbeat): one edge at a time
    const int j = __ffsll((long long)dm) - 1;
    dm &= dm - 1;
    const double s = edge_score_wave(d, rowBase + j, lds);
    if (lane == j) {
      Slive = s;
      dirty = false;
      dirtyUp = false;
    }
  }
  const bool cand = base && Slive >= d.gossipThr;
  const int n = __popcll(__ballot(cand));
  int target = d.Dlazy;
  const int factor = (int)(d.GossipFactor * (double)n);
  if (factor > target) target = factor;
  bool sel = cand;
  if (target < n) {
    const uint64_t key = gs_key64(d.seed, GS_SITE_EMIT_PEERS, v, (uint32_t)hop, vcol, t);
    sel = select_k_lds(cand, key, target, (uint64_t*)lds);
  }
  return sel ? (1ull << t) : 0;
}

// number of lanes of this lane's half with x set
__device__ __forceinline__ int half_count(bool x) {
  const unsigned long long b = __ballot(x);
  return __popc((uint32_t)(b >> (lane_id() & 32)));
}

// The joined-topic loop of k_heartbeat<true>: pairs of joined topics (ta, tb)
// ascending, half h = lane >> 5 handles topic (ta, tb)[h] of every edge (lane
// & 31).  Per pair:
//   1. mesh maintenance decisions of both topics (they read the heartbeat memo
//      S and the topic's own mesh / backoff bits only, so the two topics are
//      independent): negative-score prune, Dlo graft, Dhi prune (serially per
//      half: it ranks by value through LDS), Dout graft, opportunistic graft;
//   2. ta's stats writes (peerScore.Prune / Graft, backoff), then emitGossip's
//      live-score refresh for ta's candidates; tb's writes, then tb's refresh
//      starting from ta's live-score state — the serial topic order, so every
//      live score emitGossip compares equals the serial loop's;
//   3. both topics' IHAVE peer selections (key draw + select) at once.
__device__ __forceinline__ void hb_pair(const Dev& d, int v, int64_t base, int deg, bool vm, int64_t e, int vcol,
                                        int64_t hop, int64_t now, uint64_t ticks, int head, uint64_t joined,
                                        uint64_t subv, double S, bool dir, bool ob, bool graftSpam, int nmT,
                                        uint64_t& meshl, uint64_t& boM, double& Slive, bool& dirty, bool& dirtyUp,
                                        uint64_t& tograft, uint64_t& toprune, uint64_t& ihave, uint64_t& spamGraft,
                                        int* plst, int* obs, int* posOf, double* lds, unsigned long long& cyMesh,
                                        unsigned long long& cyEmit, unsigned long long& cySel) {
  const int lane = lane_id();
  const int h = lane >> 5;
  const uint32_t hw = (uint32_t)hop;
  const bool noFwd = behaves(d, v, GS_BEHAVE_NO_FORWARD);
  const bool ihaveSpam = behaves(d, v, GS_BEHAVE_IHAVE_SPAM);
  const bool oppTick = ticks % d.OGT == 0;
  // Steady topics: step 1 changes nothing for a topic
  // whose mesh has no member scored below 0, is not above Dhi, and is below
  // Dlo (or short of Dout outbound members) only where no candidate peer
  // could be grafted (negative-score prune, Dlo / Dhi / Dout below;
  // opportunistic ticks and GRAFT spammers are never steady).  Counted for
  // every topic at once: lane t of a transposed edge mask holds topic t's
  // edges (the lower half's edges are all of them).
  const bool lo = lane < 32 && vm;
  const uint64_t mL = lo ? meshl : 0ull;
  // graft candidates of getPeers' filter in step 1: topic peers not in the
  // mesh nor in backoff, not direct, score >= 0
  const uint64_t cL = (lo && !dir && S >= 0) ? (subv & ~meshl & ~boM) : 0ull;
  const int cntT = __popcll(wave_transpose64(mL)), outT = __popcll(wave_transpose64(ob ? mL : 0ull));
  const bool negT = wave_transpose64(S < 0 ? mL : 0ull) != 0;
  const bool candT = wave_transpose64(cL) != 0, obCandT = wave_transpose64(ob ? cL : 0ull) != 0;
  const bool busyT = lane < d.T && ((joined >> lane) & 1) &&
                     (negT || cntT > d.Dhi || (cntT < d.Dlo && candT) || (cntT >= d.Dlo && outT < d.Dout && obCandT));
  const uint64_t busy = (oppTick || graftSpam) ? ~0ull : __ballot(busyT);
  uint64_t jm = joined;
  uint64_t myT = 0;  // the topics this half handled
  while (jm) {
    const unsigned long long c0 = GS_CLK();
    const int ta = __ffsll((long long)jm) - 1;
    jm &= jm - 1;
    const int tb = jm ? __ffsll((long long)jm) - 1 : -1;
    if (jm) jm &= jm - 1;
    const int t = h ? tb : ta;  // this half's topic, -1: none
    const bool act = t >= 0;
    const int tt = act ? t : 0;
    const uint64_t bit = act ? 1ull << t : 0ull;
    const bool inTopic = vm && act && ((subv >> tt) & 1);
    bool m = vm && act && (meshl & bit);
    bool pr = false, gr = false;  // pruned / grafted at t in this pass
    // both topics steady: step 1 changes nothing (wave-uniform)
    const bool fast = !((busy >> ta) & 1) && (tb < 0 || !((busy >> tb) & 1));
    if (!fast) {
    // ---- 1. decisions
    if (m && (S < 0 || (graftSpam && ticks == 1))) {
      pr = true;
      m = false;
    }
    bool bo = (boM & bit) != 0 || pr;  // a prune adds backoff
    int cnt = half_count(m);
    if (cnt < d.Dlo) {
      const bool cand = inTopic && !m && !bo && !dir && S >= 0;
      const uint64_t key = gs_key64(d.seed, GS_SITE_GP_DLO, v, hw, vcol, tt);
      if (select_k_half(cand, key, d.D - cnt)) {
        gr = true;
        m = true;
      }
      cnt = half_count(m);
    }
    // too many peers: ranked by value through LDS, one half at a time
    const int cntA = lane_get(cnt, 0), cntB = lane_get(cnt, 32);
    for (int hh = 0; hh < 2; ++hh) {
      if ((hh ? cntB : cntA) <= d.Dhi) continue;
      const int cnth = hh ? cntB : cntA;
      const bool mh = m && h == hh;
      const uint64_t k1 = gs_key64(d.seed, GS_SITE_DHI_SHUFFLE, v, hw, vcol, tt);
      int rank1 = 0;
      unsigned long long mm = __ballot(mh);
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const double sj = lane_getf(S, j);
        const uint64_t kj = lane_get64(k1, j);
        if (sj > S || (sj == S && (kj < k1 || (kj == k1 && j < lane)))) rank1++;
      }
      const bool tail = mh && rank1 >= d.Dscore;
      const uint64_t k2 = gs_key64(d.seed, GS_SITE_DHI_TAIL, v, hw, vcol, tt);
      int rank2 = 0;
      mm = __ballot(tail);
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const uint64_t kj = lane_get64(k2, j);
        if (kj < k2 || (kj == k2 && j < lane)) rank2++;
      }
      const int pos = tail ? d.Dscore + rank2 : rank1;
      if (mh) plst[pos] = lane;
      obs[lane] = ob ? 1 : 0;
      __syncthreads();
      if (lane == 0) {
        // keep D_out outbound peers among the first D (gossipsub.go:1389-1429)
        int outbound = 0;
        for (int i = 0; i < d.D; ++i) outbound += obs[plst[i]];
        if (outbound < d.Dout) {
          if (outbound > 0) {
            int ih = outbound;
            for (int i = 1; i < d.D && ih > 0; ++i) {
              if (obs[plst[i]]) {
                const int p = plst[i];
                for (int j = i; j > 0; --j) plst[j] = plst[j - 1];
                plst[0] = p;
                ih--;
              }
            }
          }
          int ineed = d.Dout - outbound;
          for (int i = d.D; i < cnth && ineed > 0; ++i) {
            if (obs[plst[i]]) {
              const int p = plst[i];
              for (int j = i; j > 0; --j) plst[j] = plst[j - 1];
              plst[0] = p;
              ineed--;
            }
          }
        }
        for (int i = 0; i < cnth; ++i) posOf[plst[i]] = i;
      }
      __syncthreads();
      if (mh && posOf[lane] >= d.D) {
        pr = true;
        bo = true;
        m = false;
      }
      __syncthreads();
    }
    cnt = half_count(m);
    // do we have enough outbound peers?
    if (cnt >= d.Dlo) {
      const int outb = half_count(m && ob);
      if (outb < d.Dout) {
        const bool cand = inTopic && !m && !bo && !dir && ob && S >= 0;
        const uint64_t key = gs_key64(d.seed, GS_SITE_GP_DOUT, v, hw, vcol, tt);
        if (select_k_half(cand, key, d.Dout - outb)) {
          gr = true;
          m = true;
        }
        cnt = half_count(m);
      }
    }
    // opportunistic grafting (median of the memoised mesh scores), one half at a time
    if (oppTick) {
      const int ca = lane_get(cnt, 0), cb = lane_get(cnt, 32);
      for (int hh = 0; hh < 2; ++hh) {
        const int cnth = hh ? cb : ca;
        if (cnth <= 1) continue;
        const bool mh = m && h == hh;
        int rank = 0;
        unsigned long long mm = __ballot(mh);
        while (mm) {
          const int j = __ffsll((long long)mm) - 1;
          mm &= mm - 1;
          const double sj = lane_getf(S, j);
          if (sj < S || (sj == S && j < lane)) rank++;
        }
        const unsigned long long ml = __ballot(mh && rank == cnth / 2);
        const double median = lane_getf(S, __ffsll((long long)ml) - 1);
        if (median < d.oppThr) {
          const bool cand = h == hh && inTopic && !m && !bo && !dir && S > median;
          const uint64_t key = gs_key64(d.seed, GS_SITE_GP_OPPORTUNISTIC, v, hw, vcol, tt);
          if (select_k_half(cand, key, d.OGP)) {
            gr = true;
            m = true;
          }
        }
      }
    }
    // a GRAFT spammer re-GRAFTs the topic peers it is in backoff with
    if (graftSpam && ticks > 1 && inTopic && !m && bo) {
      if (pr) {
        spamGraft |= bit;  // the backoff just added expires after now
      } else {
        const int64_t be = d.backoff[tix(d, tt, e)];
        if (be != 0 && be > now) spamGraft |= bit;
      }
    }
    }  // (!fast)
    const unsigned long long c1 = GS_CLK();
    // ---- 2. stats writes and emitGossip's live scores, in topic order
    const int nmA = lane_get(nmT, ta), nmB = tb >= 0 ? lane_get(nmT, tb) : 0;
    const int nm = act ? (h ? nmB : nmA) : 0;  // message ids of t in the gossip windows
    const bool emits = nm > 0 && !noFwd && !ihaveSpam;
    const bool baseE = emits && vm && inTopic && !m && !dir;
    bool cand = false;
    // and no live score of this pair's candidates needs a refresh: step 2
    // changes nothing either (the halves' live-score states are equal at a
    // pair boundary and stay so)
    if (fast && !__ballot(baseE && (dirty || (dirtyUp && !(Slive >= d.gossipThr)))))
      cand = baseE && Slive >= d.gossipThr;
    else
    for (int hh = 0; hh < 2; ++hh) {
      if (h == hh) {
        if (pr) {
          stats_prune(d, e, tt);
          add_backoff(d, e, tt, now, d.PruneBackoff);
        }
        if (gr) stats_graft(d, e, tt, now);
        dirty = dirty || pr;
        dirtyUp = dirtyUp || gr;
      }
      unsigned long long dm = __ballot(h == hh && baseE && (dirty || (dirtyUp && !(Slive >= d.gossipThr))));
      while (dm) {  // rare (a peer pruned earlier in this heartbeat): one edge at a time
        const int j = __ffsll((long long)dm) - 1;
        dm &= dm - 1;
        const double sj = edge_score_wave(d, base + (j & 31), lds);
        if (lane == j) {
          Slive = sj;
          dirty = false;
          dirtyUp = false;
        }
      }
      if (h == hh) cand = baseE && Slive >= d.gossipThr;
      // the other half continues from this half's live-score state
      const double sx = xor32_f64(Slive);
      const uint32_t fx = xor32_u32((dirty ? 1u : 0u) | (dirtyUp ? 2u : 0u));
      if (h != hh) {
        Slive = sx;
        dirty = (fx & 1) != 0;
        dirtyUp = (fx & 2) != 0;
      }
    }
    // ---- 3. IHAVE peer selection of both topics
    const unsigned long long c2 = GS_CLK();
    uint64_t ih = 0;
    if (ihaveSpam) {
      ih = (nm > 0 && !noFwd && vm && inTopic) ? bit : 0;  // every topic peer, any score
    } else if (emits) {
      const int n = half_count(cand);
      int target = d.Dlazy;
      const int factor = (int)(d.GossipFactor * (double)n);
      if (factor > target) target = factor;
      bool sel = cand;
      if (target < n) {
        const uint64_t key = gs_key64(d.seed, GS_SITE_EMIT_PEERS, v, hw, vcol, tt);
        sel = select_k_half(cand, key, target);
      }
      ih = sel ? bit : 0;
    }
    // ---- this half's topic bits (a half reads and writes only its own
    // topics' bits; the halves are merged once, after the loop)
    myT |= bit;
    meshl = (meshl & ~bit) | (m ? bit : 0ull);
    if (pr) {
      boM |= bit;
      toprune |= bit;
    }
    if (gr) tograft |= bit;
    ihave |= ih;
    cyMesh += c1 - c0;
    cyEmit += c2 - c1;
    cySel += GS_CLK() - c2;
  }
  // merge: each half's topics from that half (the rest of meshl is unchanged
  // in both)
  const uint64_t otherT = xor32_u64(myT);
  meshl = (meshl & ~otherT) | (xor32_u64(meshl) & otherT);
  boM |= xor32_u64(boM) & otherT;
  toprune |= xor32_u64(toprune);
  tograft |= xor32_u64(tograft);
  ihave |= xor32_u64(ihave);
  spamGraft |= xor32_u64(spamGraft);
}

// ---------------------------------------------------------------- heartbeat
// GossipSubRouter.heartbeat (gossipsub.go:1299-1552) for one node: mesh
// maintenance per joined topic (ascending), emitGossip, fanout expiry and
// maintenance, sendGraftPrune (outbox), mcache.Shift.  Scores are the
// heartbeat memo (score1, computed after applyIwantPenalties); emitGossip
// re-scores peers whose stats changed during this heartbeat (live Score()).
// PAIR (every node has at most 32 peers): the joined topics are handled two at
// a time, one per half-wave: lanes 32..63 mirror the edges of lanes 0..31 for
// the topic loop (mesh maintenance and emitGossip's peer selection of topic
// t0 + 1 next to t0's), with the live-score bookkeeping of emitGossip kept in
// the serial topic order (hb_pair below).
template <bool PAIR>
__global__ __launch_bounds__(64) GS_OCC_HB void k_heartbeat(Dev d, int64_t hop, int64_t now, uint64_t ticks, int cur,
                                                  int head, int newhead, int allExact) {
  __shared__ int plst[64];
  __shared__ int obs[64];
  __shared__ int posOf[64];
  __shared__ double sterm[64];
  __shared__ uint64_t sgw[64 * GS_MAX_WPL];
  const int v = d.n0 + blockIdx.x;
  if (!gossip_host(d, v)) return;  // only gossipsub hosts run a heartbeat
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const int el = PAIR ? (lane & 31) : lane;  // the lane's edge (PAIR: both halves)
  const bool valid = lane < deg;             // PAIR: deg <= 32, the lower half only
  const bool vm = el < deg;                  // valid, mirrored into the upper half
  const int64_t e = base + el;
  const int vcol = vm ? d.col[e] : -1;
  GS_STAMPH(0, GS_CLK());
  // mcache.GetGossipIDs windows 0..HG-1 (mcache.go:82-92): this heartbeat's
  // IHAVE payload, kept as the node's gw row for the receivers' handleIHave
  {
    // windows in pairs, the pair's 2 x GS_MAX_WPL loads in flight at once
    uint64_t x[GS_MAX_WPL] = {};
    for (int k0 = 0; k0 < d.HG; k0 += 2) {
      uint64_t y[2][GS_MAX_WPL];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint64_t* src = d.hist + ((int64_t)((head + k0 + k) % d.R) * d.nOwnH + (v - d.n0)) * d.W;
#pragma unroll
        for (int j = 0; j < GS_MAX_WPL; ++j) {
          const int w = lane + 64 * j;
          y[k][j] = (k0 + k < d.HG && w < d.W) ? src[w] : 0ull;
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < GS_MAX_WPL; ++j) x[j] |= y[k][j];
    }
#pragma unroll
    for (int j = 0; j < GS_MAX_WPL; ++j) {
      const int w = lane + 64 * j;
      if (w < d.W) {
        sgw[w] = x[j];
        d.gw[(int64_t)v * d.W + w] = x[j];
      }
    }
  }
  __syncthreads();
  GS_STAMPH(1, GS_CLK());
  // lane t: message ids of topic t in the gossip windows (emitGossip's mids)
  int nmT = 0;
  if (lane < d.T)
    for (int w = lane * d.Wt; w < (lane + 1) * d.Wt; ++w) nmT += __popcll(sgw[w]);
  const uint64_t subv = vm && edge_up(d, e) ? d.subA[vcol] : 0;  // topic peers: connected, announced
  // the candidates of getPeers and emitGossip: mesh-capable topic peers
  // (GossipSubFeatureMesh, gossipsub.go:1681, 1849)
  const bool mc = vm && mesh_peer(d, e);
  const uint64_t subvM = mc ? subv : 0;
  uint64_t meshl = vm ? d.mesh[e] : 0;
  uint64_t fanl = valid ? d.fanout[e] : 0;
  uint64_t boM = vm ? d.boMask[e] : 0;  // topics in backoff with this peer
  double S = vm ? d.score1[e] : 0.0;
  const uint64_t joined = d.sub[v];
  const bool hbNoPX = vm && S < 0 && (meshl & joined) != 0;  // pruned for its negative score: noPX
  if (d.scoring && !allExact) {
    // score1 is exact only where k_score_rows<4> recomputed it; the Dhi
    // ranking compares scores as values, so the mesh members of a topic that
    // may exceed Dhi get their exact heartbeat-start score now, before any
    // stats change in this heartbeat
    bool needX = false;
    for (int t = 0; t < d.T; ++t) {
      const bool mt = valid && ((meshl >> t) & 1) && ((joined >> t) & 1);
      if (__popcll(__ballot(mt)) > d.Dhi) needX |= mt;
    }
    const bool exact = valid && (d.sdirty[e] != 0 || !(d.score0[e] >= 0.0));
    __syncthreads();  // sgw (read for nmT above) becomes the batch's term table
    edge_scores_batch(d, base, __ballot(needX && !exact), S, (double*)sgw);
    if (PAIR) S = __shfl(S, el);  // the upper half mirrors the exact scores
  }
  GS_STAMPH(2, GS_CLK());
  unsigned long long cyMesh = 0, cyEmit = 0, cySel = 0;  // GS_STAMPS: cycles in mesh maintenance / emitGossip
  double Slive = S;  // live Score(p) for emitGossip
  const bool dir = vm && d.direct[e];
  const bool ob = vm && d.outbound[e];
  bool dirty = false;    // a PRUNE lowered the peer's score since Slive
  bool dirtyUp = false;  // a GRAFT (never lowers it) changed it since Slive
  uint64_t tograft = 0, toprune = 0, ihave = 0;
  const uint32_t hw = (uint32_t)hop;
  const bool graftSpam = behaves(d, v, GS_BEHAVE_GRAFT_SPAM);
  uint64_t spamGraft = 0;  // GRAFTs without a mesh change (not traced as Graft)
  if constexpr (PAIR) {
    hb_pair(d, v, base, deg, vm, e, vcol, hop, now, ticks, head, joined, subvM, S, dir, ob, graftSpam, nmT, meshl, boM,
            Slive, dirty, dirtyUp, tograft, toprune, ihave, spamGraft, plst, obs, posOf, (double*)sgw, cyMesh, cyEmit,
            cySel);
    if (!valid) tograft = toprune = ihave = spamGraft = 0;  // the mirror half is done
  } else
  for (int t = 0; t < d.T; ++t) {
    if (!((joined >> t) & 1)) continue;
    const unsigned long long c0 = GS_CLK();
    const uint64_t bit = 1ull << t;
    const bool inTopic = valid && ((subvM >> t) & 1);
    bool m = valid && (meshl & bit);
    // drop all peers with negative score, without PX; a GRAFT spammer first
    // leaves its whole mesh (gossipsub_spam_test.go:428-446)
    if (m && (S < 0 || (graftSpam && ticks == 1))) {
      stats_prune(d, e, t);
      meshl &= ~bit;
      add_backoff(d, e, t, now, d.PruneBackoff);
      boM |= bit;
      toprune |= bit;
      dirty = true;
      m = false;
    }
    int cnt = __popcll(__ballot(m));
    // do we have enough peers?
    if (cnt < d.Dlo) {
      const bool bo = (boM & bit) != 0;
      const bool cand = inTopic && !m && !bo && !dir && S >= 0;
      const uint64_t key = gs_key64(d.seed, GS_SITE_GP_DLO, v, hw, vcol, t);
      if (select_k_lds(cand, key, d.D - cnt, (uint64_t*)sterm)) {
        stats_graft(d, e, t, now);
        meshl |= bit;
        tograft |= bit;
        dirtyUp = true;
        m = true;
      }
      cnt = __popcll(__ballot(m));
    }
    // do we have too many peers?
    if (cnt > d.Dhi) {
      const uint64_t k1 = gs_key64(d.seed, GS_SITE_DHI_SHUFFLE, v, hw, vcol, t);
      int rank1 = 0;
      unsigned long long mm = __ballot(m);
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const double sj = lane_getf(S, j);
        const uint64_t kj = lane_get64(k1, j);
        if (sj > S || (sj == S && (kj < k1 || (kj == k1 && j < lane)))) rank1++;
      }
      const bool tail = m && rank1 >= d.Dscore;
      const uint64_t k2 = gs_key64(d.seed, GS_SITE_DHI_TAIL, v, hw, vcol, t);
      int rank2 = 0;
      mm = __ballot(tail);
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const uint64_t kj = lane_get64(k2, j);
        if (kj < k2 || (kj == k2 && j < lane)) rank2++;
      }
      const int pos = tail ? d.Dscore + rank2 : rank1;
      if (m) plst[pos] = lane;
      obs[lane] = ob ? 1 : 0;
      __syncthreads();
      if (lane == 0) {
        // keep D_out outbound peers among the first D (gossipsub.go:1389-1429)
        int outbound = 0;
        for (int i = 0; i < d.D; ++i) outbound += obs[plst[i]];
        if (outbound < d.Dout) {
          if (outbound > 0) {
            int ih = outbound;
            for (int i = 1; i < d.D && ih > 0; ++i) {
              if (obs[plst[i]]) {
                const int p = plst[i];
                for (int j = i; j > 0; --j) plst[j] = plst[j - 1];
                plst[0] = p;
                ih--;
              }
            }
          }
          int ineed = d.Dout - outbound;
          for (int i = d.D; i < cnt && ineed > 0; ++i) {
            if (obs[plst[i]]) {
              const int p = plst[i];
              for (int j = i; j > 0; --j) plst[j] = plst[j - 1];
              plst[0] = p;
              ineed--;
            }
          }
        }
        for (int i = 0; i < cnt; ++i) posOf[plst[i]] = i;
      }
      __syncthreads();
      if (m && posOf[lane] >= d.D) {
        stats_prune(d, e, t);
        meshl &= ~bit;
        add_backoff(d, e, t, now, d.PruneBackoff);
        boM |= bit;
        toprune |= bit;
        dirty = true;
        m = false;
      }
      __syncthreads();
      cnt = __popcll(__ballot(m));
    }
    // do we have enough outbound peers?
    if (cnt >= d.Dlo) {
      const int outb = __popcll(__ballot(m && ob));
      if (outb < d.Dout) {
        const bool bo = (boM & bit) != 0;
        const bool cand = inTopic && !m && !bo && !dir && ob && S >= 0;
        const uint64_t key = gs_key64(d.seed, GS_SITE_GP_DOUT, v, hw, vcol, t);
        if (select_k_lds(cand, key, d.Dout - outb, (uint64_t*)sterm)) {
          stats_graft(d, e, t, now);
          meshl |= bit;
          tograft |= bit;
          dirtyUp = true;
          m = true;
        }
        cnt = __popcll(__ballot(m));
      }
    }
    // opportunistic grafting (median of the memoised mesh scores)
    if (ticks % d.OGT == 0 && cnt > 1) {
      int rank = 0;
      unsigned long long mm = __ballot(m);
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const double sj = lane_getf(S, j);
        if (sj < S || (sj == S && j < lane)) rank++;
      }
      const unsigned long long ml = __ballot(m && rank == cnt / 2);
      const double median = lane_getf(S, __ffsll((long long)ml) - 1);
      if (median < d.oppThr) {
        const bool bo = (boM & bit) != 0;
        const bool cand = inTopic && !m && !bo && !dir && S > median;
        const uint64_t key = gs_key64(d.seed, GS_SITE_GP_OPPORTUNISTIC, v, hw, vcol, t);
        if (select_k_lds(cand, key, d.OGP, (uint64_t*)sterm)) {
          stats_graft(d, e, t, now);
          meshl |= bit;
          tograft |= bit;
          dirtyUp = true;
          m = true;
        }
      }
    }
    // a GRAFT spammer re-GRAFTs the topic peers it is in backoff with, leaving
    // its own mesh as it is (gossipsub_spam_test.go:449-500)
    if (graftSpam && ticks > 1 && inTopic && !m && (boM & bit)) {
      const int64_t be = d.backoff[tix(d, t, e)];
      if (be != 0 && be > now) spamGraft |= bit;
    }
    const unsigned long long c1 = GS_CLK();
    ihave |= emit_gossip(d, v, t, hop, head, valid, vcol, inTopic, m, dir, Slive, dirty, dirtyUp, base, (double*)sgw,
                         lane_get(nmT, t));
    cyMesh += c1 - c0;
    cyEmit += GS_CLK() - c1;
  }
  if (d.doPX) {
    // makePrune with PX for every PRUNE of this heartbeat (sendGraftPrune,
    // gossipsub.go:1636-1647), with the live scores after every mesh change;
    // none for a peer dropped for its negative score (noPX, :1350-1356)
    uint64_t any = 0;
    // v1.0 peers get no PX (makePrune gossipsub.go:1804-1807)
    const bool pxTo = valid && !hbNoPX && px_peer(d, e);
    for (int o = 0; o < 64; ++o) any |= lane_get64(pxTo ? toprune : 0ull, o);
    const bool ok = any ? px_score_ok(d, base, deg, sterm) : true;
    for (uint64_t mm = any; mm; mm &= mm - 1) {
      const int t = __ffsll((long long)mm) - 1;
      unsigned long long pl = __ballot(pxTo && ((toprune >> t) & 1));
      while (pl) {  // one list per pruned peer
        const int p = __ffsll((long long)pl) - 1;
        pl &= pl - 1;
        const uint64_t list = px_sel(d, v, base, deg, t, hop, p, ok);
        if (lane == p) px_append(d, cur, rxi(d, e, d.rev[e]), t, list, base);
      }
    }
  }
  GS_STAMPH(3, GS_CLK());
  GS_STAMPH(6, cyMesh);
  GS_STAMPH(7, cyEmit);
  GS_STAMPH(4, cySel);  // PAIR: the selection part of cyEmit
  // expire fanout for topics we haven't published to in a while
  uint64_t fpres = d.fanoutPresent[v];
  {
    const int64_t lp = lane < d.T ? d.lastpub[(int64_t)v * d.T + lane] : INT64_MIN;  // lane = topic
    const bool expired = lp != INT64_MIN && lp + d.FanoutTTL < now;
    const uint64_t xm = __ballot(expired);
    fpres &= ~xm;
    fanl &= ~xm;
    if (expired) d.lastpub[(int64_t)v * d.T + lane] = INT64_MIN;
  }
  // maintain our fanout for topics we are publishing but have not joined
  for (int t = 0; t < d.T; ++t) {
    if (!((fpres >> t) & 1)) continue;
    const uint64_t bit = 1ull << t;
    const bool inTopic = valid && ((subv >> t) & 1);
    bool f = valid && (fanl & bit);
    if (f && !(inTopic && S >= d.publishThr)) {
      f = false;
      fanl &= ~bit;
    }
    const int cnt = __popcll(__ballot(f));
    if (cnt < d.D) {
      const bool cand = inTopic && mc && !f && !dir && S >= d.publishThr;
      const uint64_t key = gs_key64(d.seed, GS_SITE_GP_FANOUT_HB, v, hw, vcol, t);
      if (select_k_lds(cand, key, d.D - cnt, (uint64_t*)sterm)) {
        fanl |= bit;
        f = true;
      }
    }
    ihave |= emit_gossip(d, v, t, hop, head, valid, vcol, inTopic && mc, f, dir, Slive, dirty, dirtyUp, base,
                         (double*)sgw, lane_get(nmT, t));
  }
  // sendGraftPrune + flush: one heartbeat RPC per peer with any control
  if (valid && is_traced(d, v)) {  // prunePeer / graftPeer, gossipsub.go:1334, 1343
    for (uint64_t m = toprune; m; m &= m - 1) trace_emit(d, hop, GS_TRACE_PRUNE, v, vcol, __ffsll((long long)m) - 1, -1, 4);
    for (uint64_t m = tograft; m; m &= m - 1) trace_emit(d, hop, GS_TRACE_GRAFT, v, vcol, __ffsll((long long)m) - 1, -1, 4);
  }
  tograft |= spamGraft;
  if (behaves(d, v, GS_BEHAVE_NO_FORWARD)) tograft = toprune = ihave = 0;  // a squatter sends nothing
  if (d.rpcB != nullptr) {
    // the heartbeat RPC (sendGraftPrune + piggybacked gossip / flush): IHAVE
    // entries of min(ids, MaxIHaveLength) ids, GRAFT and PRUNE entries
    if (lane < d.T) sterm[lane] = (double)min(nmT, d.MaxIHaveLength);
    __syncthreads();
    if (valid && (tograft | toprune | ihave)) {
      int64_t body = 0;
      for (uint64_t m = ihave; m; m &= m - 1) {
        const int t = __ffsll((long long)m) - 1;
        body += gs_pb_field(d.acc[t].ihaveHead + (int64_t)sterm[t] * d.acctIdF);
      }
      for (uint64_t m = tograft; m; m &= m - 1) body += d.acc[__ffsll((long long)m) - 1].graftEnt;
      const int64_t pxA = d.doPX ? d.cPx[cur][rxi(d, e, d.rev[e])] : -1;  // the PRUNEs' PX lists
      for (uint64_t m = toprune; m; m &= m - 1) {
        const int t = __ffsll((long long)m) - 1;
        body += prune_entry(d, e, t, px_count(d, cur, pxA, 1ull << t));
      }
      acct_send(d, e, gs_pb_field(body), 1);
    }
  }
  if (valid) {
    d.mesh[e] = meshl;
    d.fanout[e] = fanl;
    if (tograft | toprune | ihave) {
      const int64_t re = rxi(d, e, d.rev[e]);  // outbox records are indexed by the receiver's in-edge
      d.cGraftHb[cur][re] = tograft;
      d.cPruneHb[cur][re] = toprune;
      d.cIhave[cur][re] = ihave;
      d.cHb[cur][re] = 1;
      if (rpc_traced(d, v, vcol)) {
        // the heartbeat RPC (sendGraftPrune with the piggybacked gossip): its
        // IHAVE ids are the gossip windows of each topic (every id: the host
        // applies emitGossip's MaxIHaveLength cut, include/gs_trace.h)
        auto gwWord = [&](int w) {
          uint64_t x = 0;
          for (int k = 0; k < d.HG; ++k) x |= d.hist[((int64_t)((head + k) % d.R) * d.nOwnH + (v - d.n0)) * d.W + w];
          return x;
        };
        int nIh = 0;
        for (uint64_t m = ihave; m; m &= m - 1) {
          const int t = __ffsll((long long)m) - 1;
          for (int w = t * d.Wt; w < (t + 1) * d.Wt; ++w) nIh += __popcll(gwWord(w));
        }
        const int64_t pxr = d.doPX ? d.cPx[cur][re] : -1;
        rpc_trace(d, hop, v, vcol, 4, 3, GS_RPC_ORD(4, 0),
                  1 + __popcll(tograft) + __popcll(toprune) + nIh + px_count(d, cur, pxr, toprune),
                  [&](auto put) {
                    put(GS_RPC_ITEM_CTL, -1, -1);
                    for (uint64_t m = tograft; m; m &= m - 1) put(GS_RPC_ITEM_GRAFT, __ffsll((long long)m) - 1, -1);
                    for (uint64_t m = toprune; m; m &= m - 1) put(GS_RPC_ITEM_PRUNE, __ffsll((long long)m) - 1, -1);
                    px_each(d, cur, pxr, toprune, [&](int tt, int q) { put(GS_RPC_ITEM_PX, tt, q); });
                    for (uint64_t m = ihave; m; m &= m - 1) {
                      const int t = __ffsll((long long)m) - 1;
                      for (int w = t * d.Wt; w < (t + 1) * d.Wt; ++w)
                        for (uint64_t y = gwWord(w); y; y &= y - 1)
                          put(GS_RPC_ITEM_IHAVE, t, d.slotMid[(int64_t)w * 64 + __ffsll((long long)y) - 1]);
                    }
                  });
      }
    }
  }
  const int g = wave_sum_int(__popcll(tograft));
  const int p = wave_sum_int(__popcll(toprune));
  const int ih = wave_sum_int(__popcll(ihave));
  if (lane == 0) {
    d.fanoutPresent[v] = fpres;
    if (g) ctr_add(d, C_GRAFTS, (unsigned long long)g);
    if (p) ctr_add(d, C_PRUNES, (unsigned long long)p);
    if (ih) ctr_add(d, C_IHAVE, (unsigned long long)ih);
  }
  // mcache.Shift (mcache.go:94-104): clear the ring slot that becomes window 0
  // (the peertx counters of the messages leaving the cache are dropped by
  // k_ptx_rebuild after this launch).  The dropped window stays readable as
  // the "ghost" slot until the next shift (IHAVE payload of this heartbeat).
  for (int w = lane; w < d.W; w += 64) d.hist[((int64_t)newhead * d.nOwnH + (v - d.n0)) * d.W + w] = 0;
  GS_STAMPH(5, GS_CLK());
}

// mcache.Shift's peertx part (mcache.go:94-104): the counters of the
// messages leaving the cache (pre-shift window `last`, still readable after
// k_heartbeat) are dropped and the node's table is rebuilt without them (an
// open-addressing table cannot delete in place).  One wave per node, the table
// staged in LDS (dynamic: 4 << ptxBits bytes); a node without entries is
// skipped.
__global__ __launch_bounds__(64) void k_ptx_rebuild(Dev d, int last) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sT[];
  const int v = d.n0 + blockIdx.x;
  if (d.ptxN[v] == 0) return;
  const int lane = lane_id();
  const int hN = 1 << d.ptxBits;
  uint32_t* const row = ptx_row(d, v);
  const uint64_t* lastw = d.hist + ((int64_t)last * d.nOwnH + (v - d.n0)) * d.W;
  for (int k = lane; k < hN / 4; k += 64) ((uint4*)sT)[k] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  int kept = 0;
  for (int k0 = 0; k0 < hN; k0 += 64 * 4) {
    // (a table smaller than the wave's 256 entries: the lanes past it read
    // nothing, not the next nodes' rows)
    const int qi = (k0 >> 2) + lane;
    const uint4 q = qi < (hN >> 2) ? ((const uint4*)row)[qi] : make_uint4(0u, 0u, 0u, 0u);
    uint32_t ent[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t x = ent[j];
      if (!x) continue;
      const int slot = (int)(x >> 14);
      if ((lastw[slot >> 6] >> (slot & 63)) & 1) continue;  // leaves the cache
      int hsl = ptx_hash(x & ~0xFFu, d.ptxBits);
      while (atomicCAS(&sT[hsl], 0u, x) != 0u) hsl = (hsl + 1) & (hN - 1);
      ++kept;
    }
  }
  __syncthreads();
  for (int k = lane; k < hN / 4; k += 64) ((uint4*)row)[k] = ((const uint4*)sT)[k];
  kept = wave_sum_int(kept);
  if (lane == 0) d.ptxN[v] = kept;
}

// The overflow table's part of the rebuild, after k_ptx_rebuild: the entries
// whose message stays in the cache are collected and the table cleared, then
// each goes back to its node's (rebuilt) table if a slot is free there, else
// to the overflow table.  Launched every heartbeat over the whole table; a
// table without entries returns at once.
__global__ void k_ptxo_collect(Dev d, int last) {
  if (d.ptxOCnt[0] == 0u) return;
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >> d.ptxOBits) return;
  const unsigned long long x = d.ptxO[k];
  if (x == 0ull) return;
  d.ptxO[k] = 0ull;
  const int v = (int)(x >> 32) - 1;
  const int slot = (int)(((uint32_t)x) >> 14);
  const uint64_t* lastw = d.hist + ((int64_t)last * d.nOwnH + (v - d.n0)) * d.W;
  if ((lastw[slot >> 6] >> (slot & 63)) & 1) return;  // leaves the cache
  d.ptxOStage[atomicAdd(&d.ptxOCnt[2], 1u)] = x;
}
__global__ void k_ptxo_reinsert(Dev d) {
  if (d.ptxOCnt[0] == 0u) return;
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)d.ptxOCnt[2]) return;
  const unsigned long long x = d.ptxOStage[k];
  const int v = (int)(x >> 32) - 1;
  const uint32_t ent = (uint32_t)x;
  uint32_t* const row = ptx_row(d, v);
  const int hmask = (1 << d.ptxBits) - 1;
  int hsl = ptx_hash(ent & ~0xFFu, d.ptxBits);
  for (int probe = 0; probe <= hmask; ++probe) {
    if (atomicCAS(&row[hsl], 0u, ent) == 0u) {
      atomicAdd(&d.ptxN[v], 1);
      return;
    }
    hsl = (hsl + 1) & hmask;
  }
  const uint64_t mask = (1ull << d.ptxOBits) - 1;
  uint64_t hs = ptxo_hash(x & ~0xFFull, d.ptxOBits);
  while (atomicCAS(&d.ptxO[hs], 0ull, x) != 0ull) hs = (hs + 1) & mask;  // (it held them all before)
  atomicAdd(&d.ptxOCnt[1], 1u);
}
__global__ void k_ptxo_fin(Dev d) {
  d.ptxOCnt[0] = d.ptxOCnt[1];
  d.ptxOCnt[1] = 0u;
  d.ptxOCnt[2] = 0u;
}

// gs_read_deliveries gather
__global__ void k_read_deliv(Dev d, int slot, int64_t pubhop, int32_t* hop, int32_t* from) {
  // needs GS_FLAG_RECORD_DELIVERIES (age / ffrom kept per slot)
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= d.N) return;
  if (v < d.n0 || v >= d.n1) { hop[v] = -1; from[v] = -1; return; }  // another rank's node
  bool s = (d.seen[(int64_t)v * d.W + (slot >> 6)] >> (slot & 63)) & 1;
  // a rejected / ignored message is seen but never delivered (the author's own
  // publish is), a phantom id is never delivered at all
  const int kind = d.slotKind[slot];
  const int t = slot / d.St;
  if (kind == GS_MSG_PHANTOM) s = false;
  if ((kind == GS_MSG_REJECT || kind == GS_MSG_IGNORE) && ((d.topicVal >> t) & 1) && d.slotSrc[slot] != v) s = false;
  if (!s) { hop[v] = -1; from[v] = -1; return; }
  hop[v] = (int32_t)(pubhop + d.age[(int64_t)v * d.S + slot]);
  const uint8_t f = d.ffrom[(int64_t)v * d.S + slot];
  from[v] = f == 255 ? -1 : d.col[d.rowptr[v] + f];
}

// ---------------------------------------------------------------- churn events
// (gs_schedule_events, applied at the start of their hop)
//
// A connection goes down: one wave per directed edge e = (u -> v), run for
// both directions.  handleDeadPeers + GossipSubRouter.RemovePeer (pubsub.go:
// 521-551, gossipsub.go:534-547): out of the mesh and fanout, no pending
// gossip, the RPCs u sent to v during the previous hop are lost (outbox and
// forwarding sets of parity prv).  tracer.RemovePeer -> peerScore.RemovePeer
// (score.go:602-635): a positive score drops the record, otherwise it is
// retained for RetainScore with firstMessageDeliveries reset and the mesh
// delivery penalty applied (lane = topic).
__global__ __launch_bounds__(64) void k_edge_down(Dev d, const int32_t* __restrict__ edges, int64_t hop,
                                                  int64_t now, int prv) {
  __shared__ double sterm[64];
  const int64_t e = edges[blockIdx.x];
  const int lane = lane_id();
  const int u = d.esrc[e], v = d.col[e];
  const int64_t re = d.rev[e];
  // A partitioned rank does the part it owns: u's side of the connection
  // (edge e: its state and what it was about to send) and, at re = rev[e] in
  // v's in-edge order, the RPCs u sent to v in the previous hop (their records
  // live with the receiver).  Unpartitioned: both.
  const bool ownE = e >= d.e0 && e < d.e1;
  const bool ownR = re >= d.e0 && re < d.e1;
  double s = 0.0;
  if (ownE && d.scoring && d.rstate != nullptr && d.rstate[e] == 1) s = edge_score_wave(d, e, sterm);
  if (lane == 0 && ownR) {
    d.cPre[prv][re] = 0; d.cHb[prv][re] = 0; d.cGraftJoin[prv][re] = 0; d.cGraftHb[prv][re] = 0;
    d.cPruneReply[prv][re] = 0; d.cPruneHb[prv][re] = 0; d.cIhave[prv][re] = 0;
    d.cIwant[prv][re] = -1; d.cIresp[prv][re] = -1;
    if (d.cSpam[prv] != nullptr) { d.cSpam[prv][re] = -1; d.cNSrv[prv][re] = 0; }
    if (d.doPX) d.cPx[prv][re] = -1;
    d.fwdIn[prv][re] = make_ulonglong2(0ull, 0ull);
  }
  if (!ownE) return;
  if (lane == 0) {
    d.alive[e] = 0;
    d.mesh[e] = 0;
    d.fanout[e] = 0;
    d.fwdRelay[prv][e] = 0;
    d.fwdPub[prv][e] = 0;
    d.sdirty[e] = 1;
    if (is_traced(d, u)) trace_emit(d, hop, GS_TRACE_REMOVE_PEER, u, v, -1, -1, 0);  // trace.go:215
    if (d.gater) {  // peerGater.RemovePeer (peer_gater.go:374-383) on the IP's stats object
      const int64_t g = d.rowptr[u] + d.gGrp[e];
      atomicSub(&d.gConn[g], 1);
      d.gExp[g] = now + d.gRetain;  // every removal of this hop writes the same expiry
    }
  }
  if (!d.scoring || d.rstate == nullptr || d.rstate[e] != 1) return;
  const bool drop = s > 0;
  for (int t = lane; t < d.T; t += 64) {
    const int64_t i = tix(d, t, e);
    if (drop) {
      d.fmd[i] = 0; d.mmd[i] = 0; d.mfp[i] = 0; d.imd[i] = 0; dlt_put(d, i, 0);
      d.meshTime[i] = 0; d.graftTime[i] = 0; d.flags[i] = 0;
      continue;
    }
    if (!d.tp[t].scored) continue;
    const TopicP& tp = d.tp[t];
    const uint32_t q = dlt_get(d, i);
    const double mm = eff_mmd(tp, d.mmd[i], q);  // the pending mesh deliveries count
    d.mmd[i] = mm;
    d.fmd[i] = 0;
    dlt_put(d, i, 0);
    const uint8_t fl = d.flags[i];
    if ((fl & 1) && (fl & 2) && mm < tp.MmdThreshold) {
      const double deficit = tp.MmdThreshold - mm;
      d.mfp[i] += deficit * deficit;
    }
    if (fl & 1) d.meshTime[i] = mesh_time_of(d.lastRefresh, d.graftTime[i]);  // the retained record's
    d.flags[i] = fl & ~1;
  }
  if (lane == 0) {
    if (drop) {
      d.bp[e] = 0;
      d.rstate[e] = 0;
    } else {
      d.rstate[e] = 2;
      d.rexpire[e] = now + d.RetainScore;
    }
  }
}

// A connection comes back: AddPeer (gossipsub.go:505-532; peerScore.AddPeer
// score.go:586-600 revives a retained record or starts an empty one).
__global__ void k_edge_up(Dev d, const int32_t* __restrict__ edges, int n, int64_t hop) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int64_t e = edges[k];
  if (e < d.e0 || e >= d.e1) return;  // another rank's connection side
  d.alive[e] = 1;
  if (d.rstate != nullptr) d.rstate[e] = 1;
  d.sdirty[e] = 1;
  if (d.gater) atomicAdd(&d.gConn[d.rowptr[d.esrc[e]] + d.gGrp[e]], 1);  // peerGater.AddPeer (:366-372)
  if (is_traced(d, d.esrc[e]))  // the connection's protocol in `reason` (mixed networks)
    trace_emit(d, hop, GS_TRACE_ADD_PEER, d.esrc[e], d.col[e], -1, -1, 0, d.proto ? d.proto[e] : 0);
}

// ipColocationFactor (score.go:335-379) after the record set changed: per
// observer (one wave per node, lane = edge) the peers with a record that share
// the edge's IP.
__global__ __launch_bounds__(64) void k_p6(Dev d, double* __restrict__ p6) {
  const int v = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const uint32_t ip = valid ? d.ipv4[d.col[e]] : 0u;
  const bool rec = valid && ip != 0 && has_record(d, e);
  int cnt = 0;
  for (int j = 0; j < deg; ++j) {
    const uint32_t ipj = (uint32_t)__builtin_amdgcn_readlane((int)ip, j);
    const int recj = __builtin_amdgcn_readlane(rec ? 1 : 0, j);
    cnt += (recj && ipj == ip) ? 1 : 0;
  }
  if (!valid) return;
  double f = 0.0;
  if (ip != 0 && !d.ipWL[d.col[e]] && cnt > d.IPThr) {
    const double s = (double)(cnt - d.IPThr);
    f = s * s;
  }
  p6[e] = f;
}

// Leave(topic) at node v (handleRemoveSubscription pubsub.go:665-686 ->
// gossipsub.go:1062-1078): tracer.Leave, then for every mesh peer
// tracer.Prune and a PRUNE RPC (sendPrune: a reply-group RPC of this hop).
// One wave per node (items: node, topic mask lo, hi), its topics ascending;
// lane = edge.
__global__ __launch_bounds__(64) void k_leave(Dev d, const int32_t* __restrict__ items, int64_t hop, int cur) {
  __shared__ double sterm[64];
  const int v = items[3 * blockIdx.x];
  const uint64_t mask = (uint64_t)(uint32_t)items[3 * blockIdx.x + 1] | ((uint64_t)(uint32_t)items[3 * blockIdx.x + 2] << 32);
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const bool traced = is_traced(d, v);
  const bool silent = behaves(d, v, GS_BEHAVE_NO_FORWARD);  // a squatter sends no control
  uint64_t meshl = valid ? d.mesh[e] : 0;
  uint64_t pruned = 0;
  int np = 0;
  for (uint64_t mm = mask; mm; mm &= mm - 1) {
    const int t = __ffsll((long long)mm) - 1;
    const uint64_t bit = 1ull << t;
    const int rv = router_of(d, v);
    if (lane == 0 && traced) trace_emit(d, hop, rv == GS_ROUTER_RANDOMSUB ? GS_TRACE_JOIN : GS_TRACE_LEAVE, v, -1, t, -1, 0);
    if (rv != GS_ROUTER_GOSSIPSUB) continue;  // floodsub / randomsub (randomsub.go:166-168 traces a Join)
    const bool m = valid && (meshl & bit);
    // makePrune's live scores: the mesh peers are pruned one after another
    // (ascending), each PRUNE's list made right after its peer's Prune — so a
    // peer's score counts its own Prune once the list is for it or a later peer
    const bool pxOn = d.doPX && !silent && __ballot(m) != 0;
    const bool okPre = pxOn ? px_score_ok(d, base, deg, sterm) : true;
    if (m) {
      meshl &= ~bit;
      pruned |= bit;
      stats_prune(d, e, t);
      if (traced) trace_emit(d, hop, GS_TRACE_PRUNE, v, d.col[e], t, -1, 0);
    }
    if (pxOn) {  // sendPrune's makePrune(p, topic, gs.doPX) (:1087)
      const bool okPost = px_score_ok(d, base, deg, sterm);
      unsigned long long pl = __ballot(m && px_peer(d, e));  // no PX to v1.0 peers (:1804-1807)
      while (pl) {
        const int p = __ffsll((long long)pl) - 1;
        pl &= pl - 1;
        const uint64_t list = px_sel(d, v, base, deg, t, hop, p, (m && lane <= p) ? okPost : okPre);
        if (lane == p) px_append(d, cur, rxi(d, e, d.rev[e]), t, list, base);
      }
    }
    np += __popcll(__ballot(m));
  }
  if (valid && pruned) {
    d.mesh[e] = meshl;
    if (!silent) {
      const int64_t re = rxi(d, e, d.rev[e]);
      d.cPruneReply[cur][re] |= pruned;
      d.cPre[cur][re] = (uint8_t)(d.cPre[cur][re] + __popcll(pruned));  // one sendPrune RPC per topic
      if (d.rpcB != nullptr) {
        int64_t b = 0;
        const int64_t pxA = d.doPX ? d.cPx[cur][re] : -1;  // the PRUNEs' PX lists
        for (uint64_t m = pruned; m; m &= m - 1) {
          const int t = __ffsll((long long)m) - 1;
          b += gs_pb_field(prune_entry(d, e, t, px_count(d, cur, pxA, 1ull << t)));
        }
        acct_send(d, e, b, __popcll(pruned));
      }
      if (rpc_traced(d, v, d.col[e]))
        for (uint64_t m = pruned; m; m &= m - 1) {
          const int t = __ffsll((long long)m) - 1;
          const int64_t pxr = d.doPX ? d.cPx[cur][rxi(d, e, d.rev[e])] : -1;
          rpc_trace(d, hop, v, d.col[e], 0, 3, GS_RPC_ORD(0, GS_RPC_O_LEAVE + t), 2 + px_count(d, cur, pxr, 1ull << t),
                    [&](auto put) {
            put(GS_RPC_ITEM_CTL, -1, -1);
            put(GS_RPC_ITEM_PRUNE, t, -1);
            px_each(d, cur, pxr, 1ull << t, [&](int tt, int q) { put(GS_RPC_ITEM_PX, tt, q); });
          });
        }
    }
  }
  if (lane == 0 && np && !silent) ctr_add(d, C_PRUNES, (unsigned long long)np);
}

// Join(topic) at node v after the start (handleAddSubscription pubsub.go:
// 692-713 -> gossipsub.go:1011-1060): reuse the fanout (dropping peers with a
// negative score) topped up by getPeers, or getPeers(D); tracer.Join, then
// tracer.Graft and one GRAFT RPC per peer.  One wave per node, its topics
// ascending.  Scores are exact: a memo below 0 or after a score change is
// recomputed (the filter compares with 0).
__global__ __launch_bounds__(64) void k_join_pairs(Dev d, const int32_t* __restrict__ items, int64_t hop,
                                                   int64_t now, int cur) {
  __shared__ double sterm[64];
  const int v = items[3 * blockIdx.x];
  const uint64_t mask = (uint64_t)(uint32_t)items[3 * blockIdx.x + 1] | ((uint64_t)(uint32_t)items[3 * blockIdx.x + 2] << 32);
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const bool traced = is_traced(d, v);
  const bool silent = behaves(d, v, GS_BEHAVE_NO_FORWARD);
  const int vcol = valid ? d.col[e] : -1;
  const bool dir = valid && d.direct[e];
  uint64_t meshl = valid ? d.mesh[e] : 0, fanl = valid ? d.fanout[e] : 0, grafted = 0;
  uint64_t fpres = d.fanoutPresent[v];
  double s = valid ? d.score0[e] : 0.0;
  bool stale = valid && d.scoring && (d.sdirty[e] != 0 || !(s >= 0.0));
  if (!d.scoring) s = 0.0;
  int ng = 0;
  for (uint64_t mm = mask; mm; mm &= mm - 1) {
    const int t = __ffsll((long long)mm) - 1;
    const uint64_t bit = 1ull << t;
    if (lane == 0 && traced) trace_emit(d, hop, GS_TRACE_JOIN, v, -1, t, -1, 0);
    if (!gossip_host(d, v)) continue;
    unsigned long long xm = __ballot(stale);
    while (xm) {  // exact Score(p) where the memo may be off
      const int j = __ffsll((long long)xm) - 1;
      xm &= xm - 1;
      const double sj = edge_score_wave(d, base + j, sterm);
      if (lane == j) {
        s = sj;
        stale = false;
      }
    }
    const bool inTopic = valid && edge_up(d, e) && mesh_peer(d, e) && ((d.subA[vcol] >> t) & 1);
    const uint64_t key = gs_key64(d.seed, GS_SITE_GP_JOIN, v, (uint32_t)hop, vcol, t);
    bool g;
    if ((fpres >> t) & 1) {
      g = valid && (fanl & bit) && s >= 0;
      const int have = __popcll(__ballot(g));
      if (have < d.D) g = g || select_k(inTopic && !g && !dir && s >= 0, key, d.D - have);
      fanl &= ~bit;
      fpres &= ~bit;
      if (lane == 0) d.lastpub[(int64_t)v * d.T + t] = INT64_MIN;
    } else {
      g = select_k(inTopic && !dir && s >= 0, key, d.D);
    }
    if (g) {
      meshl |= bit;
      grafted |= bit;
      stats_graft(d, e, t, now);
      stale = true;  // a graft may raise the score (P3 switched off)
      if (traced) trace_emit(d, hop, GS_TRACE_GRAFT, v, vcol, t, -1, 0);  // gossipsub.go:1057
    }
    ng += __popcll(__ballot(g));
  }
  if (valid) {
    d.mesh[e] = meshl;
    d.fanout[e] = fanl;
    if (grafted && !silent) {
      const int64_t re = rxi(d, e, d.rev[e]);
      d.cGraftJoin[cur][re] |= grafted;
      d.cPre[cur][re] = (uint8_t)(d.cPre[cur][re] + __popcll(grafted));  // one sendGraft RPC per topic
      if (d.rpcB != nullptr) {
        int64_t b = 0;
        for (uint64_t m = grafted; m; m &= m - 1) b += gs_pb_field(d.acc[__ffsll((long long)m) - 1].graftEnt);
        acct_send(d, e, b, __popcll(grafted));
      }
      if (rpc_traced(d, v, vcol))
        for (uint64_t m = grafted; m; m &= m - 1) {
          const int t = __ffsll((long long)m) - 1;
          rpc_trace(d, hop, v, vcol, 0, 3, GS_RPC_ORD(0, t), 2, [&](auto put) {
            put(GS_RPC_ITEM_CTL, -1, -1);
            put(GS_RPC_ITEM_GRAFT, t, -1);
          });
        }
    }
  }
  if (lane == 0) {
    d.fanoutPresent[v] = fpres;
    if (ng && !silent) ctr_add(d, C_GRAFTS, (unsigned long long)ng);
  }
}
