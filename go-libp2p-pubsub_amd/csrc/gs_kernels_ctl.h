// gs_kernels_ctl.h — control-plane kernels: HandleRPC (phase B) and the
// heartbeat.  One wave per node; per-sender / per-topic work is serialised in
// the canonical order (senders ascending, RPCs in send order, topics
// ascending) because GRAFT acceptance depends on the running mesh size.
#pragma once
#include "gs_device.h"

// handleGraft for one topic from sender edge e (gossipsub.go:713-792).
// Scalar (wave-uniform) code; meshcnt is held by lane t.  Returns true when a
// PRUNE for t must be sent back.
__device__ __forceinline__ bool graft_one(const Dev& d, int64_t e, int v, int t, double sc, int64_t now,
                                          int& meshcnt_lane, uint64_t& meshE, bool& dirty) {
  if (!((d.sub[v] >> t) & 1)) return false;  // unknown topic: ignore
  if ((meshE >> t) & 1) return false;         // already in mesh
  if (d.direct[e]) return true;
  const int64_t bi = tix(d, t, e);
  const int64_t be = d.backoff[bi];
  if (be != 0 && now < be) {
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
    add_backoff(d, e, t, now, d.PruneBackoff);
    return true;
  }
  const int mc = __shfl(meshcnt_lane, t);
  if (mc >= d.Dhi && !d.outbound[e]) {
    add_backoff(d, e, t, now, d.PruneBackoff);
    return true;
  }
  stats_graft(d, e, t, now);
  dirty = true;
  meshE |= 1ull << t;
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
    stats_prune(d, e, t);
    if (d.scoring) dirty = true;
    if ((meshE >> t) & 1) {
      meshE &= ~(1ull << t);
      if (lane_id() == t) meshcnt_lane--;
    }
    add_backoff(d, e, t, now, d.PruneRecv);
  }
}

template <int WPL>
__global__ __launch_bounds__(64) void k_phase_b(Dev d, int64_t h, int64_t now, int cur, int head) {
  __shared__ unsigned long long reqb[64 * GS_MAX_WPL];
  __shared__ unsigned long long ptx[GS_PTX];
  __shared__ double sterm[64];
  const int v = blockIdx.x;
  const int lane = lane_id();
  const int prv = cur ^ 1;
  const int W = d.W;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  // lane t: current mesh size of topic t
  uint64_t myMesh = lane < deg ? d.mesh[base + lane] : 0;
  int meshcnt = 0;
  for (int t = 0; t < d.T; ++t) {
    const int c = __popcll(__ballot((myMesh >> t) & 1));
    if (lane == t) meshcnt = c;
  }
  // graylist (AcceptFrom) on the hop-start memo, as in phase A
  bool gl = false;
  if (lane < deg && d.scoring) gl = !d.direct[base + lane] && d.score0[base + lane] < d.graylistThr;
  const unsigned long long glmask = __ballot(gl);
  // node tables: lane q = entry q
  int promN = d.promN[v];
  int64_t pMid = lane < promN ? d.promMid[(int64_t)v * GS_TABLE + lane] : -1;
  int64_t pExp = lane < promN ? d.promExp[(int64_t)v * GS_TABLE + lane] : 0;
  int32_t pSlot = lane < promN ? d.promSlot[(int64_t)v * GS_TABLE + lane] : 0;
  int pEdge = lane < promN ? d.promEdge[(int64_t)v * GS_TABLE + lane] : 0;
  bool promDirty = false;
  // mcache.peertx for this node: (slot, requester edge) -> count, staged in LDS
  int ptxN = d.ptxN[v];
  for (int q = lane; q < ptxN; q += 64) ptx[q] = d.ptx[(int64_t)v * GS_PTX + q];
  __syncthreads();
  bool ptxDirty = false;
  long long cPrunes = 0, cIwantSent = 0, cServed = 0, cGray = 0;
  // senders with control RPCs this hop (lane i = in-edge i), then visit only those
  int64_t rL = 0;
  int npreL = 0, hbL = 0;
  if (lane < deg) {
    rL = d.rev[base + lane];
    npreL = d.cPre[prv][rL];
    hbL = d.cHb[prv][rL];
  }
  unsigned long long cmask = __ballot(npreL != 0 || hbL != 0);
  while (cmask) {
    const int i = __ffsll((long long)cmask) - 1;
    cmask &= cmask - 1;
    const int64_t e = base + i;
    const int u = d.col[e];
    const int64_t r = (int64_t)shfl_u64((uint64_t)rL, i);
    const int npre = __shfl(npreL, i);
    const int hb = __shfl(hbL, i);
    const uint64_t gJoin = d.cGraftJoin[prv][r];
    const uint64_t gHb = d.cGraftHb[prv][r];
    const uint64_t pRep = d.cPruneReply[prv][r];
    const uint64_t pHb = d.cPruneHb[prv][r];
    const uint64_t ihaveT = d.cIhave[prv][r];
    const int64_t iwRec = d.cIwant[prv][r];
    // consume the outbox entry (the sender re-writes it two hops later)
    if (lane == 0) {
      d.cPre[prv][r] = 0;
      d.cHb[prv][r] = 0;
      d.cGraftJoin[prv][r] = 0;
      d.cGraftHb[prv][r] = 0;
      d.cPruneReply[prv][r] = 0;
      d.cPruneHb[prv][r] = 0;
      d.cIhave[prv][r] = 0;
      d.cIwant[prv][r] = -1;
      d.cIresp[prv][r] = -1;
    }
    if ((glmask >> i) & 1) {  // AcceptNone: the whole RPC is dropped
      cGray += npre + hb;
      continue;
    }
    uint64_t meshE = __shfl(myMesh, i);
    bool dirty = false;
    double sc = d.scoring ? d.score1[e] : 0.0;
    int ph = d.peerhave[e];
    int ia = d.iasked[e];
    uint64_t pruneOut = 0;
    int nReplies = 0;
    int64_t respRec = -1, iwantRec = -1;
    // (1) Join RPCs: one GRAFT each (gossipsub.go:1080-1084)
    const int nJoin = __popcll(gJoin);
    {
      uint64_t gj = gJoin;
      while (gj) {
        const int t = __ffsll((long long)gj) - 1;
        gj &= gj - 1;
        if (dirty) { sc = edge_score_wave(d, e, sterm); dirty = false; }
        if (sc >= d.gossipThr) ph++;  // handleIHave's counter (no IHAVE entries)
        if (graft_one(d, e, v, t, sc, now, meshcnt, meshE, dirty)) {
          pruneOut |= 1ull << t;
          nReplies++;
        }
      }
    }
    // (2) reply RPCs: IWANT requests and PRUNEs answering our own control
    const int nRep = npre - nJoin;
    if (nRep > 0) {
      if (dirty) { sc = edge_score_wave(d, e, sterm); dirty = false; }
      const bool gossipOK = sc >= d.gossipThr;
      if (gossipOK) ph += nRep;
      if (gossipOK && iwRec >= 0) {
        // handleIWant (gossipsub.go:674-711): serve cached messages, counting
        // per-peer retransmissions (mcache.GetForPeer)
        uint64_t served[WPL];
        int nServed = 0;
        arena_read(d, prv, iwRec, reqb);
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
          const int w = lane + 64 * j;
          uint64_t req = 0, cache = 0;
          if (w < W) {
            req = reqb[w];
            if (req)
              for (int k = 0; k < d.HL; ++k) cache |= d.hist[((int64_t)((head + k) % d.R) * d.N + v) * W + w];
          }
          uint64_t cand = req & cache;
          served[j] = 0;
          // serialise the retransmission-table updates over the wave
          unsigned long long lanesWith = __ballot(cand != 0);
          while (lanesWith) {
            const int src = __ffsll((long long)lanesWith) - 1;
            lanesWith &= lanesWith - 1;
            uint64_t cw = shfl_u64(cand, src);
            while (cw) {
              const int b = __ffsll((long long)cw) - 1;
              cw &= cw - 1;
              const int slot = (src + 64 * j) * 64 + b;
              // GetForPeer (mcache.go:66-80): ++peertx[mid][p]
              const uint64_t key = ((uint64_t)(uint32_t)slot << 32) | ((uint64_t)i << 8);
              int found = -1;
              for (int q = lane; q < ptxN; q += 64)
                if ((ptx[q] & ~0xFFull) == key) found = q;
              const unsigned long long hit = __ballot(found >= 0);
              int count;
              if (hit) {
                const int fl = __ffsll((long long)hit) - 1;
                const int q = __shfl(found, fl);
                if (lane == 0) {
                  const uint64_t c = ptx[q] & 0xFF;
                  ptx[q] = key | (c < 255 ? c + 1 : 255);
                }
                __syncthreads();
                count = (int)(ptx[q] & 0xFF);
              } else {
                if (ptxN >= GS_PTX) {
                  if (lane == 0) set_err(d, E_PEERTX);
                } else {
                  if (lane == 0) ptx[ptxN] = key | 1;
                  ptxN++;
                  __syncthreads();
                }
                count = 1;
              }
              ptxDirty = true;
              if (count <= d.GR && lane == src) served[j] |= 1ull << b;
            }
          }
          nServed += __popcll(served[j]);
        }
        nServed = wave_sum_int(nServed);
        if (nServed > 0) {
          respRec = arena_write<WPL>(d, cur, served);
          nReplies++;
          cServed += nServed;
        }
      }
      prune_topics(d, e, v, pRep, now, meshcnt, meshE, dirty);
    }
    // (3) heartbeat RPC: IHAVE, GRAFT, PRUNE (gossipsub.go:1618-1654 sends it last)
    if (hb) {
      if (dirty) { sc = edge_score_wave(d, e, sterm); dirty = false; }
      bool iwantAny = false;
      if (sc >= d.gossipThr) {
        ph++;
        if (ph <= d.MaxIHaveMessages && ia < d.MaxIHaveLength && ihaveT) {
          // handleIHave (gossipsub.go:610-672): IHAVE payload = the sender's
          // gossip windows at its heartbeat, now ring slots 1..HG after Shift
          uint64_t want[WPL];
          int nWant = 0, nMids = 0;
          uint64_t bestKey = ~0ull;
          int64_t bestMid = INT64_MAX;
          int bestSlot = -1;
#pragma unroll
          for (int j = 0; j < WPL; ++j) {
            const int w = lane + 64 * j;
            want[j] = 0;
            if (w >= W) continue;
            const int tw = w / d.Wt;
            if (!((ihaveT >> tw) & 1)) continue;
            uint64_t mids = 0;
            mids = d.gw[(int64_t)u * W + w];
            nMids += __popcll(mids);
            if (!((sv >> tw) & 1)) continue;  // topic not in our mesh map
            want[j] = mids & ~d.seen[(int64_t)v * W + w];
            nWant += __popcll(want[j]);
            uint64_t y = want[j];
            while (y) {
              const int b = __ffsll((long long)y) - 1;
              y &= y - 1;
              const int64_t mid = d.slotMid[(int64_t)w * 64 + b];
              const uint64_t k = gs_key64(d.seed, GS_SITE_IWANT, v, u, (uint32_t)mid, (uint32_t)h);
              if (k < bestKey || (k == bestKey && mid < bestMid)) { bestKey = k; bestMid = mid; bestSlot = w * 64 + b; }
            }
          }
          nWant = wave_sum_int(nWant);
          nMids = wave_sum_int(nMids);
          if (nMids > d.MaxIHaveLength * __popcll(ihaveT)) {
            if (lane == 0) set_err(d, E_TRUNCATE);  // per-peer IHAVE truncation: not built yet
          }
          if (nWant > 0) {
            int iask = nWant;
            if (iask + ia > d.MaxIHaveLength) {
              iask = d.MaxIHaveLength - ia;
              if (lane == 0) set_err(d, E_TRUNCATE);
            }
            // wave argmin over (key, mid): the promised message (gossip_tracer.go:53)
            for (int o = 32; o > 0; o >>= 1) {
              const uint64_t ok = shfl_u64(bestKey, lane ^ o);
              const int64_t om = (int64_t)shfl_u64((uint64_t)bestMid, lane ^ o);
              const int os = __shfl(bestSlot, lane ^ o);
              if (ok < bestKey || (ok == bestKey && om < bestMid)) { bestKey = ok; bestMid = om; bestSlot = os; }
            }
            iwantRec = arena_write<WPL>(d, cur, want);
            ia += iask;
            cIwantSent += iask;
            iwantAny = true;
            if (d.scoring) {  // gossipTracer.AddPromise (gossip_tracer.go:48-75)
              const unsigned long long ex = __ballot(lane < promN && pMid == bestMid && pEdge == i);
              if (!ex) {
                if (promN >= GS_TABLE) {
                  if (lane == 0) set_err(d, E_PROMISES);
                } else {
                  if (lane == promN) {
                    pMid = bestMid;
                    pSlot = bestSlot;
                    pEdge = i;
                    pExp = now + d.IWantFollowupTime;
                  }
                  promN++;
                  promDirty = true;
                }
              }
            }
          }
        }
      }
      {
        uint64_t g = gHb;
        uint64_t prunes = 0;
        while (g) {
          const int t = __ffsll((long long)g) - 1;
          g &= g - 1;
          if (graft_one(d, e, v, t, sc, now, meshcnt, meshE, dirty)) prunes |= 1ull << t;
        }
        prune_topics(d, e, v, pHb, now, meshcnt, meshE, dirty);
        pruneOut |= prunes;
        if (iwantAny || prunes) nReplies++;
      }
    }
    // write back per-edge state and our reply RPCs to u
    if (lane == i) myMesh = meshE;
    if (lane == 0) {
      d.mesh[e] = meshE;
      d.peerhave[e] = ph;
      d.iasked[e] = ia;
      if (nReplies) {
        d.cPre[cur][e] = (uint8_t)(d.cPre[cur][e] + nReplies);
        d.cPruneReply[cur][e] |= pruneOut;
        if (iwantRec >= 0) d.cIwant[cur][e] = iwantRec;
        if (respRec >= 0) d.cIresp[cur][e] = respRec;
      }
    }
    cPrunes += __popcll(pruneOut);
  }
  if (promDirty) {
    if (lane < promN && lane < GS_TABLE) {
      d.promMid[(int64_t)v * GS_TABLE + lane] = pMid;
      d.promExp[(int64_t)v * GS_TABLE + lane] = pExp;
      d.promSlot[(int64_t)v * GS_TABLE + lane] = pSlot;
      d.promEdge[(int64_t)v * GS_TABLE + lane] = (uint8_t)pEdge;
    }
    if (lane == 0) d.promN[v] = promN < GS_TABLE ? promN : GS_TABLE;
  }
  if (ptxDirty) {
    __syncthreads();
    const int n = ptxN < GS_PTX ? ptxN : GS_PTX;
    for (int q = lane; q < n; q += 64) d.ptx[(int64_t)v * GS_PTX + q] = ptx[q];
    if (lane == 0) d.ptxN[v] = n;
  }
  if (lane == 0) {
    if (cPrunes) ctr_add(d, C_PRUNES, (unsigned long long)cPrunes);
    if (cIwantSent) ctr_add(d, C_IWANT_SENT, (unsigned long long)cIwantSent);
    if (cServed) ctr_add(d, C_IWANT_SERVED, (unsigned long long)cServed);
    if (cGray) ctr_add(d, C_GRAYLISTED, (unsigned long long)cGray);
  }
}

// ---------------------------------------------------------------- heartbeat prelude
// clearBackoff (every 15 ticks, slack 2 * GossipSubHeartbeatInterval = 2 s,
// gossipsub.go:1573-1592), clearIHaveCounters (:1554-1564) and
// applyIwantPenalties (:1566-1571 -> gossip_tracer.go:79-115, score.go:382).
// A promise is fulfilled iff its message has been delivered since (it was
// unseen when promised), so "fulfilled" == "seen now".
__global__ __launch_bounds__(64) void k_hb_pre(Dev d, int64_t now, uint64_t ticks) {
  const int v = blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  if (valid) {
    d.peerhave[e] = 0;
    d.iasked[e] = 0;
    if (ticks % 15 == 0) {
      for (int t = 0; t < d.T; ++t) {
        const int64_t i = tix(d, t, e);
        const int64_t be = d.backoff[i];
        if (be != 0 && be + 2000000000LL < now) d.backoff[i] = 0;
      }
    }
  }
  if (!d.scoring) return;
  const int n = d.promN[v];
  if (n == 0) return;
  const int64_t ti = (int64_t)v * GS_TABLE + lane;
  int64_t mid = -1, exp = 0;
  int slot = 0, edge = 0;
  if (lane < n) {
    mid = d.promMid[ti];
    exp = d.promExp[ti];
    slot = d.promSlot[ti];
    edge = d.promEdge[ti];
  }
  bool live = lane < n, broken = false;
  if (live) {
    const bool seen = (d.seen[(int64_t)v * d.W + (slot >> 6)] >> (slot & 63)) & 1;
    if (seen) live = false;
    else if (exp < now) { live = false; broken = true; }
  }
  // per-peer broken counts -> AddPenalty(p, count) once per peer
  unsigned long long bm = __ballot(broken);
  int total = __popcll(bm);
  while (bm) {
    const int q = __ffsll((long long)bm) - 1;
    const int pe = __shfl(edge, q);
    const unsigned long long same = __ballot(broken && edge == pe);
    bm &= ~same;
    if (lane == 0) {
      d.bp[base + pe] += (double)__popcll(same);
      d.sdirty[base + pe] = 1;
    }
  }
  // compact the surviving entries
  const unsigned long long lm = __ballot(live);
  const int pos = __popcll(lm & ((1ull << lane) - 1));
  if (live) {
    const int64_t to = (int64_t)v * GS_TABLE + pos;
    d.promMid[to] = mid;
    d.promExp[to] = exp;
    d.promSlot[to] = slot;
    d.promEdge[to] = (uint8_t)edge;
  }
  if (lane == 0) {
    d.promN[v] = __popcll(lm);
    if (total) ctr_add(d, C_PROMISES_BROKEN, (unsigned long long)total);
  }
}

// emitGossip (gossipsub.go:1658-1712) for topic t of node v; lanes = edges.
// The peer filter uses the live Score(p) (:1681): Slive caches it per lane and
// is recomputed (one wave-parallel score per lane) only after the peer's stats
// changed earlier in this heartbeat.
__device__ __forceinline__ uint64_t emit_gossip(const Dev& d, int v, int t, int64_t hop, int head, bool valid,
                                                int vcol, bool inTopic, bool excl, bool dir, double& Slive,
                                                bool& dirty, int64_t rowBase, double* lds,
                                                const uint64_t* sgw) {
  const int lane = lane_id();
  int nm = 0;
  for (int w = t * d.Wt + lane; w < (t + 1) * d.Wt; w += 64) nm += __popcll(sgw[w]);
  nm = wave_sum_int(nm);
  if (nm == 0) return 0;
  if (nm > d.MaxIHaveLength && lane == 0) set_err(d, E_TRUNCATE);
  const bool base = valid && inTopic && !excl && !dir;
  unsigned long long dm = __ballot(base && dirty);
  while (dm) {
    const int j = __ffsll((long long)dm) - 1;
    dm &= dm - 1;
    const double s = edge_score_wave(d, rowBase + j, lds);
    if (lane == j) {
      Slive = s;
      dirty = false;
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
    sel = select_k(cand, key, target);
  }
  return sel ? (1ull << t) : 0;
}

// ---------------------------------------------------------------- heartbeat
// GossipSubRouter.heartbeat (gossipsub.go:1299-1552) for one node: mesh
// maintenance per joined topic (ascending), emitGossip, fanout expiry and
// maintenance, sendGraftPrune (outbox), mcache.Shift.  Scores are the
// heartbeat memo (score1, computed after applyIwantPenalties); emitGossip
// re-scores peers whose stats changed during this heartbeat (live Score()).
__global__ __launch_bounds__(64) void k_heartbeat(Dev d, int64_t hop, int64_t now, uint64_t ticks, int cur,
                                                  int head, int newhead) {
  __shared__ int plst[64];
  __shared__ int obs[64];
  __shared__ int posOf[64];
  __shared__ double sterm[64];
  __shared__ uint64_t sgw[64 * GS_MAX_WPL];
  const int v = blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const int vcol = valid ? d.col[e] : -1;
  // mcache.GetGossipIDs windows 0..HG-1 (mcache.go:82-92): this heartbeat's
  // IHAVE payload, kept as the node's gw row for the receivers' handleIHave
  for (int w = lane; w < d.W; w += 64) {
    uint64_t x = 0;
    for (int k = 0; k < d.HG; ++k) x |= d.hist[((int64_t)((head + k) % d.R) * d.N + v) * d.W + w];
    sgw[w] = x;
    d.gw[(int64_t)v * d.W + w] = x;
  }
  __syncthreads();
  const uint64_t subv = valid ? d.sub[vcol] : 0;
  uint64_t meshl = valid ? d.mesh[e] : 0;
  uint64_t fanl = valid ? d.fanout[e] : 0;
  const double S = valid ? d.score1[e] : 0.0;
  double Slive = S;  // live Score(p) for emitGossip
  const bool dir = valid && d.direct[e];
  const bool ob = valid && d.outbound[e];
  bool dirty = false;
  uint64_t tograft = 0, toprune = 0, ihave = 0;
  const uint64_t joined = d.sub[v];
  const uint32_t hw = (uint32_t)hop;
  for (int t = 0; t < d.T; ++t) {
    if (!((joined >> t) & 1)) continue;
    const uint64_t bit = 1ull << t;
    const bool inTopic = valid && ((subv >> t) & 1);
    bool m = valid && (meshl & bit);
    // drop all peers with negative score, without PX
    if (m && S < 0) {
      stats_prune(d, e, t);
      meshl &= ~bit;
      add_backoff(d, e, t, now, d.PruneBackoff);
      toprune |= bit;
      dirty = true;
      m = false;
    }
    int cnt = __popcll(__ballot(m));
    // do we have enough peers?
    if (cnt < d.Dlo) {
      const bool bo = valid && d.backoff[tix(d, t, e)] != 0;
      const bool cand = inTopic && !m && !bo && !dir && S >= 0;
      const uint64_t key = gs_key64(d.seed, GS_SITE_GP_DLO, v, hw, vcol, t);
      if (select_k(cand, key, d.D - cnt)) {
        stats_graft(d, e, t, now);
        meshl |= bit;
        tograft |= bit;
        dirty = true;
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
        const double sj = __shfl(S, j);
        const uint64_t kj = shfl_u64(k1, j);
        if (sj > S || (sj == S && (kj < k1 || (kj == k1 && j < lane)))) rank1++;
      }
      const bool tail = m && rank1 >= d.Dscore;
      const uint64_t k2 = gs_key64(d.seed, GS_SITE_DHI_TAIL, v, hw, vcol, t);
      int rank2 = 0;
      mm = __ballot(tail);
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const uint64_t kj = shfl_u64(k2, j);
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
        const bool bo = valid && d.backoff[tix(d, t, e)] != 0;
        const bool cand = inTopic && !m && !bo && !dir && ob && S >= 0;
        const uint64_t key = gs_key64(d.seed, GS_SITE_GP_DOUT, v, hw, vcol, t);
        if (select_k(cand, key, d.Dout - outb)) {
          stats_graft(d, e, t, now);
          meshl |= bit;
          tograft |= bit;
          dirty = true;
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
        const double sj = __shfl(S, j);
        if (sj < S || (sj == S && j < lane)) rank++;
      }
      const unsigned long long ml = __ballot(m && rank == cnt / 2);
      const double median = __shfl(S, __ffsll((long long)ml) - 1);
      if (median < d.oppThr) {
        const bool bo = valid && d.backoff[tix(d, t, e)] != 0;
        const bool cand = inTopic && !m && !bo && !dir && S > median;
        const uint64_t key = gs_key64(d.seed, GS_SITE_GP_OPPORTUNISTIC, v, hw, vcol, t);
        if (select_k(cand, key, d.OGP)) {
          stats_graft(d, e, t, now);
          meshl |= bit;
          tograft |= bit;
          dirty = true;
          m = true;
        }
      }
    }
    ihave |= emit_gossip(d, v, t, hop, head, valid, vcol, inTopic, m, dir, Slive, dirty, base, sterm, sgw);
  }
  // expire fanout for topics we haven't published to in a while
  uint64_t fpres = d.fanoutPresent[v];
  for (int t = 0; t < d.T; ++t) {
    const int64_t lp = d.lastpub[(int64_t)v * d.T + t];
    if (lp != INT64_MIN && lp + d.FanoutTTL < now) {
      fpres &= ~(1ull << t);
      fanl &= ~(1ull << t);
      if (lane == 0) d.lastpub[(int64_t)v * d.T + t] = INT64_MIN;
    }
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
      const bool cand = inTopic && !f && !dir && S >= d.publishThr;
      const uint64_t key = gs_key64(d.seed, GS_SITE_GP_FANOUT_HB, v, hw, vcol, t);
      if (select_k(cand, key, d.D - cnt)) {
        fanl |= bit;
        f = true;
      }
    }
    ihave |= emit_gossip(d, v, t, hop, head, valid, vcol, inTopic, f, dir, Slive, dirty, base, sterm, sgw);
  }
  // sendGraftPrune + flush: one heartbeat RPC per peer with any control
  if (valid) {
    d.mesh[e] = meshl;
    d.fanout[e] = fanl;
    if (tograft | toprune | ihave) {
      d.cGraftHb[cur][e] = tograft;
      d.cPruneHb[cur][e] = toprune;
      d.cIhave[cur][e] = ihave;
      d.cHb[cur][e] = 1;
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
  // mcache.Shift (mcache.go:94-104): drop the IWANT retransmission counters of
  // messages leaving the cache (pre-shift window HL-1), then clear the ring
  // slot that becomes window 0.  The dropped window stays readable as the
  // "ghost" slot until the next shift (IHAVE payload of this heartbeat).
  const int n = d.ptxN[v];
  if (n > 0) {
    const int last = (head + d.HL - 1) % d.R;
    const uint64_t* lastw = d.hist + ((int64_t)last * d.N + v) * d.W;
    int kept = 0;
    for (int base = 0; base < n; base += 64) {
      const int q = base + lane;
      uint64_t ent = 0;
      bool live = q < n;
      if (live) {
        ent = d.ptx[(int64_t)v * GS_PTX + q];
        const int slot = (int)(ent >> 32);
        if ((lastw[slot >> 6] >> (slot & 63)) & 1) live = false;
      }
      const unsigned long long lm = __ballot(live);
      const int pos = kept + __popcll(lm & ((1ull << lane) - 1));
      if (live) d.ptx[(int64_t)v * GS_PTX + pos] = ent;  // pos <= q: in-place compaction is safe
      kept += __popcll(lm);
    }
    if (lane == 0) d.ptxN[v] = kept;
  }
  for (int w = lane; w < d.W; w += 64) d.hist[((int64_t)newhead * d.N + v) * d.W + w] = 0;
}

// gs_read_deliveries gather
__global__ void k_read_deliv(Dev d, int slot, int64_t pubhop, int32_t* hop, int32_t* from) {
  // needs GS_FLAG_RECORD_DELIVERIES (age / ffrom kept per slot)
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= d.N) return;
  const bool s = (d.seen[(int64_t)v * d.W + (slot >> 6)] >> (slot & 63)) & 1;
  if (!s) { hop[v] = -1; from[v] = -1; return; }
  hop[v] = (int32_t)(pubhop + d.age[(int64_t)v * d.S + slot]);
  const uint8_t f = d.ffrom[(int64_t)v * d.S + slot];
  from[v] = f == 255 ? -1 : d.col[d.rowptr[v] + f];
}
