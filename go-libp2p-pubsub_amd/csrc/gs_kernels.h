// gs_kernels.h — HIP kernels of the gossip engine (gfx950, wave64).
//
// Kernel map (one hop):
//   k_score        thread/edge   peerScore.score            score.go:256-333
//   k_refresh      thread/edge   refreshScores              score.go:495-556
//   k_join         wave/node     Join at hop 0              gossipsub.go:1011-1060
//   k_fanout_pub   wave/pair     Publish fanout creation    gossipsub.go:977-994
//   k_fwd          thread/edge   forwarding-target snapshot gossipsub.go:953-999, floodsub.go:85, randomsub.go:115
//   k_pubmask      thread/msg    slots published this hop (retire mask)
//   k_phase_a      wave/node     payload messages: handleIncomingRPC/pushMsg/
//                                DeliverMessage/DuplicateMessage, senders ascending
//                                                           pubsub.go:946-1022, score.go:693-964
//   k_publish      thread/msg    local publish bookkeeping  pubsub.go:1056, mcache.go:55
//   k_rs_select    wave/(node,msg) randomsub target masks   randomsub.go:115-149
//   k_phase_b      wave/node     HandleRPC per control RPC  gossipsub.go:591-838
//   k_hb_pre       wave/node     clearBackoff, clearIHaveCounters, applyIwantPenalties
//   k_heartbeat    wave/node     mesh maintenance, emitGossip, fanout, mcache.Shift
//                                                           gossipsub.go:1299-1552, 1658-1712
#pragma once
#include "gs_device.h"

// ---------------------------------------------------------------- score
__global__ void k_score(Dev d, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.E) return;
  out[e] = edge_score(d, e);
}

// refreshScores — score.go:495-556 (every peer is connected: no retention path)
__global__ void k_refresh(Dev d, int64_t now) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.E) return;
  for (int t = 0; t < d.T; ++t) {
    const TopicP& tp = d.tp[t];
    if (!tp.scored) continue;
    const int64_t i = (int64_t)t * d.E + e;
    double x = d.fmd[i] * tp.FmdDecay;
    if (x < d.DecayToZero) x = 0;
    d.fmd[i] = x;
    x = d.mmd[i] * tp.MmdDecay;
    if (x < d.DecayToZero) x = 0;
    d.mmd[i] = x;
    x = d.mfp[i] * tp.MfpDecay;
    if (x < d.DecayToZero) x = 0;
    d.mfp[i] = x;
    x = d.imd[i] * tp.ImdDecay;
    if (x < d.DecayToZero) x = 0;
    d.imd[i] = x;
    const uint8_t fl = d.flags[i];
    if (fl & 1) {
      const int64_t mt = now - d.graftTime[i];
      d.meshTime[i] = mt;
      if (mt > tp.MmdActivation) d.flags[i] = fl | 2;
    }
  }
  double b = d.bp[e] * d.BPDecay;
  if (b < d.DecayToZero) b = 0;
  d.bp[e] = b;
}

// SetTopicScoreParams recap — score.go:215-229
__global__ void k_recap(Dev d, int t, double fmdCap, double mmdCap) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.E) return;
  const int64_t i = (int64_t)t * d.E + e;
  if (d.fmd[i] > fmdCap) d.fmd[i] = fmdCap;
  if (d.mmd[i] > mmdCap) d.mmd[i] = mmdCap;
}

// ---------------------------------------------------------------- join (hop 0)
// GossipSubRouter.Join for every subscribed topic, ascending (gossipsub.go:1011-1060).
// At hop 0 no fanout exists, so Join takes getPeers(D, !direct && score >= 0).
__global__ __launch_bounds__(64) void k_join(Dev d, int64_t hop, int64_t now, int cur) {
  const int u = blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const int v = valid ? d.col[e] : 0;
  const uint64_t subv = valid ? d.sub[v] : 0;
  const bool dir = valid && d.direct[e];
  const double s = valid ? d.score0[e] : 0.0;
  uint64_t meshl = 0, gj = 0;
  const uint64_t joined = d.sub[u];
  for (int t = 0; t < d.T; ++t) {
    if (!((joined >> t) & 1)) continue;
    const bool cand = valid && ((subv >> t) & 1) && !dir && s >= 0;
    const uint64_t key = gs_key64(d.seed, GS_SITE_GP_JOIN, u, (uint32_t)hop, v, t);
    const bool sel = select_k(cand, key, d.D);
    if (sel) {
      meshl |= 1ull << t;
      gj |= 1ull << t;
      stats_graft(d, e, t, now);
    }
  }
  if (valid) {
    d.mesh[e] = meshl;
    d.cGraftJoin[cur][e] = gj;
    d.cPre[cur][e] = (uint8_t)__popcll(gj);
  }
  int g = wave_sum_int(valid ? __popcll(gj) : 0);
  if (lane == 0 && g) ctr_add(d, C_GRAFTS, (unsigned long long)g);
}

// ---------------------------------------------------------------- publish-time fanout
// GossipSubRouter.Publish for a topic the node has not joined (gossipsub.go:977-994):
// reuse the fanout, or pick getPeers(D, !direct && score >= publishThreshold);
// lastpub = now.  One wave per (node, topic) pair publishing this hop.
__global__ __launch_bounds__(64) void k_fanout_pub(Dev d, const int32_t* __restrict__ pairs, int npairs,
                                                    int64_t hop, int64_t now) {
  const int p = blockIdx.x;
  if (p >= npairs) return;
  const int u = pairs[2 * p];
  const int t = pairs[2 * p + 1];
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const int v = valid ? d.col[e] : 0;
  uint64_t fo = valid ? d.fanout[e] : 0;
  const bool present = (d.fanoutPresent[u] >> t) & 1;
  const int have = __popcll(__ballot((fo >> t) & 1));
  if (!present || have == 0) {
    const bool cand = valid && ((d.sub[v] >> t) & 1) && !d.direct[e] && d.score0[e] >= d.publishThr;
    const uint64_t key = gs_key64(d.seed, GS_SITE_GP_FANOUT_PUB, u, (uint32_t)hop, v, t);
    const bool sel = select_k(cand, key, d.D);
    const unsigned long long any = __ballot(sel);
    if (any) {
      if (valid) d.fanout[e] = sel ? (fo | (1ull << t)) : fo;
      if (lane == 0) d.fanoutPresent[u] |= 1ull << t;
    }
  }
  if (lane == 0) d.lastpub[(int64_t)u * d.T + t] = now;
}

// ---------------------------------------------------------------- forwarding snapshot
// Topics for which the owner of edge e forwards to col[e] during this hop:
// relay = messages first delivered here, pub = the owner's own publishes.
__global__ void k_fwd(Dev d, int cur) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.E) return;
  const int u = d.esrc[e];
  const uint64_t sv = d.sub[d.col[e]];
  uint64_t relay, pub;
  if (d.router != 2) {  // floodsub.go:85-99 / randomsub.go:115-150: every topic peer
    relay = sv;
    pub = sv;
  } else {
    const uint64_t joined = d.sub[u];
    const uint64_t m = d.mesh[e];
    const bool dir = d.direct[e];
    relay = joined & (m | (dir ? sv : 0));
    if (d.floodPublish) {
      pub = (dir || d.score0[e] >= d.publishThr) ? sv : 0;
    } else {
      pub = (dir ? sv : 0) | (m & joined) | (d.fanout[e] & ~joined);
    }
  }
  d.fwdRelay[cur][e] = relay;
  d.fwdPub[cur][e] = pub;
}

__global__ void k_pubmask(Dev d, int b, int n, int cur) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int slot = d.mSlot[b + i];
  atomicOr((unsigned long long*)&d.pubmask[cur][slot >> 6], 1ull << (slot & 63));
}

// ---------------------------------------------------------------- phase A
// RandomSubRouter.Publish target choice (randomsub.go:115-149) for message
// `slot` first held by node u (first deliverer = neighbour slot ff, 255 = own
// publish): every topic peer except ReceivedFrom and the author, and if more
// than RandomSubD (6) remain, the keyed-shuffle prefix of max(6, ceil(sqrt(size))).
// Wave-cooperative, lanes = u's neighbours; stores the chosen neighbour mask.
__device__ __forceinline__ void rs_select(const Dev& d, int u, int deg, int p, uint64_t subp, int slot, int ff) {
  const int lane = lane_id();
  const int t = slot / d.St;
  const int origin = d.slotSrc[slot];
  const bool cand = lane < deg && ((subp >> t) & 1) && lane != ff && p != origin;
  const int n = __popcll(__ballot(cand));
  bool sel = cand;
  if (n > 6) {
    int target = d.rsTarget < n ? d.rsTarget : n;
    if (target < n) {
      const uint64_t key = gs_key64(d.seed, GS_SITE_RANDOMSUB, u, (uint32_t)d.slotMid[slot], p, 0);
      sel = select_k(cand, key, target);
    }
  }
  const unsigned long long m = __ballot(sel);
  if (lane == 0) d.sel[(int64_t)u * d.S + slot] = m;
}

// Word sets of the message window (W <= 256 words): bit w set = word w may
// hold a message published within the delivery age bound.
struct WMask {
  uint64_t m[4];
};
__device__ __forceinline__ bool wm_has(const WMask& a, int w) { return (a.m[w >> 6] >> (w & 63)) & 1; }
__device__ __forceinline__ int wm_rank(const WMask& a, int w) {
  int r = 0;
  for (int k = 0; k < (w >> 6); ++k) r += __popcll(a.m[k]);
  return r + __popcll(a.m[w >> 6] & ((1ull << (w & 63)) - 1));
}

// Phase A — one wave per receiving node v; lane j*64+l holds word w = l + 64 j
// of v's bitsets.  The frontier of a node (what it forwards this hop) is a
// bitset restricted to the active words amR (messages young enough to be in
// flight) plus a compact array ffc of its first deliverers in slot order, so
// a receiver can skip what a sender got from it (ReceivedFrom exclusion,
// gossipsub.go:1003) by reading ~one cache line instead of per-slot bytes.
// Senders are scanned in ascending node id — the canonical arrival order.
template <int WPL>
__global__ __launch_bounds__(64) void k_phase_a(Dev d, int64_t h, int cur, int head, WMask amR, WMask amW) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* xrb = (unsigned long long*)smem;  // [64*WPL] IWANT-response bits of one sender
  int* cntF = (int*)(smem + 64 * WPL * 8);               // [64] per-topic fresh counts
  int* cntD = cntF + 64;                                  // [64] per-topic creditable duplicates
  int* wscan = cntD + 64;                                 // [64*WPL] exclusive fresh-rank scan per word
  uint8_t* ffTmp = (uint8_t*)(wscan + 64 * WPL);          // [popc(amR)*64] first deliverer per active slot
  const int v = blockIdx.x;
  const int lane = lane_id();
  const int prv = cur ^ 1;
  const int W = d.W;
  const int Wt = d.Wt;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  const int64_t S = d.S;
  cntF[lane] = 0;
  cntD[lane] = 0;
  // in-edge metadata, lane i = in-edge i (one coalesced/gathered load each)
  int uL = 0, jrL = 0;
  uint64_t relayL = 0, pubL = 0;
  int64_t irL = -1;
  bool gl = false;
  if (lane < deg) {
    const int64_t e = base + lane;
    uL = d.col[e];
    const int64_t r = d.rev[e];
    jrL = (int)(r - d.rowptr[uL]);
    relayL = d.fwdRelay[prv][r] & sv;
    pubL = d.fwdPub[prv][r] & sv;
    irL = d.cIresp[prv][r];
    gl = d.router == 2 && d.scoring && !d.direct[e] && d.score0[e] < d.graylistThr;
  }
  unsigned long long amask = __ballot(lane < deg && ((relayL | pubL) != 0 || irL >= 0));
  const unsigned long long glmask = __ballot(gl);
  const int myPeer = (d.router == 1 && lane < deg) ? uL : -1;
  const uint64_t myPeerSub = myPeer >= 0 ? d.sub[myPeer] : 0;
  uint64_t seen[WPL], facc[WPL];
  unsigned loaded = 0;
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    seen[j] = 0;
    facc[j] = 0;
    if (w < W && wm_has(amR, w)) {
      seen[j] = d.seen[(int64_t)v * W + w];
      loaded |= 1u << j;
    }
  }
  long long nDeliv = 0, nDup = 0, nSent = 0, nGray = 0;
  while (amask) {
    const int i = __ffsll((long long)amask) - 1;
    amask &= amask - 1;
    const int u = __shfl(uL, i);
    const int jr = __shfl(jrL, i);
    const uint64_t relay = shfl_u64(relayL, i);
    const uint64_t pub = shfl_u64(pubL, i);
    const int64_t iresp = (int64_t)shfl_u64((uint64_t)irL, i);
    const bool gray = (glmask >> i) & 1;
    const int64_t e = base + i;
    if (iresp >= 0) arena_read(d, prv, iresp, xrb);
    // the sender's frontier words of the topics it forwards to us
    uint64_t nwv[WPL], pmv[WPL];
    int fc[WPL];
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      const int w = lane + 64 * j;
      nwv[j] = 0;
      pmv[j] = 0;
      if (w < W && wm_has(amR, w) && (((relay | pub) >> (w / Wt)) & 1)) {
        nwv[j] = d.newb[prv][(int64_t)u * W + w];
        pmv[j] = d.pubmask[prv][w];
      }
      fc[j] = __popcll(nwv[j] & ~pmv[j]);
    }
    // exclusive scan of the sender's relayed-bit counts over ascending words
    // (only needed when a duplicate candidate must be checked against ffc)
    int running = 0;
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      int incl = fc[j];
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      wscan[lane + 64 * j] = running + incl - fc[j];
      running += __shfl(incl, 63);
    }
    __syncthreads();
    // step 1 (lane = word): what the sender hands us, split fresh / already seen
    uint64_t X[WPL], FR[WPL], DU[WPL];
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      const int w = lane + 64 * j;
      X[j] = FR[j] = DU[j] = 0;
      if (w >= W) continue;
      const int tw = w / Wt;
      const uint64_t nw = nwv[j], pm = pmv[j];
      uint64_t x = (nw & ~pm & (((relay >> tw) & 1) ? ~0ull : 0ull)) |
                   (nw & pm & (((pub >> tw) & 1) ? ~0ull : 0ull));
      if (d.router == 1 && x) {  // randomsub: per-message target sets
        uint64_t y = x, keep = 0;
        while (y) {
          const int b = __ffsll((long long)y) - 1;
          y &= y - 1;
          if ((d.sel[(int64_t)u * S + (int64_t)w * 64 + b] >> jr) & 1) keep |= 1ull << b;
        }
        x = keep;
      }
      const uint64_t xr = iresp >= 0 ? (uint64_t)xrb[w] : 0ull;
      const uint64_t xa = x | xr;
      if (!xa) continue;
      if (!((loaded >> j) & 1)) {  // an IWANT response outside the active window
        seen[j] = d.seen[(int64_t)v * W + w];
        loaded |= 1u << j;
      }
      X[j] = x;
      FR[j] = xa & ~seen[j];
      DU[j] = xa & seen[j];
      if (!gray) {
        seen[j] |= FR[j];
        facc[j] |= FR[j];
      }
    }
    // step 2 (lane = bit of one active word): exclusion, P3 window, records.
    // Every per-message load is one coalesced vector access per word.
    int nF = 0, nDupK = 0, nCred = 0;
    long long sent = 0, rpcs = 0;
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      unsigned long long act = __ballot((FR[j] | DU[j]) != 0);
      while (act) {
        const int o = __ffsll((long long)act) - 1;
        act &= act - 1;
        const int w = o + 64 * j;
        const int tw = w / Wt;
        const uint64_t fresh = shfl_u64(FR[j], o), dup = shfl_u64(DU[j], o), x = shfl_u64(X[j], o);
        const uint64_t nw = shfl_u64(nwv[j], o), pm = shfl_u64(pmv[j], o);
        const uint64_t bit = 1ull << lane;
        const int64_t slot = (int64_t)w * 64 + lane;
        const bool isF = fresh & bit, isD = dup & bit;
        const bool cand = isD && (x & bit);  // ReceivedFrom / author exclusion (gossipsub.go:1003)
        const bool needPh = isF || (isD && !gray && d.needAge);
        const int64_t ph = needPh ? d.slotPubHop[slot] : 0;
        int sSrc = -1, ffb = -1;
        if (cand) {
          sSrc = d.slotSrc[slot];
          if (!(pm & bit)) {
            const int rank = (d.T > 1 ? d.fpre[prv][(int64_t)u * d.T + tw] : 0) + (wscan[w] - wscan[tw * Wt]) +
                             __popcll(nw & ~pm & (bit - 1));
            if (rank < d.fcap) ffb = d.ffc[prv][(int64_t)u * d.fcap + rank];
          }
        }
        const int ag = (isD && !gray && d.needAge) ? d.age[(int64_t)v * S + slot] : 0;
        const bool excl = cand && (sSrc == v || ffb == jr);
        const bool dupK = isD && !excl;
        const int64_t window = d.tp[tw].MmdWindow;
        const bool cred = dupK && (!d.needAge || !((h - (ph + ag)) * d.hop_ns > window));
        const int kD = __popcll(__ballot(dupK));
        const int kF = __popcll(fresh);
        sent += kF + kD;
        rpcs += __popcll(__ballot((isF || dupK) && (x & bit)));
        if (gray) continue;
        const int kC = __popcll(__ballot(cred));
        if (isF) {
          const int64_t a = h - ph;
          const bool inWin = wm_has(amR, w);
          if (a > d.maxAge || !inWin) set_err(d, E_LATE);
          if (inWin) ffTmp[wm_rank(amR, w) * 64 + lane] = (uint8_t)i;
          if (d.needAge) d.age[(int64_t)v * S + slot] = (int16_t)a;
          if (d.record) d.ffrom[(int64_t)v * S + slot] = (uint8_t)i;
        }
        nF += kF;
        nDupK += kD;
        nCred += kC;
        if (d.scoring && d.T > 1 && lane == 0) {
          cntF[tw] += kF;
          cntD[tw] += kC;
        }
      }
    }
    const int myF = nF, myNd = nCred, myDup = nDupK;
    nSent += sent;
    if (gray) {
      nGray += rpcs;  // the IWANT-response RPC is counted with the control RPCs in phase B
      continue;
    }
    nDeliv += myF;
    nDup += myDup;
    // score counters of edge (v <- u): fmd += fresh, mmd += fresh + creditable dups
    if (d.scoring && (myF > 0 || myNd > 0)) {
      const int nfT1 = myF;
      const int ndT1 = myNd;
      __syncthreads();
      if (lane < d.T) {
        const int nf = d.T == 1 ? nfT1 : cntF[lane];
        const int nd = d.T == 1 ? ndT1 : cntD[lane];
        const TopicP& tp = d.tp[lane];
        if ((nf || nd) && tp.scored) {
          const int64_t ti = (int64_t)lane * d.E + e;
          if (nf) d.fmd[ti] = add_ones_capped(d.fmd[ti], nf, tp.FmdCap);
          if (d.flags[ti] & 1) d.mmd[ti] = add_ones_capped(d.mmd[ti], nf + nd, tp.MmdCap);
        }
        cntF[lane] = 0;
        cntD[lane] = 0;
      }
      __syncthreads();
    }
  }
  // ---- write back: seen, frontier (active words of this hop), mcache Put
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    if (w >= W) continue;
    if ((loaded >> j) & 1) d.seen[(int64_t)v * W + w] = seen[j];
    if (wm_has(amW, w)) d.newb[cur][(int64_t)v * W + w] = facc[j];
    else if (facc[j]) set_err(d, E_LATE);
    if (d.router == 2 && facc[j]) d.hist[((int64_t)head * d.N + v) * W + w] |= facc[j];
  }
  // ---- first deliverers in slot order (ffc) and per-topic rank prefixes (fpre);
  // written bit-parallel, one coalesced byte store per active word
  {
    int running = 0;
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      const int w = lane + 64 * j;
      const int c = __popcll(facc[j]);
      int incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      const int rankW = running + incl - c;
      if (d.T > 1 && w < W && (w % Wt) == 0) d.fpre[cur][(int64_t)v * d.T + w / Wt] = rankW;
      unsigned long long act = __ballot(facc[j] != 0);
      while (act) {
        const int o = __ffsll((long long)act) - 1;
        act &= act - 1;
        const int wo = o + 64 * j;
        const uint64_t f = shfl_u64(facc[j], o);
        const int r0 = __shfl(rankW, o);
        const uint64_t bit = 1ull << lane;
        if (f & bit) {
          const int rank = r0 + __popcll(f & (bit - 1));
          if (rank < d.fcap && wm_has(amR, wo))
            d.ffc[cur][(int64_t)v * d.fcap + rank] = ffTmp[wm_rank(amR, wo) * 64 + lane];
          else
            set_err(d, E_LATE);
        }
      }
      running += __shfl(incl, 63);
    }
  }
  // ---- randomsub: choose the targets of every message first delivered here
  if (d.router == 1) {
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      unsigned long long lanesWith = __ballot(facc[j] != 0);
      while (lanesWith) {
        const int src = __ffsll((long long)lanesWith) - 1;
        lanesWith &= lanesWith - 1;
        uint64_t fw = shfl_u64(facc[j], src);
        const int w = src + 64 * j;
        if (!wm_has(amR, w)) continue;  // E_LATE already raised
        const int cw = wm_rank(amR, w);
        while (fw) {
          const int b = __ffsll((long long)fw) - 1;
          fw &= fw - 1;
          rs_select(d, v, deg, myPeer, myPeerSub, w * 64 + b, ffTmp[cw * 64 + b]);
        }
      }
    }
  }
  const long long sums[4] = {nDeliv, nDup, nSent, nGray};  // wave-uniform
  if (lane == 0) {
    if (sums[0]) ctr_add(d, C_DELIVERIES, (unsigned long long)sums[0]);
    if (sums[1]) ctr_add(d, C_DUPLICATES, (unsigned long long)sums[1]);
    if (sums[2]) ctr_add(d, C_TRANSMISSIONS, (unsigned long long)sums[2]);
    if (sums[3]) ctr_add(d, C_GRAYLISTED, (unsigned long long)sums[3]);
  }
}

// Clears the seen bits of recycled message slots (the slots published in
// this hop held messages retired from the window).  One thread per
// (node, word) of the words[] list.
__global__ void k_retire(Dev d, int cur, const int32_t* __restrict__ words, int nwords) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)d.N * nwords) return;
  const int v = (int)(k / nwords);
  const int w = words[k % nwords];
  d.seen[(int64_t)v * d.W + w] &= ~d.pubmask[cur][w];
}

// ---------------------------------------------------------------- local publish
// Topic.Publish -> markSeen -> publishMessage -> router Publish bookkeeping:
// seen, frontier, mcache.Put (gossipsub), slot metadata.
__global__ void k_publish(Dev d, int b, int n, int64_t h, int cur, int head) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int slot = d.mSlot[b + i];
  const int src = d.mSrc[b + i];
  d.slotSrc[slot] = src;
  d.slotPubHop[slot] = h;
  d.slotMid[slot] = d.mId[b + i];
  const int w = slot >> 6;
  const unsigned long long bit = 1ull << (slot & 63);
  atomicOr((unsigned long long*)&d.seen[(int64_t)src * d.W + w], bit);
  atomicOr((unsigned long long*)&d.newb[cur][(int64_t)src * d.W + w], bit);
  if (d.router == 2) atomicOr((unsigned long long*)&d.hist[((int64_t)head * d.N + src) * d.W + w], bit);
  if (d.needAge) d.age[(int64_t)src * d.S + slot] = 0;
  if (d.record) d.ffrom[(int64_t)src * d.S + slot] = 255;
  ctr_add(d, C_PUBLISHED, 1ull);
}

// Randomsub targets of the messages published this hop (one wave per message).
__global__ __launch_bounds__(64) void k_publish_rs(Dev d, int b) {
  const int i = blockIdx.x;
  const int slot = d.mSlot[b + i];
  const int u = d.mSrc[b + i];
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const int p = lane < deg ? d.col[base + lane] : -1;
  const uint64_t subp = p >= 0 ? d.sub[p] : 0;
  rs_select(d, u, deg, p, subp, slot, 255);
}
