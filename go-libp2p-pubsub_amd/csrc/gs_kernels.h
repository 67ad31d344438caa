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
  if (lane == 0 && g) atomicAdd(&d.ctr[C_GRAFTS], (unsigned long long)g);
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

// One wave per receiving node; lanes hold the node's bitset words
// (word w = lane + 64*j).  Senders are scanned in ascending node id — the
// canonical arrival order — so "first deliverer" is the lowest sender.
template <int WPL>
__global__ __launch_bounds__(64) void k_phase_a(Dev d, int64_t h, int cur, int head) {
  __shared__ int cntF[64];
  __shared__ int cntD[64];
  __shared__ unsigned long long xrb[64 * GS_MAX_WPL];
  const int v = blockIdx.x;
  const int lane = lane_id();
  const int prv = cur ^ 1;
  const int W = d.W;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  const int64_t S = d.S;
  cntF[lane] = 0;
  cntD[lane] = 0;
  // randomsub: this lane's neighbour (for the target selection)
  const int myPeer = (d.router == 1 && lane < deg) ? d.col[base + lane] : -1;
  const uint64_t myPeerSub = myPeer >= 0 ? d.sub[myPeer] : 0;
  uint64_t seen[WPL], facc[WPL];
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    seen[j] = (w < W) ? (d.seen[(int64_t)v * W + w] & ~d.pubmask[cur][w]) : 0;  // retire recycled slots
    facc[j] = 0;
  }
  // AcceptFrom graylist (gossipsub.go:578-589) from the hop-start memo S0
  bool gl = false;
  if (lane < deg && d.router == 2 && d.scoring) {
    const int64_t e = base + lane;
    gl = !d.direct[e] && d.score0[e] < d.graylistThr;
  }
  const unsigned long long glmask = __ballot(gl);
  long long nDeliv = 0, nDup = 0, nSent = 0, nGray = 0;
  for (int i = 0; i < deg; ++i) {
    const int64_t e = base + i;
    const int u = d.col[e];
    const int64_t r = d.rev[e];
    const int jr = (int)(r - d.rowptr[u]);
    const uint64_t relay = d.fwdRelay[prv][r];
    const uint64_t pub = d.fwdPub[prv][r];
    const int64_t iresp = d.cIresp[prv][r];
    if ((relay | pub) == 0 && iresp < 0) continue;
    if (iresp >= 0) arena_read(d, prv, iresp, xrb);
    const bool gray = (glmask >> i) & 1;
    int myF = 0, myDup = 0;
    long long sent = 0, rpcs = 0;
    uint64_t freshJ[WPL];
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      freshJ[j] = 0;
      const int w = lane + 64 * j;
      if (w >= W) continue;
      const int tw = w / d.Wt;
      const uint64_t nw = d.newb[prv][(int64_t)u * W + w];
      const uint64_t pm = d.pubmask[prv][w];
      uint64_t x = (nw & ~pm & (((relay >> tw) & 1) ? ~0ull : 0ull)) |
                   (nw & pm & (((pub >> tw) & 1) ? ~0ull : 0ull));
      if (d.router == 1 && x) {  // randomsub: per-message target sets
        uint64_t y = x, keep = 0;
        while (y) {
          const int b = __ffsll((long long)y) - 1;
          y &= y - 1;
          const int64_t slot = (int64_t)w * 64 + b;
          if ((d.sel[(int64_t)u * S + slot] >> jr) & 1) keep |= 1ull << b;
        }
        x = keep;
      }
      const uint64_t xr = iresp >= 0 ? xrb[w] : 0;
      if (x & xr) set_err(d, E_DOUBLE);
      const uint64_t tmask = ((sv >> tw) & 1) ? ~0ull : 0ull;
      const uint64_t xa = (x | xr) & tmask;
      if (!xa) continue;
      const uint64_t fresh = xa & ~seen[j];
      uint64_t dup = xa & seen[j];
      // ReceivedFrom / author exclusion (the sender skipped us): only the
      // forwarded part, and only already-seen messages can be affected
      uint64_t y = dup & x;
      while (y) {
        const int b = __ffsll((long long)y) - 1;
        y &= y - 1;
        const int64_t slot = (int64_t)w * 64 + b;
        const bool own = (pm >> b) & 1;
        if (d.slotSrc[slot] == v || (!own && d.ffrom[(int64_t)u * S + slot] == jr)) dup &= ~(1ull << b);
      }
      sent += __popcll(fresh) + __popcll(dup);
      rpcs += __popcll((fresh | dup) & x);
      if (gray) continue;
      seen[j] |= fresh;
      facc[j] |= fresh;
      freshJ[j] = fresh;
      int nf = 0, nd = 0;
      y = fresh;
      while (y) {
        const int b = __ffsll((long long)y) - 1;
        y &= y - 1;
        const int64_t slot = (int64_t)w * 64 + b;
        const int64_t a = h - d.slotPubHop[slot];
        if (a > d.maxAge) set_err(d, E_LATE);
        d.age[(int64_t)v * S + slot] = (int16_t)a;
        d.ffrom[(int64_t)v * S + slot] = (uint8_t)i;
        nf++;
      }
      y = dup;
      const int64_t window = d.tp[tw].MmdWindow;
      while (y) {
        const int b = __ffsll((long long)y) - 1;
        y &= y - 1;
        const int64_t slot = (int64_t)w * 64 + b;
        const int64_t validated = d.slotPubHop[slot] + d.age[(int64_t)v * S + slot];
        if (!((h - validated) * d.hop_ns > window)) nd++;
        myDup++;
      }
      if (nf || nd) {
        atomicAdd(&cntF[tw], nf);
        atomicAdd(&cntD[tw], nd);
      }
      myF += nf;
    }
    nSent += sent;
    if (gray) {
      nGray += rpcs;  // the IWANT-response RPC is counted with the control RPCs in phase B
      continue;
    }
    nDeliv += myF;
    nDup += myDup;
    if (d.router == 1) {
#pragma unroll
      for (int j = 0; j < WPL; ++j) {
        unsigned long long lanesWith = __ballot(freshJ[j] != 0);
        while (lanesWith) {
          const int src = __ffsll((long long)lanesWith) - 1;
          lanesWith &= lanesWith - 1;
          uint64_t fw = shfl_u64(freshJ[j], src);
          while (fw) {
            const int b = __ffsll((long long)fw) - 1;
            fw &= fw - 1;
            rs_select(d, v, deg, myPeer, myPeerSub, (src + 64 * j) * 64 + b, i);
          }
        }
      }
    }
    const int anyF = __any(myF > 0 || myDup > 0);
    if (anyF && d.scoring) {
      __syncthreads();
      if (lane < d.T) {
        const int nf = cntF[lane], nd = cntD[lane];
        const TopicP& tp = d.tp[lane];
        if ((nf || nd) && tp.scored) {
          const int64_t ti = (int64_t)lane * d.E + e;
          if (nf) d.fmd[ti] = add_ones_capped(d.fmd[ti], nf, tp.FmdCap);
          if (d.flags[ti] & 1) d.mmd[ti] = add_ones_capped(d.mmd[ti], nf + nd, tp.MmdCap);
        }
      }
      __syncthreads();
      cntF[lane] = 0;
      cntD[lane] = 0;
      __syncthreads();
    }
  }
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    if (w >= W) continue;
    d.seen[(int64_t)v * W + w] = seen[j];
    d.newb[cur][(int64_t)v * W + w] = facc[j];
    if (d.router == 2 && facc[j]) d.hist[((int64_t)head * d.N + v) * W + w] |= facc[j];
  }
  long long sums[4] = {nDeliv, nDup, nSent, nGray};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    long long x = sums[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    sums[k] = x;
  }
  if (lane == 0) {
    if (sums[0]) atomicAdd(&d.ctr[C_DELIVERIES], (unsigned long long)sums[0]);
    if (sums[1]) atomicAdd(&d.ctr[C_DUPLICATES], (unsigned long long)sums[1]);
    if (sums[2]) atomicAdd(&d.ctr[C_TRANSMISSIONS], (unsigned long long)sums[2]);
    if (sums[3]) atomicAdd(&d.ctr[C_GRAYLISTED], (unsigned long long)sums[3]);
  }
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
  d.age[(int64_t)src * d.S + slot] = 0;
  d.ffrom[(int64_t)src * d.S + slot] = 255;
  atomicAdd(&d.ctr[C_PUBLISHED], 1ull);
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
