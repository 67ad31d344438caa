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

// Exclusive prefix-OR of a 64-bit value over ascending lanes (lane 0 gets 0).
__device__ __forceinline__ uint64_t wave_prefix_or_excl(uint64_t x) {
  const int lane = lane_id();
  uint64_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = shfl_u64(incl, (lane - o) & 63);
    if (lane >= o) incl |= y;
  }
  const uint64_t prev = shfl_u64(incl, (lane - 1) & 63);
  return lane == 0 ? 0ull : prev;
}

__device__ __forceinline__ unsigned long long wave_sum_ll(long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return (unsigned long long)v;
}

// Phase A — handleIncomingRPC / pushMsg for the payload of every RPC sent to
// node v in the previous hop (pubsub.go:946-1022, score.go:693-964).  One
// wave per receiving node; lane i = in-edge i, i.e. sender u_i = col[base+i],
// so the lanes are in the canonical arrival order (senders ascending).
// Topics are walked ascending and the words of a topic ascending; per word,
//   A_i      = what sender i hands over (relay/publish frontier + IWANT response),
//   P_i      = OR of A_j over non-graylisted senders j < i  (exclusive prefix-OR),
//   fresh_i  = A_i & ~seen & ~P_i            (DeliverMessage from sender i),
//   dup_i    = A_i & (seen | P_i) minus the copies the sender never sent
//              (ReceivedFrom / author exclusion, gossipsub.go:1003),
// which is exactly the sender-by-sender scan of the reference with each
// sender's messages in ascending slot order.  The per-(edge, topic) score
// counters of a topic are then updated for all senders at once, one
// coalesced access per array (state is topic-major [t][E]).
// Exclusion: a sender never returns a message to the neighbour it first got
// it from.  The receiver checks its duplicate candidates against the sender's
// first-deliverer table ffc[u][t][rank] (written by u one hop earlier, ranks
// are u's fresh bits of topic t in slot order).
template <int WPL>
__global__ __launch_bounds__(64) void k_phase_a(Dev d, int64_t h, int cur, int head, WMask amR, WMask amW) {
  __shared__ uint64_t sseen[64 * WPL];  // v's seen words (amR + lazily loaded)
  __shared__ uint64_t sU[64 * WPL];     // v's fresh union per word (its next frontier)
  __shared__ uint64_t spm[64 * WPL];    // slots published in the previous hop
  __shared__ uint64_t sold[64 * WPL];   // slots too old for a first delivery
  const int v = blockIdx.x;
  const int lane = lane_id();
  const int prv = cur ^ 1;
  const int W = d.W;
  const int Wt = d.Wt;
  const int T = d.T;
  const int Kt = d.Kt;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  const bool valid = lane < deg;
  // in-edge metadata (lane = in-edge)
  int u = 0, jr = 0;
  uint64_t relay = 0, pub = 0;
  bool gray = false;
  int irOff = 0, irN = 0;
  if (valid) {
    const int64_t e = base + lane;
    u = d.col[e];
    const int64_t r = d.rev[e];
    jr = (int)(r - d.rowptr[u]);
    relay = d.fwdRelay[prv][r] & sv;
    pub = d.fwdPub[prv][r] & sv;
    const int64_t ir = d.cIresp[prv][r];
    if (ir >= 0) {
      irOff = (int)(ir >> 24);
      irN = (int)(ir & 0xFFFFFF);
    }
    gray = d.router == 2 && d.scoring && !d.direct[e] && d.score0[e] < d.graylistThr;
  }
  int irPos = 0;
  int nextSlot = irN > 0 ? d.pool[prv][irOff] : 0x7FFFFFFF;
  const bool authV = d.nAuth[v] > 0;  // v authored a live message: author exclusion possible
  WMask loaded = amR;
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    if (w < W) {
      sseen[w] = wm_has(amR, w) ? d.seen[(int64_t)v * W + w] : 0ull;
      sU[w] = 0ull;
      spm[w] = d.pubmask[prv][w];
      sold[w] = d.oldm[w];
    }
  }
  long long nDeliv = 0, nDup = 0, nSent = 0, nGray = 0;
  const uint8_t* ffcU = d.ffc[prv] + (int64_t)u * T * Kt;
  uint8_t* ffcV = d.ffc[cur] + (int64_t)v * T * Kt;
  const bool scoring = d.scoring != 0;
  const int64_t eIdx = base + lane;

  // ---- software pipeline over chunks (topic t, words w0..w0+3): the loads of
  // the next chunk (sender frontier words; at a topic start also the sender's
  // first-deliverer window and the edge's score counters) are issued before
  // the current chunk is processed, so their latency overlaps its work.
  auto nextTopic = [&](int t0) {
    const uint64_t rest = t0 < 64 ? (sv >> t0) : 0ull;
    return rest ? t0 + __ffsll((long long)rest) - 1 : T;
  };
  uint64_t pnw[4];
  uint64_t pLo = 0, pHi = 0;
  double pF = 0.0, pM = 0.0;
  uint8_t pFl = 0;
  auto issue = [&](int tt, int ww0, bool start) {
    const uint64_t tb = 1ull << tt;
    const bool fw = ((relay | pub) & tb) != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int w = ww0 + k;
      pnw[k] = 0;
      if (fw && w < (tt + 1) * Wt && wm_has(amR, w)) pnw[k] = d.newb[prv][(int64_t)u * W + w];
    }
    if (start) {
      pLo = pHi = 0;
      if (relay & tb) {
        const uint64_t* p = (const uint64_t*)(ffcU + (int64_t)tt * Kt);
        pLo = p[0];
        pHi = p[1];
      }
      pF = pM = 0.0;
      pFl = 0;
      if (scoring && valid && (fw || nextSlot < (tt + 1) * d.St)) {
        const int64_t ti = (int64_t)tt * d.E + eIdx;
        pFl = d.flags[ti];
        pF = d.fmd[ti];
        pM = d.mmd[ti];
      }
    }
  };
  __syncthreads();
  int t = nextTopic(0);
  int w0 = t * Wt;
  if (t < T) issue(t, w0, true);
  int nf = 0, ndc = 0;  // this lane's fresh / creditable-duplicate counts in topic t
  int rankT = 0;        // v's fresh count in topic t so far (wave-uniform)
  int uRank = 0;        // sender's relayed-fresh count in topic t before the current word
  int cBase = 0;        // cached 16-byte window of the sender's ffc row for topic t
  uint64_t cLo = 0, cHi = 0;
  double curF = 0.0, curM = 0.0;
  uint8_t curFl = 0;
  bool start = true;
  while (t < T) {
    uint64_t nwv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) nwv[k] = pnw[k];
    if (start) {
      cLo = pLo;
      cHi = pHi;
      cBase = 0;
      curF = pF;
      curM = pM;
      curFl = pFl;
      nf = ndc = rankT = uRank = 0;
    }
    const int tEnd = (t + 1) * Wt;
    int nt = t, nw0 = w0 + 4;
    bool nStart = false;
    if (nw0 >= tEnd) {
      nt = nextTopic(t + 1);
      nw0 = nt * Wt;
      nStart = true;
    }
    if (nt < T) issue(nt, nw0, nStart);
    const uint64_t tb = 1ull << t;
    const bool fwdRelay = (relay & tb) != 0, fwdPub = (pub & tb) != 0;
    if (__ballot(fwdRelay || fwdPub || nextSlot < tEnd * 64)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int w = w0 + k;
        if (w >= tEnd) break;
        const uint64_t nw = nwv[k];
        const uint64_t pm = spm[w];
        uint64_t x = (fwdRelay ? (nw & ~pm) : 0ull) | (fwdPub ? (nw & pm) : 0ull);
        if (d.router == 1 && x) {  // randomsub: per-message target sets of the sender
          uint64_t y = x, keep = 0;
          while (y) {
            const int b = __ffsll((long long)y) - 1;
            y &= y - 1;
            if ((d.sel[(int64_t)u * d.S + (int64_t)w * 64 + b] >> jr) & 1) keep |= 1ull << b;
          }
          x = keep;
        }
        uint64_t xr = 0;  // IWANT response (slot ids ascending)
        while (nextSlot < (w + 1) * 64) {
          if (nextSlot >= w * 64) xr |= 1ull << (nextSlot & 63);
          ++irPos;
          nextSlot = irPos < irN ? d.pool[prv][irOff + irPos] : 0x7FFFFFFF;
        }
        const uint64_t A = x | xr;
        const uint64_t relF = nw & ~pm;  // the sender's relayed-fresh bits of this word
        if (!__ballot(A != 0)) {
          uRank += __popcll(relF);
          continue;
        }
        if (!wm_has(loaded, w)) {  // IWANT response outside the active window
          if (lane == 0) sseen[w] = d.seen[(int64_t)v * W + w];
          loaded.m[w >> 6] |= 1ull << (w & 63);
          __syncthreads();
        }
        const uint64_t S = sseen[w];
        // ---- copies the sender never sent (it got them from us / we are the author)
        uint64_t excl = 0;
        uint64_t cand = x & ~pm & S;
        while (cand) {
          const int b = __ffsll((long long)cand) - 1;
          cand &= cand - 1;
          const int rank = uRank + __popcll(relF & ((1ull << b) - 1));
          int ffb = -1;  // rank >= Kt: the sender raised E_FCAP when it stored this rank
          if (rank < Kt) {
            const int cb = rank & ~15;
            if (cb != cBase) {
              const uint64_t* p = (const uint64_t*)(ffcU + (int64_t)t * Kt + cb);
              cLo = p[0];
              cHi = p[1];
              cBase = cb;
            }
            const int o = rank - cb;
            ffb = (int)(((o < 8 ? cLo >> (8 * o) : cHi >> (8 * (o - 8)))) & 0xFF);
          }
          if (ffb == jr) excl |= 1ull << b;
        }
        if (authV) {
          uint64_t c2 = x & S & ~excl;
          while (c2) {
            const int b = __ffsll((long long)c2) - 1;
            c2 &= c2 - 1;
            if (d.slotSrc[w * 64 + b] == v) excl |= 1ull << b;
          }
        }
        uRank += __popcll(relF);
        // ---- dedup in sender order
        const uint64_t Ag = gray ? 0ull : A;
        const uint64_t P = wave_prefix_or_excl(Ag);
        const uint64_t fresh = Ag & ~S & ~P;
        const uint64_t U = shfl_u64(P | Ag, 63) & ~S;
        const uint64_t sentBits = A & ~excl;
        nSent += __popcll(sentBits);
        if (gray) nGray += __popcll(x & ~excl);  // one RPC per relayed message, all dropped
        const uint64_t dupK = gray ? 0ull : (sentBits & ~fresh);
        uint64_t cred = dupK;
        if (d.needAge && dupK) {
          // markDuplicateMessageDelivery window (score.go:955): first delivered at
          // pubHop + age; copies of messages first delivered earlier in this hop
          // (bits in P) are within any window
          const int64_t window = d.tp[t].MmdWindow;
          uint64_t y = dupK & S;
          while (y) {
            const int b = __ffsll((long long)y) - 1;
            y &= y - 1;
            const int64_t slot = (int64_t)w * 64 + b;
            const int64_t firstHop = d.slotPubHop[slot] + d.age[(int64_t)v * d.S + slot];
            if ((h - firstHop) * d.hop_ns > window) cred &= ~(1ull << b);
          }
        }
        nf += __popcll(fresh);
        ndc += __popcll(cred);
        nDeliv += __popcll(fresh);
        nDup += __popcll(dupK);
        // ---- v's first deliverers (ffc), ranks in slot order within topic t
        uint64_t f = fresh;
        while (f) {
          const int b = __ffsll((long long)f) - 1;
          f &= f - 1;
          const int rank = rankT + __popcll(U & ((1ull << b) - 1));
          if (rank < Kt) ffcV[(int64_t)t * Kt + rank] = (uint8_t)lane;
          else set_err(d, E_FCAP);
          if (d.needAge || d.record) {
            const int64_t slot = (int64_t)w * 64 + b;
            const int64_t a = h - d.slotPubHop[slot];
            if (d.needAge) d.age[(int64_t)v * d.S + slot] = (int16_t)a;
            if (d.record) d.ffrom[(int64_t)v * d.S + slot] = (uint8_t)lane;
          }
        }
        if (U) {
          if (lane == 0) {
            if ((U & sold[w]) || !wm_has(amW, w)) set_err(d, E_LATE);
            sseen[w] = S | U;
            sU[w] = U;
          }
          rankT += __popcll(U);
          if (d.router == 1) {  // randomsub: targets of every message first delivered here
            uint64_t y = U;
            while (y) {
              const int b = __ffsll((long long)y) - 1;
              y &= y - 1;
              const int ff = __ffsll((long long)__ballot((fresh >> b) & 1)) - 1;
              rs_select(d, v, deg, valid ? u : -1, valid ? d.sub[u] : 0, w * 64 + b, ff);
            }
          }
        }
      }
    }
    if (nStart || nt >= T) {
      // score counters of the in-edges for topic t: fmd += fresh, mmd += fresh +
      // creditable duplicates while in the mesh (score.go:915-928, 945-963)
      if (scoring && valid && (nf | ndc) && d.tp[t].scored) {
        const TopicP& tp = d.tp[t];
        const int64_t ti = (int64_t)t * d.E + eIdx;
        if (nf) d.fmd[ti] = add_ones_capped(curF, nf, tp.FmdCap);
        if (curFl & 1) d.mmd[ti] = add_ones_capped(curM, nf + ndc, tp.MmdCap);
      }
    }
    t = nt;
    w0 = nw0;
    start = nStart;
  }
  __syncthreads();
  // ---- write back: seen, frontier (active words of this hop), mcache Put
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    if (w >= W) continue;
    const uint64_t U = sU[w];
    if (wm_has(loaded, w)) d.seen[(int64_t)v * W + w] = sseen[w];
    if (wm_has(amW, w)) d.newb[cur][(int64_t)v * W + w] = U;
    if (d.router == 2 && U) d.hist[((int64_t)head * d.N + v) * W + w] |= U;
  }
  const unsigned long long s0 = wave_sum_ll(nDeliv), s1 = wave_sum_ll(nDup), s2 = wave_sum_ll(nSent),
                           s3 = wave_sum_ll(nGray);
  if (lane == 0) {
    if (s0) ctr_add(d, C_DELIVERIES, s0);
    if (s1) ctr_add(d, C_DUPLICATES, s1);
    if (s2) ctr_add(d, C_TRANSMISSIONS, s2);
    if (s3) ctr_add(d, C_GRAYLISTED, s3);
  }
}

// Slots whose message was published more than maxAge hops ago: a first
// delivery of one of them in hop h is outside the engine's window (E_LATE).
__global__ void k_oldmask(Dev d, int64_t h) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  const bool old = s < d.S && d.slotSrc[s] >= 0 && d.slotPubHop[s] < h - d.maxAge;
  const unsigned long long m = __ballot(old);
  if (s < d.S && (s & 63) == 0) d.oldm[s >> 6] = m;
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
  const int prevAuthor = d.slotSrc[slot];  // the retired message of this slot
  if (prevAuthor >= 0) atomicSub(&d.nAuth[prevAuthor], 1);
  atomicAdd(&d.nAuth[src], 1);
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
