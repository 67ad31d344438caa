// gs_kernels.h — HIP kernels of the gossip engine (gfx950, wave64).
//
// Kernel map (one hop):
//   k_score_rows   wave/64 edges peerScore.score (+ memos)  score.go:256-333
//   k_refresh_rows wave/1024 pairs refreshScores (+ exact S0) score.go:495-556
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
#include <type_traits>

#include "gs_device.h"

// ---------------------------------------------------------------- score
// peerScore.score (score.go:256-333) of score_wave_edges(T) consecutive edges
// per wave.  The topic terms of one edge are one contiguous row of each state
// array (full lines), loaded by T lanes; terms go to LDS and lane j then adds
// edge j's terms in ascending topic order, exactly as the reference's loop does.
// Only the edges that need it are computed, so a sparse recompute costs the
// rows it touches, not the whole table.
//   MODE 0: every edge -> out
//   MODE 1: memo S0.  Every consumer of S0 only asks "score >= threshold" for
//     thresholds <= PublishThreshold (AcceptFrom graylist, publish / fanout
//     filters; thresholds are <= 0 by validation, score_params.go:34-51), and
//     between two recomputations the score can only rise unless a graft,
//     prune, penalty or refresh touched the edge (message deliveries raise P2
//     and lower the P3 deficit; FirstMessageDeliveriesWeight >= 0 and
//     MeshMessageDeliveriesWeight <= 0 by validation).  So a memo that is
//     >= PublishThreshold and not dirty gives the same decisions as the exact
//     score; everything else is recomputed exactly.
//   MODE 2: memo S1 for HandleRPC (after the message phase): its decisions
//     compare with 0 and GossipThreshold (<= 0), and only deliveries happened
//     since S0, so a non-negative S0 decides exactly like the exact score.
//   MODE 3: every edge exact -> score1, right after k_refresh_rows left exact
//     scores in S0: only the edges dirtied since (penalties) are recomputed.
//   MODE 4: heartbeat memo -> score1 without a refresh in this hop: exact where
//     a score-lowering change happened or S0 < 0, else S0 (a lower bound >= 0
//     of the exact score, so every heartbeat threshold test — 0, Gossip- and
//     PublishThreshold, all <= 0 — decides exactly).  k_heartbeat recomputes
//     the few scores it needs as values (Dhi ranking) from the same rule.
#define GS_SB 8   // passes per load batch
#ifndef GS_RB
#define GS_RB 8   // refresh: pairs per lane per load batch
#endif
#define GS_RP 1024  // (edge, topic) pairs of one wave's LDS term table
__device__ __forceinline__ int rp_pad(int pl) { return pl + (pl >> 6); }
// Edges per wave of k_score_rows: lane = edge for the need test, and the
// needy edges' T-topic rows fill the lanes in passes of 64 / T edges.
__host__ __device__ __forceinline__ int score_wave_edges(int T) { return T * 64 <= GS_RP ? 64 : GS_RP / T; }
// A wave tests GS_SCW consecutive edges (four per lane) and recomputes the
// needy ones in chunks of score_wave_edges(T) (the LDS term table's edges):
// at T = 64 a wave per 16 edges made 2M waves per launch for a test that
// rarely finds work.
#define GS_SCW 256
template <int MODE, bool LANE_T>
__global__ __launch_bounds__(64) void k_score_rows(Dev d, double* __restrict__ out) {
  __shared__ double sT[GS_RP + GS_RP / 64];  // [edge][topic], padded: conflict-free column reads
  __shared__ uint16_t sList[GS_SCW];         // the needy edges (offsets from eb)
  const int lane = lane_id();
  const int T = d.T;
  const int sgw = score_wave_edges(T);
  const int64_t eb = d.e0 + (int64_t)blockIdx.x * GS_SCW;
  int nNeed = 0;
#pragma unroll
  for (int k = 0; k < GS_SCW / 64; ++k) {
    const int64_t e = eb + 64 * k + lane;
    const bool in = e < d.e1;
    double s0 = 0.0;
    bool need = false;
    if (in) {
      if (MODE == 0) {
        need = true;
      } else {
        s0 = d.score0[e];
        need = MODE == 1 ? (d.sdirty[e] != 0 || !(s0 >= d.publishThr))
               : MODE == 2 ? !(s0 >= 0.0)
               : MODE == 4 ? (d.sdirty[e] != 0 || !(s0 >= 0.0))
                           : d.sdirty[e] != 0;
      }
    }
    if (!d.scoring) {
      if (in) {
        if (MODE == 0) out[e] = 0.0;
        if (MODE == 1) { d.score0[e] = 0.0; d.sdirty[e] = 0; }
        if (MODE >= 2) d.score1[e] = 0.0;
      }
      continue;
    }
    if (MODE >= 2 && in && !need) d.score1[e] = s0;
    const unsigned long long m = __ballot(need);
    if (need) sList[nNeed + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)(64 * k + lane);
    nNeed += __popcll(m);
  }
  if (!d.scoring || nNeed == 0) return;
  __syncthreads();
  // LANE_T (T divides 64): lane = (edge of the pass, topic); else one edge
  // per pass, lane = topic
  const int G = LANE_T ? 64 / T : 1;
  const int gi = LANE_T ? lane / T : 0;
  const int tl = LANE_T ? (lane & (T - 1)) : (lane < T ? lane : 0);
  const bool lt = LANE_T || lane < T;
  const bool scoredL = lt && d.tp[tl].scored;
  const uint64_t scoredT = __ballot(lane < T && d.tp[lane < T ? lane : 0].scored);
  for (int c0 = 0; c0 < nNeed; c0 += sgw) {
    const int nc = min(sgw, nNeed - c0);  // the chunk's edges: positions 0 .. nc - 1
    const int P = (nc + G - 1) / G;
    for (int p0 = 0; p0 < P; p0 += GS_SB) {
      // GS_SB passes per batch: every load of the batch in flight at once
      int js[GS_SB];
#pragma unroll
      for (int k = 0; k < GS_SB; ++k) {
        const int q = (p0 + k) * G + gi;
        js[k] = (lt && q < nc) ? q : -1;
      }
      TermIn x[GS_SB];
#pragma unroll
      for (int k = 0; k < GS_SB; ++k)
        x[k] = term_load(d, (eb + sList[c0 + (js[k] < 0 ? 0 : js[k])]) * T + tl);
#pragma unroll
      for (int k = 0; k < GS_SB; ++k)
        if (js[k] >= 0) sT[rp_pad(js[k] * T + tl)] = scoredL ? term_eval(d.tp[tl], x[k]) : 0.0;
    }
    __syncthreads();
    for (int j = lane; j < nc; j += 64) {
      const int64_t e = eb + sList[c0 + j];
      double score = 0.0;
      for (int t = 0; t < T; ++t)
        if ((scoredT >> t) & 1) score += sT[rp_pad(j * T + t)];
      score = has_record(d, e) ? score_tail(d, e, score) : 0.0;
      if (MODE == 0) out[e] = score;
      if (MODE == 1 || MODE == 3) { d.score0[e] = score; d.sdirty[e] = 0; }
      if (MODE >= 2) d.score1[e] = score;
    }
    __syncthreads();  // the term table is the next chunk's
  }
}

// refreshScores — score.go:495-556, and the exact score of every edge from
// the refreshed state into S0 (sdirty cleared): nothing but refreshScores
// changed the state since the hop's message phase, so this is the value the
// next S0 pass would compute.
// A wave owns GS_RP consecutive (edge, topic) pairs — GS_RP / T whole edges —
// and lane l takes pairs l, l + 64, ...: every lane busy for any T (at T = 1
// a wave covers 1024 edges, at T = 64 sixteen, one topic per lane).  LANE_T:
// T divides 64, so a lane's topic is fixed (lane % T) and its params stay in
// registers; otherwise each pair finds its own.  Terms go to LDS (one pad
// word per 64: conflict-free at T = 64) and the sum per edge runs in
// ascending topic order, as the reference's loop does.
// CHURN: some connection may be down (gs_schedule_events): retained records
// are not decayed and expire; the honest instantiation carries none of it.
template <bool CHURN, bool LANE_T, bool NDLT>
__global__ __launch_bounds__(64) GS_OCC_RF void k_refresh_rows(Dev d, int64_t now) {
  __shared__ double sT[GS_RP + GS_RP / 64];
  const int lane = lane_id();
  const int T = d.T;
  const int epw = GS_RP / T;
  const int64_t e0 = d.e0 + (int64_t)blockIdx.x * epw;
  const int ng = (int)min((int64_t)epw, d.e1 - e0);
  const int np = ng * T;
  const int64_t p0 = e0 * T;
  const int tl = lane < T ? lane : 0;
  const uint64_t scoredT = __ballot(lane < T && d.tp[tl].scored);
  const int tLane = LANE_T ? (lane & (T - 1)) : 0;
  // the score tail's per-edge inputs (P5 app score through col, P6, P7) of the
  // lane's edge, loaded with the first batch instead of after the topic sums
  // (one edge per lane when the wave covers at most 64 edges)
  double tApp = 0.0, tP6 = 0.0, tBp = 0.0;
  if (epw <= 64 && lane < ng) {
    const int64_t e = e0 + lane;
    tApp = d.app[d.col[e]];
    tP6 = d.p6[e];
    tBp = d.bp[e];
  }
  for (int k0 = 0; 64 * k0 < np; k0 += GS_RB) {
    uint32_t q[GS_RB];
    double fmd[GS_RB], mmd[GS_RB], mfp[GS_RB], imd[GS_RB];
    int64_t gt[GS_RB];
    uint8_t fl[GS_RB];
#pragma unroll
    for (int k = 0; k < GS_RB; ++k) {
      const int pl = min(lane + 64 * (k0 + k), np - 1);
      const int64_t i = p0 + pl;
      q[k] = dlt_get_t<NDLT>(d, i);
      fmd[k] = d.fmd[i];
      mmd[k] = d.mmd[i];
      mfp[k] = d.mfp[i];
      imd[k] = d.anyImd ? d.imd[i] : 0.0;
      gt[k] = d.graftTime[i];
      fl[k] = d.flags[i];
    }
#pragma unroll
    for (int k = 0; k < GS_RB; ++k) {
      const int pl = lane + 64 * (k0 + k);
      if (pl >= np) break;
      const int64_t i = p0 + pl;
      int t = tLane;
      int64_t e = 0;
      if (!LANE_T || CHURN) {
        pair_split(d, i, e, t);
        if (LANE_T) t = tLane;
      }
      const TopicP& tp = d.tp[t];
      const bool act = (scoredT >> t) & 1;
      double term = 0.0;
      uint8_t st = 1;
      if (CHURN && d.rstate != nullptr) st = d.rstate[e];
      if (CHURN && st != 1) {
        // a retained record is not decayed; past its expiry it is dropped
        // (score.go:500-509); the host then recounts P6 (removeIPs)
        if (st == 2 && now > d.rexpire[e]) {
          d.fmd[i] = 0; d.mmd[i] = 0; d.mfp[i] = 0; d.imd[i] = 0; dlt_put_t<NDLT>(d, i, 0);
          d.meshTime[i] = 0; d.graftTime[i] = 0; d.flags[i] = 0;
        } else if (act) {
          term = topic_term(d, tp, i);  // the stored record as it is
        }
      } else if (act) {
        TermIn x;
        x.q = 0;
        double v = eff_fmd(tp, fmd[k], q[k]) * tp.FmdDecay;
        if (v < d.DecayToZero) v = 0;
        x.fmd = v;
        v = eff_mmd(tp, mmd[k], q[k]) * tp.MmdDecay;
        if (v < d.DecayToZero) v = 0;
        x.mm = v;
        v = mfp[k] * tp.MfpDecay;
        if (v < d.DecayToZero) v = 0;
        x.mfp = v;
        v = imd[k] * tp.ImdDecay;
        if (v < d.DecayToZero) v = 0;
        x.im = v;
        x.fl = fl[k];
        x.mt = 0;
        // unchanged counters (mostly zeros staying zero) are not written back
        if (q[k]) dlt_put_t<NDLT>(d, i, 0);
        if (x.fmd != fmd[k]) d.fmd[i] = x.fmd;
        if (x.mm != mmd[k]) d.mmd[i] = x.mm;
        if (x.mfp != mfp[k]) d.mfp[i] = x.mfp;
        if (d.anyImd && x.im != imd[k]) d.imd[i] = x.im;
        if (x.fl & 1) {
          x.mt = now - gt[k];  // meshTime (score.go:518-520): mesh_time_of() from here on
          if (x.mt > tp.MmdActivation) {
            x.fl |= 2;
            d.flags[i] = x.fl;
          }
        }
        term = term_eval(tp, x);
      }
      sT[rp_pad(pl)] = term;
    }
  }
  __syncthreads();
  for (int j = lane; j < ng; j += 64) {
    const int64_t e = e0 + j;
    bool frozen = false, dropped = false;
    if (CHURN && d.rstate != nullptr) {
      const uint8_t st = d.rstate[e];
      frozen = st != 1;
      dropped = st == 2 && now > d.rexpire[e];
    }
    const bool pre = epw <= 64;  // tail inputs already in registers (lane j == edge j)
    double b = pre ? tBp : d.bp[e];
    if (dropped) {
      b = 0;
      d.bp[e] = 0;
      d.rstate[e] = 0;
    } else if (!frozen) {
      b *= d.BPDecay;
      if (b < d.DecayToZero) b = 0;
      d.bp[e] = b;
    }
    double score = 0.0;
    if (d.scoring && !dropped && (!CHURN || has_record(d, e))) {
      for (int t = 0; t < T; ++t)
        if ((scoredT >> t) & 1) score += sT[rp_pad(j * T + t)];
      // score_tail with the refreshed P7 (d.bp[e] == b after the store above)
      score = pre ? score_tail_v(d, score, tApp, tP6, b) : score_tail(d, e, score);
    }
    d.score0[e] = score;
    d.sdirty[e] = 0;
  }
}

// Folds the pending deliveries of every pair into fmd / mmd.
__global__ void k_fold_all(Dev d) {
  const int64_t p = d.e0 * d.T + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= d.e1 * d.T) return;
  const uint32_t q = dlt_get(d, p);
  if (!q) return;
  int64_t e;
  int t;
  pair_split(d, p, e, t);
  const TopicP& tp = d.tp[t];
  d.fmd[p] = eff_fmd(tp, d.fmd[p], q);
  d.mmd[p] = eff_mmd(tp, d.mmd[p], q);
  dlt_put(d, p, 0);
}

// gs_read_topic_stats_edges: the counters of n chosen edges, out[i*T + t],
// pending deliveries applied (eff_fmd / eff_mmd) without writing them back.
// Output arrays are packed after each other in `out` (8-byte fields first).
__global__ void k_gather_pairs(Dev d, const int64_t* __restrict__ edges, int64_t n, uint8_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nk = n * d.T;
  if (k >= nk) return;
  const int64_t e = edges[k / d.T];
  const int t = (int)(k % d.T);
  double* o = (double*)out;
  int64_t* oi = (int64_t*)out;
  uint8_t* of = out + 48 * nk;
  if (e < d.e0 || e >= d.e1) {
    for (int a = 0; a < 6; ++a) o[a * nk + k] = 0.0;
    of[k] = 0;
    return;
  }
  const int64_t i = tix(d, t, e);
  const TopicP& tp = d.tp[t];
  const uint32_t q = dlt_get(d, i);
  o[k] = eff_fmd(tp, d.fmd[i], q);
  o[nk + k] = eff_mmd(tp, d.mmd[i], q);
  o[2 * nk + k] = d.mfp[i];
  o[3 * nk + k] = d.imd[i];
  oi[4 * nk + k] = (d.flags[i] & 1) ? mesh_time_of(d.lastRefresh, d.graftTime[i]) : d.meshTime[i];
  oi[5 * nk + k] = d.graftTime[i];
  of[k] = d.flags[i];
}

// gs_read_backoff_edges: the backoff expiries of n chosen edges, out[i*T + t]
// (0 = no entry; an edge outside this rank's range reads 0).
__global__ void k_gather_backoff(Dev d, const int64_t* __restrict__ edges, int64_t n, int64_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n * d.T) return;
  const int64_t e = edges[k / d.T];
  const int t = (int)(k % d.T);
  out[k] = (e < d.e0 || e >= d.e1) ? 0 : d.backoff[tix(d, t, e)];
}

// Folds the pending deliveries of topic t into fmd / mmd.
__global__ void k_fold(Dev d, int t) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  const int64_t i = tix(d, t, e);
  const uint32_t q = dlt_get(d, i);
  if (!q) return;
  const TopicP& tp = d.tp[t];
  d.fmd[i] = eff_fmd(tp, d.fmd[i], q);
  d.mmd[i] = eff_mmd(tp, d.mmd[i], q);
  dlt_put(d, i, 0);
}

// SetTopicScoreParams recap — score.go:215-229
__global__ void k_recap(Dev d, int t, double fmdCap, double mmdCap) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  const int64_t i = tix(d, t, e);
  if (d.fmd[i] > fmdCap) d.fmd[i] = fmdCap;
  if (d.mmd[i] > mmdCap) d.mmd[i] = mmdCap;
}

// ---------------------------------------------------------------- join (hop 0)
// GossipSubRouter.Join for every subscribed topic, ascending (gossipsub.go:1011-1060).
// At hop 0 no fanout exists, so Join takes getPeers(D, !direct && score >= 0).
__global__ __launch_bounds__(64) void k_join(Dev d, int64_t hop, int64_t now, int cur) {
  const int u = d.n0 + blockIdx.x;
  if (!gossip_host(d, u)) return;  // floodsub.go:102-104, randomsub.go:162-164: Join only traces
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const int v = valid ? d.col[e] : 0;
  const uint64_t subv = valid ? d.subA[v] : 0;
  const bool dir = valid && d.direct[e];
  const double s = valid ? d.score0[e] : 0.0;
  uint64_t meshl = 0, gj = 0;
  const uint64_t joined = d.sub[u];
  for (int t = 0; t < d.T; ++t) {
    if (!((joined >> t) & 1)) continue;
    const bool cand = valid && edge_up(d, e) && mesh_peer(d, e) && ((subv >> t) & 1) && !dir && s >= 0;
    const uint64_t key = gs_key64(d.seed, GS_SITE_GP_JOIN, u, (uint32_t)hop, v, t);
    const bool sel = select_k(cand, key, d.D);
    if (sel) {
      meshl |= 1ull << t;
      gj |= 1ull << t;
      stats_graft(d, e, t, now);
      if (is_traced(d, u)) trace_emit(d, hop, GS_TRACE_GRAFT, u, v, t, -1, 0);  // gossipsub.go:1057
    }
  }
  const bool silent = behaves(d, u, GS_BEHAVE_NO_FORWARD);  // a squatter sends no control
  if (silent) gj = 0;
  if (valid) {
    d.mesh[e] = meshl;
    const int64_t rj = rxi(d, e, d.rev[e]);
    d.cGraftJoin[cur][rj] = gj;
    d.cPre[cur][rj] = (uint8_t)__popcll(gj);
    if (d.rpcB != nullptr && gj) {  // one sendGraft RPC per topic (gossipsub.go:1080-1084)
      int64_t b = 0;
      for (uint64_t m = gj; m; m &= m - 1) b += gs_pb_field(d.acc[__ffsll((long long)m) - 1].graftEnt);
      acct_send(d, e, b, __popcll(gj));
    }
    if (gj && rpc_traced(d, u, v))
      for (uint64_t m = gj; m; m &= m - 1) {
        const int t = __ffsll((long long)m) - 1;
        rpc_trace(d, hop, u, v, 0, 3, GS_RPC_ORD(0, t), 2, [&](auto put) {
          put(GS_RPC_ITEM_CTL, -1, -1);
          put(GS_RPC_ITEM_GRAFT, t, -1);
        });
      }
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
    const bool cand = valid && edge_up(d, e) && mesh_peer(d, e) && ((d.subA[v] >> t) & 1) && !d.direct[e] &&
                      d.score0[e] >= d.publishThr;
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
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  const int u = d.esrc[e];
  const uint64_t sv = d.subA[d.col[e]];  // the peer's subscriptions as u knows them
  uint64_t relay, pub;
  if (!gossip_host(d, u)) {  // floodsub.go:85-99 / randomsub.go:115-150: every topic peer
    relay = sv;
    pub = sv;
  } else {
    const uint64_t joined = d.sub[u];
    const uint64_t m = d.mesh[e];
    const bool dir = d.direct[e];
    // a floodsub-protocol peer gets every message of its topics at score >=
    // PublishThreshold (gossipsub.go:969-975)
    const uint64_t fs = (!mesh_peer(d, e) && d.score0[e] >= d.publishThr) ? sv : 0;
    relay = joined & (m | (dir ? sv : 0) | fs);
    if (behaves(d, u, GS_BEHAVE_NO_FORWARD)) relay = 0;  // a squatter relays nothing
    if (d.floodPublish) {
      pub = (dir || d.score0[e] >= d.publishThr) ? sv : 0;
    } else {
      pub = (dir ? sv : 0) | (m & joined) | (d.fanout[e] & ~joined) | fs;
    }
  }
  if (!edge_up(d, e)) relay = pub = 0;  // no connection: nothing is sent
  if (d.fwdRelay[cur][e] == relay && d.fwdPub[cur][e] == pub) return;
  // partitioned engine: a forwarding set that changed since this parity was
  // last exchanged must reach the receiver's rank (gs_exchange.h)
  if (d.xmark) d.xmark[e] = 1;
  d.fwdRelay[cur][e] = relay;
  d.fwdPub[cur][e] = pub;
  d.fwdIn[cur][rxi(d, e, d.rev[e])] = make_ulonglong2(relay, pub);
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
// Floodsub-protocol peers are always sent to (randomsub.go:117-118); only the
// randomsub-protocol candidates are sampled.
__device__ __forceinline__ void rs_select(const Dev& d, int u, int64_t base, int deg, int p, uint64_t subp, int slot,
                                          int ff) {
  const int lane = lane_id();
  const int t = slot / d.St;
  const int origin = d.slotSrc[slot];
  const bool cand = lane < deg && ((subp >> t) & 1) && lane != ff && p != origin;
  const bool fs = cand && d.proto != nullptr && d.proto[base + lane] == GS_PROTO_FLOODSUB;
  const bool rc = cand && !fs;
  const int n = __popcll(__ballot(rc));
  bool sel = cand;
  if (n > 6) {
    int target = d.rsTarget < n ? d.rsTarget : n;
    if (target < n) {
      const uint64_t key = gs_key64(d.seed, GS_SITE_RANDOMSUB, u, (uint32_t)d.slotMid[slot], p, 0);
      sel = fs || select_k(rc, key, target);
    }
  }
  const unsigned long long m = __ballot(sel);
  if (lane == 0) d.sel[(int64_t)u * d.S + slot] = m;
}
// rs_select for two messages at once on a node of degree <= 32: half h =
// lane >> 5 takes message (slotA, slotB)[h] over every edge (lane & 31), the
// same candidates, keys and lowest-lane tie rule (select_k_half), so each
// message's mask equals rs_select's.  p / subp hold lane el's values in lanes
// 0..31 (mirrored here).
__device__ __forceinline__ void rs_select2(const Dev& d, int u, int64_t base, int deg, int pIn, uint64_t subpIn,
                                           int slotA, int ffA, int slotB, int ffB) {
  const int lane = lane_id();
  const int h = lane >> 5, el = lane & 31;
  const int p = __shfl(pIn, el);
  const uint64_t subp = shfl_u64(subpIn, el);
  const int slot = h ? slotB : slotA;
  const int ff = h ? ffB : ffA;
  const int t = slot / d.St;
  const int origin = d.slotSrc[slot];
  const bool cand = el < deg && ((subp >> t) & 1) && el != ff && p != origin;
  const bool fs = cand && d.proto != nullptr && d.proto[base + el] == GS_PROTO_FLOODSUB;
  const bool rc = cand && !fs;
  const int n = __popc((uint32_t)(__ballot(rc) >> (32 * h)));  // this half's candidates
  bool sel = cand;
  const int target = d.rsTarget < n ? d.rsTarget : n;
  if (n > 6 && target < n) {  // (per half: select_k_half runs under divergence)
    const uint64_t key = gs_key64(d.seed, GS_SITE_RANDOMSUB, u, (uint32_t)d.slotMid[slot], p, 0);
    sel = fs || select_k_half(rc, key, target);
  }
  const unsigned long long m = __ballot(sel);
  if (lane == 0) d.sel[(int64_t)u * d.S + slotA] = m & 0xFFFFFFFFull;
  if (lane == 32) d.sel[(int64_t)u * d.S + slotB] = m >> 32;
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

__device__ __forceinline__ int wave_min_int(int x) {
  for (int o = 32; o > 0; o >>= 1) {
    const int y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}

#define GS_NO_SLOT 0x7FFFFFFF

// Debug build only (-DGS_STAMPS): cycle stamps at pass boundaries of every
// 1024th node, read with gs_debug_stamps.
#ifdef GS_STAMPS
// every stamp index is checked against the allocation ((N / 1024 + 1) * 24
// words: phase A | phase B | heartbeat, 8 stamps per sampled node); an index
// past it (never expected: k <= 7, blockIdx.x < N) flags E_STAMP, no write
#define GS_STAMP_AT(region, k, val)                                                                \
  do {                                                                                             \
    if ((blockIdx.x & 1023) == 0 && lane == 0) {                                                   \
      const int64_t _i = ((int64_t)d.N / 1024 + 1) * 8 * (region) + (blockIdx.x >> 10) * 8 + (k);  \
      if ((k) >= 0 && (k) < 8 && _i < ((int64_t)d.N / 1024 + 1) * 24) d.stamps[_i] = (val);        \
      else set_err(d, E_STAMP);                                                                    \
    }                                                                                              \
  } while (0)
#define GS_STAMP(k) GS_STAMP_AT(0, k, clock64())
#define GS_STAMPB(k) GS_STAMP_AT(1, k, clock64())
// heartbeat: stamp k = value v (a clock or an accumulated cycle count)
#define GS_STAMPH(k, v) GS_STAMP_AT(2, k, v)
// a node wave that returns early leaves no stale stamps of an earlier hop
// behind (round 5's negative phase-B intervals were such stale stamps)
#define GS_STAMPB_CLEAR()                                  \
  do {                                                     \
    for (int _k = 0; _k < 8; ++_k) GS_STAMP_AT(1, _k, 0ull); \
  } while (0)
#define GS_CLK() clock64()
#else
#define GS_STAMPH(k, v) \
  do {                  \
  } while (0)
#define GS_CLK() 0ull
#define GS_STAMP(k) \
  do {              \
  } while (0)
#define GS_STAMPB(k) \
  do {               \
  } while (0)
#define GS_STAMPB_CLEAR() \
  do {                    \
  } while (0)
#endif

// Phase A — handleIncomingRPC / pushMsg for the payload of every RPC sent to
// node v in the previous hop (pubsub.go:946-1022, score.go:693-964).  One
// wave per receiving node; lane i = in-edge i, i.e. sender u_i = col[base+i],
// in the canonical arrival order (senders ascending).
//
// What a sender forwarded is its frontier list fl[u]: the slots it first
// received in the previous hop, tagged with the in-edge they came from, and
// its own publishes (tag 255), ascending by slot, filtered here by the
// sender's per-edge forwarding topics.  A copy the sender never sent — back to
// the neighbour it got the message from, or to the author (gossipsub.go:1003)
// — is dropped by its tag.
//   pass 1 (every 16-byte block of every sender's list is a work item, spread
//          over the lanes): each delivered copy records the lowest non-
//          graylisted sender per slot (LDS byte min) and its count per
//          (topic, sender);
//   pass 2 (lane = word):   fresh = delivered & ~seen; the first deliverer of a
//          fresh slot is its lowest sender, exactly the reference's sender-by-
//          sender scan (DeliverMessage from that sender, DuplicateMessage from
//          every other copy); seen, mcache and v's own frontier list are written;
//   pass 3 (lane = edge):   fmd / mmd of every (topic, in-edge) updated once.
// LDS slot tables cover the words of the active window amR (messages young
// enough to be in flight), indexed by the word's rank in amR; the lowest-
// deliverer table holds one byte per YOUNG slot only (published in the last
// maxAge + 1 hops: d.yTab gives each amR word's young-slot mask and prefix),
// which halves it at config4 (about half of an amR word's slots hold older
// messages): less LDS per wave, more waves per CU.  A copy of an older slot
// can only be a duplicate (or E_LATE).
// NARROW: the host proved that no sender can deliver more than 255 copies of
// one topic in this hop (every topic has <= 255 live message slots), so the
// (sender, topic) counters are 8-bit copies | 8-bit first deliveries, two per
// LDS word: half the counter table, more waves per CU.
// ADV (the adversarial model: topic validators, the peer gater, attacker
// behaviours; host-selected, so the honest path compiles without it):
//   * every payload RPC passes AcceptFrom's peer gater (peer_gater.go:320-363)
//     on the hop-start gater state: payload RPCs carry one draw each
//     (GS_SITE_GATER, key = message id), a sender's control RPCs share one;
//     AcceptControl drops the payload and throttles the peer's promises;
//   * a fresh message of a topic with a validator is validated (validation.go:
//     274-351): REJECT / IGNORE verdicts mark it seen without delivering it
//     (P4 for every copy of a rejected message); with a bounded validation
//     queue only the first valQueue fresh messages in arrival order (first
//     deliverer, then message id) are validated, the copies of the rest are
//     RejectValidationQueueFull (not seen; the gater's throttle counter);
//   * an IWANT spammer re-requests every message it received, per sender.
// ADV takes the Dev record from device memory (the engine uploads it before
// the launch): as a by-value argument the compiler copied all 1.5 KB of it to
// every lane's scratch in the adversarial instantiations.  The honest path
// keeps the kernel-argument copy (a little faster there).
template <bool ADV>
using PhaseADev = std::conditional_t<ADV, const Dev*, Dev>;
__device__ __forceinline__ const Dev& dev_of(const Dev& d) { return d; }
__device__ __forceinline__ const Dev& dev_of(const Dev* d) { return *d; }
// occupancy floor: 3 waves/SIMD (<= 168 VGPRs, GS_WPE_PA); the honest wide-
// counter instantiation (config3: T = 1, St > 254) 4 (<= 128 VGPRs): it is not
// LDS-bound (a few KB per wave) and ran 98.9 -> 82.7 ms per round at 4 waves
#ifndef GS_WPE_PA_WIDE
#define GS_WPE_PA_WIDE 4
#endif
template <bool NARROW, bool ADV>
constexpr int pa_waves = (!NARROW && !ADV) ? GS_WPE_PA_WIDE : GS_WPE_PA;
// DENSE (one topic, honest, one rank; gs_engine.hip denseGossip): pass 1 reads
// the senders' frontier bitmaps fb instead of their lists (see "pass 1, dense"
// below); passes 1b, 2 and 3 are the same code.  amF: the words the node's fb
// row of this parity may hold bits in (written over in pass 2b).
template <int WPL, bool NARROW, bool ADV, bool DENSE = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(pa_waves<NARROW, ADV>))) void k_phase_a(
    PhaseADev<ADV> dArg, int64_t h, int cur, int head,
                                                WMask amR, WMask amW, WMask amP, WMask amF, int nR, int nY) {
  static_assert(!(DENSE && ADV), "the dense pass 1 is honest-only");
  const Dev& d = dev_of(dArg);
  extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
  const int nCnt = (d.T * d.maxDeg + 7) & ~7;
  const int nCntW = NARROW ? nCnt / 2 : nCnt;             // LDS words of the counter table
  uint32_t* scnt = smem32;  // [MD][T] copies | fresh << 16 (NARROW: u16 copies | fresh << 8)
  uint64_t* sD = (uint64_t*)(scnt + nCntW);               // [nR] delivered young slots (non-graylisted)
  // scnt word of pair (sender i, topic t).  (Rotating each sender's row so
  // that one topic's copies from different senders fall into different LDS
  // banks measured slower at config4, 96.1 -> 100.3 ms per round: the address
  // arithmetic in passes 2 and 3 cost more than the conflicts it removed.)
  const int cT = d.T;
  auto cword = [&](int i, int t) -> int { return NARROW ? (i * cT + t) >> 1 : i * cT + t; };
  uint64_t* sYm = sD + nR;                                // [nR] young-slot mask of each amR word
  uint16_t* sRk = (uint16_t*)(sYm + nR);                  // [W] rank of word w in amR, 0xFFFF = outside
  uint16_t* sYp = sRk + d.W;                              // [nR] young slots in the amR words before it
  uint8_t* sFirst = (uint8_t*)(sYm + nR) + ((2 * (d.W + nR) + 15) & ~15);  // [nY] lowest deliverer per young slot
  uint32_t* sUnc = (uint32_t*)(sFirst + nY);              // [MD][T] uncredited duplicates (needAge / pmask)
  // drec.peers of this node (score.go:786-818): the senders whose duplicate
  // of a message was already counted — tracked only for nodes that re-request
  // messages they have (IWANT spammers), the only receivers of repeats
  const int prow = (ADV && d.pmaskRow != nullptr) ? d.pmaskRow[d.n0 + blockIdx.x] : -1;
  const bool hasUnc = d.needAge || (ADV && d.pmaskRow != nullptr);
  // ADV tables after sUnc (present only in the ADV launch)
  uint32_t* sInv = sUnc + (hasUnc ? nCnt : 0);            // [MD][T] copies of rejected messages
  uint32_t* sPer = sInv + nCnt;                           // [4][64] per sender: accepted copies, valid /
                                                          // rejected / ignored first deliveries
  double* sGThr = (double*)(sPer + 4 * 64);               // [64] gater threshold per sender, < 0 = accept
  uint64_t* sDrop = (uint64_t*)(sGThr + 64);              // [nR] fresh messages dropped by a full queue
  // block -> sender without a search: a bit per list block where a non-empty
  // sender's list starts (the first GS_BMAP * 64 blocks), and the non-empty
  // senders in ascending order as first block | sender << 24 | copies << 32
  // (past the map: a binary search over the first blocks)
  __shared__ uint64_t sStart[GS_BMAP];
  __shared__ uint64_t sComp[64];
  __shared__ uint64_t sRelay[64], sPub[64];
  __shared__ int sSnd[64];        // sender node | jr << 24 | graylisted << 31
  __shared__ uint32_t sAddr[64];  // a sender's copies: its pushed segment (in 8-slot units), or its list
  __shared__ uint32_t sQ[GS_QCAP];         // sent copies awaiting delivery: slot | sender << 16
  const int v = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int prv = cur ^ 1;
  const int W = d.W;
  const int T = d.T;
  const int FC = d.FC;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  const bool valid = lane < deg;
  const bool gossipV = gossip_host(d, v);  // peerScore, gater and mcache exist on gossipsub hosts only
  const bool scoring = d.scoring != 0 && gossipV;
  // in-edge metadata (lane = in-edge)
  int u = 0, jr = -1, Ln = 0;
  int64_t pOff = -1;  // the pushed segment of this in-edge (k_push), -1 = the sender's list
  uint64_t relay = 0, pub = 0, relayAll = 0, pubAll = 0;
  bool gray = false;
  int irOff = 0, irN = 0;
  if (valid) {
    const int64_t e = base + lane;
    u = d.col[e];
    jr = d.jrIn[e];
    // only copies of v's own topics are handled (pubsub.go:959); what the
    // sender sent on other topics (a peer that left is still in the sender's
    // mesh until its PRUNE arrives) only counts as transmitted (uSent below)
    const ulonglong2 fw = d.fwdIn[prv][e];
    relayAll = fw.x;
    pubAll = fw.y;
    relay = relayAll & sv;
    pub = pubAll & sv;
    const int64_t ir = d.cIresp[prv][e];
    if (ir >= 0) {
      irOff = (int)(ir >> 24);
      irN = (int)(ir & 0xFFFFFF);
    }
    gray = scoring && !d.direct[e] && d.score0[e] < d.graylistThr;
    if (relayAll | pubAll) {
      // the sender pushed this edge's copies (k_push; a remote sender's record
      // and segment arrived with the exchange): read that segment
      if (d.ibxRec[0] != nullptr) {
        const int64_t rec = d.ibxRec[prv][e];
        if (rec >= 0) {
          pOff = rec >> 24;
          Ln = (int)(rec & 0xFFFFFF);
        }
      }
      if (pOff < 0) Ln = d.fln[prv][u];
    }
  }
  // DENSE: the sender's frontier row is read when it relays to v or (as an
  // author) publishes to v; exD = the copies it did not send v because v had
  // delivered them to it first (ReceivedFrom, counted by the sender: fex)
  bool liveD = false, authU = false;
  int exD = 0;
  if constexpr (DENSE) {
    authU = valid && d.nAuth[u] > 0;
    if (valid && (relayAll | pubAll)) {
      liveD = d.fbN[prv][u] != 0 && (relayAll != 0 || authU);
      exD = d.fex[prv][d.rev[base + lane]];
    }
    Ln = 0;
  }
  const uint64_t authM = __ballot(authU);  // DENSE: the neighbours that author a live message
  const uint64_t pushM = __ballot(pOff >= 0);  // senders whose copies were pushed
  GS_STAMP(0);
  const bool authV = d.nAuth[v] > 0;  // v authored a live message: author exclusion possible
  for (int k = lane; k < nCntW / 4; k += 64) ((uint4*)scnt)[k] = make_uint4(0, 0, 0, 0);
  const bool acct = d.rpcB != nullptr;
  if (hasUnc)
    for (int k = lane; k < nCnt / 4; k += 64) ((uint4*)sUnc)[k] = make_uint4(0, 0, 0, 0);
  for (int k = lane; k < nR; k += 64) {
    sD[k] = 0;
    sYm[k] = d.yTab[k];
    sYp[k] = (uint16_t)d.yTab[d.W + k];
  }
  {
    int rb = 0;  // rank of word 64 j + lane in amR
#pragma unroll
    for (int j = 0; j < GS_MAX_WPL; ++j) {
      const uint64_t m = amR.m[j];
      if (64 * j + lane < W)
        sRk[64 * j + lane] = ((m >> lane) & 1) ? (uint16_t)(rb + __popcll(m & ((1ull << lane) - 1))) : (uint16_t)0xFFFF;
      rb += __popcll(m);
    }
  }
  for (int k = lane; k < nY / 16; k += 64) ((uint4*)sFirst)[k] = make_uint4(~0u, ~0u, ~0u, ~0u);
  // ---- ADV: the hop-start peer-gater decision inputs (lane = in-edge)
  bool ctlGated = false;  // the sender's control RPCs of this hop got AcceptControl
  int nSrvRpc = 0;        // reply RPCs of the sender carrying served messages
  if constexpr (ADV) {
    for (int k = lane; k < nCnt / 4; k += 64) ((uint4*)sInv)[k] = make_uint4(0, 0, 0, 0);
    for (int k = lane; k < 4 * 64; k += 64) sPer[k] = 0;
    for (int k = lane; k < nR; k += 64) sDrop[k] = 0;
    double thr = -1.0;
    if (d.gater && gossipV && valid && !gray && !d.direct[base + lane]) {
      // AcceptFrom's circuit breaker on this node's hop-start counters (:329-342)
      const int64_t last = d.gLast[v];
      const double gv = d.gValidate[v], gt = d.gThrottle[v];
      const bool active = !(last == INT64_MIN || h * d.hop_ns - last > d.gQuiet) && gt != 0 &&
                          !(gv != 0 && gt / gv < d.gThreshold);
      if (active) {
        const int64_t ge = base + d.gGrp[base + lane];
        const double de = d.gSt[ge], du = d.gSt[d.eOwn + ge], ig = d.gSt[2 * d.eOwn + ge], rj = d.gSt[3 * d.eOwn + ge];
        const double total = de + d.gDupW * du + d.gIgnW * ig + d.gRejW * rj;
        if (total != 0) thr = (1 + de) / (1 + total);
      }
    }
    sGThr[lane] = thr;
    if (valid && thr >= 0 && (d.cPre[prv][base + lane] != 0 || d.cHb[prv][base + lane] != 0)) {
      const double uu = gs_key_to_unit(gs_key64(d.seed, GS_SITE_GATER, v, u, (uint32_t)h, 0xFFFFFFFFu));
      ctlGated = !(uu < thr);
    }
    if (valid && d.cNSrv[prv] != nullptr) nSrvRpc = d.cNSrv[prv][base + lane];
    else if (irN) nSrvRpc = 1;
  }
  // per-sender view for the block-parallel walk
#ifndef GS_PB8
#define GS_PB8 1  // timing A/B: -DGS_PB8=0 reads pushed segments 4 slots (8 B) per block
#endif
  constexpr int EPBP = GS_PB8 ? 8 : 4;  // slots per block of a pushed segment (16 B: 8 slots)
  // 16-byte blocks of the sender's list (4 entries) or pushed segment (8 slots)
  const int nb = pOff >= 0 ? (Ln + EPBP - 1) / EPBP : (Ln + 3) >> 2;
  const int bincl = wave_incl_sum(nb);
  const int totalBlk = wave_last(bincl);
  const int nNE = __popcll(__ballot(nb > 0));  // non-empty senders
  {
    const uint64_t ne = __ballot(nb > 0);
    for (int k = lane; k < GS_BMAP; k += 64) sStart[k] = 0ull;
    __syncthreads();
    const int fb = bincl - nb;
    if (nb > 0) {
      sComp[__popcll(ne & ((1ull << lane) - 1))] =
          (uint64_t)(unsigned)fb | ((uint64_t)lane << 24) | ((uint64_t)(unsigned)Ln << 32);
      if (fb < 64 * GS_BMAP) atomicOr((unsigned long long*)&sStart[fb >> 6], 1ull << (fb & 63));
    }
  }
  sRelay[lane] = relay;
  sPub[lane] = pub;
  // sender node | jr << 24 | randomsub sender << 30 | graylisted << 31
  sSnd[lane] = valid ? (u | (jr << 24) | (rs_host(d, u) ? (1 << 30) : 0) | (gray ? (1 << 31) : 0)) : 0;
  // (pushed segments are 8-aligned; N * FC <= 2^31 entries, checked in gs_engine.hip start)
  sAddr[lane] = pOff >= 0 ? (uint32_t)(pOff >> 3) : (uint32_t)u * (uint32_t)FC;
  const uint64_t scoredT = __ballot(lane < T && scoring && d.tp[lane].scored);  // scored topics
  // ---- prefetch (phase A is LDS-bound at ~10 waves per CU, so registers are
  // free to hold loads in flight across pass 1): pass 3's 16-bit pending
  // words when the node's fit one batch, and pass 2's seen / mcache / old-slot
  // words of the active window; none of them is written before this wave's
  // own passes 2b / 3
  constexpr int PF3 = 16;
#ifndef GS_PF
#define GS_PF 1  // timing A/B: -DGS_PF=0 builds the phase A without the prefetch
#endif
  constexpr bool kPf = GS_PF != 0;
  const int nWdPf = (kPf && NARROW && scoring && d.dltN != nullptr) ? (deg * T) >> 1 : 0;
  const bool pf3 = nWdPf > 0 && nWdPf <= 64 * PF3;
  uint32_t q3[PF3];
  if (pf3) {
    const uint32_t* const pw = (const uint32_t*)(d.dltN + base * T);
#pragma unroll
    for (int k = 0; k < PF3; ++k) {
      const int wi = lane + 64 * k;
      q3[k] = pw[wi < nWdPf ? wi : nWdPf - 1];
    }
  }
  // (the honest instantiation only: the adversarial one has no registers to spare)
  uint64_t Sp[WPL], Hp[WPL], Op[WPL];
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    Sp[j] = Hp[j] = Op[j] = 0;
    if constexpr (!ADV && kPf) {
      const bool act = w < W && wm_has(amR, w);
      if (act || (w < W && wm_has(amP, w))) Sp[j] = d.seen[(int64_t)v * W + w];
      if (act) {
        Op[j] = d.oldm[w];
        if (gossipV) Hp[j] = d.hist[((int64_t)head * d.nOwnH + (v - d.n0)) * W + w];
      }
    }
  }
  __syncthreads();
  GS_STAMP(1);

  int nSent = 0, nGray = 0;
  long long nCopies = 0;  // delivered copies (non-graylisted)
  int nGatedCopies = 0;   // ADV: payload RPCs dropped by the gater
  uint64_t throttled = 0; // ADV: senders throttled this hop (ThrottlePeer), lane-uniform after the ballot
  // ADV: the verdict of slot's message: its kind on a topic with a validator
  auto kindOf = [&](int slot, int t) -> int {
    if constexpr (!ADV) return GS_MSG_VALID;
    return ((d.topicVal >> t) & 1) ? (int)d.slotKind[slot] : GS_MSG_VALID;
  };
  // ADV: the gater's AcceptFrom for the payload RPC carrying slot from sender i
  auto gated = [&](int i, int slot) -> bool {
    if constexpr (!ADV) return false;
    const double thr = sGThr[i];
    if (thr < 0) return false;
    const uint32_t mid = (uint32_t)d.slotMid[slot];
    const double uu = gs_key_to_unit(gs_key64(d.seed, GS_SITE_GATER, v, d.col[base + i], (uint32_t)h, mid));
    return !(uu < thr);
  };
  // One delivered copy of `slot` from sender i (sent, not graylisted).
  const bool trv = is_traced(d, v);
  auto deliver = [&](int i, int slot, bool payloadRpc) {
    if (payloadRpc && gated(i, slot)) {  // AcceptControl: payload ignored (pubsub.go:951-955)
      ++nGatedCopies;
      throttled |= 1ull << i;
      return;
    }
    const int w = slot >> 6;
    const int t = (int)__umulhi((unsigned)slot, d.stMagic);
    if (trv) trace_emit(d, h, GS_TRACE_COPY, v, d.col[base + i], t, d.slotMid[slot], 2);
    const int kind = kindOf(slot, t);
    if constexpr (ADV) {
      atomicAdd(&sPer[i], 1u);
      if (kind == GS_MSG_REJECT) atomicAdd(&sInv[i * T + t], 1u);
    }
    if (kind == GS_MSG_VALID) {
      if (NARROW) {
        // no-return add: the host proved the 8-bit count cannot overflow
        const int pl = i * T + t;
        atomicAdd(&scnt[cword(i, t)], 1u << (16 * (pl & 1)));
      } else {
        atomicAdd(&scnt[cword(i, t)], 1u);
      }
    }
    ++nCopies;
    const int rk = sRk[w];
    const uint64_t ym = rk == 0xFFFF ? 0ull : sYm[rk];
    const bool young = (ym >> (slot & 63)) & 1;
    unsigned long long pold = 0;  // this node's drec.peers of the message before the copy
    if (prow >= 0 && kind == GS_MSG_VALID)
      pold = atomicOr((unsigned long long*)&d.pmask[(int64_t)prow * d.S + slot], 1ull << i);
    if (d.needAge || !young || prow >= 0) {
      const bool had = (d.seen[(int64_t)v * W + w] >> (slot & 63)) & 1;
      // markDuplicateMessageDelivery window (score.go:955): a copy of a message
      // first delivered before this hop is credited only within the window;
      // a second duplicate from the same peer is not counted (score.go:801-805)
      if (had && kind == GS_MSG_VALID) {
        bool unc = (pold >> i) & 1;
        if (d.needAge && !unc) {
          const int64_t firstHop = d.slotPubHop[slot] + d.age[(int64_t)v * d.S + slot];
          unc = (h - firstHop) * d.hop_ns > d.tp[t].MmdWindow;
        }
        if (unc) atomicAdd(&sUnc[i * T + t], 1u);
      }
      if (!young) {
        // outside the young slots only an old duplicate is possible; a first
        // delivery there is later than the engine's window allows
        if (!had) set_err(d, E_LATE);
        return;
      }
    }
    const int ix = sYp[rk] + __popcll(ym & ((1ull << (slot & 63)) - 1));
    // (an atomic per copy: reading the word first to skip repeats measured
    // slower, 96.0 -> 97.3 ms per round at config4)
    atomicOr((unsigned long long*)&sD[rk], 1ull << (slot & 63));
    // byte-wise min of the lowest deliverer (senders ascending)
    uint32_t* wp = (uint32_t*)(sFirst + (ix & ~3));
    const int sh = 8 * (ix & 3);
    uint32_t old = *wp;
    while ((int)((old >> sh) & 0xFF) > i) {
      const uint32_t nw = (old & ~(0xFFu << sh)) | ((uint32_t)i << sh);
      const uint32_t prev = atomicCAS(wp, old, nw);
      if (prev == old) break;
      old = prev;
    }
  };
  // ---- pass 1a: every 16-byte block of every sender's list is one work item;
  // lane l takes items l, l+64, ...  (PB loads in flight per lane).  The
  // entries actually sent (about a quarter: the sender's per-edge topic masks)
  // are compacted into an LDS queue and handed to fn 64 at a time by all lanes.
  // fn(i, slot) sees every sent, non-graylisted copy; walk() also counts
  // nSent / nGray when `count` (the first walk).
  // block kb of sender i: four list entries (16 B), or four pushed slots (8 B)
  const uint32_t* const flPrv = prv ? d.fl[1] : d.fl[0];
  const uint16_t* const ibxPrv = prv ? d.ibx[1] : d.ibx[0];
  auto load_block = [&](int i, int kb) -> uint4 {
    if ((pushM >> i) & 1) {
      if constexpr (EPBP == 8) return *(const uint4*)(ibxPrv + 8 * (size_t)sAddr[i] + 8 * kb);
      const uint2 p = *(const uint2*)(ibxPrv + 8 * (size_t)sAddr[i] + 4 * kb);
      return make_uint4(p.x, p.y, 0u, 0u);
    }
    return *(const uint4*)(flPrv + (size_t)sAddr[i] + 4 * kb);
  };
  auto walk = [&](auto&& fn, bool count) {
    int qh = 0, qt = 0;  // queue head / tail (wave-uniform)
    int rankPrev = -1;   // rank (among non-empty senders) of the sender of the block before the window
    constexpr int PB = 8;
    for (int b0 = 0; b0 < totalBlk; b0 += 64 * PB) {
      int si[PB], kb[PB];  // kb: block index | the sender's copies << 16
      uint4 q[PB];
#pragma unroll
      for (int rr = 0; rr < PB; ++rr) {
        const int B = b0 + rr * 64;  // the window's first block (wave-uniform, a multiple of 64)
        const int bidx = B + lane;
        si[rr] = -1;
        kb[rr] = 0;
        q[rr] = make_uint4(0, 0, 0, 0);
        if (B < 64 * GS_BMAP) {
          // sender of block B + lane: the non-empty sender whose rank is the
          // window's starting rank plus the list starts at offsets <= lane
          const uint64_t mb = sStart[B >> 6];
          const int rank = rankPrev + __popcll(mb & ((2ull << lane) - 1));
          rankPrev += __popcll(mb);
          if (bidx < totalBlk) {
            const uint64_t ce = sComp[rank];
            si[rr] = (int)((ce >> 24) & 63);
            const int k = bidx - (int)(ce & 0xFFFFFF);
            kb[rr] = k | (int)((ce >> 32) << 16);
            q[rr] = load_block(si[rr], k);
          }
        } else if (bidx < totalBlk) {
          int lo = 0, hi = nNE - 1;  // last non-empty sender whose first block is <= bidx
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((int)(sComp[mid] & 0xFFFFFF) <= bidx) lo = mid; else hi = mid - 1;
          }
          const uint64_t ce = sComp[lo];
          si[rr] = (int)((ce >> 24) & 63);
          const int k = bidx - (int)(ce & 0xFFFFFF);
          kb[rr] = k | (int)((ce >> 32) << 16);
          q[rr] = load_block(si[rr], k);
        }
      }
#pragma unroll
      for (int rr = 0; rr < PB; ++rr) {
        if (b0 + rr * 64 >= totalBlk) break;  // (wave-uniform) no block of this window is left
        uint32_t en[EPBP];
        bool sn[EPBP];
        bool wide = false;  // a pushed block with more than 4 slots
        {
          const int i = si[rr] < 0 ? 0 : si[rr];
          const int snd = sSnd[i];
          const int uu = snd & 0xFFFFFF;
          const int jri = (snd >> 24) & 0x3F;
          const bool rsS = (snd >> 30) & 1;
          const bool isGray = snd < 0;
          const uint64_t rl = sRelay[i], pb = sPub[i];
          const bool pushed = (pushM >> i) & 1;
          const int epb = pushed ? EPBP : 4;
          const int n = si[rr] < 0 ? 0 : min(epb, (kb[rr] >> 16) - epb * (kb[rr] & 0xFFFF));
          wide = n > 4;
#pragma unroll
          for (int c = 4; c < EPBP; ++c) {
            sn[c] = false;
            en[c] = 0;
          }
          if (pushed) {
            // pushed: every copy was sent; the topics v left are only counted
#pragma unroll
            for (int c = 0; c < EPBP; ++c) {
              const uint32_t wd = c < 2 ? q[rr].x : c < 4 ? q[rr].y : c < 6 ? q[rr].z : q[rr].w;
              const int slot = (int)((c & 1) ? (wd >> 16) : (wd & 0xFFFFu));
              const int t = (int)__umulhi((unsigned)slot, d.stMagic);
              const bool sent = c < n && !(authV && d.slotSrc[slot] == v);  // never to the author
              if (count) {
                nSent += sent;
                if (sent && isGray) ++nGray;
              }
              sn[c] = sent && !isGray && ((sv >> t) & 1);
              en[c] = (uint32_t)slot | ((uint32_t)i << 16);
            }
          } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint32_t ent = c == 0 ? q[rr].x : (c == 1 ? q[rr].y : (c == 2 ? q[rr].z : q[rr].w));
            const int slot = (int)(ent & 0xFFFF);
            const int tag = (int)(ent >> 16);
            const int t = (int)__umulhi((unsigned)slot, d.stMagic);
            bool sent = c < n && (tag == 255 ? ((pb >> t) & 1) : ((rl >> t) & 1));
            sent = sent && tag != jri;  // ReceivedFrom exclusion (gossipsub.go:1003)
            if (sent && rsS) sent = (d.sel[(int64_t)uu * d.S + slot] >> jri) & 1;
            if (sent && authV && d.slotSrc[slot] == v) sent = false;  // never to the author
            if (count) {
              nSent += sent;
              if (sent && isGray) ++nGray;  // one RPC per relayed message, all dropped
            }
            sn[c] = sent && !isGray;
            en[c] = (uint32_t)slot | ((uint32_t)i << 16);
          }
          }
        }
        // c-major positions (delivery order does not matter: every update is
        // a commutative LDS atomic), four entries per lane between drains
        // (the queue holds 63 pending + 256 appended)
        const bool wideAny = EPBP > 4 && __ballot(wide) != 0;
#pragma unroll
        for (int g = 0; g < EPBP / 4; ++g) {
          if (g > 0 && !wideAny) break;
#pragma unroll
          for (int c = 4 * g; c < 4 * g + 4; ++c) {
            const uint64_t m = __ballot(sn[c]);
            if (sn[c]) sQ[qt + lane_rank(m)] = en[c];
            qt += __popcll(m);
          }
          __syncthreads();
          if (qt >= 64) {
            while (qt - qh >= 64) {
              const uint32_t ent = sQ[qh + lane];
              fn((int)(ent >> 16), (int)(ent & 0xFFFF));
              qh += 64;
            }
            // move the (< 64) pending copies to the front
            const uint32_t rest = lane < qt - qh ? sQ[qh + lane] : 0u;
            __syncthreads();
            if (lane < qt - qh) sQ[lane] = rest;
            qt -= qh;
            qh = 0;
            __syncthreads();
          }
        }
      }
    }
    if (lane < qt - qh) {
      const uint32_t ent = sQ[qh + lane];
      fn((int)(ent >> 16), (int)(ent & 0xFFFF));
    }
    __syncthreads();
  };
  long long nValidated = 0, nRejected = 0, nThrottledCopies = 0;
  // ADV: a copy of a message dropped by a full validation queue (the second
  // walk below): RejectValidationQueueFull, neither a delivery nor a duplicate
  bool dropPass = false;
  auto drop = [&](int i, int slot, bool payloadRpc) {
    const int rk = sRk[slot >> 6];
    if (rk == 0xFFFF || !((sDrop[rk] >> (slot & 63)) & 1)) return;
    if (payloadRpc && gated(i, slot)) return;
    const int t = (int)__umulhi((unsigned)slot, d.stMagic);
    const int kind = kindOf(slot, t);
    atomicSub(&sPer[i], 1u);
    if (kind == GS_MSG_REJECT) atomicSub(&sInv[i * T + t], 1u);
    if (kind == GS_MSG_VALID) {
      if (NARROW) {
        const int pl = i * T + t;
        atomicSub(&scnt[cword(i, t)], 1u << (16 * (pl & 1)));
      } else {
        atomicSub(&scnt[cword(i, t)], 1u);
      }
    }
    ++nThrottledCopies;
    --nCopies;
    if (trv)  // validation.go:240
      trace_emit(d, h, GS_TRACE_REJECT_MESSAGE, v, d.col[base + i], t, d.slotMid[slot], 2, GS_REJECT_QUEUE_FULL);
  };
  // one walk instantiation for both passes (a second one made the compiler
  // copy the kernel arguments to scratch)
  auto onCopy = [&](int i, int slot) {
    if (ADV && dropPass) drop(i, slot, true);
    else deliver(i, slot, true);
  };
  if constexpr (DENSE) {
    // ---- pass 1, dense (lane = rank of a word in the active window amR): the
    // senders that sent v anything, ascending; sender i's copies are its
    // frontier row fb[u] (its first deliveries of the previous hop plus its own
    // publishes), all of it where it relays to v, its own messages only where it
    // just publishes to v, less v's own messages (the author exclusion).  A bit
    // the senders before i did not deliver and v has not seen is a first
    // delivery by i.  The copies u did not send because v delivered them to u
    // first (tag == jr in the list) are not in the bitmap's reach and leave the
    // counts through exD.  Per-copy state the list walk keeps (sD, sFirst, the
    // (sender, topic) counts, nSent / nGray / nCopies) comes out equal.  The
    // rows hold bits in amR words only (what a sender first received in the
    // previous hop was published within its window), so rank space reads just
    // those: one word per lane at config3, eight senders' rows in flight.
    int* const sLv = (int*)sComp;  // (the list walk's LDS, unused here)
    int* const sCs = (int*)sPub;   // per sender: the copies its row holds for v
    const uint64_t lmD = __ballot(liveD);
    const int nLv = __popcll(lmD);
    if (liveD) sLv[__popcll(lmD & ((1ull << lane) - 1))] = lane;
    sCs[lane] = 0;
    // (one topic, T == 1: a sender relays / publishes to v or not, and v
    // either holds the topic or left it, dropping every copy)
    const bool svT = sv & 1;
    __syncthreads();
    const uint64_t* const fbPrv = d.fb[prv];
    uint64_t lateM = 0;
    for (int r0 = 0; r0 < nR; r0 += 64) {
      const int k = r0 + lane;
      const bool act = k < nR;
      const int w = act ? (int)(d.yTab[W + k] >> 32) : 0;  // the word of rank k (host table)
      const uint64_t Y = act ? sYm[k] : 0ull;
      const uint64_t Sv = act ? d.seen[(int64_t)v * W + w] : 0ull;
      const uint64_t O = (act && authV) ? d.own[(int64_t)v * W + w] : 0ull;
      const int yp = act ? (int)sYp[k] : 0;
      uint64_t D = 0;
      for (int k0 = 0; k0 < nLv; k0 += 8) {
        uint64_t F[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int i = k0 + q < nLv ? sLv[k0 + q] : -1;
          F[q] = (i >= 0 && act) ? fbPrv[(int64_t)(sSnd[i] & 0xFFFFFF) * W + w] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (k0 + q >= nLv) break;
          const int i = sLv[k0 + q];
          const bool r = lane_get64(relayAll, i) & 1, p = lane_get64(pubAll, i) & 1;
          // its own messages matter where the relay and pub masks differ (a
          // peer it publishes to but does not relay to, or the reverse): rare
          uint64_t A = 0;
          if (r != p) {
            const int uq = sSnd[i] & 0xFFFFFF;
            if (d.nAuth[uq] > 0 && act) A = d.own[(int64_t)uq * W + w];
          }
          const uint64_t f = F[q];
          const uint64_t sb = (r ? (p ? f : f & ~A) : (p ? f & A : 0ull)) & ~O;
          const int cs = wave_last(wave_incl_sum(__popcll(sb)));
          if (lane == 0) sCs[i] += cs;
          if (!svT || sSnd[i] < 0) continue;  // v left the topic / i is graylisted: dropped
          lateM |= sb & ~Y & ~Sv;
          const uint64_t y = sb & Y;
          for (uint64_t nb = y & ~D & ~Sv; nb; nb &= nb - 1)
            sFirst[yp + __popcll(Y & ((1ull << (__ffsll((long long)nb) - 1)) - 1))] = (uint8_t)i;
          D |= y;
        }
      }
      if (act) sD[k] = D;
    }
    if (lateM) set_err(d, E_LATE);  // a first delivery older than the window
    __syncthreads();
    if (liveD) {  // lane = sender: its copies, less the ReceivedFrom ones
      const int c = sCs[lane] - ((relayAll & 1) ? exD : 0);
      nSent += c;
      if (gray) {
        nGray += c;
      } else if (svT) {
        nCopies += c;
        if (c) atomicAdd(&scnt[cword(lane, 0)], NARROW ? (uint32_t)c << (16 * (lane & 1)) : (uint32_t)c);
      }
    }
    if (trv && valid && !gray && (relay | pub)) {
      // a traced receiver's copy events, exactly per sent copy (its senders'
      // lists carry the ReceivedFrom tags the bitmaps do not)
      const uint32_t* L = d.fl[prv] + (int64_t)u * FC;
      const int nL = d.fln[prv][u];
      for (int k = 0; k < nL; ++k) {
        const uint32_t ent = L[k];
        const int slot = (int)(ent & 0xFFFF), tag = (int)(ent >> 16);
        const int t = (int)__umulhi((unsigned)slot, d.stMagic);
        bool sent = tag == 255 ? ((pub >> t) & 1) : ((relay >> t) & 1);
        sent = sent && tag != jr;
        if (sent && authV && d.slotSrc[slot] == v) sent = false;
        if (sent) trace_emit(d, h, GS_TRACE_COPY, v, u, t, d.slotMid[slot], 2);
      }
    }
    __syncthreads();
  } else {
  walk(onCopy, true);
  if (__ballot(((relayAll | pubAll) & ~sv) != 0)) {
    // copies of topics v is not subscribed to: transmitted, then ignored
    // (churn runs only: a mesh or announced peer that has just left)
    const uint64_t ru = relayAll & ~sv, pu = pubAll & ~sv;
    if ((ru | pu) && valid && pOff < 0) {  // (a pushed segment's were counted by the walk)
      const uint32_t* L = d.fl[prv] + (int64_t)u * FC;
      for (int k = 0; k < Ln; ++k) {
        const uint32_t ent = L[k];
        const int slot = (int)(ent & 0xFFFF), tag = (int)(ent >> 16);
        const int t = (int)__umulhi((unsigned)slot, d.stMagic);
        bool sent = tag == 255 ? ((pu >> t) & 1) : ((ru >> t) & 1);
        sent = sent && tag != jr;
        if (sent && rs_host(d, u)) sent = (d.sel[(int64_t)u * d.S + slot] >> jr) & 1;
        if (sent && authV && d.slotSrc[slot] == v) sent = false;
        if (sent) {
          ++nSent;
          if (gray) ++nGray;
        }
      }
    }
  }
  }
  // ---- pass 1b: IWANT responses (in the sender's reply RPCs): every served
  // id of every accepted sender is one work item, spread over the lanes (an
  // IWANT spammer gets hundreds from one sender)
  nSent += irN;
  if (!gray && ADV && ctlGated) nGatedCopies += nSrvRpc;  // the served replies' payload is ignored
  const int myIr = (!gray && !(ADV && ctlGated)) ? irN : 0;
  const int irTot = wave_last(wave_incl_sum(myIr));
  // exclusive prefix of the accepted senders' served ids and their arena
  // offsets, in the walk queue's LDS (free outside a walk): written by each
  // call, since the ADV path walks again in between
  int* const sIrP = (int*)sQ;       // [64]
  int* const sIrO = (int*)sQ + 64;  // [64]
  // fn(sender, slot) for every accepted served id
  auto eachIr = [&](auto&& fn) {
    if (irTot == 0) return;
    const int incl = wave_incl_sum(myIr);
    sIrP[lane] = incl - myIr;
    sIrO[lane] = irOff;
    __syncthreads();
    for (int idx = lane; idx < irTot; idx += 64) {
      int lo = 0, hi = 63;  // last sender whose first item is <= idx
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sIrP[mid] <= idx) lo = mid; else hi = mid - 1;
      }
      fn(lo, d.pool[prv][sIrO[lo] + idx - sIrP[lo]]);
    }
    __syncthreads();  // the queue's LDS again
  };
  eachIr([&](int i, int slot) {
    if ((sv >> (int)__umulhi((unsigned)slot, d.stMagic)) & 1) deliver(i, slot, false);
  });
  if constexpr (ADV) {
    if (ctlGated) throttled |= 1ull << lane;
    // lane-uniform set of throttled senders
    uint64_t all = 0;
    for (int o = 0; o < 64; ++o) all |= lane_get64(throttled, o);
    throttled = all;
  }
  __syncthreads();

  GS_STAMP(2);
  // ---- pass 2 (lane = word of the active window): first deliveries.  All
  // loads of the pass are issued before its first store (on gfx9 a load's
  // wait also waits for every older store).
  uint32_t* Lv = d.fl[cur] + (int64_t)v * FC;
  // pass 3's in-edge mesh words replace the relay masks in sRelay; the ADV
  // launch still walks the lists again (queue drops) and loads them later
  if (!ADV && scoring) sRelay[lane] = valid ? d.mesh[base + lane] : 0ull;
  long long nDeliv = 0;
  // the slots published this hop (words amP, slots pubmask[cur]) recycle their
  // previous messages (mcache.go:94-104 has let them go, retireHops): their
  // seen bits are cleared here, in the write of the node's seen word that pass
  // 2b does anyway for most of them.  No copy of either occupant can arrive in
  // this hop (the new one is published after phase A, the old one is past
  // every delivery horizon), so clearing before or after the deliveries is the
  // same.  k_publish then sets the authors' bits.
  uint64_t Uw[WPL], Sw[WPL], Hw[WPL], Ow[WPL], Rw[WPL];
  uint64_t Xw[WPL];  // ADV: fresh messages validated as REJECT / IGNORE (seen, not delivered)
  int rkw[WPL];  // rank of the lane's word in amR
  // index of young slot b of the amR word of rank rk in sFirst
  auto fidx = [&](int rk, int b) -> int { return sYp[rk] + __popcll(sYm[rk] & ((1ull << b) - 1)); };
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    Uw[j] = Sw[j] = Hw[j] = Ow[j] = Xw[j] = Rw[j] = 0;
    rkw[j] = 0;
    const bool ret = w < W && wm_has(amP, w);
    if (ret) Rw[j] = d.pubmask[cur][w];
    if constexpr (!ADV && kPf) {
      Sw[j] = Sp[j];  // (prefetched at wave start)
      if (w < W && wm_has(amR, w)) {
        rkw[j] = wm_rank(amR, w);
        const uint64_t D = sD[rkw[j]];
        if (D) {
          Uw[j] = D;  // & ~seen below
          Ow[j] = Op[j];
          Hw[j] = Hp[j];
        }
      }
    } else {
      if (w < W && wm_has(amR, w)) {
        rkw[j] = wm_rank(amR, w);
        const uint64_t D = sD[rkw[j]];
        if (D) {
          // the pass's loads in one round trip: seen, and (for the first
          // deliveries it may hold) the old-slot mask and the mcache window
          Sw[j] = d.seen[(int64_t)v * W + w];
          Uw[j] = D;  // & ~seen below
          Ow[j] = d.oldm[w];
          if (gossipV) Hw[j] = d.hist[((int64_t)head * d.nOwnH + (v - d.n0)) * W + w];
        } else if (ret) {
          Sw[j] = d.seen[(int64_t)v * W + w];
        }
      } else if (ret) {
        Sw[j] = d.seen[(int64_t)v * W + w];
      }
    }
  }
  bool anyDrop = false;
  bool staged = false;          // ADV: the validator topics' fresh messages staged (cs / ck)
  int cs[4] = {-1, -1, -1, -1};
  unsigned long long ck[4] = {0, 0, 0, 0};
  if constexpr (ADV) {
    // ---- the validation queue: the first valQueue fresh messages of topics
    // with a validator, in arrival order (first deliverer, then message id),
    // are validated; the rest are dropped (RejectValidationQueueFull)
    int nCand = 0;
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      const int w = lane + 64 * j;
      const int t = (int)__umulhi((unsigned)(w * 64), d.stMagic);
      if (!((d.topicVal >> t) & 1)) continue;
      nCand += __popcll(Uw[j] & ~Sw[j]);
    }
    const int candIncl = wave_incl_sum(nCand);
    const int nAll = wave_last(candIncl);
    // up to 256 candidates are staged in registers (four per lane, slot and
    // key ff << 56 | mid, their loads in flight together): the selection and
    // the verdicts below run lane-parallel instead of one lane per word
    staged = nAll <= 256;
    if (staged && nAll > 0) {
      int pos = candIncl - nCand;
#pragma unroll
      for (int j = 0; j < WPL; ++j) {
        const int w = lane + 64 * j;
        const int t = (int)__umulhi((unsigned)(w * 64), d.stMagic);
        if (!((d.topicVal >> t) & 1)) continue;
        for (uint64_t y = Uw[j] & ~Sw[j]; y; y &= y - 1) sQ[pos++] = (uint32_t)(w * 64 + __ffsll((long long)y) - 1);
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) cs[k] = lane + 64 * k < nAll ? (int)sQ[lane + 64 * k] : -1;
      __syncthreads();  // sQ is the selection's histogram below
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (cs[k] < 0) continue;
        const int slot = cs[k];
        ck[k] = ((unsigned long long)sFirst[fidx(sRk[slot >> 6], slot & 63)] << 56) |
                (unsigned long long)d.slotMid[slot];
      }
    }
    if (d.valQueue > 0 && nAll > d.valQueue) {
      unsigned long long K;
      long long M;
      if (staged) {
        auto each = [&](auto&& fn) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (cs[k] >= 0) fn(ck[k], (long long)d.slotMid[cs[k]]);
        };
        select_kth(each, d.valQueue, sQ, K, M);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (cs[k] < 0 || ck[k] <= K) continue;
          const int slot = cs[k];
          atomicOr((unsigned long long*)&sDrop[sRk[slot >> 6]], 1ull << (slot & 63));
          if (prow >= 0) d.pmask[(int64_t)prow * d.S + slot] = 0;  // never seen: no record
        }
      } else {
      // the valQueue-th smallest key ff << 56 | mid (radix select over the
      // lanes' own fresh words; the walk queue's LDS is free now)
      auto each = [&](auto&& fn) {
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
          const int w = lane + 64 * j;
          const int t = (int)__umulhi((unsigned)(w * 64), d.stMagic);
          if (!((d.topicVal >> t) & 1)) continue;
          uint64_t y = Uw[j] & ~Sw[j];
          while (y) {
            const int b = __ffsll((long long)y) - 1;
            y &= y - 1;
            const long long mid = d.slotMid[w * 64 + b];
            fn(((unsigned long long)sFirst[fidx(rkw[j], b)] << 56) | (unsigned long long)mid, mid);
          }
        }
      };
      select_kth(each, d.valQueue, sQ, K, M);
#pragma unroll
      for (int j = 0; j < WPL; ++j) {
        const int w = lane + 64 * j;
        const int t = (int)__umulhi((unsigned)(w * 64), d.stMagic);
        if (!((d.topicVal >> t) & 1)) continue;
        uint64_t y = Uw[j] & ~Sw[j];
        while (y) {
          const int b = __ffsll((long long)y) - 1;
          y &= y - 1;
          const unsigned long long key =
              ((unsigned long long)sFirst[fidx(rkw[j], b)] << 56) | (unsigned long long)d.slotMid[w * 64 + b];
          if (key > K) {
            atomicOr((unsigned long long*)&sDrop[rkw[j]], 1ull << b);
            if (prow >= 0) d.pmask[(int64_t)prow * d.S + w * 64 + b] = 0;  // never seen: no record
          }
        }
      }
      }
      anyDrop = true;
      __syncthreads();
    }
    if (staged && nAll > 0) {
      // verdicts of the staged candidates that were not dropped: REJECT /
      // IGNORE are seen but not delivered; sD (pass 1's delivered words, read
      // above) collects them per word rank
      for (int k = lane; k < nR; k += 64) sD[k] = 0ull;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (cs[k] < 0) continue;
        const int slot = cs[k], rk = sRk[slot >> 6];
        if (anyDrop && ((sDrop[rk] >> (slot & 63)) & 1)) continue;
        const int kd = d.slotKind[slot];
        if (kd == GS_MSG_REJECT || kd == GS_MSG_IGNORE) atomicOr((unsigned long long*)&sD[rk], 1ull << (slot & 63));
      }
      __syncthreads();
    }
    nValidated = nAll < d.valQueue || d.valQueue == 0 ? nAll : d.valQueue;
  }
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    Uw[j] &= ~Sw[j];
    if constexpr (ADV) {
      if (Uw[j]) {
        if (anyDrop) Uw[j] &= ~sDrop[rkw[j]];
        const int t = (int)__umulhi((unsigned)(w * 64), d.stMagic);
        if (staged) {
          if ((d.topicVal >> t) & 1) Xw[j] = sD[rkw[j]] & Uw[j];  // the staged verdicts
        } else if ((d.topicVal >> t) & 1) {
          // verdicts: REJECT / IGNORE are seen but not delivered
          uint64_t y = Uw[j];
          while (y) {
            const int b = __ffsll((long long)y) - 1;
            y &= y - 1;
            const int k = d.slotKind[w * 64 + b];
            if (k == GS_MSG_REJECT || k == GS_MSG_IGNORE) Xw[j] |= 1ull << b;
          }
        }
      }
    }
  }
  // first deliveries per (topic, first deliverer) for the counters of pass 3
  if (scoring) {
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      uint64_t y = Uw[j] & ~Xw[j];
      const int t = (int)__umulhi((unsigned)((lane + 64 * j) * 64), d.stMagic);
      while (y) {
        const int b = __ffsll((long long)y) - 1;
        y &= y - 1;
        const int ff = sFirst[fidx(rkw[j], b)];
        const int pl = ff * T + t;
        if (NARROW) atomicAdd(&scnt[cword(ff, t)], 1u << (16 * (pl & 1) + 8));
        else atomicAdd(&scnt[cword(ff, t)], 1u << 16);
      }
    }
  }
  if constexpr (ADV) {
    // per first deliverer: valid / rejected / ignored first deliveries (gater
    // DeliverMessage / RejectMessage, peer_gater.go:397-432), REJECT traces
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      uint64_t y = Uw[j];
      const int w = lane + 64 * j;
      while (y) {
        const int b = __ffsll((long long)y) - 1;
        y &= y - 1;
        const int ff = sFirst[fidx(rkw[j], b)];
        const bool x = (Xw[j] >> b) & 1;
        const int slot = w * 64 + b;
        const int k = x ? d.slotKind[slot] : GS_MSG_VALID;
        atomicAdd(&sPer[(k == GS_MSG_VALID ? 1 : k == GS_MSG_REJECT ? 2 : 3) * 64 + ff], 1u);
        if (x) {
          ++nRejected;
          if (trv)  // validation.go:333 / :351
            trace_emit(d, h, GS_TRACE_REJECT_MESSAGE, v, d.col[base + ff], (int)__umulhi((unsigned)slot, d.stMagic),
                       d.slotMid[slot], 2, k == GS_MSG_REJECT ? GS_REJECT_VALIDATION_FAILED : GS_REJECT_VALIDATION_IGNORED);
        }
      }
    }
    if (anyDrop) {
      // ---- second walk: every copy of a dropped message is RejectValidation-
      // QueueFull: neither a delivery nor a duplicate (its counts leave the
      // tables), the gater's throttle, and it fulfils promises (gossip_tracer.go:133)
      dropPass = true;
      walk(onCopy, false);
      eachIr([&](int i, int slot) { drop(i, slot, false); });
      __syncthreads();
    }
    if (scoring && (anyDrop || throttled)) {
      // promises: a dropped message fulfils its promises, a throttled peer
      // loses its own (gossip_tracer.go:119-126, 163-181); lane = table entry
      const int n = d.promN[v];
      if (n > 0) {
        int kept = 0;  // the table in banks of 64 (lane = entry), compacted in place
        for (int b0 = 0; b0 < n; b0 += 64) {
          const int64_t ti = (int64_t)v * d.promCap + b0 + lane;
          int64_t pm = -1, pe = 0;
          int ps = 0, pg = 0;
          bool live = b0 + lane < n;
          if (live) {
            pm = d.promMid[ti];
            pe = d.promExp[ti];
            ps = d.promSlot[ti];
            pg = d.promEdge[ti];
            if ((throttled >> pg) & 1) live = false;
            const int rk = sRk[ps >> 6];
            if (anyDrop && rk != 0xFFFF && ((sDrop[rk] >> (ps & 63)) & 1)) live = false;
          }
          const unsigned long long lm = __ballot(live);
          const int pos = kept + __popcll(lm & ((1ull << lane) - 1));
          __syncthreads();
          if (live) {  // pos <= b0 + lane: never past an entry not yet read
            const int64_t to = (int64_t)v * d.promCap + pos;
            d.promMid[to] = pm;
            d.promExp[to] = pe;
            d.promSlot[to] = ps;
            d.promEdge[to] = (uint8_t)pg;
          }
          kept += __popcll(lm);
        }
        if (lane == 0) d.promN[v] = kept;
      }
    }
    if (scoring) sRelay[lane] = valid ? d.mesh[base + lane] : 0ull;
  }
  __syncthreads();
  GS_STAMP(3);
  // ---- pass 3 (lane = in-edge): fmd += fresh, mmd += fresh + creditable
  // duplicates while in the mesh (score.go:915-928, 945-963).  inMesh of a
  // scored topic is the edge's mesh bit (tracer.Graft / tracer.Prune accompany
  // every mesh change).  Batches of 8 topics, the next batch's loads issued
  // before this batch's stores.
  if (scoring) {
    // The counts go to the pending-delivery words dlt (eff_counters).  v's
    // in-edges own the contiguous pairs [base*T, (base+deg)*T), pair index
    // pl = i*T + t (== the scnt index): lane l takes pairs l, l+64, ... — one
    // coalesced, branch-free read-modify-write per pair, every load of a batch
    // issued before its first store (no full-queue drains).
    const int nP = deg * T;
    uint32_t* const scr = (uint32_t*)(d.pad + ((int64_t)(blockIdx.x & 255) * 64 + lane) * 2);
    if (NARROW && d.dltN != nullptr) {
      // (narrow pending words imply narrow phase-A counters: St <= 254)
      // 16-bit pending words (Dev::dltN), two pairs per lane: word wi of v's
      // rows holds pairs 2 wi (in-edge i, topic t) and 2 wi + 1 (i, t + 1; T is
      // even), so one 4-byte load covers both and a wave moves 128 pairs
      const int nWd = nP >> 1;
      uint32_t* const pw = (uint32_t*)(d.dltN + base * T);
      const int q128 = 128 / T, r128 = 128 - q128 * T;
      int ic = (2 * lane) / T, tc = 2 * lane - ((2 * lane) / T) * T;
#ifndef GS_UPD2P
#define GS_UPD2P 1  // timing A/B: -DGS_UPD2P=0 updates the two pairs of a word one after the other
#endif
      auto upd2 = [&](int wi, int i, int t, uint32_t q) -> uint32_t {
        if (GS_UPD2P && !hasUnc) {
          // both pairs of the word at once, a byte per field: counts
          // [copies | fresh << 8] and pending [fmd | mmd << 8] per 16-bit half;
          // fmd += fresh, mmd += fresh + credited duplicates = copies while in
          // the mesh (no uncredited copies without needAge / pmask)
          const uint32_t sm = (((scoredT >> t) & 1) ? 0x0000FFFFu : 0u) | (((scoredT >> (t + 1)) & 1) ? 0xFFFF0000u : 0u);
          const uint32_t c = scnt[cword(i, t)] & sm;
          const uint64_t rl = sRelay[i] >> t;
          const uint32_t mm = ((rl & 1) ? 0x0000FFFFu : 0u) | ((rl & 2) ? 0xFFFF0000u : 0u);
          const uint32_t f = (q & 0x00FF00FFu) + ((c >> 8) & 0x00FF00FFu);
          const uint32_t m = ((q >> 8) & 0x00FF00FFu) + (c & mm & 0x00FF00FFu);
          if ((f | m) & 0xFF00FF00u) set_err(d, E_DELTA);
          return f | (m << 8);
        }
        uint32_t out = 0;
        bool over = false;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int pl = 2 * wi + hh, tt = t + hh;
          const bool sc = (scoredT >> tt) & 1;
          uint32_t c = 0;
          if (sc) c = NARROW ? ((scnt[cword(i, t)] >> (16 * hh)) & 0xFFFF) : scnt[cword(i, tt)];
          const int copies = NARROW ? (int)(c & 0xFF) : (int)(c & 0xFFFF);
          const int nf = NARROW ? (int)(c >> 8) : (int)(c >> 16);
          int credited = copies - nf;
          if (hasUnc && sc) credited -= (int)sUnc[pl];
          const uint32_t addM = ((sRelay[i] >> tt) & 1) ? (uint32_t)(nf + credited) : 0u;
          const uint32_t old = (q >> (16 * hh)) & 0xFFFF;
          const uint32_t f = (old & 0xFF) + (uint32_t)nf, m = (old >> 8) + addM;
          over |= f > 0xFF || m > 0xFF;
          out |= (f | (m << 8)) << (16 * hh);
        }
        if (over) set_err(d, E_DELTA);
        return out;
      };
      auto rmw2 = [&](auto bsC) {
        constexpr int BS = decltype(bsC)::value;
        uint32_t q[BS];
        int iv[BS], tv[BS];
        for (int k0 = 0; 64 * k0 < nWd; k0 += BS) {
#pragma unroll
          for (int kk = 0; kk < BS; ++kk) {
            const int wi = lane + 64 * (k0 + kk);
            q[kk] = pw[wi < nWd ? wi : nWd - 1];
            iv[kk] = ic;
            tv[kk] = tc;
            ic += q128;
            tc += r128;
            if (tc >= T) { tc -= T; ++ic; }
          }
#pragma unroll
          for (int kk = 0; kk < BS; ++kk) {
            const int wi = lane + 64 * (k0 + kk);
            const bool ok = wi < nWd;
            const uint32_t nq = upd2(ok ? wi : 0, ok ? iv[kk] : 0, ok ? tv[kk] : 0, q[kk]);
            *(ok ? pw + wi : scr) = nq;
          }
        }
      };
      if (pf3) {
        // the words prefetched at wave start: one batch
#pragma unroll
        for (int kk = 0; kk < PF3; ++kk) {
          const int wi = lane + 64 * kk;
          const bool ok = wi < nWd;
          const int iv = ic, tv = tc;
          ic += q128;
          tc += r128;
          if (tc >= T) { tc -= T; ++ic; }
          const uint32_t nq = upd2(ok ? wi : 0, ok ? iv : 0, ok ? tv : 0, q3[kk]);
          *(ok ? pw + wi : scr) = nq;
        }
      } else if (nWd > 8 * 64) {
        rmw2(std::integral_constant<int, 16>{});
      } else if (nWd > 2 * 64) {
        rmw2(std::integral_constant<int, 8>{});
      } else if (nWd > 64) {
        rmw2(std::integral_constant<int, 2>{});
      } else {
        rmw2(std::integral_constant<int, 1>{});
      }
    } else {
    uint32_t* const pv = d.dlt + base * T;
    const int q64 = 64 / T, r64 = 64 - q64 * T;
    int ic = lane / T, tc = lane - (lane / T) * T;  // (in-edge, topic) of the lane's next pair
    auto upd = [&](int pl, int i, int t, uint32_t q) -> uint32_t {
      uint32_t c = ((scoredT >> t) & 1) ? scnt[cword(i, t)] : 0u;
      if (NARROW) c = (c >> (16 * (pl & 1))) & 0xFFFF;
      const int copies = NARROW ? (int)(c & 0xFF) : (int)(c & 0xFFFF);
      const int nf = NARROW ? (int)(c >> 8) : (int)(c >> 16);
      int credited = copies - nf;
      if (hasUnc && ((scoredT >> t) & 1)) credited -= (int)sUnc[pl];  // unscored: no counts at all
      const uint32_t addM = ((sRelay[i] >> t) & 1) ? (uint32_t)(nf + credited) : 0u;
      if ((q & 0xFFFF) + nf > 0xFFFF || (q >> 16) + addM > 0xFFFF) set_err(d, E_DELTA);
      return q + (uint32_t)nf + (addM << 16);
    };
    auto rmw = [&](auto bsC) {
      constexpr int BS = decltype(bsC)::value;
      uint32_t q[BS];
      int iv[BS], tv[BS];
      for (int k0 = 0; 64 * k0 < nP; k0 += BS) {
#pragma unroll
        for (int kk = 0; kk < BS; ++kk) {
          const int pl = lane + 64 * (k0 + kk);
          q[kk] = pv[pl < nP ? pl : nP - 1];
          iv[kk] = ic;
          tv[kk] = tc;
          ic += q64;
          tc += r64;
          if (tc >= T) { tc -= T; ++ic; }
        }
#pragma unroll
        for (int kk = 0; kk < BS; ++kk) {
          const int pl = lane + 64 * (k0 + kk);
          const bool ok = pl < nP;
          const uint32_t nq = upd(ok ? pl : 0, ok ? iv[kk] : 0, ok ? tv[kk] : 0, q[kk]);
          *(ok ? pv + pl : scr) = nq;
        }
      }
    };
    // a batch no larger than the node's pairs need: a batch slot past nP is a
    // scratch store (config3: 32 pairs, one slot)
    if (nP > 16 * 64) {
      rmw(std::integral_constant<int, 32>{});
    } else if (nP > 4 * 64) {
      rmw(std::integral_constant<int, 16>{});
    } else if (nP > 64) {
      rmw(std::integral_constant<int, 4>{});
    } else {
      rmw(std::integral_constant<int, 1>{});
    }
    }
    GS_STAMP(5);
    if constexpr (ADV) {
      // P4: every non-dropped copy of a rejected message is an invalid delivery
      // of its sender (RejectMessage, then DuplicateMessage on the invalid
      // record: score.go:766-783, 808-810), +1 steps, uncapped
      for (int pl = lane; pl < nP; pl += 64) {
        const int t = pl % T;
        const uint32_t n = ((scoredT >> t) & 1) ? sInv[pl] : 0u;
        if (!n) continue;
        double x = d.imd[base * T + pl];
        x = gs_add_ones(x, n);  // +1 steps (include/gs_fp.h)
        d.imd[base * T + pl] = x;
        d.sdirty[base + pl / T] = 1;  // a score-lowering change
      }
    }
  }
  if constexpr (ADV) {
    __syncthreads();
    if (d.gater && gossipV) {
      // peerGater counters (peer_gater.go:390-440): per IP group (+1 steps)
      // and per node; lane = in-edge, its group's stats edge gets the sums
      const int cp = valid ? (int)sPer[lane] : 0;
      const int fv = valid ? (int)sPer[64 + lane] : 0, fr = valid ? (int)sPer[128 + lane] : 0,
                fi = valid ? (int)sPer[192 + lane] : 0;
      const int dup = cp - fv - fr - fi;
      const int g = valid ? d.gGrp[base + lane] : 0;
      __syncthreads();
      for (int k = lane; k < 4 * 64; k += 64) sPer[k] = 0;
      __syncthreads();
      if (valid) {
        if (fv) atomicAdd(&sPer[g], (uint32_t)fv);
        if (dup) atomicAdd(&sPer[64 + g], (uint32_t)dup);
        if (fi) atomicAdd(&sPer[128 + g], (uint32_t)fi);
        if (fr) atomicAdd(&sPer[192 + g], (uint32_t)fr);
      }
      __syncthreads();
      if (valid && g == lane) {
        for (int k = 0; k < 4; ++k) {
          const uint32_t n = sPer[k * 64 + lane];
          if (!n) continue;
          double x = d.gSt[k * d.eOwn + base + lane];
          x = gs_add_ones(x, n);
          d.gSt[k * d.eOwn + base + lane] = x;
        }
      }
      const long long thc = (long long)wave_sum_ll(nThrottledCopies);
      if (lane == 0) {
        if (nValidated) {
          double x = d.gValidate[v];
          x = gs_add_ones(x, nValidated);
          d.gValidate[v] = x;
        }
        if (thc) {
          double x = d.gThrottle[v];
          x = gs_add_ones(x, thc);
          d.gThrottle[v] = x;
          d.gLast[v] = h * d.hop_ns;
        }
      }
    }
    GS_STAMP(6);
    if (d.cSpam[cur] != nullptr && valid && !gray && behaves(d, v, GS_BEHAVE_IWANT_SPAM) && mesh_peer(d, base + lane)) {
      // IWANT spam (gossipsub_spam_test.go:113-128): one request per message
      // received from this sender (its accepted copies), in an extra RPC
      auto each = [&](auto&& fn) {
        const uint32_t* L = d.fl[prv] + (int64_t)u * FC;
        const int nL = pOff >= 0 ? d.fln[prv][u] : Ln;  // the sender's whole list
        for (int k = 0; k < nL; ++k) {
          const uint32_t ent = L[k];
          const int slot = (int)(ent & 0xFFFF), tag = (int)(ent >> 16);
          const int t = (int)__umulhi((unsigned)slot, d.stMagic);
          bool sent = tag == 255 ? ((pub >> t) & 1) : ((relay >> t) & 1);
          sent = sent && tag != jr;
          if (sent && authV && d.slotSrc[slot] == v) sent = false;
          if (sent && !gated(lane, slot)) fn(slot);
        }
        if (!ctlGated)
          for (int k = 0; k < irN; ++k) fn(d.pool[prv][irOff + k]);
      };
      int n = 0;
      each([&](int) { ++n; });
      if (n) {
        const unsigned long long off = pool_take(d, cur, (unsigned long long)n);
        if (off == ~0ull) {  // arena full (E_POOL)
        } else {
          int p = (int)off;
          each([&](int slot) { d.pool[cur][p++] = slot; });
          const int64_t rl = rxi(d, base + lane, d.rev[base + lane]);  // the receiver's in-edge (or its stage slot)
          d.cSpam[cur][rl] = ((int64_t)off << 24) | (int64_t)n;
          d.cPre[cur][rl] = (uint8_t)(d.cPre[cur][rl] + 1);
          // RPC{control: {iwant: [{n ids}]}}
          if (acct) acct_send(d, base + lane, gs_pb_field(gs_pb_field((int64_t)n * d.acctIdF)), 1);
          ctr_add(d, C_IWANT_SENT, (unsigned long long)n);
          if (rpc_traced(d, v, u))
            rpc_trace(d, h, v, u, 2, 3, GS_RPC_ORD(2, GS_RPC_O_SPAM), 1 + n, [&](auto put) {
              put(GS_RPC_ITEM_CTL, -1, -1);
              for (int q = 0; q < n; ++q) put(GS_RPC_ITEM_IWANT, -1, d.slotMid[d.pool[cur][off + q]]);
            });
        }
      }
    }
  }
  GS_STAMP(7);
  // ---- pass 2b: the stores of the first deliveries (after pass 3's loads,
  // which would otherwise wait for them)
  int running = 0;  // rank of the next entry of v's own frontier list
  // loop invariants read once (the ADV Dev lives in device memory, and every
  // store below could alias it for the compiler)
  const bool noFwd = behaves(d, v, GS_BEHAVE_NO_FORWARD);  // a squatter relays nothing
  const bool needAge = d.needAge, record = d.record;
  int16_t* const ageRow = needAge ? d.age + (int64_t)v * d.S : nullptr;
  uint8_t* const ffRow = record ? d.ffrom + (int64_t)v * d.S : nullptr;
  const int64_t* const pubHop = d.slotPubHop;
  uint64_t* const pmRow = prow >= 0 ? d.pmask + (int64_t)prow * d.S : nullptr;
  // randomsub targets (rs_select): a node of degree <= 32 draws two messages'
  // masks per wave step (rs_select2), the odd one last
  const bool rsV = rs_host(d, v);
  const bool pair2 = deg <= 32;
  const int rsP = valid ? u : -1;
  const uint64_t rsSub = (rsV && valid && edge_up(d, base + lane)) ? d.subA[u] : 0ull;
  int pendSlot = -1, pendFf = 0;
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    const uint64_t U = Uw[j];
    const uint64_t Ud = U & ~Xw[j];  // delivered (valid) fresh messages
    const int k = __popcll(Ud);
    const int incl = wave_incl_sum(k);
    int rank = running + incl - k;
    running += wave_last(incl);
    if (U | Rw[j]) d.seen[(int64_t)v * W + w] = (Sw[j] & ~Rw[j]) | U;
    // DENSE: v's frontier row of the next hop (k_publish adds own publishes);
    // amF also covers the words this parity's row held two hops ago
    if (DENSE && w < W && wm_has(amF, w)) d.fb[cur][(int64_t)v * W + w] = Ud;
    if (U) {
      if ((U & Ow[j]) || !wm_has(amW, w)) set_err(d, E_LATE);
      if (gossipV && Ud) d.hist[((int64_t)head * d.nOwnH + (v - d.n0)) * W + w] = Hw[j] | Ud;
      nDeliv += k;
      // one first delivery: trace, drec.peers, v's frontier list, age / deliverer
      auto put = [&](int b, int64_t ph) {
        const int slot = w * 64 + b;
        const int ff = sFirst[fidx(rkw[j], b)];
        if (trv)  // pubsub.go:1057, ReceivedFrom = the first deliverer
          trace_emit(d, h, GS_TRACE_DELIVER_MESSAGE, v, d.col[base + ff], (int)__umulhi((unsigned)slot, d.stMagic),
                     d.slotMid[slot], 2);
        if (pmRow != nullptr)  // DeliverMessage does not add the deliverer to drec.peers
          atomicAnd((unsigned long long*)&pmRow[slot], ~(1ull << ff));
        // v will not send it back to ff (fex below) unless ff authored it (the
        // author check needs a load only for a neighbour that authors at all)
        if (DENSE && (!((authM >> ff) & 1) || d.slotSrc[slot] != (sSnd[ff] & 0xFFFFFF)))
          atomicAdd((int*)sStart + ff, 1);
        if (!noFwd) {
          if (rank < FC) Lv[rank] = (uint32_t)slot | ((uint32_t)ff << 16);
          else set_err(d, E_FCAP);
        }
        ++rank;
        if (needAge) ageRow[slot] = (int16_t)(h - ph);
        if (record) ffRow[slot] = (uint8_t)ff;
      };
      uint64_t y = Ud;
      if (needAge) {
        while (y) {  // four messages at a time: their publish hops in flight together
          int bs[4];
          int64_t ph[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            bs[q] = y ? __ffsll((long long)y) - 1 : -1;
            y &= y ? y - 1 : 0ull;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) ph[q] = bs[q] >= 0 ? pubHop[w * 64 + bs[q]] : 0;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (bs[q] >= 0) put(bs[q], ph[q]);
        }
      } else {
        while (y) {
          const int b = __ffsll((long long)y) - 1;
          y &= y - 1;
          put(b, 0);
        }
      }
    }
    if (rsV) {  // randomsub: targets of every message first delivered here
      unsigned long long lanesWith = __ballot(Ud != 0);
      while (lanesWith) {
        const int src = __ffsll((long long)lanesWith) - 1;
        lanesWith &= lanesWith - 1;
        uint64_t y = lane_get64(Ud, src);
        const int wsrc = src + 64 * j;
        const int rks = lane_get(rkw[j], src);
        while (y) {
          const int b = __ffsll((long long)y) - 1;
          y &= y - 1;
          const int slot = wsrc * 64 + b, ff = sFirst[fidx(rks, b)];
          if (!pair2) {
            rs_select(d, v, base, deg, rsP, rsSub, slot, ff);
          } else if (pendSlot < 0) {
            pendSlot = slot;
            pendFf = ff;
          } else {
            rs_select2(d, v, base, deg, rsP, rsSub, pendSlot, pendFf, slot, ff);
            pendSlot = -1;
          }
        }
      }
    }
  }
  if (pendSlot >= 0) rs_select(d, v, base, deg, rsP, rsSub, pendSlot, pendFf);
  GS_STAMP(4);
  if (lane == 0) d.fln[cur][v] = behaves(d, v, GS_BEHAVE_NO_FORWARD) ? 0 : (running < FC ? running : FC);
  if constexpr (DENSE) {
    // per out-edge: the fresh messages of this hop each neighbour delivered
    // first (and did not author), which v's copies of the next hop leave out
    __syncthreads();
    if (valid) d.fex[cur][base + lane] = ((const int*)sStart)[lane];
    if (lane == 0) d.fbN[cur][v] = running;
  }
  const long long deliv = (long long)wave_sum_ll(nDeliv);
  const unsigned long long copies = wave_sum_ll(nCopies), s2 = wave_sum_ll(nSent), s3 = wave_sum_ll(nGray);
  if (lane == 0) {
    if (deliv) ctr_add(d, C_DELIVERIES, (unsigned long long)deliv);
    if (s2) ctr_add(d, C_TRANSMISSIONS, s2);
    if (s3) ctr_add(d, C_GRAYLISTED, s3);
  }
  if constexpr (ADV) {
    const unsigned long long rej = wave_sum_ll(nRejected), thc = wave_sum_ll(nThrottledCopies);
    const unsigned long long gc = wave_sum_ll(nGatedCopies);
    if (lane == 0) {
      const unsigned long long dups = copies - (unsigned long long)deliv - rej;
      if (dups) ctr_add(d, C_DUPLICATES, dups);
      if (rej) ctr_add(d, C_REJECTED, rej);
      if (thc) ctr_add(d, C_THROTTLED, thc);
      if (gc) ctr_add(d, C_GATED, gc);
    }
  } else {
    if (lane == 0 && copies - deliv) ctr_add(d, C_DUPLICATES, copies - deliv);
  }
}

// Floodsub on dense frontiers (FloodSubRouter.Publish floodsub.go:76-100 for
// every host that forwarded in the previous hop; pushMsg pubsub.go:978-1022).
// a frontier is a W-word bitmap fb[u] of the messages
// u first received (or published) in the previous hop, which u sent to every
// topic peer except ReceivedFrom and the author; receiver v ORs its senders'
// bitmaps in ascending sender order, so the first sender holding a bit is its
// first deliverer.  One wave per receiver, lane = word of v's topics in the
// active window: every sender's row is one coalesced read, the algorithm's
// (E_fwd + 3N) * W * 8 bytes per hop.  What a bitmap does not carry -- the
// copies u did not send v -- is counted exactly all the same: v drops the
// bits of its own messages (own[v], the author exclusion) itself, and u
// counted in its previous hop, per in-edge, the fresh messages that sender
// delivered first and did not author (fex[u's edge to v], ReceivedFrom), so
// transmissions / duplicates are the reference's per-copy counts.  Used by a
// floodsub engine without tracing, RPC accounting, churn, mixed routers or
// partitioning (gs_engine.hip denseFlood); k_phase_a's list walk covers the
// rest.
template <int WPL>
__global__ __launch_bounds__(64) void k_flood_a(Dev d, int64_t h, int cur, WMask amR, WMask amW, WMask amP) {
  __shared__ int sNb[64];         // v's neighbours, ascending
  __shared__ uint64_t sSubN[64];  // their subscriptions (what v's topic maps hold)
  __shared__ int sAuth[64];       // they author a live message (nAuth > 0)
  __shared__ int sEx[64];         // this hop's ReceivedFrom exclusions toward each neighbour
  __shared__ int sLive[64];       // the senders whose frontier is not empty, ascending
  const int v = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int prv = cur ^ 1;
  const int W = d.W, Wt = d.Wt;
  const int64_t base = d.rowptr[v];
  const int deg = (int)(d.rowptr[v + 1] - base);
  const uint64_t sv = d.sub[v];
  const bool valid = lane < deg;
  int ex = 0;  // copies sender `lane` did not send v (v had delivered them to it)
  bool live = false;
  if (valid) {
    const int64_t e = base + lane;
    const int u = d.col[e];
    sNb[lane] = u;
    sSubN[lane] = d.subA[u];
    sAuth[lane] = d.nAuth[u] > 0;
    ex = d.fex[prv][d.rev[e]];
    live = d.fbN[prv][u] != 0;  // (an empty frontier's row is all zero and is not read)
  }
  sEx[lane] = 0;
  const uint64_t lm = __ballot(live);
  const int nLive = __popcll(lm);
  if (live) sLive[__popcll(lm & ((1ull << lane) - 1))] = lane;
  const int oldN = d.fbN[cur][v];  // this parity's row is all zero iff its count is
  bool anyRet = false;
#pragma unroll
  for (int j = 0; j < GS_MAX_WPL; ++j) anyRet |= amP.m[j] != 0;
  if (nLive == 0 && !anyRet) {
    // nothing arrives and no slot is recycled: seen and counters stay; the
    // frontier of the next hop is empty (k_publish may add own publishes)
    if (oldN != 0) {
      for (int w = lane; w < W; w += 64) d.fb[cur][(int64_t)v * W + w] = 0ull;
      if (lane == 0) d.fbN[cur][v] = 0;
    }
    if (valid) d.fex[cur][base + lane] = 0;
    return;
  }
  uint64_t acc[WPL], S[WPL], R[WPL], O[WPL];
  bool act[WPL];
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    // v handles the messages of its own topics only (pubsub.go:959)
    act[j] = w < W && wm_has(amR, w) && ((sv >> (w / Wt)) & 1);
    const bool ret = w < W && wm_has(amP, w);
    S[j] = (act[j] || ret) ? d.seen[(int64_t)v * W + w] : 0ull;
    O[j] = act[j] ? d.own[(int64_t)v * W + w] : 0ull;  // v's own messages: nobody sends them back
    R[j] = ret ? d.pubmask[cur][w] : 0ull;
    acc[j] = 0;
  }
  __syncthreads();
  const uint64_t* const fbPrv = d.fb[prv];
  int16_t* const ageRow = d.needAge ? d.age + (int64_t)v * d.S : nullptr;
  uint8_t* const ffRow = d.record ? d.ffrom + (int64_t)v * d.S : nullptr;
  long long sent = 0;
  for (int k0 = 0; k0 < nLive; k0 += 4) {  // four live senders' rows in flight
    uint64_t F[4][WPL], A[4][WPL];  // the senders' frontiers, and the messages they authored
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int uq = k0 + q < nLive ? sNb[sLive[k0 + q]] : -1;
      const bool au = uq >= 0 && sAuth[sLive[k0 + q]] != 0;
#pragma unroll
      for (int j = 0; j < WPL; ++j) {
        F[q][j] = (uq >= 0 && act[j]) ? fbPrv[(int64_t)uq * W + lane + 64 * j] : 0ull;
        A[q][j] = (au && act[j]) ? d.own[(int64_t)uq * W + lane + 64 * j] : 0ull;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (k0 + q >= nLive) break;
      const int i = sLive[k0 + q];  // senders ascending: the first holding a bit delivers it
      const uint64_t subI = sSubN[i];
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < WPL; ++j) {
        const uint64_t f = F[q][j];
        sent += __popcll(f & ~O[j]);
        const uint64_t nb = f & ~acc[j] & ~S[j];  // first deliveries by sender i
        acc[j] |= f;
        if (!nb) continue;
        const int w = lane + 64 * j;
        if ((subI >> (w / Wt)) & 1) {
          // v will not send them back to i (ReceivedFrom); those i authored
          // are i's own messages, which i drops itself (O above)
          cnt += __popcll(nb & ~A[q][j]);
        }
        if (ageRow || ffRow)
          for (uint64_t y = nb; y; y &= y - 1) {
            const int slot = w * 64 + __ffsll((long long)y) - 1;
            if (ageRow) ageRow[slot] = (int16_t)(h - d.slotPubHop[slot]);
            if (ffRow) ffRow[slot] = (uint8_t)i;
          }
      }
      if (cnt) atomicAdd(&sEx[i], cnt);
    }
  }
  // fresh messages: seen (recycled slots' old bits cleared, k_publish sets the
  // author's), the frontier of the next hop (k_publish adds own publishes)
  long long nDeliv = 0;
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int w = lane + 64 * j;
    if (w >= W) continue;
    const uint64_t fr = acc[j] & ~S[j];
    if (fr) {
      nDeliv += __popcll(fr);
      if ((fr & d.oldm[w]) || !wm_has(amW, w)) set_err(d, E_LATE);
    }
    if (fr | R[j]) d.seen[(int64_t)v * W + w] = (S[j] & ~R[j]) | fr;
  }
  const long long deliv = (long long)wave_sum_ll(nDeliv);
  if (deliv != 0 || oldN != 0) {  // (a row whose count is 0 stays all zero)
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
      const int w = lane + 64 * j;
      if (w < W) d.fb[cur][(int64_t)v * W + w] = acc[j] & ~S[j];
    }
  }
  __syncthreads();
  if (lane == 0) d.fbN[cur][v] = (int)deliv;
  if (valid) d.fex[cur][base + lane] = sEx[lane];
  const long long copies = (long long)wave_sum_ll(sent) - (long long)wave_sum_ll(ex);
  if (lane == 0) {
    if (deliv) ctr_add(d, C_DELIVERIES, (unsigned long long)deliv);
    if (copies) ctr_add(d, C_TRANSMISSIONS, (unsigned long long)copies);
    if (copies - deliv) ctr_add(d, C_DUPLICATES, (unsigned long long)(copies - deliv));
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

// Clears the adversarial model's per-slot state of recycled message slots
// (the slots published in this hop held messages retired from the window):
// the IWANT spammers' drec.peers bits and peertx nibbles.  One thread per
// (node, word) of the words[] list.  (The seen bits themselves are cleared by
// phase A's pass 2b, the amP / Rw masks, and k_publish then sets the authors'
// bits; this kernel runs only when spammers exist.)
__global__ void k_retire(Dev d, int cur, const int32_t* __restrict__ words, int nwords) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)(d.n1 - d.n0) * nwords) return;
  const int v = d.n0 + (int)(k / nwords);
  const int w = words[k % nwords];
  if (d.spamRow != nullptr && d.pubmask[cur][w]) {
    // a recycled slot starts with no peertx counts from v's spammer peers
    const uint64_t pm = d.pubmask[cur][w];
    for (int64_t e = d.rowptr[v]; e < d.rowptr[v + 1]; ++e) {
      const int row = d.spamRow[e];
      if (row < 0) continue;
      uint32_t* c = d.spamCnt + (int64_t)row * (d.S >> 3) + w * 8;
      for (int q = 0; q < 8; ++q) {
        const uint32_t b = (uint32_t)(pm >> (8 * q)) & 0xFFu;
        if (!b) continue;
        uint32_t m = 0;
        for (int j = 0; j < 8; ++j)
          if ((b >> j) & 1) m |= 0xFu << (4 * j);
        c[q] &= ~m;
      }
    }
  }
  if (d.pmaskRow != nullptr && d.pmaskRow[v] >= 0) {  // a recycled slot starts a fresh record
    uint64_t y = d.pubmask[cur][w];
    while (y) {
      const int b = __ffsll((long long)y) - 1;
      y &= y - 1;
      d.pmask[(int64_t)d.pmaskRow[v] * d.S + w * 64 + b] = 0;
    }
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
  const int prevAuthor = d.slotSrc[slot];  // the retired message of this slot
  // slot metadata is replicated on every rank; the rest belongs to src's rank
  if (prevAuthor >= d.n0 && prevAuthor < d.n1) {
    atomicSub(&d.nAuth[prevAuthor], 1);
    if (d.own != nullptr)  // k_flood_a's author exclusion: the retired message is no longer prevAuthor's
      atomicAnd((unsigned long long*)&d.own[(int64_t)prevAuthor * d.W + (slot >> 6)], ~(1ull << (slot & 63)));
  }
  d.slotSrc[slot] = src;
  d.slotPubHop[slot] = h;
  d.slotMid[slot] = d.mId[b + i];
  const uint8_t kind = d.mKind[b + i];
  d.slotKind[slot] = kind;
  if (src < d.n0 || src >= d.n1) return;
  atomicAdd(&d.nAuth[src], 1);
  if (kind == GS_MSG_PHANTOM) {
    // an advertised-only id: in the author's seen set and mcache (emitGossip
    // lists it), never sent or traced (IHAVE spam, gossipsub_spam_test.go:196-203)
    const int w = slot >> 6;
    const unsigned long long bit = 1ull << (slot & 63);
    atomicOr((unsigned long long*)&d.seen[(int64_t)src * d.W + w], bit);
    if (gossip_host(d, src)) atomicOr((unsigned long long*)&d.hist[((int64_t)head * d.nOwnH + (src - d.n0)) * d.W + w], bit);
    if (d.needAge) d.age[(int64_t)src * d.S + slot] = 0;
    if (d.record) d.ffrom[(int64_t)src * d.S + slot] = 255;
    return;
  }
  if (is_traced(d, src)) {  // validation.go:217, then pubsub.go:1057 with ReceivedFrom = self
    trace_emit(d, h, GS_TRACE_PUBLISH_MESSAGE, src, -1, d.mTopic[b + i], d.mId[b + i], 1);
    trace_emit(d, h, GS_TRACE_DELIVER_MESSAGE, src, src, d.mTopic[b + i], d.mId[b + i], 1);
  }
  const int w = slot >> 6;
  const unsigned long long bit = 1ull << (slot & 63);
  atomicOr((unsigned long long*)&d.seen[(int64_t)src * d.W + w], bit);
  if (gossip_host(d, src)) atomicOr((unsigned long long*)&d.hist[((int64_t)head * d.nOwnH + (src - d.n0)) * d.W + w], bit);
  if (d.fb[0] != nullptr) {  // k_flood_a: the frontier of the next hop, and the author's own messages
    atomicOr((unsigned long long*)&d.fb[cur][(int64_t)src * d.W + w], bit);
    atomicAdd(&d.fbN[cur][src], 1);
    atomicOr((unsigned long long*)&d.own[(int64_t)src * d.W + w], bit);
  }
  if (d.needAge) d.age[(int64_t)src * d.S + slot] = 0;
  if (d.record) d.ffrom[(int64_t)src * d.S + slot] = 255;
  ctr_add(d, C_PUBLISHED, 1ull);
}

// Adds this hop's local publishes to the publisher's frontier list (tag 255 =
// own publish, forwarded on the edges of fwdPub), keeping the list sorted by
// slot.  One thread per message; the thread of a node's first message of the
// hop inserts all of that node's messages.
__global__ void k_publist(Dev d, int b, int n, int cur) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int src = d.mSrc[b + i];
  if (src < d.n0 || src >= d.n1) return;
  for (int j = 0; j < i; ++j)
    if (d.mSrc[b + j] == src) return;
  uint32_t* L = d.fl[cur] + (int64_t)src * d.FC;
  int len = d.fln[cur][src];
  for (int j = i; j < n; ++j) {
    if (d.mSrc[b + j] != src || d.mKind[b + j] == GS_MSG_PHANTOM) continue;  // phantoms are never sent
    const uint32_t slot = (uint32_t)d.mSlot[b + j];
    if (len >= d.FC) {
      set_err(d, E_FCAP);
      break;
    }
    int pos = len;
    while (pos > 0 && (L[pos - 1] & 0xFFFFu) > slot) {
      L[pos] = L[pos - 1];
      --pos;
    }
    L[pos] = slot | (255u << 16);
    ++len;
  }
  d.fln[cur][src] = len;
}

// Lane t gets column t of the 64 x 64 bit matrix whose row j is lane j's x:
// bit j of the result = bit t of lane j's x (butterfly block swaps).
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x) {
  const int lane = lane_id();
  const uint64_t lo[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                          0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int s = 32 >> k;
    const uint64_t m = lo[k];
    const uint64_t y = shfl_u64(x, lane ^ s);
    x = (lane & s) ? (((y & ~m) >> s) | (x & ~m)) : ((x & m) | ((y & m) << s));
  }
  return x;
}

// Push (Dev::ibx): the copies owned sender u sends on each edge to an owned
// receiver in the next hop's phase A — its frontier list fl[cur][u] (first
// deliveries of this hop and its publishes) filtered per edge as the
// receiver's list walk would: the edge's forwarding sets (relay for first
// deliveries, pub for tag 255; every topic of the sets, the receiver drops
// the topics it left), never back to the first deliverer (tag == the
// receiver's position in u's row, gossipsub.go:1003), and randomsub's
// targets.  The author exclusion stays with the receiver (a cheap test there).
// One wave per sender: the edges' sets transposed to per-topic edge masks,
// then lane = list entry: its edge mask, a count pass (LDS counters), the
// segments laid out 8-aligned in row order in the sender's own region of the
// arena (GS_PUSHR slots, no allocation), staged in LDS (order within a
// segment is free: the receiver's updates commute) and stored coalesced.
// Records go to the receiver's in-edge (a receiver on another rank gets the
// record and the segment through the exchange, gs_exchange.h); every edge of
// a sender whose copies overflow its region gets -1: the receiver walks the
// sender's list.
__global__ __launch_bounds__(64) void k_push(Dev d, int cur) {
  __shared__ uint64_t sMR[64], sMP[64];
  __shared__ uint16_t sSlot[64];
  __shared__ __attribute__((aligned(16))) uint16_t sOut[GS_PUSHR];
  const int u = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const int64_t e = base + lane;
  const uint32_t* L = d.fl[cur] + (int64_t)u * d.FC;
  // everything the wave needs first, loaded at once: the list length, the
  // first 64 entries (speculatively: a list slot past fln holds stale data),
  // the edges' sets
  const int Ln0 = d.fln[cur][u];
  const uint32_t ent0 = L[lane];
  // the second 64 entries too (a list holds ~100 at config4), within the row
  const uint32_t ent1 = L[64 + lane < d.FC ? 64 + lane : d.FC - 1];
  // every out-edge gets a record; one to a receiver on another rank travels
  // with the hop's exchange (gs_exchange.h k_xp_pack)
  const bool local = lane < deg;
  uint64_t relay = 0, pub = 0;
  int64_t re = 0;
  if (local) {
    re = rxi(d, e, d.rev[e]);
    relay = d.fwdRelay[cur][e];
    pub = d.fwdPub[cur][e];
  }
  const int Ln = __ballot((relay | pub) != 0) ? Ln0 : 0;
  if (Ln == 0) {
    if (local) d.ibxRec[cur][re] = 0;  // nothing sent
    return;
  }
  sMR[lane] = wave_transpose64(relay);  // edges whose relay set holds topic `lane`
  sMP[lane] = wave_transpose64(pub);
  __syncthreads();
  const bool rs = rs_host(d, u);
  // the edges entry k goes out on
  auto dest = [&](uint32_t ent, int& slot) -> uint64_t {
    slot = (int)(ent & 0xFFFF);
    const int tag = (int)(ent >> 16);
    const int t = (int)__umulhi((unsigned)slot, d.stMagic);
    uint64_t m = tag == 255 ? sMP[t] : (sMR[t] & ~(1ull << (tag & 63)));
    if (rs) m &= d.sel[(int64_t)u * d.S + slot];
    return m;
  };
  // lane = entry: its edge mask; transposed, lane = edge: its entries of the
  // chunk (the first two chunks' kept in registers for the write pass)
  const int nch = (Ln + 63) >> 6;
  int s0 = 0, s1 = 0;
  const uint64_t E0 = wave_transpose64(lane < Ln ? dest(ent0, s0) : 0ull);
  const uint64_t E1 = nch > 1 ? wave_transpose64(64 + lane < Ln ? dest(ent1, s1) : 0ull) : 0ull;
  int cnt = __popcll(E0) + __popcll(E1);
  for (int c = 2; c < nch; ++c) {
    int slot;
    cnt += __popcll(wave_transpose64(64 * c + lane < Ln ? dest(L[64 * c + lane], slot) : 0ull));
  }
  const int seg = (cnt + 7) & ~7;
  const int incl = wave_incl_sum(seg);
  const int total = wave_last(incl);
  const int pre = incl - seg;
  if (total > GS_PUSHR) {
    if (local) d.ibxRec[cur][re] = -1;  // region overflow: the receiver walks u's list
    if (lane == 0 && d.pushOvf != nullptr) *d.pushOvf = 1;
    return;
  }
  // lane j (edge j) writes its entries of each chunk contiguously from its
  // segment start
  int run = pre;
  auto put = [&](uint64_t E, int slot) {
    sSlot[lane] = (uint16_t)slot;
    __syncthreads();
    for (; E; E &= E - 1) sOut[run++] = sSlot[__ffsll((long long)E) - 1];
    __syncthreads();
  };
  put(E0, s0);
  if (nch > 1) put(E1, s1);
  for (int c = 2; c < nch; ++c) {
    int slot = 0;
    const uint64_t E = wave_transpose64(64 * c + lane < Ln ? dest(L[64 * c + lane], slot) : 0ull);
    put(E, slot);
  }
  const int64_t A = (int64_t)(u - d.n0) * GS_PUSHR;
  const uint4* src = (const uint4*)sOut;
  uint4* dst = (uint4*)(d.ibx[cur] + A);
  for (int k = lane; k < total / 8; k += 64) dst[k] = src[k];
  if (local) d.ibxRec[cur][re] = ((A + pre) << 24) | (int64_t)cnt;
}

// Randomsub targets of the messages published this hop (one wave per message).
__global__ __launch_bounds__(64) void k_publish_rs(Dev d, int b) {
  const int i = blockIdx.x;
  const int slot = d.mSlot[b + i];
  const int u = d.mSrc[b + i];
  if (u < d.n0 || u >= d.n1 || !rs_host(d, u)) return;  // another rank's host (its mask travels with
                                                       // its list), or another router's publish
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const int p = lane < deg ? d.col[base + lane] : -1;
  const uint64_t subp = p >= 0 && edge_up(d, base + lane) ? d.subA[p] : 0;
  rs_select(d, u, base, deg, p, subp, slot, 255);
}

// ---------------------------------------------------------------- peer gater decay
// peerGater.decayStats (peer_gater.go:219-259) every gater DecayInterval: the
// node counters (thread per node) and the per-IP stats held on group edges
// (thread per edge).  A stats object with a connected peer decays; one whose
// peers all disconnected is frozen until its expiry (RemovePeer + RetainStats,
// :374-383), then deleted — its counters restart from zero.
__device__ __forceinline__ double gdecay(double x, double f, double z) {
  x *= f;
  return x < z ? 0.0 : x;
}
// RPC accounting: the payload RPCs u sent in the hop of parity p (its list and
// forwarding sets; forwarded and published messages, one RPC each,
// rpcWithMessages), counted at the end of the hop — the filter of phase A's
// list walk seen from the sender.  A wave per sender, lane = out-edge, the
// list's entries broadcast one at a time.
__global__ __launch_bounds__(64) void k_acct_payload(Dev d, int p) {
  const int u = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const uint64_t ru = valid ? d.fwdRelay[p][e] : 0, pu = valid ? d.fwdPub[p][e] : 0;
  if (!__ballot((ru | pu) != 0)) return;
  const int w = valid ? d.col[e] : 0;
  // the receiver authored a live message (nAuth is kept for owned nodes only)
  const bool authW = valid && (d.world > 1 || d.nAuth[w] > 0);
  const int Ln = d.fln[p][u];
  const uint32_t* L = d.fl[p] + (int64_t)u * d.FC;
  const bool rsU = rs_host(d, u);
  unsigned long long b = 0, n = 0;
  for (int k0 = 0; k0 < Ln; k0 += 64) {
    const uint32_t mine = k0 + lane < Ln ? L[k0 + lane] : 0u;
    const int cnt = min(64, Ln - k0);
    for (int k = 0; k < cnt; ++k) {
      const uint32_t ent = (uint32_t)lane_get((int)mine, k);
      const int slot = (int)(ent & 0xFFFF), tag = (int)(ent >> 16);
      const int t = (int)__umulhi((unsigned)slot, d.stMagic);
      bool sent = tag == 255 ? ((pu >> t) & 1) : ((ru >> t) & 1);
      sent = sent && tag != lane;  // not back to the deliverer (gossipsub.go:1003)
      if (sent && rsU) sent = (d.sel[(int64_t)u * d.S + slot] >> lane) & 1;
      if (sent && authW && d.slotSrc[slot] == w) sent = false;  // never to the author
      if (sent) {
        b += (unsigned long long)d.acc[t].msgF;
        ++n;
      }
    }
  }
  if (valid && n) acct_send(d, e, (int64_t)b, (int)n);
}

// RPC accounting: (edge, bytes) pairs of the host-side RPCs of a hop
// RPC trace of this hop's payload RPCs (gs_set_trace_rpc): one RPC per
// forwarded or published message and receiver, the walk of k_acct_payload;
// only senders that are traced or have a traced peer do any work.
__global__ __launch_bounds__(64) void k_trace_payload(Dev d, int p, int64_t hop) {
  const int u = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int64_t base = d.rowptr[u];
  const int deg = (int)(d.rowptr[u + 1] - base);
  const bool valid = lane < deg;
  const int64_t e = base + lane;
  const int w = valid ? d.col[e] : 0;
  const bool tr = valid && (is_traced(d, u) || is_traced(d, w));
  if (!__ballot(tr)) return;
  const uint64_t ru = valid ? d.fwdRelay[p][e] : 0, pu = valid ? d.fwdPub[p][e] : 0;
  const int Ln = d.fln[p][u];
  const uint32_t* L = d.fl[p] + (int64_t)u * d.FC;
  for (int k0 = 0; k0 < Ln; k0 += 64) {
    const uint32_t mine = k0 + lane < Ln ? L[k0 + lane] : 0u;
    const int cnt = min(64, Ln - k0);
    for (int k = 0; k < cnt; ++k) {
      const uint32_t ent = (uint32_t)lane_get((int)mine, k);
      const int slot = (int)(ent & 0xFFFF), tag = (int)(ent >> 16);
      const int t = (int)__umulhi((unsigned)slot, d.stMagic);
      bool sent = tr && (tag == 255 ? ((pu >> t) & 1) : ((ru >> t) & 1));
      sent = sent && tag != lane;  // not back to the deliverer (gossipsub.go:1003)
      if (sent && rs_host(d, u)) sent = (d.sel[(int64_t)u * d.S + slot] >> lane) & 1;
      if (sent && d.slotSrc[slot] == w) sent = false;  // never to the author
      if (sent) {
        const int sp = tag == 255 ? 1 : 2;  // local publish / forward
        const int64_t mid = d.slotMid[slot];
        rpc_trace(d, hop, u, w, sp, 2, GS_RPC_ORD(sp, mid), 1, [&](auto put) { put(GS_RPC_ITEM_MSG, t, mid); });
      }
    }
  }
}

__global__ void k_acct_add(Dev d, const int64_t* __restrict__ pairs, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  // one edge may get several (a node announcing two topics): atomics
  atomicAdd(&d.rpcB[pairs[2 * k]], (unsigned long long)pairs[2 * k + 1]);
  atomicAdd(&d.rpcN[pairs[2 * k]], 1ull);
}

__global__ void k_gater_decay(Dev d, int64_t now) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.n1 - d.n0) {
    const int v = d.n0 + (int)i;
    d.gValidate[v] = gdecay(d.gValidate[v], d.gGlobalDecay, d.gDecayToZero);
    d.gThrottle[v] = gdecay(d.gThrottle[v], d.gGlobalDecay, d.gDecayToZero);
  }
  const int64_t e = d.e0 + i;
  if (e >= d.e1) return;
  if (d.rowptr[d.esrc[e]] + d.gGrp[e] != e) return;  // not a group's stats edge
  if (d.gConn[e] > 0) {
    for (int k = 0; k < 4; ++k) d.gSt[k * d.eOwn + e] = gdecay(d.gSt[k * d.eOwn + e], d.gSourceDecay, d.gDecayToZero);
  } else if (d.gExp[e] < now) {
    for (int k = 0; k < 4; ++k) d.gSt[k * d.eOwn + e] = 0.0;  // delete(pg.ipStats, ip)
  }
}
