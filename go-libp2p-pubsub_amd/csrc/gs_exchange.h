// gs_exchange.h — per-hop exchange of a partitioned engine (one rank per GPU,
// SURVEY.md §8e).
//
// Every piece of router state belongs to the observing node, so the only
// cross-rank traffic is what a node sends to its neighbours in one hop: the
// RPCs of handleIncomingRPC's next call (pubsub.go:946-969).  In this engine a
// receiver reads, through the reverse edge r = rev[e], what its sender wrote
// in the previous hop (parity prv):
//   - the sender's frontier list fl[u] / fln[u] (the payload of its RPCs),
//   - the forwarding sets fwdRelay[r] / fwdPub[r] (the sender's mesh, fanout,
//     direct and flood-publish choice for that edge),
//   - the control outbox of edge r (GRAFT / PRUNE / IHAVE / IWANT entries, an
//     IWANT spammer's re-request list) and the slot-id arena lists its
//     records point at,
//   - after a heartbeat, the sender's IHAVE payload row gw[u].
// Each rank keeps a full-size mirror of these arrays: its own nodes' entries
// are written by its kernels, every other entry by the unpack kernels below.
// At the end of hop h the parity written in h is exchanged:
//   broadcast part (all-gather, equal chunks):
//     [node header: (off << 16 | len) per owned node][list entries]
//     [randomsub target masks of the entries, engines with randomsub hosts]
//     [the rank's arena segment][gw rows of owned nodes, heartbeat hops only]
//   edge records (all-to-all-v, block per destination rank): one XRec per
//     owned edge whose receiver lives on another rank and whose forwarding set
//     changed or whose control outbox is not empty.  Records are moved: the
//     sender's copy of the outbox entry is cleared once packed (the receiver's
//     phase B clears its mirror after consuming it, exactly as for local edges).
#pragma once
#include "gs_device.h"

struct XRec {  // 96 bytes
  int32_t e;   // the sender's edge (receiver reads it as rev[e'])
  uint8_t pre, hb;
  uint8_t nsrv;  // reply RPCs carrying served messages (IWANT-spam runs)
  uint8_t pad;
  uint64_t relay, pub, gj, ghb, prep, phb, ihave;
  int64_t iwant, iresp;
  int64_t spam;  // an IWANT spammer's re-request list (arena record), -1 = none
  int64_t px;    // the PRUNEs' peer-exchange lists (arena record), -1 = none
};
static_assert(sizeof(XRec) == 96, "XRec layout");

__device__ __forceinline__ bool x_needed(const Dev& d, int cur, int64_t e, int& dest) {
  dest = d.nodeRank[d.col[e]];
  if (dest == d.rank) return false;
  const int64_t ri = rxi(d, e, d.rev[e]);  // the receiver's records of edge e: its stage slot here
  return d.xmark[e] || d.cPre[cur][ri] || d.cHb[cur][ri];
}

// Records per destination rank.
__global__ void k_x_count(Dev d, int cur, unsigned long long* __restrict__ cnt) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  int dest;
  if (x_needed(d, cur, e, dest)) atomicAdd(&cnt[dest], 1ull);
}

// Packs the records at off[dest] + (running index) and clears what was moved.
__global__ void k_x_pack(Dev d, int cur, const int64_t* __restrict__ off, unsigned long long* __restrict__ cursor,
                         XRec* __restrict__ out) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  int dest;
  if (!x_needed(d, cur, e, dest)) return;
  const int64_t k = off[dest] + (int64_t)atomicAdd(&cursor[dest], 1ull);
  const int64_t ri = rxi(d, e, d.rev[e]);  // the stage slot of edge e
  XRec x;
  x.e = (int32_t)e;
  x.pre = d.cPre[cur][ri];
  x.hb = d.cHb[cur][ri];
  x.pad = 0;
  x.relay = d.fwdRelay[cur][e];
  x.pub = d.fwdPub[cur][e];
  if (x.pre | x.hb) {
    x.gj = d.cGraftJoin[cur][ri];
    x.ghb = d.cGraftHb[cur][ri];
    x.prep = d.cPruneReply[cur][ri];
    x.phb = d.cPruneHb[cur][ri];
    x.ihave = d.cIhave[cur][ri];
    x.iwant = d.cIwant[cur][ri];
    x.iresp = d.cIresp[cur][ri];
    x.spam = d.cSpam[cur] != nullptr ? d.cSpam[cur][ri] : -1;
    x.nsrv = d.cNSrv[cur] != nullptr ? d.cNSrv[cur][ri] : 0;
    x.px = d.doPX ? d.cPx[cur][ri] : -1;
    if (d.doPX) d.cPx[cur][ri] = -1;
    if (d.cSpam[cur] != nullptr) {
      d.cSpam[cur][ri] = -1;
      d.cNSrv[cur][ri] = 0;
    }
    d.cPre[cur][ri] = 0;
    d.cHb[cur][ri] = 0;
    d.cGraftJoin[cur][ri] = 0;
    d.cGraftHb[cur][ri] = 0;
    d.cPruneReply[cur][ri] = 0;
    d.cPruneHb[cur][ri] = 0;
    d.cIhave[cur][ri] = 0;
    d.cIwant[cur][ri] = -1;
    d.cIresp[cur][ri] = -1;
  } else {
    x.gj = x.ghb = x.prep = x.phb = x.ihave = 0;
    x.iwant = x.iresp = x.spam = x.px = -1;
    x.nsrv = 0;
  }
  d.xmark[e] = 0;
  out[k] = x;
}

__global__ void k_x_unpack(Dev d, int cur, const XRec* __restrict__ in, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const XRec x = in[k];
  const int64_t e = x.e;
  const int64_t ri = d.rev[e];  // this rank's in-edge (the sender's sets live with the sender)
  d.fwdIn[cur][ri] = make_ulonglong2(x.relay, x.pub);
  d.cPre[cur][ri] = x.pre;
  d.cHb[cur][ri] = x.hb;
  d.cGraftJoin[cur][ri] = x.gj;
  d.cGraftHb[cur][ri] = x.ghb;
  d.cPruneReply[cur][ri] = x.prep;
  d.cPruneHb[cur][ri] = x.phb;
  d.cIhave[cur][ri] = x.ihave;
  d.cIwant[cur][ri] = x.iwant;
  d.cIresp[cur][ri] = x.iresp;
  if (d.cSpam[cur] != nullptr) {
    d.cSpam[cur][ri] = x.spam;
    d.cNSrv[cur][ri] = x.nsrv;
  }
  if (d.doPX) d.cPx[cur][ri] = x.px;
}

// Frontier lists of the owned nodes: one wave per node, entries appended at a
// bump offset (their order in the chunk is irrelevant: the header locates
// them).  `cap` entries fit; the bump keeps counting past it so the host can
// grow the buffer and pack again.
__global__ __launch_bounds__(64) void k_x_lists(Dev d, int cur, unsigned long long* __restrict__ bump,
                                                int64_t* __restrict__ hdr, uint32_t* __restrict__ ent, int64_t cap) {
  const int v = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int len = d.fln[cur][v];
  unsigned long long off = 0;
  if (lane == 0) off = len ? atomicAdd(bump, (unsigned long long)len) : 0ull;
  off = lane_get64(off, 0);
  if (lane == 0) hdr[blockIdx.x] = ((int64_t)off << 16) | len;
  if ((int64_t)(off + len) > cap) return;
  const uint32_t* L = d.fl[cur] + (int64_t)v * d.FC;
  for (int i = lane; i < len; i += 64) ent[off + i] = L[i];
}

// Randomsub target masks of the packed entries (d.sel: a receiver's list walk
// keeps a randomsub sender's copy only on the edges of its mask, randomsub.go:
// 115-149), one u64 per entry in the entries' order; 0 for other routers'.
__global__ __launch_bounds__(64) void k_x_sel(Dev d, const int64_t* __restrict__ hdr, const uint32_t* __restrict__ ent,
                                              uint64_t* __restrict__ sel) {
  const int v = d.n0 + blockIdx.x;
  const int lane = lane_id();
  const int64_t h = hdr[blockIdx.x];
  const int len = (int)(h & 0xFFFF);
  const int64_t off = h >> 16;
  const bool rs = rs_host(d, v);
  for (int i = lane; i < len; i += 64) sel[off + i] = rs ? d.sel[(int64_t)v * d.S + (ent[off + i] & 0xFFFF)] : 0ull;
}

// Another rank's lists into the mirror: nodes [n0r, n0r + nr); with `sel`, the
// randomsub senders' target masks of those entries too.
__global__ __launch_bounds__(64) void k_x_unlists(Dev d, int cur, const int64_t* __restrict__ hdr,
                                                  const uint32_t* __restrict__ ent, const uint64_t* __restrict__ sel,
                                                  int n0r) {
  const int u = n0r + blockIdx.x;
  const int lane = lane_id();
  const int64_t h = hdr[blockIdx.x];
  const int len = (int)(h & 0xFFFF);
  const int64_t off = h >> 16;
  uint32_t* L = d.fl[cur] + (int64_t)u * d.FC;
  const bool rs = sel != nullptr && rs_host(d, u);
  for (int i = lane; i < len; i += 64) {
    const uint32_t x = ent[off + i];
    L[i] = x;
    if (rs) d.sel[(int64_t)u * d.S + (x & 0xFFFF)] = sel[off + i];
  }
  if (lane == 0) d.fln[cur][u] = len;
}

// ---- pushed copies of cross-rank edges (k_push's segments, Dev::ibx) ----
// A sender's k_push lays out the copies of EVERY out-edge, and writes each
// edge's record at ibxRec[cur][rev[e]] (the receiver's in-edge).  For an edge
// whose receiver lives on another rank, the record and its slots travel in a
// second all-to-all-v, one block per destination rank:
//   [PRec x nRec][slots, each segment 8-aligned]
// and the receiver's alltoallv lands the blocks right behind its own senders'
// regions in ibx[cur], so its phase A reads a remote sender's copies exactly
// like a local one's (pOff into ibx), instead of walking the sender's whole
// frontier list.  A record travels for every edge the sender forwards on
// (fwdRelay | fwdPub != 0 -- exactly the edges whose fwdIn mirror makes the
// receiver read its record); -1 (the sender's region overflowed) keeps the
// list walk.
struct PRec {  // 16 bytes
  int32_t ri;   // the receiver's in-edge (rev[e])
  int32_t n;    // copies, -1 = walk the sender's list
  int64_t off;  // first slot of the segment, in slots from the block's slot region
};
static_assert(sizeof(PRec) == 16, "PRec layout");

__device__ __forceinline__ bool xp_needed(const Dev& d, int cur, int64_t e, int& dest) {
  dest = d.nodeRank[d.col[e]];
  if (dest == d.rank) return false;
  return (d.fwdRelay[cur][e] | d.fwdPub[cur][e]) != 0;
}
__device__ __forceinline__ int xp_slots(int64_t rec) {  // slots a record's segment occupies (8-aligned)
  return rec > 0 ? (int)(((rec & 0xFFFFFF) + 7) & ~7) : 0;
}

// Records and slots per destination rank: cnt[dest], cnt[world + dest].
__global__ void k_xp_count(Dev d, int cur, unsigned long long* __restrict__ cnt) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  int dest;
  if (!xp_needed(d, cur, e, dest)) return;
  atomicAdd(&cnt[dest], 1ull);
  const int ns = xp_slots(d.ibxRec[cur][rxi(d, e, d.rev[e])]);
  if (ns) atomicAdd(&cnt[d.world + dest], (unsigned long long)ns);
}

// Packs the records and segments; boff[dest] = block byte offset in `out`,
// nrec[dest] = the block's record count, cursors [world] records, [world] slots.
__global__ void k_xp_pack(Dev d, int cur, const int64_t* __restrict__ boff, const int64_t* __restrict__ nrec,
                          unsigned long long* __restrict__ cursor, uint8_t* __restrict__ out) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.e1) return;
  int dest;
  if (!xp_needed(d, cur, e, dest)) return;
  const int64_t ri = d.rev[e];
  const int64_t rec = d.ibxRec[cur][rxi(d, e, ri)];
  const int ns = xp_slots(rec);
  uint8_t* blk = out + boff[dest];
  const int64_t k = (int64_t)atomicAdd(&cursor[dest], 1ull);
  int64_t so = 0;
  if (ns) {
    so = (int64_t)atomicAdd(&cursor[d.world + dest], (unsigned long long)ns);
    const uint4* src = (const uint4*)(d.ibx[cur] + (rec >> 24));  // 8-aligned segment: 16-B aligned
    uint4* dst = (uint4*)(blk + 16 * nrec[dest] + 2 * so);
    for (int j = 0; j < ns / 8; ++j) dst[j] = src[j];
  }
  PRec p;
  p.ri = (int32_t)ri;
  p.n = rec < 0 ? -1 : (int32_t)(rec & 0xFFFFFF);
  p.off = so;
  ((PRec*)blk)[k] = p;
}

// One source rank's block, received at slot index `slot0` of ibx[cur] (its
// slot region starts after the records): the receiver's records point at it.
__global__ void k_xp_unpack(Dev d, int cur, const PRec* __restrict__ in, int64_t n, int64_t slotBase) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const PRec p = in[k];
  d.ibxRec[cur][p.ri] = p.n < 0 ? -1 : (((slotBase + p.off) << 24) | (int64_t)p.n);
}

__global__ void k_set_u64(unsigned long long* p, unsigned long long v) { *p = v; }
