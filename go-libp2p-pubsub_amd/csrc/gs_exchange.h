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
  const int64_t ri = d.rev[e];  // outbox records are indexed by the receiver's in-edge
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
  const int64_t ri = d.rev[e];
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
  const int64_t ri = d.rev[e];
  d.fwdRelay[cur][e] = x.relay;
  d.fwdPub[cur][e] = x.pub;
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

// Another rank's lists into the mirror: nodes [n0r, n0r + nr).
__global__ __launch_bounds__(64) void k_x_unlists(Dev d, int cur, const int64_t* __restrict__ hdr,
                                                  const uint32_t* __restrict__ ent, int n0r) {
  const int u = n0r + blockIdx.x;
  const int lane = lane_id();
  const int64_t h = hdr[blockIdx.x];
  const int len = (int)(h & 0xFFFF);
  const int64_t off = h >> 16;
  uint32_t* L = d.fl[cur] + (int64_t)u * d.FC;
  for (int i = lane; i < len; i += 64) L[i] = ent[off + i];
  if (lane == 0) d.fln[cur][u] = len;
}

__global__ void k_set_u64(unsigned long long* p, unsigned long long v) { *p = v; }
