// gs_device.h — device-side state and helpers of the MI355X gossip engine.
//
// Layout: message slots are topic-segmented, slot s belongs to
// topic s / St; a node bitset is W = T*Wt 64-bit words.  Per-node arrays are
// row-major [node][word]; per-edge arrays are indexed by the CSR edge id e
// (observer u = edge_src[e], neighbour col[e]); per-(edge,topic) state
// (score counters, backoff) is tiled [e/64][t][e%64] (tix): a wave of 64
// consecutive edges reads one contiguous 512-byte row per topic, and all the
// topics of a node's edges lie within a few KiB, so per-node passes stay
// inside a handful of pages instead of touching T pages E*8 bytes apart.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gossip_engine.h"
#include "../../include/gs_rng.h"
#include "../../include/gs_rpcsize.h"
#include "../../include/gs_trace.h"
#include "../../include/gs_fp.h"

#define GS_WAVE 64
// Occupancy hints (waves per SIMD the register allocator must allow) of the
// latency-bound node-wave kernels; -DGS_WPE_<K>=n overrides for experiments.
#define GS_WPE_(n) __attribute__((amdgpu_waves_per_eu(n)))
// heartbeat: 6 waves/SIMD (80 VGPRs) measured 43 -> 34 ms per launch at
// config4 against the allocator's own 4 (97 VGPRs); 8 spills and loses
#ifndef GS_WPE_HB
#define GS_WPE_HB 6
#endif
#ifdef GS_WPE_HB
#define GS_OCC_HB GS_WPE_(GS_WPE_HB)
#else
#define GS_OCC_HB
#endif
// refresh: 4 waves/SIMD (<= 128 VGPRs): at 141 VGPRs (3 waves) the config4
// refresh took 44 ms per launch instead of 33 (round 5)
#ifndef GS_WPE_RF
#define GS_WPE_RF 4
#endif
#ifdef GS_WPE_RF
#define GS_OCC_RF GS_WPE_(GS_WPE_RF)
#else
#define GS_OCC_RF
#endif
// phase A: at least 3 waves/SIMD (<= 168 VGPRs): the adversarial 3-word
// instantiation at 171 VGPRs ran 2 waves and config5's phase A went 185 -> 228
// ms per round (round 5); LDS keeps phase A at about 10 waves per CU anyway
#ifndef GS_WPE_PA
#define GS_WPE_PA 3
#endif
#ifdef GS_WPE_PA
#define GS_OCC_PA GS_WPE_(GS_WPE_PA)
#else
#define GS_OCC_PA
#endif
#ifdef GS_WPE_PB
#define GS_OCC_PB GS_WPE_(GS_WPE_PB)
#else
#define GS_OCC_PB
#endif
#define GS_MAX_WPL 4   // words per lane in the node-wave kernels: W <= 256
#ifndef GS_SBATCH
#define GS_SBATCH 2    // edge_scores_batch: edges whose loads are in flight together (<= 4)
#endif
#define GS_QCAP 320    // phase A delivery queue (>= 63 pending + 256 appended per sub-round)
#define GS_BMAP 32     // phase A: list blocks mapped to senders without a search (64 per entry)
// push arena: a region of this many 16-bit slots per owned sender
#define GS_PUSHR 2048
#define GS_PTX_BITS 10 // mcache.peertx hash slots per node: 2^10 (2^12 when IWANT spammers run)
#define GS_CUTS 64     // IHAVE items above MaxIHaveLength whose cut key one node keeps in LDS per hop
                       // (more spill into the per-rank table Dev::cutSpK / cutSpM)
#define GS_CUTSPILL (1 << 20)  // spilled cut keys per rank per hop
// phase B dynamic LDS: the MaxIHaveLength-cut tables (cut mode): radix
// histogram, per-word cut-bit prefix, item / sender cut keys, cut bits, count
#define GS_CUTLDS (256 * 4 + 128 * 4 + GS_CUTS * 16 + 64 * 16 + 128 * 4 + 16)

// device counter slots (same order as gs_counters)
enum {
  C_HOPS = 0, C_HEARTBEATS, C_PUBLISHED, C_DELIVERIES, C_DUPLICATES, C_TRANSMISSIONS, C_GRAFTS,
  C_PRUNES, C_IHAVE, C_IWANT_SENT, C_IWANT_SERVED, C_PROMISES_BROKEN, C_GRAYLISTED, C_REJECTED,
  C_THROTTLED, C_GATED, C_NCOUNTERS = 16
};
// device error codes (first one wins)
enum {
  E_NONE = 0, E_POOL = 1, E_PROMISES = 2, E_PEERTX = 3, E_LATE = 4, E_TRUNCATE = 5, E_DOUBLE = 6,
  E_FCAP = 7, E_DELTA = 8, E_TRACE = 9, E_STAMP = 10  // (E_STAMP: GS_STAMPS debug builds only)
};

struct TopicP {  // TopicScoreParams (score_params.go:98-148) + scored flag
  double TopicWeight, TimeInMeshWeight;
  int64_t TimeInMeshQuantum;
  double TimeInMeshCap;
  double FmdWeight, FmdDecay, FmdCap;
  double MmdWeight, MmdDecay, MmdCap, MmdThreshold;
  int64_t MmdWindow, MmdActivation;
  double MfpWeight, MfpDecay, ImdWeight, ImdDecay;
  int32_t scored;
  int32_t pad;
  uint64_t qMagic;  // floor(2^64 / TimeInMeshQuantum) for a quantum >= 2, else 0 (quantum_div)
};

// meshTime / TimeInMeshQuantum without a 64-bit divide (include/gs_fp.h)
__device__ __forceinline__ int64_t quantum_div(int64_t mt, const TopicP& tp) {
  return gs_quantum_div(mt, tp.TimeInMeshQuantum, tp.qMagic);
}

// RPC byte accounting (gs_set_rpc_accounting): per topic, the sizes of the
// RPC parts that carry it (include/gs_rpcsize.h)
struct AcctT {
  int32_t msgF;       // RPC.publish entry of a message of the topic
  int32_t graftEnt;   // ControlMessage.graft entry
  int32_t pruneBody;  // ControlPrune body (makePrune: topic + backoff; PX entries add acctPiF each)
  int32_t pruneEnt10; // the same to a gossipsub v1.0 peer (topic only, gossipsub.go:1804-1807)
  int32_t ihaveHead;  // ControlIHave topicID field (the ids add acctIdF each)
};

struct Dev {
  // sizes
  int32_t N, T, Wt, W, St, S, R, HL, HG;
  int64_t E;
  int32_t router, scoring, floodPublish, rsTarget, maxAge;
  // mixed networks (gs_set_routers / gs_set_graph_ex): the router of every host
  // (GS_ROUTER_*, the v1.0 variant folded into gossipsub) and the protocol of
  // every connection (GS_PROTO_*); nullptr: every host runs `router` and every
  // connection its own protocol
  const uint8_t* nrouter;
  const uint8_t* proto;
  // partition (gs_set_partition): this rank owns nodes [n0, n1) and their CSR
  // rows, i.e. edges [e0, e1).  Node kernels run one wave per owned node, edge
  // kernels one lane per owned edge; per-(edge, topic) state is allocated for
  // the owned edges only.  Unpartitioned: n0 = 0, n1 = N, e0 = 0, e1 = E.
  // Per-edge arrays are owned-only too (a base shifted by e0): the sender's
  // state at its own edge e, and the receiver-indexed records (outbox, fwdIn,
  // ibxRec: at the receiver's in-edge ri = rev[e]) with a stage behind the
  // owned range for the records whose receiver lives on another rank (rxi).
  int32_t n0, n1, rank, world;
  int64_t e0, e1, eOwn;
  uint8_t* xmark;   // [E] forwarding set changed since its parity was exchanged (world > 1)
  // RPC byte accounting (gs_set_rpc_accounting); rpcB == nullptr: off
  unsigned long long* rpcB;    // [E] bytes of the RPCs sent over the sender's edge e
  unsigned long long* rpcN;    // [E] RPCs sent over edge e
  const AcctT* acc;            // [T]
  int32_t acctIdF;             // one message id inside an IHAVE / IWANT
  int32_t acctPiF;             // one PX PeerInfo inside a ControlPrune
  // EventTracer of the hosts with traced[u] != 0 (gs_set_trace); nullptr = off
  const uint8_t* traced;
  gs_trace_event* trace;
  unsigned long long* traceN;
  int64_t traceCap;
  int32_t traceRpc;  // gs_set_trace_rpc: RECV_RPC / SEND_RPC blocks of the traced hosts
  const uint8_t* nodeRank;  // [N] owning rank of every node (world > 1)
  uint32_t seed;
  int64_t hop_ns;
  // graph (static)
  const int64_t* rowptr;
  const int32_t* col;
  const int32_t* esrc;
  const int32_t* rev;
  const uint8_t* outbound;
  const uint8_t* direct;
  const uint64_t* sub;      // [N] the node's own subscriptions (p.mySubs)
  const uint64_t* subA;     // [N] its announced subscriptions: what its peers' topic maps hold
  // connection churn (gs_schedule_events); nullptr: every connection up, every
  // peer's score record present and connected
  uint8_t* alive;           // [E] the connection of the edge is up
  uint8_t* rstate;          // [E] peerScore record of the edge's peer: 0 none, 1 connected, 2 retained
  int64_t* rexpire;         // [E] retained record expiry (score.go:634)
  const uint32_t* ipv4;     // [N] (P6 recount)
  const uint8_t* ipWL;      // [N] the node's IP is whitelisted for P6
  int64_t RetainScore;
  int32_t IPThr;
  // score params
  const TopicP* tp;
  const double* app;
  const double* p6;
  double TopicScoreCap, AppW, IPW, BPW, BPThr, BPDecay, DecayToZero;
  double gossipThr, publishThr, graylistThr, oppThr;
  // gossipsub params (gossipsub.go:62-195)
  int32_t D, Dlo, Dhi, Dscore, Dout, Dlazy, GR, OGP, MaxIHaveLength, MaxIHaveMessages;
  double GossipFactor;
  int64_t PruneBackoff, GraftFloodThreshold, IWantFollowupTime, FanoutTTL, PruneRecv;
  uint64_t OGT;
  // per-node state
  uint64_t* seen;
  uint64_t* hist;  // [R][N][W]
  uint64_t* gw;    // [N][W] IHAVE payload of the node's last heartbeat (gossip windows)
  int16_t* age;    // [N][S] first-delivery hop - publish hop   (record / short-window mode)
  uint8_t* ffrom;  // [N][S] first-deliverer neighbour slot, 255 = self (record mode)
  uint32_t* fl[2]; // [N][FC] frontier list of hop h: slots first delivered in hop h
                   // (| in-edge index << 16) and own publishes (| 255 << 16), ascending
  int32_t* fln[2]; // [N] list lengths
  int32_t FC;      // list capacity per node (multiple of 4)
  // floodsub on dense frontiers (k_flood_a; nullptr: the lists above): the
  // messages a node first received or published in hop h as a W-word row, and
  // per edge the copies the sender will not send the receiver next hop
  uint64_t* fb[2]; // [N][W]
  int32_t* fex[2]; // [E]
  int32_t* fbN[2]; // [N] bits in the fb row (0: the row is all zero and is not read)
  uint64_t* own;   // [N][W] the live messages the node authored
  uint32_t stMagic; // ceil(2^32 / St): topic of slot s = umulhi(s, stMagic) (s < 2^16)
  uint64_t tDivM;   // ceil(2^64 / T) (0 when T == 1): edge of pair p = umul64hi(p, tDivM)
  int32_t maxDeg;  // largest node degree (<= 64)
  uint64_t* oldm;  // [W] slots whose message is too old to be first-delivered this hop
  uint64_t* yTab;  // [2][W] phase A: young-slot mask of the amR word of rank k, then its slot prefix | word << 32
  int32_t* nAuth;  // [N] live message slots authored by the node
  int32_t needAge, record;
  uint64_t* sel;   // [N][S] randomsub target mask (randomsub only)
  // ---- adversarial model (gs_publish_ex / gs_set_validation / gs_set_behaviour / gater)
  uint8_t* slotKind;     // [S] GS_MSG_* of the slot's message
  uint64_t topicVal;     // topics with a validator (RegisterTopicValidator)
  int32_t valQueue;      // validation-queue entries per node per hop, 0 = unlimited
  int32_t anyBehave;     // some node has a GS_BEHAVE_* bit
  const uint8_t* behave; // [N] GS_BEHAVE_* bits (nullptr: all honest)
  int64_t* cSpam[2];     // [E] IWANT-spam request list (arena record), -1 = none
  int32_t* pmaskRow;     // [N] row of an IWANT spammer in pmask, -1 = none (nullptr: no spammers)
  uint64_t* pmask;       // [spammers][S] drec.peers: in-edges whose duplicate was counted
  uint8_t* pflag[2];     // IWANT-spam runs: per arena entry, the served verdict of that request
  int32_t* spamRow;      // [E] row of in-edge e in spamCnt when col[e] is an IWANT spammer, else -1
  uint32_t* spamCnt;     // [rows][S / 8] mcache.peertx counts of those requesters, a nibble per slot
  uint8_t* cNSrv[2];     // [E] reply RPCs carrying served messages (0..2)
  // peer gater (peer_gater.go), one per node; stats per (observer, IP) kept on
  // the observer's first edge to a peer of that IP (gGrp = its in-row index)
  int32_t gater;
  double gThreshold, gGlobalDecay, gSourceDecay, gDecayToZero, gDupW, gIgnW, gRejW;
  int64_t gQuiet;
  double* gValidate;     // [N]
  double* gThrottle;     // [N]
  int64_t* gLast;        // [N] lastThrottle, INT64_MIN = never
  double* gSt;           // [4][E] deliver, duplicate, ignore, reject (at group edges)
  uint8_t* gGrp;         // [E] in-row index of the edge holding this peer's IP stats
  // the stats object's lifecycle (peer_gater.go:366-383, 219-259), at group
  // edges: connected peers of the IP, and the expiry set by the last RemovePeer
  int32_t* gConn;        // [E]
  int64_t* gExp;         // [E]
  int64_t gRetain;       // RetainStats
  int64_t* lastpub;        // [N][T], INT64_MIN = none
  uint64_t* fanoutPresent; // [N]
  int32_t nOwnH;      // owned nodes n1 - n0: the mcache ring is [R][nOwnH][W] (v - n0)
  int32_t promCap;   // promise-table entries per node: a multiple of 64 (banks of one wave)
  int64_t* promMid;  // [N][promCap] (owned rows only: the pointer is shifted by n0 rows)
  int64_t* promExp;
  int32_t* promSlot;
  uint8_t* promEdge;
  int32_t* promN;
  // mcache.peertx per node: an open-addressing hash in HBM, 2^ptxBits 32-bit
  // entries slot << 14 | in-edge << 8 | count (0 = empty), linear probing
  uint32_t* ptxT;    // [N][2^ptxBits] (owned rows only: shifted by n0 rows)
  int32_t ptxBits;
  int32_t* ptxN;     // [N] entries in the table
  // the rank's overflow table: a node whose table is full takes further keys
  // here (mcache.peertx is an unbounded map, mcache.go:66-80), 2^ptxOBits
  // 64-bit entries (node + 1) << 32 | peertx entry, linear probing
  unsigned long long* ptxO;
  int32_t ptxOBits;
  unsigned int* ptxOCnt;           // [0] live entries, [1] kept by the heartbeat's rebuild, [2] staged
  unsigned long long* ptxOStage;   // [2^ptxOBits] the rebuild's survivors
  // per-edge state
  uint64_t* mesh;
  uint64_t* fanout;
  uint64_t* fwdRelay[2];
  uint64_t* fwdPub[2];
  // the same sets in the receiver's order: fwdIn[p][rev[e]] = {relay, pub} of
  // edge e, so a receiver reads its in-edges' sets as one coalesced row
  // (maintained by k_fwd on change, k_edge_down and the exchange)
  ulonglong2* fwdIn[2];
  // push: the copies each owned sender sends on each edge to an owned receiver
  // (its frontier list filtered by the edge's forwarding sets, the ReceivedFrom
  // exclusion and randomsub's targets), k_push after the hop's publishes; the
  // receiver's phase A reads its in-edges' segments instead of the senders'
  // whole lists.  A segment is n 16-bit slots at an 8-aligned offset of the
  // sender's GS_PUSHR-slot region; ibxRec[p][rev[e]] = off << 24 | n, -1 =
  // read the list (the sender's copies overflowed its region)
  uint16_t* ibx[2];  // [owned senders][GS_PUSHR]
  int64_t* ibxRec[2];
  int32_t* pushOvf;  // a sender's copies overflowed its region this hop (partitioned: its rank ships its lists)
  uint8_t* jrIn;  // [E] position of the receiver in the sender's row: rev[e] - rowptr[col[e]]
  double* score0;  // hop-start score memo (S0)
  double* score1;  // after the message phase (S1) / heartbeat memo
  uint8_t* sdirty; // [E] a score-lowering change (graft/prune/penalty/refresh) since score0
  int64_t* backoff;  // [T][E], 0 = none
  uint64_t* boMask;  // [E] bit t: backoff of (e, t) is set (the heartbeat's candidate filter
                     // reads one coalesced word per edge instead of a strided expiry per topic)
  double *fmd, *mmd, *mfp, *imd;  // per-(edge, topic) rows (tix)
  int32_t anyImd;                 // 0: no invalid delivery ever recorded, imd is all 0 (P4 = 0)
  uint32_t* dlt;                  // [E][T]: deliveries not yet folded into fmd / mmd,
                                  // (+1s to fmd) | (+1s to mmd) << 16 (see eff_fmd)
  uint16_t* dltN;                 // the narrow layout (exactly one of dlt / dltN is set):
                                  // (+1s to fmd) | (+1s to mmd) << 8, used when at most
                                  // 255 messages per topic can be delivered between two
                                  // folds (slots per topic <= 255, T even; the host folds
                                  // early otherwise, gs_engine.hip foldDue).  Half the
                                  // bytes of phase A's per-hop read-modify-write.
  int64_t *graftTime, *meshTime;  // [T][E]; meshTime holds the value of a pair that left the
                                  // mesh (a mesh pair's is mesh_time_of(): refreshScores
                                  // no longer writes it)
  int64_t lastRefresh;            // time of the last refreshScores, INT64_MIN = none yet
  uint8_t* flags;                 // [T][E] bit0 inMesh, bit1 P3 active
  double* bp;                     // [E] behaviourPenalty
  int32_t *peerhave, *iasked;     // [E]
  // control outbox, double-buffered by hop parity; written by the sender on
  // its own edge, read by the receiver through rev[]
  uint8_t* cPre[2];   // number of control RPCs before the heartbeat RPC (join + reply RPCs)
  uint8_t* cHb[2];    // heartbeat RPC present
  uint64_t* cGraftJoin[2];
  uint64_t* cGraftHb[2];
  uint64_t* cPruneReply[2];
  uint64_t* cPruneHb[2];
  uint64_t* cIhave[2];
  int64_t* cIwant[2];  // IWANT request list: arena record (off << 24 | count), -1 = none
  int64_t* cIresp[2];  // messages served for an IWANT: arena record, -1 = none;
                       // indexed by the receiver's in-edge (rev of the sender's edge)
  int32_t* pool[2];    // slot-id arena for IWANT lists / responses (and PX lists)
  // peer exchange (GS_FLAG_PEER_EXCHANGE, unscored engines): a PRUNE's peer
  // list per (edge, topic) as arena entries topic << 26 | peer node, one record
  // per edge and hop parity; the dial requests of the hop (v << 32 | peer)
  int32_t doPX, PrunePeers;
  int64_t* cPx[2];
  unsigned long long* pxq;
  unsigned long long* pxqN;
  int64_t pxqCap;
  double acceptPX;
  // each rank's arena segment [rank * poolSeg, +poolSeg) is split into poolSub
  // sub-arenas of poolSubCap ids, each with its own bump counter (128 B apart)
  unsigned long long* poolCnt;  // [2][poolSub * 16]
  int64_t poolCap;     // ids per arena
  int64_t poolBase0;   // rank * poolSeg
  int64_t poolSubCap;
  int32_t poolSub;
  int32_t poolS0Mask;  // first sub-arena tried = block % poolSub & mask (0: sub-arena 0 first, tests)
  // MaxIHaveLength item cuts past a node's GS_CUTS in LDS: (key, id) thresholds
  // taken by bump (cutSpN, reset per hop) from GS_CUTSPILL entries per rank
  unsigned long long* cutSpK;
  int64_t* cutSpM;
  unsigned long long* cutSpN;
  // message slots
  int32_t* slotSrc;
  int64_t* slotPubHop;
  int64_t* slotMid;
  uint64_t* pubmask[2];  // slots published in hop h (also the retire mask of hop h)
  const int32_t* mSrc;
  const int32_t* mTopic;
  const int32_t* mSlot;
  const int64_t* mId;
  const uint8_t* mKind;
  // counters / error
  unsigned long long* stamps;  // debug builds only (GS_STAMPS)
  double* pad;                 // [256][64][2] scratch targets of branch-free predicated accesses
  unsigned long long* ctr;
  int32_t* err;
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// ---- mixed networks (gossip_engine.h gs_set_routers / gs_set_graph_ex)
__device__ __forceinline__ int router_of(const Dev& d, int u) { return d.nrouter ? (int)d.nrouter[u] : d.router; }
__device__ __forceinline__ bool gossip_host(const Dev& d, int u) { return router_of(d, u) == GS_ROUTER_GOSSIPSUB; }
// a randomsub host (its per-message target masks live in d.sel)
__device__ __forceinline__ bool rs_host(const Dev& d, int u) {
  return d.sel != nullptr && router_of(d, u) == GS_ROUTER_RANDOMSUB;
}
// gs.feature(GossipSubFeatureMesh / GossipSubFeaturePX, gs.peers[p]) of the
// connection of edge e (gossipsub_feat.go:27-38); symmetric in e
__device__ __forceinline__ bool mesh_peer(const Dev& d, int64_t e) {
  return d.proto == nullptr || d.proto[e] >= GS_PROTO_GOSSIPSUB_V10;
}
__device__ __forceinline__ bool px_peer(const Dev& d, int64_t e) {
  return d.proto == nullptr || d.proto[e] == GS_PROTO_GOSSIPSUB_V11;
}
// makePrune's ControlPrune entry size for the peer of edge e (RPC accounting)
__device__ __forceinline__ int64_t prune_entry(const Dev& d, int64_t e, int t, int npx);
__device__ __forceinline__ bool behaves(const Dev& d, int v, unsigned bit) {
  return d.behave != nullptr && (d.behave[v] & bit) != 0;
}

// ---- trace events (gossip_engine.h gs_trace_event) -----------------------
#define GS_TRACE_COPY 100  // internal: one delivered copy; the host turns every
                           // copy but the delivering one into DUPLICATE_MESSAGE
__device__ __forceinline__ bool is_traced(const Dev& d, int v) { return d.traced != nullptr && d.traced[v] != 0; }
__device__ __forceinline__ bool edge_up(const Dev& d, int64_t e) { return d.alive == nullptr || d.alive[e] != 0; }
// Score(p) of an observer without a record of p is 0 (score.go:246-249)
// mcache.peertx (mcache.go:66-80) of a requester that is an IWANT spammer: a
// nibble per (in-edge, slot) in HBM instead of the node's LDS hash, which would
// need an entry per (message, spammer).  A count only matters while its
// message is cached (GetForPeer), so it is cleared when the slot is recycled
// (k_retire) rather than at mcache.Shift.  handleIWant only compares the count
// with GossipRetransmission (GR), so a nibble is held at GR + 1: one atomic add
// per request returns the count, and an add past GR + 1 is taken back (the
// nibble peaks at GR + 2 < 16, so no carry reaches a neighbour; one request
// list names a slot once and a spammer's two lists are counted one after the
// other, so no two adds race on one nibble).  The host requires GR < 14.
__device__ __forceinline__ uint32_t* spam_word(const Dev& d, int row, int slot) {
  return d.spamCnt + (int64_t)row * (d.S >> 3) + (slot >> 3);
}
__device__ __forceinline__ int spam_incr(const Dev& d, int row, int slot) {
  uint32_t* w = spam_word(d, row, slot);
  const int sh = (slot & 7) * 4;
  const int c = (int)((atomicAdd(w, 1u << sh) >> sh) & 0xF) + 1;
  if (c > d.GR + 1) atomicSub(w, 1u << sh);
  return c;
}
__device__ __forceinline__ int spam_count(const Dev& d, int row, int slot) {
  const uint32_t x = __hip_atomic_load(spam_word(d, row, slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (int)((x >> ((slot & 7) * 4)) & 0xF);
}
// count one or more RPCs of `bytes` in total sent over the sender's edge e
__device__ __forceinline__ void acct_send(const Dev& d, int64_t e, int64_t bytes, int n) {
  d.rpcB[e] += (unsigned long long)bytes;
  d.rpcN[e] += (unsigned long long)n;
}
__device__ __forceinline__ bool has_record(const Dev& d, int64_t e) { return d.rstate == nullptr || d.rstate[e] != 0; }
// the ControlMessage.prune entry of topic t to e's peer carrying npx PX peers
__device__ __forceinline__ int64_t prune_entry(const Dev& d, int64_t e, int t, int npx) {
  return px_peer(d, e) ? gs_pb_field((int64_t)d.acc[t].pruneBody + (int64_t)npx * d.acctPiF) : d.acc[t].pruneEnt10;
}
__device__ __forceinline__ void set_err(const Dev& d, int code);
// n ids of this hop's arena (cur) for one wave or lane; ~0 = full (E_POOL
// set).  The sub-arena is picked by blockIdx: a single counter serialised
// about a million per-wave atomics at one L2 address.  A full sub-arena hands
// the request on to the next ones (its counter stays past the cap, so later
// requests skip it after one add), so skewed loads (high-degree or
// IWANT-heavy nodes on one sub-arena) use the whole segment before E_POOL.
__device__ __forceinline__ unsigned long long pool_take(const Dev& d, int cur, unsigned long long n) {
  const int s0 = (int)(blockIdx.x % (unsigned)d.poolSub) & d.poolS0Mask;
  for (int k = 0; k < d.poolSub; ++k) {
    const int s = (s0 + k) & (d.poolSub - 1);  // poolSub is a power of two
    const unsigned long long o = atomicAdd(&d.poolCnt[((int64_t)cur * d.poolSub + s) * 16], n);
    if ((int64_t)(o + n) <= d.poolSubCap) return (unsigned long long)(d.poolBase0 + (int64_t)s * d.poolSubCap) + o;
  }
  set_err(d, E_POOL);
  return ~0ull;
}
__device__ __forceinline__ void trace_emit(const Dev& d, int64_t hop, int type, int node, int peer, int topic,
                                           int64_t msg, int phase, int reason = 0) {
  const unsigned long long k = atomicAdd(d.traceN, 1ull);
  if ((int64_t)k >= d.traceCap) {
    set_err(d, E_TRACE);
    return;
  }
  gs_trace_event e;
  e.hop = hop;
  e.msg = msg;
  e.type = type;
  e.node = node;
  e.peer = peer;
  e.topic = (int16_t)topic;
  e.phase = (uint8_t)phase;
  e.reason = (uint8_t)reason;
  d.trace[k] = e;
}

// ---- RPC trace events (gs_set_trace_rpc, include/gs_trace.h) -------------
// One RPC sent by `snd` to `rcv` in hop `hop`: a SEND_RPC block for a traced
// sender (its send phase sPhase) and a RECV_RPC block for a traced receiver,
// stamped hop + 1 (the receiver handles it in the next hop; the host holds it
// back until that hop ran, and drops it if the connection closed at its start).
// A block is the RPC event and its nItems items, contiguous in the buffer;
// gen(put) must call put(kind, topic, msg) exactly nItems times.  One lane.
template <class G>
__device__ __forceinline__ void rpc_trace(const Dev& d, int64_t hop, int snd, int rcv, int sPhase, int rPhase, int64_t ord, int nItems,
                          G&& gen) {
  for (int dir = 0; dir < 2; ++dir) {
    const int node = dir ? rcv : snd, peer = dir ? snd : rcv;
    if (!is_traced(d, node)) continue;
    const unsigned long long k = atomicAdd(d.traceN, (unsigned long long)(1 + nItems));
    if ((int64_t)(k + 1 + nItems) > d.traceCap) {
      set_err(d, E_TRACE);
      continue;
    }
    gs_trace_event e;
    e.hop = dir ? hop + 1 : hop;
    e.msg = ord;
    e.type = dir ? GS_TRACE_RECV_RPC : GS_TRACE_SEND_RPC;
    e.node = node;
    e.peer = peer;
    e.topic = -1;
    e.phase = (uint8_t)(dir ? rPhase : sPhase);
    e.reason = 0;
    d.trace[k] = e;
    unsigned long long j = k + 1;
    e.type = GS_TRACE_RPC_ITEM;
    gen([&](int kind, int topic, int64_t msg) {
      if (j > k + (unsigned long long)nItems) return;  // never more than reserved
      e.reason = (uint8_t)kind;
      e.topic = (int16_t)topic;
      e.msg = msg;
      d.trace[j++] = e;
    });
  }
}
__device__ __forceinline__ bool rpc_traced(const Dev& d, int a, int b) {
  return d.traceRpc && (is_traced(d, a) || is_traced(d, b));
}

// Index of (edge e, topic t) in the per-(edge, topic) arrays: one row of T
// topics per edge, so one edge's state is contiguous (a wave with lane =
// topic reads it in full lines) and one node's in-edges are one contiguous
// range [rowptr[v] * T, rowptr[v + 1] * T) of pairs.
__device__ __forceinline__ int64_t tix(const Dev& d, int t, int64_t e) { return e * d.T + t; }
// (edge, topic) of pair index p (exact for p < 2^58)
__device__ __forceinline__ void pair_split(const Dev& d, int64_t p, int64_t& e, int& t) {
  e = d.T == 1 ? p : (int64_t)__umul64hi((unsigned long long)p, (unsigned long long)d.tDivM);
  t = (int)(p - e * d.T);
}

__device__ __forceinline__ void set_err(const Dev& d, int code) { atomicCAS(d.err, 0, code); }
// Event counters are spread over GS_CTR_SPREAD copies (by workgroup) so a
// million waves do not serialise on one L2 line; the host sums the copies.
#define GS_CTR_SPREAD 256
__device__ __forceinline__ void ctr_add(const Dev& d, int k, unsigned long long v) {
  atomicAdd(&d.ctr[(blockIdx.x & (GS_CTR_SPREAD - 1)) * C_NCOUNTERS + k], v);
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  return (uint64_t)__shfl((unsigned long long)v, src);
}
// Value of lane i for a wave-uniform i (v_readlane into a scalar register,
// no LDS permute).
__device__ __forceinline__ int lane_get(int x, int i) { return __builtin_amdgcn_readlane(x, i); }
// The value of lane (lane ^ 32), for the half-wave pairs: v_permlane32_swap
// swaps the halves in a VALU op (a __shfl_xor(x, 32) is a ds_bpermute round
// trip through the LDS unit).  Every lane must be active.
__device__ __forceinline__ uint32_t xor32_u32(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return lane_id() < 32 ? r[1] : r[0];
}
__device__ __forceinline__ uint64_t xor32_u64(uint64_t x) {
  return ((uint64_t)xor32_u32((uint32_t)(x >> 32)) << 32) | (uint64_t)xor32_u32((uint32_t)x);
}
__device__ __forceinline__ double xor32_f64(double x) {
  return __longlong_as_double((long long)xor32_u64((uint64_t)__double_as_longlong(x)));
}
__device__ __forceinline__ uint64_t lane_get64(uint64_t x, int i) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, i);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), i);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double lane_getf(double x, int i) {
  return __longlong_as_double((long long)lane_get64((uint64_t)__double_as_longlong(x), i));
}

__device__ __forceinline__ int wave_sum_int(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// k smallest (key, lane) among candidate lanes: the keyed "shuffle then take
// k" of gs_rng.h.  k <= 0 selects every candidate (getPeers count semantics).
// Radix selection from the key's top bit down, one ballot per bit: the
// candidates whose key has a 0 at the bit are all smaller than those with a
// 1, so either all of them are taken (and the search continues among the
// ones) or the search narrows to them.  Random keys separate n candidates
// after about log2(n) bits; equal keys fall back to the lowest lanes.
__device__ __forceinline__ bool select_k(bool cand, uint64_t key, int k) {
  const int lane = lane_id();
  unsigned long long act = __ballot(cand);
  int n = __popcll(act);
  if (k <= 0 || n <= k) return cand;
  unsigned long long sel = 0;
  int need = k;
  for (int b = 63; b >= 0; --b) {
    const unsigned long long z = __ballot(((act >> lane) & 1) && !((key >> b) & 1));
    const int nz = __popcll(z);
    if (nz <= need) {
      sel |= z;
      need -= nz;
      act &= ~z;
      n -= nz;
    } else {
      act = z;
      n = nz;
    }
    if (need == 0) break;
    if (n == need) {  // every remaining candidate is needed
      sel |= act;
      need = 0;
      break;
    }
  }
  while (need > 0 && act) {  // identical keys: lowest lanes first
    sel |= act & (~act + 1);
    act &= act - 1;
    need--;
  }
  return (sel >> lane) & 1;
}

// select_k per half-wave: each half (lanes 0..31, 32..63) selects its own k
// (a lane-varying value, uniform within the half) of its own candidates; the
// same radix selection and the same "lowest lanes first" tie rule as select_k.
// Works under divergence: a half that is not executing contributes nothing.
// (Keeping both halves' selection state in scalar registers, so that the
// lanes only test their key bit per round, measured slower: the config4
// heartbeat went 22.5 -> 28.3 ms per launch.)
__device__ __forceinline__ bool select_k_half(bool cand, uint64_t key, int k) {
  const int lane = lane_id();
  const int sh = lane & 32, bl = lane & 31;
  uint32_t act = (uint32_t)(__ballot(cand) >> sh);
  int n = __popc(act);
  if (k <= 0 || n <= k) return cand;
  uint32_t sel = 0;
  int need = k;
  for (int b = 63; b >= 0; --b) {
    const uint32_t z = (uint32_t)(__ballot(((act >> bl) & 1) && !((key >> b) & 1)) >> sh);
    const int nz = __popc(z);
    if (nz <= need) {
      sel |= z;
      need -= nz;
      act &= ~z;
      n -= nz;
    } else {
      act = z;
      n = nz;
    }
    if (need == 0) break;
    if (n == need) {
      sel |= act;
      need = 0;
      break;
    }
  }
  while (need > 0 && act) {
    sel |= act & (~act + 1);
    act &= act - 1;
    need--;
  }
  return (sel >> bl) & 1;
}

// "+1, cap" applied n times — markFirstMessageDelivery / markDuplicate-
// MessageDelivery (score.go:915-928, 960-963) one message at a time, since
// (x+1)+1 != x+2 for fractional decayed counters: gs_add_ones_capped
// (include/gs_fp.h) takes one exact add per binade, same result.
__device__ __forceinline__ double add_ones_capped(double x, int n, double cap) {
  return gs_add_ones_capped(x, n, cap);
}

// One topic's contribution topicScore * TopicWeight (score.go:265-311) for
// state index i = t*E + e.  kEager: every load is issued up front (latency-
// bound callers); otherwise meshTime / mmd are read only when P1 / P3 apply
// (the bandwidth-bound streaming pass).
// Phase A records a hop's deliveries per (edge, topic) as counts in dlt and
// leaves fmd / mmd untouched; the counts are folded in (the same "+1, cap"
// steps, score.go:915-928, 960-963) by every reader that needs the exact
// counter and for good at refreshScores, before the decay.  Applying n then m
// steps equals applying n + m steps, so the result is independent of when
// the fold happens as long as it precedes the decay.
// The pending counts of pair i as (+1s to fmd) | (+1s to mmd) << 16 in either
// layout, and their store (a narrow count is <= 255: the host's fold policy
// and phase A's E_DELTA check guarantee it).
// The slot of a receiver-indexed record (outbox, fwdIn, ibxRec) that the
// sender of its own edge e writes for the receiver's in-edge ri = rev[e]: the
// receiver's own slot when this rank owns the receiver, else the stage slot of
// e behind the owned range (the exchange packs and clears it).  Such arrays
// hold [e0, e1 + eOwn) on a partitioned rank; unpartitioned, every ri is owned.
__device__ __forceinline__ int64_t rxi(const Dev& d, int64_t e, int64_t ri) {
  return (ri >= d.e0 && ri < d.e1) ? ri : d.e1 + (e - d.e0);
}
__device__ __forceinline__ uint32_t dlt_get(const Dev& d, int64_t i) {
  if (d.dltN != nullptr) {
    const uint32_t x = d.dltN[i];
    return (x & 0xFFu) | ((x >> 8) << 16);
  }
  return d.dlt[i];
}
__device__ __forceinline__ void dlt_put(const Dev& d, int64_t i, uint32_t q) {
  if (d.dltN != nullptr) d.dltN[i] = (uint16_t)((q & 0xFFu) | ((q >> 16) << 8));
  else d.dlt[i] = q;
}
// the same with the layout known at compile time (the streaming refresh)
template <bool NDLT>
__device__ __forceinline__ uint32_t dlt_get_t(const Dev& d, int64_t i) {
  if constexpr (NDLT) {
    const uint32_t x = d.dltN[i];
    return (x & 0xFFu) | ((x >> 8) << 16);
  } else {
    return d.dlt[i];
  }
}
template <bool NDLT>
__device__ __forceinline__ void dlt_put_t(const Dev& d, int64_t i, uint32_t q) {
  if constexpr (NDLT) d.dltN[i] = (uint16_t)((q & 0xFFu) | ((q >> 16) << 8));
  else d.dlt[i] = q;
}
__device__ __forceinline__ double eff_fmd(const TopicP& tp, double fmd, uint32_t q) {
  return (q & 0xFFFF) ? add_ones_capped(fmd, (int)(q & 0xFFFF), tp.FmdCap) : fmd;
}
__device__ __forceinline__ double eff_mmd(const TopicP& tp, double mmd, uint32_t q) {
  return (q >> 16) ? add_ones_capped(mmd, (int)(q >> 16), tp.MmdCap) : mmd;
}

// One topic's contribution topicScore * TopicWeight (score.go:265-311) of
// pair i, split into its loads (all issued at once) and its arithmetic.
struct TermIn {
  double fmd, mm, mfp, im;
  int64_t mt;
  uint32_t q;
  uint8_t fl;
};
// topicStats.meshTime of a mesh pair: refreshScores sets it to now - graftTime
// (score.go:518-520) and a graft to 0, so between refreshes it is the last
// refresh's now - graftTime, or 0 for a pair grafted since (graftTime is then
// past the last refresh).  A pair out of the mesh keeps what it had when it
// left (stats_prune / RemovePeer store it).
__device__ __forceinline__ int64_t mesh_time_of(int64_t lastRefresh, int64_t gt) {
  return gt <= lastRefresh ? lastRefresh - gt : 0;
}
__device__ __forceinline__ TermIn term_load(const Dev& d, int64_t i) {
  TermIn x;
  x.fl = d.flags[i];
  x.q = dlt_get(d, i);
  x.mt = mesh_time_of(d.lastRefresh, d.graftTime[i]);  // read only for mesh pairs (fl & 1)
  x.mm = d.mmd[i];
  x.fmd = d.fmd[i];
  x.mfp = d.mfp[i];
  x.im = d.anyImd ? d.imd[i] : 0.0;
  return x;
}
__device__ __forceinline__ double term_eval(const TopicP& tp, const TermIn& x) {
  double topicScore = 0.0;
  if (x.fl & 1) {
    double p1 = (double)quantum_div(x.mt, tp);
    if (p1 > tp.TimeInMeshCap) p1 = tp.TimeInMeshCap;
    topicScore += p1 * tp.TimeInMeshWeight;
  }
  topicScore += eff_fmd(tp, x.fmd, x.q) * tp.FmdWeight;
  if (x.fl & 2) {
    const double mm = eff_mmd(tp, x.mm, x.q);
    if (mm < tp.MmdThreshold) {
      const double deficit = tp.MmdThreshold - mm;
      const double p3 = deficit * deficit;
      topicScore += p3 * tp.MmdWeight;
    }
  }
  topicScore += x.mfp * tp.MfpWeight;
  const double p4 = x.im * x.im;
  topicScore += p4 * tp.ImdWeight;
  return topicScore * tp.TopicWeight;
}
__device__ __forceinline__ double topic_term(const Dev& d, const TopicP& tp, int64_t i) {
  return term_eval(tp, term_load(d, i));
}

// The topic-independent tail of score(): cap, P5, P6, P7 (score.go:313-332).
__device__ __forceinline__ double score_tail_v(const Dev& d, double score, double app, double p6, double b) {
  if (d.TopicScoreCap > 0 && score > d.TopicScoreCap) score = d.TopicScoreCap;
  score += app * d.AppW;
  score += p6 * d.IPW;
  if (b > d.BPThr) {
    const double excess = b - d.BPThr;
    const double p7 = excess * excess;
    score += p7 * d.BPW;
  }
  return score;
}
__device__ __forceinline__ double score_tail(const Dev& d, int64_t e, double score) {
  if (d.TopicScoreCap > 0 && score > d.TopicScoreCap) score = d.TopicScoreCap;
  score += d.app[d.col[e]] * d.AppW;
  score += d.p6[e] * d.IPW;
  const double b = d.bp[e];
  if (b > d.BPThr) {
    const double excess = b - d.BPThr;
    const double p7 = excess * excess;
    score += p7 * d.BPW;
  }
  return score;
}

// Score of ONE edge computed by the whole wave (e wave-uniform): lane t loads
// topic t's state, so every load is in flight at once; the terms are then
// added in ascending topic order exactly as edge_score does.  lds: 64 doubles.
__device__ __forceinline__ double edge_score_wave(const Dev& d, int64_t e, double* lds) {
  if (!d.scoring) return 0.0;
  const int lane = lane_id();
  const int tl = lane < d.T ? lane : 0;
  const bool sc = lane < d.T && d.tp[tl].scored;
  const uint64_t scoredT = __ballot(sc);
  // every load of the score at once: the row of the edge and the tail inputs
  const TermIn x = term_load(d, tix(d, tl, e));
  const double app = d.app[d.col[e]], p6 = d.p6[e], b = d.bp[e];
  const double term = sc ? term_eval(d.tp[tl], x) : 0.0;
  __syncthreads();
  lds[lane] = term;
  __syncthreads();
  double score = 0.0;
  for (int t = 0; t < d.T; ++t)
    if ((scoredT >> t) & 1) score += lds[t];
  return has_record(d, e) ? score_tail_v(d, score, app, p6, b) : 0.0;
}

// edge_score_wave for every edge rowBase + j with bit j of `mask` (wave-
// uniform): GS_SBATCH edges per pass with all their loads in flight at once (lane
// = topic), instead of one memory round trip per edge.  Lane j receives its
// edge's score in S; other lanes keep theirs.  lds: 4 * 64 doubles.
__device__ __forceinline__ void edge_scores_batch(const Dev& d, int64_t rowBase, unsigned long long mask, double& S,
                                                  double* lds) {
  const int lane = lane_id();
  const bool mine = (mask >> lane) & 1;
  if (!d.scoring) {
    if (mine) S = 0.0;
    return;
  }
  const int T = d.T;
  const int tl = lane < T ? lane : 0;
  const bool sc = lane < T && d.tp[tl].scored;
  const uint64_t scoredT = __ballot(sc);
  double app = 0.0, p6 = 0.0, b = 0.0;
  bool rec = false;
  if (mine) {  // the tail inputs of the lane's own edge
    const int64_t e = rowBase + lane;
    app = d.app[d.col[e]];
    p6 = d.p6[e];
    b = d.bp[e];
    rec = has_record(d, e);
  }
  while (mask) {
    int js[GS_SBATCH];
#pragma unroll
    for (int k = 0; k < GS_SBATCH; ++k) {
      js[k] = mask ? __ffsll((long long)mask) - 1 : -1;
      mask &= mask ? mask - 1 : 0ull;
    }
    TermIn x[GS_SBATCH];
#pragma unroll
    for (int k = 0; k < GS_SBATCH; ++k) x[k] = term_load(d, tix(d, tl, rowBase + (js[k] < 0 ? js[0] : js[k])));
    __syncthreads();  // the previous pass's sums are done with lds
#pragma unroll
    for (int k = 0; k < GS_SBATCH; ++k) lds[k * 64 + lane] = (js[k] >= 0 && sc) ? term_eval(d.tp[tl], x[k]) : 0.0;
    __syncthreads();
    int kb = -1;
#pragma unroll
    for (int k = 0; k < GS_SBATCH; ++k)
      if (lane == js[k]) kb = k;
    if (kb >= 0) {
      double score = 0.0;
      for (int t = 0; t < T; ++t)
        if ((scoredT >> t) & 1) score += lds[kb * 64 + t];
      S = rec ? score_tail_v(d, score, app, p6, b) : 0.0;
    }
  }
  __syncthreads();
}

// peerScore.Graft — score.go:640-658 (scored topics only)
__device__ __forceinline__ void stats_graft(const Dev& d, int64_t e, int t, int64_t now) {
  if (!d.scoring || !d.tp[t].scored) return;
  const int64_t i = tix(d, t, e);
  d.sdirty[e] = 1;
  d.flags[i] = 1;  // inMesh, P3 inactive
  d.graftTime[i] = now;
  d.meshTime[i] = 0;
}

// peerScore.Prune — score.go:660-682
__device__ __forceinline__ void stats_prune(const Dev& d, int64_t e, int t) {
  if (!d.scoring || !d.tp[t].scored) return;
  const int64_t i = tix(d, t, e);
  d.sdirty[e] = 1;
  const uint8_t fl = d.flags[i];
  const TopicP& tp = d.tp[t];
  const uint32_t q = dlt_get(d, i);
  double mm = d.mmd[i];
  if (q >> 16) {  // fold the pending mesh deliveries: the deficit reads the counter
    mm = eff_mmd(tp, mm, q);
    d.mmd[i] = mm;
    dlt_put(d, i, q & 0xFFFF);
  }
  const double thr = tp.MmdThreshold;
  if ((fl & 2) && mm < thr) {
    const double deficit = thr - mm;
    d.mfp[i] += deficit * deficit;
  }
  if (fl & 1) d.meshTime[i] = mesh_time_of(d.lastRefresh, d.graftTime[i]);  // kept as it was at the prune
  d.flags[i] = fl & ~1;
}

// doAddBackoff — gossipsub.go:844-854 (0 = no entry)
__device__ __forceinline__ void add_backoff(const Dev& d, int64_t e, int t, int64_t now, int64_t interval) {
  const int64_t i = tix(d, t, e);
  const int64_t expire = now + interval;
  const int64_t cur = d.backoff[i];
  if (cur == 0 || cur < expire) d.backoff[i] = expire;
  d.boMask[e] |= 1ull << t;  // the edge's observer only: no other wave writes it
}

// ---- slot-id arena: compact IWANT request / response payloads ----------
// Writes the set bits of a wave-distributed bitset (word w = lane + 64*j) as
// slot ids in ascending slot order (phase A walks them with a cursor);
// returns the packed record (off << 24 | count) or -1 when empty.
// Inclusive prefix sum over the 64 lanes with DPP row shifts and row
// broadcasts (no LDS permutes).  Call with all 64 lanes active.
__device__ __forceinline__ int wave_incl_sum(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}
// Number of set bits of the wave mask m below this lane.
__device__ __forceinline__ int lane_rank(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
// Former LDS rank-loop variant (kept for its call sites): now select_k.
__device__ __forceinline__ bool select_k_lds(bool cand, uint64_t key, int k, uint64_t* skey) {
  (void)skey;  // the radix selection needs no LDS
  return select_k(cand, key, k);
}

// Value of lane 63 (wave-uniform).
__device__ __forceinline__ int wave_last(int x) { return __builtin_amdgcn_readlane(x, 63); }

template <int WPL>
__device__ __forceinline__ int64_t arena_write(const Dev& d, int buf, const uint64_t (&bits)[WPL]) {
  const int lane = lane_id();
  int incl[WPL], tot[WPL];
  int total = 0;
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    const int c = __popcll(bits[j]);
    const int s = wave_incl_sum(c);  // inclusive prefix over lanes of word row j
    incl[j] = s - c;
    tot[j] = wave_last(s);
    total += tot[j];
  }
  if (total == 0) return -1;
  unsigned long long off = 0;
  if (lane == 0) off = pool_take(d, buf, (unsigned long long)total);
  off = lane_get64(off, 0);
  if (off == ~0ull) return -1;
  int rowBase = (int)off;
#pragma unroll
  for (int j = 0; j < WPL; ++j) {
    int pos = rowBase + incl[j];
    uint64_t y = bits[j];
    while (y) {
      const int b = __ffsll((long long)y) - 1;
      y &= y - 1;
      d.pool[buf][pos++] = (lane + 64 * j) * 64 + b;
    }
    rowBase += tot[j];
  }
  return ((int64_t)off << 24) | (int64_t)total;
}

// Expands an arena record into the wave's LDS bitset lds[0..W).
__device__ __forceinline__ void arena_read(const Dev& d, int buf, int64_t rec, unsigned long long* lds) {
  const int lane = lane_id();
  for (int w = lane; w < d.W; w += 64) lds[w] = 0;
  __syncthreads();
  const int64_t off = rec >> 24;
  const int n = (int)(rec & 0xFFFFFF);
  for (int k = lane; k < n; k += 64) {
    const int slot = d.pool[buf][off + k];
    atomicOr(&lds[slot >> 6], 1ull << (slot & 63));
  }
  __syncthreads();
}

// The k-th smallest (key, id) of a candidate set spread over the wave: radix
// select on the 64-bit key (8 passes of 8-bit digits, a 256-bin LDS
// histogram), then the id among equal keys.  `each(fn)` calls fn(key, id) for
// this lane's share of the candidates (re-run every pass); k in [1, count].
// Taking every candidate with (key, id) <= (K, M) takes exactly k of them:
// the keyed "shuffle, then truncate" of gs_rng.h.  Wave-uniform call.
template <class F>
__device__ __forceinline__ void select_kth(F&& each, int k, uint32_t* hist, unsigned long long& K, long long& M) {
  const int lane = lane_id();
  unsigned long long prefix = 0;
  int kk = k;
  for (int pass = 7; pass >= 0; --pass) {
    const int sh = 8 * pass;
    for (int q = lane; q < 256; q += 64) hist[q] = 0u;
    __syncthreads();
    const unsigned long long hiMask = pass == 7 ? 0ull : (~0ull << (sh + 8));
    each([&](unsigned long long key, long long) {
      if ((key & hiMask) == (prefix & hiMask)) atomicAdd(&hist[(key >> sh) & 255], 1u);
    });
    __syncthreads();
    const uint32_t c0 = hist[4 * lane], c1 = hist[4 * lane + 1], c2 = hist[4 * lane + 2], c3 = hist[4 * lane + 3];
    const int sum = (int)(c0 + c1 + c2 + c3);
    const int incl = wave_incl_sum(sum);
    const int excl = incl - sum;
    const bool mine = excl < kk && kk <= incl;
    int digit = 0, below = 0, inBin = 0;
    if (mine) {
      const uint32_t cs[4] = {c0, c1, c2, c3};
      int acc = excl, dd = 0;
      for (; dd < 3; ++dd) {
        if (acc + (int)cs[dd] >= kk) break;
        acc += (int)cs[dd];
      }
      digit = 4 * lane + dd;
      below = acc;
      inBin = (int)cs[dd];
    }
    const unsigned long long m = __ballot(mine);
    __syncthreads();
    if (!m) {  // k above the candidate count: take everything
      K = ~0ull;
      M = INT64_MAX;
      return;
    }
    const int src = __ffsll((long long)m) - 1;
    digit = lane_get(digit, src);
    below = lane_get(below, src);
    inBin = lane_get(inBin, src);
    prefix |= (unsigned long long)digit << sh;
    kk -= below;
    if (inBin == 1) {
      // the k-th candidate is the only one left with this prefix: one more
      // pass reads its whole key and id (usually after 2 of the 8 digits)
      const unsigned long long pm = ~0ull << sh;
      unsigned long long bk = 0;
      long long bi = 0;
      bool found = false;
      each([&](unsigned long long key, long long id) {
        if ((key & pm) == prefix) {
          bk = key;
          bi = id;
          found = true;
        }
      });
      const unsigned long long f = __ballot(found);
      const int fl = __ffsll((long long)f) - 1;
      K = lane_get64(bk, fl);
      M = (long long)lane_get64((uint64_t)bi, fl);
      return;
    }
  }
  K = prefix;
  long long prev = INT64_MIN;  // the kk-th smallest id among the keys equal to K
  for (int q = 0; q < kk; ++q) {
    long long best = INT64_MAX;
    each([&](unsigned long long key, long long id) {
      if (key == prefix && id > prev && id < best) best = id;
    });
    for (int o = 32; o > 0; o >>= 1) {
      const long long y = __shfl_xor(best, o);
      best = y < best ? y : best;
    }
    prev = best;
  }
  M = prev;
}

// select_kth for n candidates with uniformly random keys (Philox outputs:
// emitGossip's and handleIHave's keyed shuffles), in ONE pass of `each` in
// the common case instead of about three.  The k-th smallest key's top byte
// is expected near 256 k / n (its standard deviation is about 256 *
// sqrt(k (n - k) / n^3), ~1.2 bins at config3's 5000 of 6000), so the pass
// counts the keys whose top byte lies below GS_SEL_WIN bins under that
// estimate and keeps every candidate within GS_SEL_WIN bins of it in LDS
// (cand: GS_SEL_CAP (key, id) pairs + a counter; ~117 expected at config3's
// 6000 ids, so about one select in twenty falls back).  If the k-th falls
// among the kept entries and nothing overflowed, it is ranked among them;
// otherwise select_kth runs as before.  Either way the result is the
// exact k-th smallest (key, id).  n = the number of candidates each() yields.
#define GS_SEL_WIN 2
#define GS_SEL_CAP 143
template <class F>
__device__ __forceinline__ void select_kth_est(F&& each, int k, int n, uint32_t* hist, unsigned long long* cand,
                                               unsigned long long& K, long long& M) {
  const int lane = lane_id();
  if (k >= n) {  // every candidate is taken
    K = ~0ull;
    M = INT64_MAX;
    return;
  }
  const int est = (int)((((int64_t)k << 9) / n + 1) >> 1);  // 256 k / n, rounded
  const int lo = max(0, est - GS_SEL_WIN), hi = min(255, est + GS_SEL_WIN);
  uint32_t* const cnt = (uint32_t*)(cand + 2 * GS_SEL_CAP);
  if (lane == 0) *cnt = 0u;
  __syncthreads();
  // no histogram: the keys below bin lo are only counted (a register per
  // lane), the window's are kept
  int nLo = 0;
  each([&](unsigned long long key, long long id) {
    const int top = (int)(key >> 56);
    nLo += top < lo ? 1 : 0;
    if (top >= lo && top <= hi) {
      const uint32_t pos = atomicAdd(cnt, 1u);
      if (pos < GS_SEL_CAP) {
        cand[2 * pos] = key;
        cand[2 * pos + 1] = (unsigned long long)id;
      }
    }
  });
  const int below = wave_sum_int(nLo);
  __syncthreads();
  const int nc = (int)*cnt;
  __syncthreads();
  if (!(below < k && k <= below + nc) || nc > GS_SEL_CAP) {
    select_kth(each, k, hist, K, M);  // the estimate missed: the multi-pass select
    return;
  }
  // the (k - below)-th smallest (key, id) among the kept entries
  const int kk = k - below;
  unsigned long long fk = 0;
  long long fm = 0;
  bool found = false;
  for (int j0 = 0; j0 < nc; j0 += 64) {
    const int j = j0 + lane;
    const unsigned long long key = j < nc ? cand[2 * j] : ~0ull;
    const long long id = j < nc ? (long long)cand[2 * j + 1] : INT64_MAX;
    if (j < nc) {
      int rank = 0;
      for (int q = 0; q < nc; ++q) {
        const unsigned long long qk = cand[2 * q];
        const long long qm = (long long)cand[2 * q + 1];
        rank += (qk < key || (qk == key && qm < id)) ? 1 : 0;
      }
      if (rank == kk - 1) {
        fk = key;
        fm = id;
        found = true;
      }
    }
  }
  const unsigned long long f = __ballot(found);
  const int fl = __ffsll((long long)f) - 1;
  K = lane_get64(fk, fl);
  M = (long long)lane_get64((uint64_t)fm, fl);
  __syncthreads();
}
