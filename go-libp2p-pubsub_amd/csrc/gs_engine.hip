// gs_engine.hip — product C-ABI (include/gossip_engine.h) over HIP kernels
// for gfx950.  Host side: validation, graph preprocessing (reverse edges,
// P6 colocation factors), message-slot assignment, device allocation and the
// per-hop launch schedule (DESIGN.md §4 "Canonical round").  Every kernel runs
// on one HIP stream per engine; gs_step enqueues many hops and synchronises
// once at the end to check the device error word.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <array>
#include "../../include/gs_rpcsize.h"
#include <map>
#include <set>
#include <tuple>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gossip_engine.h"
#include "../../include/gs_trace.h"
#include "../../include/gs_proto.h"
#include "gs_host.h"
#include "gs_kernels.h"
#include "gs_kernels_ctl.h"
#include "gs_exchange.h"

static thread_local std::string g_err;
void gs_set_error(const std::string& msg) { g_err = msg; }

#define HIPCHECK(expr)                                                        \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      gs_set_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
      return GS_EDEVICE;                                                      \
    }                                                                         \
  } while (0)

static const int64_t kSec = 1000000000LL;

struct gs_engine {
  gs_config cfg{};
  gs_gossipsub_params gp{};
  gs_peer_score_params sp{};
  gs_peer_score_thresholds thr{};
  std::vector<gs_topic_score_params> tps;
  std::vector<uint8_t> tscored;
  bool scoring = false, floodPublish = false, record = false;
  int N = 0, T = 0, St = 0, Wt = 0, W = 0, S = 0, R = 0;
  int64_t E = 0;
  int H = 16;  // hops per heartbeat (or a nominal 16 for floodsub/randomsub)
  int64_t retireHops = 0;
  std::vector<int32_t> topicLive;  // per-topic live message count (phase-A counter width)
  int64_t hopsSinceFold = 0, foldEvery = 1;  // pending-delivery fold cadence (dlt)
  int64_t eOwn = 0;                          // owned edges e1 - e0 (Dev::eOwn)
  // the 16-bit pending counts (Dev::dltN): counts accumulate from foldStart;
  // a pair's count is bounded by the messages of its topic that can be
  // delivered since then, so the host folds before that bound could pass 255
  bool narrowDlt = false;
  int64_t foldStart = 0;
  bool narrowFoldDue(int64_t h) {
    auto it = std::lower_bound(mHop.begin(), mHop.end(), foldStart - retireHops);
    std::fill(topicLive.begin(), topicLive.end(), 0);
    for (size_t k = (size_t)(it - mHop.begin()); k < mHop.size() && mHop[k] <= h; ++k)
      if (++topicLive[mTopic[k]] > 255) return true;
    return false;
  }
  std::vector<uint64_t> yWord, yTabH;          // phase A young-slot tables (per hop)
  int64_t refreshedHop = -1;                 // hop of the last refreshScores (S0 exact after it)
  int maxAge = 0;
  // host graph / attributes
  std::vector<int64_t> rowptr;
  std::vector<int32_t> col, rev, esrc;
  std::vector<uint8_t> outbound, direct;
  // mixed networks (gs_set_routers / gs_set_graph_ex): the router of every
  // host and the protocol of every connection (empty: cfg.router's own)
  std::vector<uint8_t> routerH, protoH;
  bool mixed = false;
  int validateMixed();
  int routerOf(int u) const {  // GS_ROUTER_* with the v1.0 variant folded into gossipsub
    const int r = routerH.empty() ? cfg.router : (int)routerH[u];
    return r == GS_ROUTER_GOSSIPSUB_V10 ? GS_ROUTER_GOSSIPSUB : r;
  }
  std::vector<uint64_t> sub;
  std::vector<double> app;
  std::vector<uint32_t> ipv4;
  std::vector<std::pair<uint32_t, uint32_t>> whitelist;
  // connection churn and subscription changes (gs_schedule_events)
  struct Event { int64_t hop; int32_t kind, a, b; };
  std::vector<Event> events;
  size_t nextEv = 0;
  struct Ann { int node, topic; bool sub; };
  std::vector<Ann> pendAnn;            // announcements arriving next hop
  std::vector<uint64_t> subA;          // announced subscriptions (host copy of d.subA)
  std::vector<uint8_t> aliveH;         // [E] host copy of d.alive
  bool churnOn = false;
  // push (k_push + phase A reading per-edge segments) pays where an edge
  // forwards a fraction of its sender's list: several topics.  With one topic
  // a forwarding edge carries the whole list and phase A reads the lists.
  bool pushOn = false;
  // floodsub on dense frontiers (k_flood_a): a single-router floodsub engine
  // with nothing that needs a per-copy record (trace, RPC accounting, churn,
  // dormant slots, validators, attackers) on one rank
  bool denseFlood = false;
  // gossipsub on one topic (config3's shape): phase A pass 1 ORs the senders'
  // frontier bitmaps (k_phase_a DENSE); the lists stay for every other reader
  bool denseGossip = false;
  int frontierMode = 0;                // gs_set_frontier_mode: 0 auto, 1 lists only
  WMask amWPar[2]{};                   // denseGossip: amW of the last hop of each parity
  bool churnWindow = false;            // events scheduled before the first publish: wide window
  uint64_t* dSubA = nullptr;
  uint64_t* dSubOwn = nullptr;
  double* dP6w = nullptr;              // writable view of d.p6 (k_p6)
  int32_t* dEv = nullptr;
  int64_t evCap = 0;
  bool p6Live() const { return scoring && sp.IPColocationFactorWeight != 0 && !ipv4.empty(); }
  int enableChurn();
  int applyEvents(int64_t h);
  int uploadList(const std::vector<int32_t>& v);
  bool graphSet = false, started = false;
  // schedule
  int64_t hop = 0;
  uint64_t ticks = 0;
  int head = 0;
  int64_t heartbeats = 0;
  std::vector<int32_t> mSrc, mTopic, mSlot;
  std::vector<int64_t> mId, mHop;
  std::vector<uint8_t> mKind;          // GS_MSG_* per message
  // adversarial model (gs_set_validation / gs_set_behaviour / WithPeerGater)
  uint64_t topicVal = 0;
  int32_t valQueue = 0;
  std::vector<uint8_t> behaveH;
  std::vector<int32_t> spamRowH;  // host copy of Dev::spamRow
  uint8_t behaveAll = 0;               // OR of every node's bits
  bool anyPhantom = false;             // a published id is advertised only (GS_MSG_PHANTOM)
  bool gaterOn = false;
  gs_peer_gater_params gaterP{};
  bool gaterDecayDue(int64_t t) const { return gaterOn && t > 0 && t % gaterP.DecayInterval == 0; }
  size_t uploaded = 0, msgCap = 0, nextMsg = 0;
  std::vector<int64_t> topicCounter, slotOwnerHop, slotOwnerId;
  // device
  Dev d{};
  std::vector<void*> allocs;
  hipStream_t stream = nullptr;
  TopicP* dTp = nullptr;
  int32_t* dPairs = nullptr;
  int pairCap = 0;
  int32_t* dRetire = nullptr;
  int retireCap = 0;
  double* dScoreTmp = nullptr;
  int32_t *dHopOut = nullptr, *dFromOut = nullptr;
  // partition (gs_set_partition; world == 1: the whole graph)
  int rank = 0, world = 1;
  gs_transport tr{};
  std::vector<int32_t> part;  // [world + 1] node boundaries
  int32_t n0 = 0, n1 = 0;
  int64_t e0 = 0, e1 = 0, poolSeg = 0;
  // exchange buffers (device) and the pinned host staging of the counts
  uint8_t *xSend = nullptr, *xRecv = nullptr, *xSendE = nullptr, *xRecvE = nullptr;
  size_t xSendCap = 0, xRecvCap = 0, xSendECap = 0, xRecvECap = 0;
  unsigned long long* xCnt = nullptr;  // device: [world] record counts, [world] cursors, bump
  int64_t* xOff = nullptr;             // device: [world] record offsets
  unsigned long long* xHost = nullptr; // pinned: world counts, bump, poolCnt, error, push counts [2 world]
  // cross-rank push (gs_exchange.h k_xp_*): send blocks, device counters
  // ([world] records, [world] slots, then the same as cursors), block offsets
  // and record counts ([world] each); a parity's receive area is ibx[k] past
  // the owned senders' regions (ibxOwnSlots), ibxCapB[k] bytes in all
  uint8_t* xSendP = nullptr;
  size_t xSendPCap = 0;
  unsigned long long* xpCnt = nullptr;
  int64_t* xpOff = nullptr;
  int64_t ibxOwnSlots = 0;
  size_t ibxCapB[2] = {0, 0};
  double xMs = 0.0;                    // host wall time spent in exchanges
  int64_t xBytes = 0;                  // bytes received by this rank
  int exchange(int cur, bool hb);
  // trace events (gs_set_trace / gs_trace_read)
  std::vector<uint8_t> traceMask;
  int64_t traceCap = 0;
  // RPC byte accounting (gs_set_rpc_accounting)
  bool acctOn = false;
  std::vector<int32_t> acctMsg, acctTl;
  int32_t acctIdLen = 0;
  int32_t acctPidLen = 38, acctRecLen = 0;  // PX PeerInfo (gs_set_rpc_px_sizes)
  std::vector<int64_t> acctPend;        // (edge, bytes) pairs sent by the host side this hop
  int64_t* dAcctPend = nullptr;
  int64_t acctPendCap = 0;
  int64_t helloBytes(uint64_t subs) const {  // getHelloPacket: one SubOpts per subscribed topic
    int64_t b = 0;
    for (int t = 0; t < T; ++t)
      if ((subs >> t) & 1) b += gs_pb_field(gs_pb_subopts(acctTl[t]));
    return b;
  }
  int flushAcct();
  std::vector<gs_trace_event> tracePending;  // converted, canonical order from traceOut
  // RPC events (gs_set_trace_rpc): RECV blocks of hops not run yet, and the
  // connections closed at the start of a hop (their in-flight RPCs are lost)
  bool traceRpc = false;
  int ptxHomeBits = -1, ptxOvfBits = -1;  // gs_set_peertx_capacity (-1: defaults)
  // peer exchange (GS_FLAG_PEER_EXCHANGE) and connections down at the start
  bool doPX = false;
  std::set<std::pair<int, int>> dormant;       // gs_set_dormant (a < b)
  std::vector<std::pair<int, int>> pxPend;     // dials of the previous hop (connected at this hop's start)
  std::vector<unsigned long long> pxqH;
  int readPx();
  // direct peers (gossipsub.go:492-502, 1594-1616): the (host, direct peer)
  // edges, dialled by the connector when down
  std::vector<std::pair<int, int>> directPairs;
  int64_t directInitHop = 0;
  void directConnect() {
    for (auto& pr : directPairs) {
      const auto bgn = col.begin() + rowptr[pr.first], fin = col.begin() + rowptr[pr.first + 1];
      if (!aliveH.empty() && !aliveH[std::lower_bound(bgn, fin, pr.second) - col.begin()])
        pxPend.push_back({std::min(pr.first, pr.second), std::max(pr.first, pr.second)});
    }
  }
  std::vector<gs_trace_event> traceFuture;
  std::vector<std::array<int64_t, 3>> rpcDowns;  // (hop, receiver, sender)
  // an RPC block recorded on the host: hello packets and announcements
  void hostRpc(int type, int node, int peer, int64_t h, int64_t ord, int topicSub, uint64_t subs, int subFlag) {
    if (!traceRpc || traceMask.empty() || !traceMask[node] || node < n0 || node >= n1) return;
    tracePending.push_back(gs_trace_event{h, ord, type, node, peer, -1, 0, 0});
    for (int t = 0; t < T; ++t)
      if (((subs >> t) & 1) || t == topicSub)
        tracePending.push_back(gs_trace_event{h, t == topicSub ? subFlag : 1, GS_TRACE_RPC_ITEM, node, peer,
                                              (int16_t)t, 0, GS_RPC_ITEM_SUB});
  }
  size_t traceOut = 0;
  int drainTrace();
  int64_t x_poolEnd() const { return (int64_t)(rank + 1) * poolSeg; }
  int growDev(uint8_t*& p, size_t& cap, size_t need, size_t keep = 0);
  // kernel timing: (kernel id, start event, end event) pending until a sync
  bool profiling = false;
  std::vector<hipEvent_t> evPool;
  size_t evUsed = 0;
  std::vector<int> pendKid;
  double kMs[GS_NUM_KERNELS] = {0};
  int64_t kLaunches[GS_NUM_KERNELS] = {0};
  hipEvent_t nextEvent() {
    if (evUsed == evPool.size()) {
      hipEvent_t ev;
      (void)hipEventCreate(&ev);
      evPool.push_back(ev);
    }
    return evPool[evUsed++];
  }
  void resolveTimings() {  // call after a stream sync
    for (size_t i = 0; i < pendKid.size(); ++i) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, evPool[2 * i], evPool[2 * i + 1]) == hipSuccess) kMs[pendKid[i]] += ms;
      kLaunches[pendKid[i]]++;
    }
    pendKid.clear();
    evUsed = 0;
  }

  // Pinned staging ring for the per-hop host-to-device uploads: the copy is
  // asynchronous on the engine stream and the host goes on preparing the next
  // hop; a slot is refilled only after the copy that used it has completed.
  struct Stage {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  static constexpr int kStages = 16;
  Dev* dDev = nullptr;  // device copy of d for the kernels that take it by pointer (k_phase_a / k_phase_b)
  Stage stages[kStages];
  int stageNext = 0;
  // uploads above kStageMax (the full N x 8 subscription rows of an
  // announcement hop: 80 MB at 10M peers) share one pinned buffer instead of
  // growing every ring slot to their size
  static constexpr size_t kStageMax = (size_t)4 << 20;
  Stage bigStage;
  int upload(void* dst, const void* src, size_t bytes) {
    if (!bytes) return GS_OK;
    Stage& st = bytes > kStageMax ? bigStage : stages[stageNext];
    if (&st != &bigStage) stageNext = (stageNext + 1) % kStages;
    if (st.used) HIPCHECK(hipEventSynchronize(st.ev));
    if (st.cap < bytes) {
      if (st.p) HIPCHECK(hipHostFree(st.p));
      st.p = nullptr;
      st.cap = std::max<size_t>(bytes, (size_t)1 << 16);
      HIPCHECK(hipHostMalloc(&st.p, st.cap, hipHostMallocDefault));
    }
    if (!st.ev) HIPCHECK(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
    std::memcpy(st.p, src, bytes);
    HIPCHECK(hipMemcpyAsync(dst, st.p, bytes, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipEventRecord(st.ev, stream));
    st.used = true;
    return GS_OK;
  }

  ~gs_engine() {
    if (stream) (void)hipStreamSynchronize(stream);  // staged uploads in flight
    for (Stage* st : {&bigStage}) {
      if (st->ev) (void)hipEventDestroy(st->ev);
      if (st->p) (void)hipHostFree(st->p);
    }
    for (Stage& st : stages) {
      if (st.ev) (void)hipEventDestroy(st.ev);
      if (st.p) (void)hipHostFree(st.p);
    }
    for (hipEvent_t ev : evPool) (void)hipEventDestroy(ev);
    for (uint8_t* p : {xSend, xRecv, xSendE, xRecvE, xSendP}) if (p) (void)hipFree(p);
    if (xHost) (void)hipHostFree(xHost);
    if (errRing) (void)hipHostFree(errRing);
    for (void* p : allocs) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
  }
  template <class X>
  X* dalloc(size_t n, int fill = 0) {
    void* p = nullptr;
    size_t bytes = std::max<size_t>(n * sizeof(X), 16);
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    allocs.push_back(p);
    (void)hipMemsetAsync(p, fill, bytes, stream);
    return (X*)p;
  }
  // Per-edge device arrays (Dev::rxi): a sender-indexed array holds the owned
  // edges [e0, e1), a receiver-indexed one (outbox, fwdIn, ibxRec) also the
  // stage [e1, e1 + eOwn) on a partitioned rank; both through a base shifted
  // by e0.  Unpartitioned: [0, E), as before.
  template <class X>
  X* ealloc(int fill = 0) {
    X* p = dalloc<X>((size_t)std::max<int64_t>(eOwn, 1), fill);
    return p ? p - e0 : nullptr;
  }
  template <class X>
  X* ralloc(int fill = 0) {
    X* p = dalloc<X>((size_t)std::max<int64_t>(world > 1 ? 2 * eOwn : eOwn, 1), fill);
    return p ? p - e0 : nullptr;
  }
  bool ageWindowNeeded() const {
    for (int t = 0; t < T; ++t)
      if (tscored[t] && tps[t].MeshMessageDeliveriesWindow < retireHops * cfg.hop_ns) return true;
    return false;
  }
  bool heartbeatDue(int64_t t) const {
    if (cfg.router != GS_ROUTER_GOSSIPSUB) return false;
    if (t < gp.HeartbeatInitialDelay) return false;
    return (t - gp.HeartbeatInitialDelay) % gp.HeartbeatInterval == 0;
  }
  bool refreshDue(int64_t t) const { return scoring && t > 0 && t % sp.DecayInterval == 0; }
  // Message-window policy: a message must be first delivered within maxAge
  // hops of its publish (phase A tracks first deliverers for those "young"
  // slots only), and its slot is recycled only after retireHops.  Honest
  // runs deliver everything within a few hops (3 heartbeats is ample); with
  // the adversarial model (validation drops, the gater, spam) messages can
  // arrive much later through gossip, so the window then spans the gossip
  // history twice over.
  void setWindow() {
    // (churn too: a peer that joins or reconnects late catches up through gossip)
    const bool adv = topicVal != 0 || gaterOn || behaveAll != 0 || churnWindow;
    maxAge = (adv ? gp.HistoryLength + gp.HistoryGossip + 3 : 3) * H;
    retireHops = maxAge + (int64_t)(gp.HistoryLength + 2) * H;
    if (cfg.router != GS_ROUTER_GOSSIPSUB) retireHops = maxAge + 2;
  }
  int start();
  int stepOne();
  int uploadMessages();
  int checkDeviceError();
  // Device error flags, copied to pinned memory after every hop so the first
  // failing hop is named; an error is sticky (the state after it is not the
  // reference's), every later gs_step returns it again.
  static constexpr int kErrRing = 64;
  int32_t* errRing = nullptr;
  int stickyRc = GS_OK;
  std::string stickyMsg;
  int drainErrors(int64_t firstHop, int n);
  int deviceErrorCode(int32_t err);
  int deviceErrorText(int32_t err, int64_t atHop);
};

// Contiguous node ranges balanced by edges: rank r owns the nodes whose CSR
// rows start in [E*r/world, E*(r+1)/world).  Identical on every rank.
static std::vector<int32_t> partition_bounds(const std::vector<int64_t>& rowptr, int N, int world) {
  const int64_t E = rowptr[N];
  std::vector<int32_t> part(world + 1, N);
  part[0] = 0;
  for (int r = 1; r < world; ++r)
    part[r] = (int32_t)(std::lower_bound(rowptr.begin(), rowptr.begin() + N, (E * r) / world) - rowptr.begin());
  for (int r = 1; r <= world; ++r) part[r] = std::max(part[r], part[r - 1]);
  return part;
}

static TopicP to_dev(const gs_topic_score_params& p, bool scored) {
  TopicP t{};
  t.TopicWeight = p.TopicWeight;
  t.TimeInMeshWeight = p.TimeInMeshWeight;
  t.TimeInMeshQuantum = p.TimeInMeshQuantum ? p.TimeInMeshQuantum : 1;
  t.TimeInMeshCap = p.TimeInMeshCap;
  t.FmdWeight = p.FirstMessageDeliveriesWeight;
  t.FmdDecay = p.FirstMessageDeliveriesDecay;
  t.FmdCap = p.FirstMessageDeliveriesCap;
  t.MmdWeight = p.MeshMessageDeliveriesWeight;
  t.MmdDecay = p.MeshMessageDeliveriesDecay;
  t.MmdCap = p.MeshMessageDeliveriesCap;
  t.MmdThreshold = p.MeshMessageDeliveriesThreshold;
  t.MmdWindow = p.MeshMessageDeliveriesWindow;
  t.MmdActivation = p.MeshMessageDeliveriesActivation;
  t.MfpWeight = p.MeshFailurePenaltyWeight;
  t.MfpDecay = p.MeshFailurePenaltyDecay;
  t.ImdWeight = p.InvalidMessageDeliveriesWeight;
  t.ImdDecay = p.InvalidMessageDeliveriesDecay;
  t.scored = scored ? 1 : 0;
  // reciprocal of the quantum for quantum_div: floor(2^64 / q), q >= 2
  t.qMagic = gs_quantum_magic(t.TimeInMeshQuantum);
  return t;
}

static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }
// k_score_rows over nEdges edges from d.e0 (lanes hold whole topic rows when
// T divides 64)
template <int MODE>
static void score_rows(const Dev& d, int64_t nEdges, int T, double* out, hipStream_t s) {
  const unsigned g = nblk(nEdges, GS_SCW);
  if (g == 0) return;
  if (64 % T == 0)
    k_score_rows<MODE, true><<<g, 64, 0, s>>>(d, out);
  else
    k_score_rows<MODE, false><<<g, 64, 0, s>>>(d, out);
}

// Launch `stmt` on g's stream; with profiling on, bracket it with HIP events
// recorded on that same stream (so the measured interval is the kernel's).
#define TIMED(g, kid, stmt)                                   \
  do {                                                        \
    if ((g)->profiling) {                                     \
      hipEvent_t _a = (g)->nextEvent(), _b = (g)->nextEvent(); \
      (void)hipEventRecord(_a, (g)->stream);                  \
      stmt;                                                   \
      (void)hipEventRecord(_b, (g)->stream);                  \
      (g)->pendKid.push_back(kid);                            \
    } else {                                                  \
      stmt;                                                   \
    }                                                         \
  } while (0)

// The rules of gs_set_routers / gs_set_graph_ex (gossip_engine.h): protocols
// both hosts speak, equal on both directions; the negotiated one by default.
int gs_engine::validateMixed() {
  auto rt = [&](int u) { return routerH.empty() ? cfg.router : (int)routerH[u]; };
  mixed = !routerH.empty() || !protoH.empty();
  const bool given = !protoH.empty();
  if (!given) protoH.assign((size_t)E, 0);
  auto edgeOf = [&](int a, int b) -> int64_t {
    return (int64_t)(std::lower_bound(col.begin() + rowptr[a], col.begin() + rowptr[a + 1], b) - col.begin());
  };
  for (int u = 0; u < N; ++u) {
    const int ru = rt(u);
    const bool gsHost = ru == GS_ROUTER_GOSSIPSUB || ru == GS_ROUTER_GOSSIPSUB_V10;
    if (gsHost && cfg.router != GS_ROUTER_GOSSIPSUB) {
      gs_set_error("gossipsub hosts need cfg.router == GS_ROUTER_GOSSIPSUB (their params come from the engine)");
      return GS_EINVAL;
    }
    if (!behaveH.empty() && behaveH[u] && !gsHost) { gs_set_error("attacker behaviours need gossipsub hosts"); return GS_EINVAL; }
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
      const int v = col[e], rv = rt(v);
      if (!gsHost && !direct.empty() && direct[e]) { gs_set_error("direct peers need a gossipsub host"); return GS_EINVAL; }
      if (!given) {
        protoH[e] = (uint8_t)gs_negotiate(ru, rv);
        continue;
      }
      const int64_t r = edgeOf(v, u);
      const int pr = protoH[e] == GS_PROTO_DEFAULT ? gs_negotiate(ru, rv) : protoH[e];
      const int pb = protoH[r] == GS_PROTO_DEFAULT ? gs_negotiate(rv, ru) : protoH[r];
      if (pr != pb || !gs_router_speaks(ru, pr) || !gs_router_speaks(rv, pr)) {
        gs_set_error("proto[e] must be a protocol both hosts speak, equal on both directions of the connection");
        return GS_EINVAL;
      }
    }
  }
  if (given)
    for (int u = 0; u < N; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        if (protoH[e] == GS_PROTO_DEFAULT) protoH[e] = (uint8_t)gs_negotiate(rt(u), rt(col[e]));
  return GS_OK;
}

int gs_engine::start() {
  {
    const int rc = validateMixed();
    if (rc) return rc;
  }
  bool anyRandom = cfg.router == GS_ROUTER_RANDOMSUB;  // some host runs randomsub (d.sel)
  pushOn = T >= 4;
  denseFlood = cfg.router == GS_ROUTER_FLOODSUB && !mixed && routerH.empty() && world == 1 && traceMask.empty() &&
               !acctOn && events.empty() && dormant.empty() && topicVal == 0 && behaveAll == 0 &&
               frontierMode != GS_FRONTIER_LISTS;
  // (no P3 window shorter than a message's lifetime: the dense pass counts
  // duplicates per sender, not per copy's age; one rank: the senders' rows)
  denseGossip = cfg.router == GS_ROUTER_GOSSIPSUB && T == 1 && !mixed && routerH.empty() && world == 1 &&
                events.empty() && dormant.empty() && !doPX && topicVal == 0 && behaveAll == 0 && !gaterOn &&
                !(scoring && ageWindowNeeded()) && frontierMode == GS_FRONTIER_BITMAPS;
  if (!routerH.empty()) {
    anyRandom = false;
    for (uint8_t r : routerH) anyRandom = anyRandom || r == GS_ROUTER_RANDOMSUB;
  }
  if (doPX && N >= (1 << 26)) {  // a PX arena entry is topic << 26 | peer (gs_kernels_ctl.h px_append)
    gs_set_error("peer exchange supports fewer than 2^26 peers in this build");
    return GS_EUNSUPPORTED;
  }
  HIPCHECK(hipSetDevice(cfg.device));
  HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  // reverse edges, edge sources, P6
  rev.assign(E, -1);
  esrc.assign(E, 0);
  int maxdeg = 0;
  for (int u = 0; u < N; ++u) {
    maxdeg = std::max<int>(maxdeg, (int)(rowptr[u + 1] - rowptr[u]));
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
      esrc[e] = u;
      const int v = col[e];
      auto b = col.begin() + rowptr[v], en = col.begin() + rowptr[v + 1];
      auto it = std::lower_bound(b, en, u);
      if (it == en || *it != u) {
        gs_set_error("graph must be symmetric");
        return GS_EINVAL;
      }
      rev[e] = (int32_t)(it - col.begin());
    }
  }
  if (maxdeg > 64) {
    gs_set_error("this build supports node degree <= 64 (one wave per node)");
    return GS_EUNSUPPORTED;
  }
  if (E > INT32_MAX) {
    gs_set_error("this build supports < 2^31 edges per engine");
    return GS_EUNSUPPORTED;
  }
  part = partition_bounds(rowptr, N, world);
  n0 = part[rank];
  n1 = part[rank + 1];
  e0 = rowptr[n0];
  e1 = rowptr[n1];
  eOwn = e1 - e0;
  // connections down at the start (gs_set_dormant): no score record, no IP
  std::vector<uint8_t> downH;
  if (!dormant.empty()) {
    downH.assign((size_t)E, 0);
    for (int u = 0; u < N; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        downH[e] = dormant.count({std::min(u, col[e]), std::max(u, col[e])}) ? 1 : 0;
  }
  auto isDown = [&](int64_t e) { return !downH.empty() && downH[e]; };
  std::vector<double> p6(E, 0.0);
  if (scoring && sp.IPColocationFactorWeight != 0 && !ipv4.empty()) {
    // ipColocationFactor (score.go:335-379): peers per IP among the observer's peers
    std::unordered_map<uint32_t, int> cnt;
    for (int u = 0; u < N; ++u) {
      cnt.clear();
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        if (ipv4[col[e]] != 0 && !isDown(e)) cnt[ipv4[col[e]]]++;
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
        const uint32_t ip = ipv4[col[e]];
        if (ip == 0 || isDown(e)) continue;
        bool wl = false;
        for (auto& nm : whitelist)
          if ((ip & nm.second) == (nm.first & nm.second)) { wl = true; break; }
        if (wl) continue;
        const int c = cnt[ip];
        if (c > sp.IPColocationFactorThreshold) {
          const double s = (double)(c - sp.IPColocationFactorThreshold);
          p6[e] = s * s;
        }
      }
    }
  }
  if (app.empty()) app.assign(N, 0.0);
  if (sub.empty()) sub.assign(N, 0);
  if (outbound.empty()) outbound.assign(E, 0);
  if (direct.empty()) direct.assign(E, 0);
  directPairs.clear();
  if (cfg.router == GS_ROUTER_GOSSIPSUB)
    for (int u = 0; u < N; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        if (direct[e]) directPairs.push_back({u, col[e]});
  directInitHop = gp.DirectConnectInitialDelay <= 0 ? 0 : (gp.DirectConnectInitialDelay + cfg.hop_ns - 1) / cfg.hop_ns;

  Dev& x = d;
  dDev = dalloc<Dev>(1);
  if (!dDev) { gs_set_error("device allocation failed (Dev record)"); return GS_ENOMEM; }
  x.N = N; x.T = T; x.Wt = Wt; x.W = W; x.St = St; x.S = S; x.R = R;
  x.HL = gp.HistoryLength; x.HG = gp.HistoryGossip; x.E = E;
  x.router = cfg.router; x.scoring = scoring; x.floodPublish = floodPublish;
  x.nrouter = nullptr;
  x.proto = nullptr;
  x.rsTarget = 6;
  if (anyRandom) {
    const int sq = (int)std::ceil(std::sqrt((double)cfg.randomsub_size));
    x.rsTarget = std::max(6, sq);
  }
  x.maxAge = maxAge; x.seed = cfg.seed; x.hop_ns = cfg.hop_ns;
  x.n0 = n0; x.n1 = n1; x.e0 = e0; x.e1 = e1; x.eOwn = eOwn; x.rank = rank; x.world = world;
  x.TopicScoreCap = sp.TopicScoreCap; x.AppW = sp.AppSpecificWeight; x.IPW = sp.IPColocationFactorWeight;
  x.BPW = sp.BehaviourPenaltyWeight; x.BPThr = sp.BehaviourPenaltyThreshold; x.BPDecay = sp.BehaviourPenaltyDecay;
  x.DecayToZero = sp.DecayToZero;
  x.gossipThr = thr.GossipThreshold; x.publishThr = thr.PublishThreshold; x.graylistThr = thr.GraylistThreshold;
  x.oppThr = thr.OpportunisticGraftThreshold;
  x.D = gp.D; x.Dlo = gp.Dlo; x.Dhi = gp.Dhi; x.Dscore = gp.Dscore; x.Dout = gp.Dout; x.Dlazy = gp.Dlazy;
  x.GR = gp.GossipRetransmission; x.OGP = gp.OpportunisticGraftPeers; x.MaxIHaveLength = gp.MaxIHaveLength;
  x.MaxIHaveMessages = gp.MaxIHaveMessages; x.GossipFactor = gp.GossipFactor;
  x.PruneBackoff = gp.PruneBackoff; x.GraftFloodThreshold = gp.GraftFloodThreshold;
  x.IWantFollowupTime = gp.IWantFollowupTime; x.FanoutTTL = gp.FanoutTTL;
  // the PRUNE we receive carries the sender's PruneBackoff in whole seconds
  // (makePrune gossipsub.go:1809, handlePrune :819-825)
  x.PruneRecv = (gp.PruneBackoff / kSec) > 0 ? (gp.PruneBackoff / kSec) * kSec : gp.PruneBackoff;
  x.OGT = gp.OpportunisticGraftTicks ? gp.OpportunisticGraftTicks : 1;

  const size_t NW = (size_t)N * W, NS = (size_t)N * S;
  // per-(edge, topic) state exists for the owned edges only: rows e*T + t,
  // addressed through a base shifted by e0*T
  const size_t TE = (size_t)T * (size_t)(e1 - e0) + 64;
  const int64_t shift = e0 * T;
  bool ok = true;
  auto chk = [&](const void* p) { if (!p) ok = false; };
  int64_t* dRowptr = dalloc<int64_t>(N + 1); chk(dRowptr);
  int32_t* dCol = dalloc<int32_t>(E); chk(dCol);
  int32_t* dEsrc = dalloc<int32_t>(E); chk(dEsrc);
  int32_t* dRev = dalloc<int32_t>(E); chk(dRev);
  uint8_t* dOut = ealloc<uint8_t>(); chk(dOut);
  uint8_t* dDir = ealloc<uint8_t>(); chk(dDir);
  uint8_t* dJrIn = ealloc<uint8_t>(); chk(dJrIn);
  uint64_t* dSub = dalloc<uint64_t>(N); chk(dSub);
  dSubA = dalloc<uint64_t>(N); chk(dSubA);
  double* dApp = dalloc<double>(N); chk(dApp);
  double* dP6 = ealloc<double>(); chk(dP6);
  dTp = dalloc<TopicP>(T); chk(dTp);
  if (!ok) { gs_set_error("device allocation failed (graph)"); return GS_ENOMEM; }
  HIPCHECK(hipMemcpyAsync(dRowptr, rowptr.data(), (N + 1) * 8, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dCol, col.data(), E * 4, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dEsrc, esrc.data(), E * 4, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dRev, rev.data(), E * 4, hipMemcpyHostToDevice, stream));
  {
    std::vector<uint8_t> jr(E);
    for (int64_t e = 0; e < E; ++e) jr[e] = (uint8_t)(rev[e] - rowptr[col[e]]);
    // on the engine's (non-blocking) stream, after dalloc's memset; the host
    // buffer must outlive the copy
    HIPCHECK(hipMemcpyAsync(dJrIn + e0, jr.data() + e0, (size_t)eOwn, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }
  HIPCHECK(hipMemcpyAsync(dOut + e0, outbound.data() + e0, (size_t)eOwn, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dDir + e0, direct.data() + e0, (size_t)eOwn, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dSub, sub.data(), N * 8, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dSubA, sub.data(), N * 8, hipMemcpyHostToDevice, stream));
  subA = sub;
  dSubOwn = dSub;
  dP6w = dP6;
  HIPCHECK(hipMemcpyAsync(dApp, app.data(), N * 8, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(dP6 + e0, p6.data() + e0, (size_t)eOwn * 8, hipMemcpyHostToDevice, stream));
  std::vector<TopicP> htp(T);
  for (int t = 0; t < T; ++t) htp[t] = to_dev(tps[t], scoring && tscored[t]);
  HIPCHECK(hipMemcpyAsync(dTp, htp.data(), T * sizeof(TopicP), hipMemcpyHostToDevice, stream));
  x.rowptr = dRowptr; x.col = dCol; x.esrc = dEsrc; x.rev = dRev; x.outbound = dOut; x.direct = dDir; x.jrIn = dJrIn;
  x.sub = dSub; x.subA = dSubA; x.app = dApp; x.p6 = dP6; x.tp = dTp;
  x.alive = nullptr; x.rstate = nullptr; x.rexpire = nullptr; x.ipv4 = nullptr; x.ipWL = nullptr;
  x.RetainScore = sp.RetainScore; x.IPThr = sp.IPColocationFactorThreshold;

  // Per-node state only the node's own wave touches (seen, the mcache ring,
  // first-delivery ages / senders, promises, peertx, drec.peers) is allocated
  // for the owned nodes [n0, n1) only: seen / age / ffrom / promises / peertx
  // through a base pointer shifted by n0 rows, the mcache ring [R][nOwn][W]
  // indexed by v - n0 (hist_row).  A partitioned rank holds 1/world of it.
  const int64_t nOwnN = n1 - n0;
  const size_t NWo = (size_t)nOwnN * W, NSo = (size_t)nOwnN * S;
  x.nOwnH = (int32_t)nOwnN;
  x.seen = dalloc<uint64_t>(NWo); chk(x.seen);
  x.hist = dalloc<uint64_t>((size_t)R * NWo); chk(x.hist);
  x.gw = cfg.router == GS_ROUTER_GOSSIPSUB ? dalloc<uint64_t>(NW) : nullptr;
  if (cfg.router == GS_ROUTER_GOSSIPSUB) chk(x.gw);
  // per-slot first-delivery hops only when read back or when the P3 window
  // check can fail: a duplicate always arrives less than retireHops after the
  // message's first delivery, so a MeshMessageDeliveriesWindow of at least
  // that long always credits it (score.go:955)
  x.record = record ? 1 : 0;
  x.needAge = (x.record || (scoring && ageWindowNeeded())) ? 1 : 0;
  x.age = x.needAge ? dalloc<int16_t>(NSo) : nullptr;
  x.ffrom = x.record ? dalloc<uint8_t>(NSo) : nullptr;
  if (x.needAge) chk(x.age);
  if (x.record) chk(x.ffrom);
  if (!ok) { gs_set_error("device allocation failed (per-node state)"); return GS_ENOMEM; }
  x.seen -= (size_t)n0 * W;
  if (x.age) x.age -= (size_t)n0 * S;
  if (x.ffrom) x.ffrom -= (size_t)n0 * S;
  // frontier lists: per node FC entries of 4 bytes (a node's first deliveries
  // of one hop plus its own publishes), at most 8 GiB per parity
  {
    const int64_t budget = 8ll << 30;
    int64_t fc = std::min<int64_t>(S + 64, budget / (4 * (int64_t)N));
    x.FC = (int32_t)std::max<int64_t>(64, fc & ~3ll);
    // the budget gives N * FC <= 2^31 entries, the bound phase A's 32-bit list
    // offsets (sAddr, in entries) rely on; only the 64-entry floor can break
    // it (N > 2^25)
    if ((int64_t)N * x.FC > (1ll << 31)) {
      gs_set_error("too many peers for the frontier lists (N * list capacity must stay <= 2^31)");
      return GS_EUNSUPPORTED;
    }
  }
  const bool denseAny = denseFlood || denseGossip;
  for (int k = 0; k < 2; ++k) {
    x.fl[k] = dalloc<uint32_t>((size_t)N * x.FC); chk(x.fl[k]);
    x.fln[k] = dalloc<int32_t>(N); chk(x.fln[k]);
    x.fb[k] = denseAny ? dalloc<uint64_t>(NW) : nullptr;
    x.fex[k] = denseAny ? dalloc<int32_t>(E) : nullptr;
    x.fbN[k] = denseAny ? dalloc<int32_t>(N) : nullptr;
    if (denseAny) { chk(x.fb[k]); chk(x.fex[k]); chk(x.fbN[k]); }
  }
  x.own = denseAny ? dalloc<uint64_t>(NW) : nullptr;
  if (denseAny) chk(x.own);
  if (!ok) { gs_set_error("device allocation failed (frontiers)"); return GS_ENOMEM; }
  // push arena: a region of GS_PUSHR slots (4 KiB) per owned sender and parity
  for (int k = 0; k < 2; ++k) {
    x.ibx[k] = nullptr;
    x.ibxRec[k] = nullptr;
    if (!pushOn) continue;
    ibxOwnSlots = (int64_t)std::max<int64_t>(nOwnN, 1) * GS_PUSHR;
    x.ibx[k] = dalloc<uint16_t>((size_t)ibxOwnSlots); chk(x.ibx[k]);
    ibxCapB[k] = (size_t)ibxOwnSlots * 2;
    x.ibxRec[k] = ralloc<int64_t>(0xFF); chk(x.ibxRec[k]);
  }
  x.pushOvf = (pushOn && world > 1) ? dalloc<int32_t>(1) : nullptr;
  x.maxDeg = std::max(1, maxdeg);
  x.stMagic = (uint32_t)(((1ull << 32) + (uint64_t)St - 1) / (uint64_t)St);
  x.tDivM = T == 1 ? 0 : ~0ull / (uint64_t)T + 1;  // ceil(2^64 / T)
  foldEvery = std::max<int64_t>(1, 65535 / (2 * (int64_t)St));  // a hop adds at most 2*St per (edge, topic)
  x.oldm = dalloc<uint64_t>(W); chk(x.oldm);
  x.yTab = dalloc<uint64_t>(2 * (size_t)W); chk(x.yTab);
  x.nAuth = dalloc<int32_t>(N); chk(x.nAuth);
  x.sel = anyRandom ? dalloc<uint64_t>(NS) : nullptr;
  if (anyRandom) chk(x.sel);
  if (mixed) {
    // the hosts' routers (v1.0 folded into gossipsub) and the connections' protocols
    uint8_t* nr = dalloc<uint8_t>(N);
    uint8_t* pr = dalloc<uint8_t>(E);
    chk(nr); chk(pr);
    if (ok) {
      std::vector<uint8_t> rh((size_t)N);
      for (int u = 0; u < N; ++u) rh[u] = (uint8_t)routerOf(u);
      HIPCHECK(hipMemcpyAsync(nr, rh.data(), (size_t)N, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipMemcpyAsync(pr, protoH.data(), (size_t)E, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipStreamSynchronize(stream));  // rh is pageable
    }
    x.nrouter = nr;
    x.proto = pr;
  }
  x.lastpub = dalloc<int64_t>((size_t)N * T); chk(x.lastpub);
  x.fanoutPresent = dalloc<uint64_t>(N); chk(x.fanoutPresent);
  // gossipTracer promises (gossip_tracer.go:48-77): at most one per IWANT,
  // i.e. per peer per heartbeat (the IHAVE rides the heartbeat RPC); a
  // promise lives until its message arrives or the first heartbeat after its
  // expiry (applyIwantPenalties), so a node holds at most
  // degree x (ceil(IWantFollowupTime / HeartbeatInterval) + 2) of them.  The
  // table is sized to that bound in banks of 64 (E_PROMISES only guards it).
  {
    int64_t live = 1;
    if (cfg.router == GS_ROUTER_GOSSIPSUB && gp.HeartbeatInterval > 0)
      live = (gp.IWantFollowupTime + gp.HeartbeatInterval - 1) / gp.HeartbeatInterval + 2;
    const int64_t bound = std::max<int64_t>(1, (int64_t)maxdeg * live);
    if (bound > (int64_t)1 << 24) {
      gs_set_error("promise table bound too large (degree x (IWantFollowupTime / HeartbeatInterval + 2) > 2^24)");
      return GS_EUNSUPPORTED;
    }
    x.promCap = (int32_t)(64 * ((bound + 63) / 64));
  }
  const size_t NQ = (size_t)nOwnN * x.promCap;
  x.promMid = dalloc<int64_t>(NQ); x.promExp = dalloc<int64_t>(NQ); x.promSlot = dalloc<int32_t>(NQ);
  x.promEdge = dalloc<uint8_t>(NQ); x.promN = dalloc<int32_t>(nOwnN);
  // mcache.peertx: a hash of 1024 slots per node in HBM.  With IWANT spammers
  // present the honest requests grow too (messages dropped by validation
  // queues come back through gossip; config5 at 1M peers: 43 live entries per
  // node on average, 881 at most), so those runs get 4096; the spammers' own
  // requests, one per (message, spammer), are counted in spamCnt
  // A node whose table fills takes further keys in the rank's overflow table.
  const bool spamRun = (behaveAll & GS_BEHAVE_IWANT_SPAM) != 0;
  x.ptxBits = ptxHomeBits >= 0 ? ptxHomeBits : (spamRun ? 12 : GS_PTX_BITS);
  x.ptxOBits = ptxOvfBits >= 0 ? ptxOvfBits : (spamRun ? 20 : 16);
  x.ptxT = dalloc<uint32_t>((size_t)nOwnN << x.ptxBits); x.ptxN = dalloc<int32_t>(nOwnN);
  x.ptxO = dalloc<unsigned long long>((size_t)1 << x.ptxOBits);
  x.ptxOStage = dalloc<unsigned long long>((size_t)1 << x.ptxOBits);
  x.ptxOCnt = dalloc<unsigned int>(4);
  chk(x.promMid); chk(x.promExp); chk(x.promSlot); chk(x.promEdge); chk(x.promN);
  chk(x.ptxT); chk(x.ptxN); chk(x.ptxO); chk(x.ptxOStage); chk(x.ptxOCnt);
  if (!ok) { gs_set_error("device allocation failed (promises / peertx)"); return GS_ENOMEM; }
  x.promMid -= (size_t)n0 * x.promCap; x.promExp -= (size_t)n0 * x.promCap;
  x.promSlot -= (size_t)n0 * x.promCap; x.promEdge -= (size_t)n0 * x.promCap; x.promN -= n0;
  x.ptxT -= (size_t)n0 << x.ptxBits; x.ptxN -= n0;
  if (gp.GossipRetransmission > 253) {  // a peertx count byte peaks at GossipRetransmission + 2
    gs_set_error("GossipRetransmission > 253 is not supported");
    return GS_EUNSUPPORTED;
  }
  x.mesh = ealloc<uint64_t>(); x.fanout = ealloc<uint64_t>();
  chk(x.mesh); chk(x.fanout);
  for (int k = 0; k < 2; ++k) {
    x.fwdRelay[k] = ealloc<uint64_t>(); x.fwdPub[k] = ealloc<uint64_t>();
    x.fwdIn[k] = ralloc<ulonglong2>();
    chk(x.fwdRelay[k]); chk(x.fwdPub[k]); chk(x.fwdIn[k]);
    x.cPre[k] = ralloc<uint8_t>(); x.cHb[k] = ralloc<uint8_t>();
    x.cGraftJoin[k] = ralloc<uint64_t>(); x.cGraftHb[k] = ralloc<uint64_t>();
    x.cPruneReply[k] = ralloc<uint64_t>(); x.cPruneHb[k] = ralloc<uint64_t>();
    x.cIhave[k] = ralloc<uint64_t>();
    x.cIwant[k] = ralloc<int64_t>(0xFF); x.cIresp[k] = ralloc<int64_t>(0xFF);
    chk(x.cPre[k]); chk(x.cHb[k]); chk(x.cGraftJoin[k]); chk(x.cGraftHb[k]); chk(x.cPruneReply[k]);
    chk(x.cPruneHb[k]); chk(x.cIhave[k]); chk(x.cIwant[k]); chk(x.cIresp[k]);
    x.pubmask[k] = dalloc<uint64_t>(W); chk(x.pubmask[k]);
  }
  x.score0 = ealloc<double>(); x.score1 = ealloc<double>();
  x.sdirty = ealloc<uint8_t>(1); chk(x.sdirty);
  x.backoff = dalloc<int64_t>(TE);
  x.boMask = ealloc<uint64_t>(); chk(x.boMask);
  x.fmd = dalloc<double>(TE); x.mmd = dalloc<double>(TE); x.mfp = dalloc<double>(TE); x.imd = dalloc<double>(TE);
  // 16-bit pending counts when a topic's slots (at most St + 1 messages live at
  // one hop) fit a byte and the pairs of an edge pack into whole words
  narrowDlt = St <= 254 && (T % 2) == 0;
  x.dlt = nullptr;
  x.dltN = nullptr;
  if (narrowDlt) {
    x.dltN = dalloc<uint16_t>(TE); chk(x.dltN);
  } else {
    x.dlt = dalloc<uint32_t>(TE); chk(x.dlt);
  }
  x.graftTime = dalloc<int64_t>(TE); x.meshTime = dalloc<int64_t>(TE); x.flags = dalloc<uint8_t>(TE);
  chk(x.backoff); chk(x.fmd); chk(x.mmd); chk(x.mfp); chk(x.imd); chk(x.graftTime); chk(x.meshTime); chk(x.flags);
  if (!ok) { gs_set_error("device allocation failed (per-(edge, topic) state)"); return GS_ENOMEM; }
  x.backoff -= shift; x.fmd -= shift; x.mmd -= shift; x.mfp -= shift; x.imd -= shift;
  if (narrowDlt) x.dltN -= shift; else x.dlt -= shift;
  x.graftTime -= shift; x.meshTime -= shift; x.flags -= shift;
  x.bp = ealloc<double>(); x.peerhave = ealloc<int32_t>(); x.iasked = ealloc<int32_t>();
  chk(x.score0); chk(x.score1); chk(x.backoff); chk(x.fmd); chk(x.mmd); chk(x.mfp); chk(x.imd);
  chk(x.graftTime); chk(x.meshTime); chk(x.flags); chk(x.bp); chk(x.peerhave); chk(x.iasked);
  // IWANT payload arena (slot ids): 4 ids per owned edge per hop, >= 16M in
  // total; rank r allocates from its own segment [r*seg, (r+1)*seg)
  poolSeg = cfg.router == GS_ROUTER_GOSSIPSUB ? std::max<int64_t>((1 << 24) / world, 4 * (e1 - e0)) : 16;
  poolSeg = (poolSeg + 63) & ~63ll;
  x.poolCap = (int64_t)(rank + 1) * poolSeg;
  // sub-arenas of at least 2^20 ids (one counter each) on an unpartitioned
  // engine; a partitioned one keeps one counter so its used ids stay one
  // prefix of its segment (the exchange ships that prefix)
  {
    int sub = 1;
    while (world == 1 && sub < 256 && (poolSeg / (2 * sub)) >= (1 << 20)) sub *= 2;
    x.poolSub = sub;
    x.poolSubCap = poolSeg / sub;
    x.poolBase0 = (int64_t)rank * poolSeg;
    x.poolS0Mask = -1;
    // tests only: small sub-arenas, every node trying sub-arena 0 first, so
    // allocations fill it and spill into the next ones (tests/test_parity_gpu.py)
    if (const char* dbg = std::getenv("GS_DEBUG_POOL_SUB_CAP"))
      if (world == 1) {
        x.poolSubCap = std::min<int64_t>(x.poolSubCap, std::max<long long>(1, std::atoll(dbg)));
        x.poolS0Mask = 0;
        // never silent: it changes the arena's capacity and allocation order
        std::fprintf(stderr, "gossip engine: GS_DEBUG_POOL_SUB_CAP=%s active (IWANT sub-arenas of %lld ids, "
                     "sub-arena 0 first; a test-only setting)\n", dbg, (long long)x.poolSubCap);
      }
  }
  for (int k = 0; k < 2; ++k) { x.pool[k] = dalloc<int32_t>((size_t)poolSeg * world); chk(x.pool[k]); }
  x.poolCnt = dalloc<unsigned long long>((size_t)2 * x.poolSub * 16); chk(x.poolCnt);
  x.cutSpK = dalloc<unsigned long long>(GS_CUTSPILL); x.cutSpM = dalloc<int64_t>(GS_CUTSPILL);
  x.cutSpN = dalloc<unsigned long long>(1);
  chk(x.cutSpK); chk(x.cutSpM); chk(x.cutSpN);
  x.doPX = doPX ? 1 : 0;
  x.PrunePeers = gp.PrunePeers;
  x.acceptPX = thr.AcceptPXThreshold;
  x.cPx[0] = x.cPx[1] = nullptr;
  x.pxq = x.pxqN = nullptr;
  x.pxqCap = 0;
  if (doPX) {
    for (int k = 0; k < 2; ++k) { x.cPx[k] = ralloc<int64_t>(0xFF); chk(x.cPx[k]); }
    x.pxqCap = std::max<int64_t>(1 << 16, 4 * (int64_t)N);
    x.pxq = dalloc<unsigned long long>((size_t)x.pxqCap); x.pxqN = dalloc<unsigned long long>(1);
    chk(x.pxq); chk(x.pxqN);
  }
  x.slotSrc = dalloc<int32_t>(S, 0xFF); x.slotPubHop = dalloc<int64_t>(S); x.slotMid = dalloc<int64_t>(S, 0xFF);
  chk(x.slotSrc); chk(x.slotPubHop); chk(x.slotMid);
  // adversarial model
  x.slotKind = dalloc<uint8_t>(S); chk(x.slotKind);
  x.topicVal = topicVal;
  x.valQueue = valQueue;
  x.anyImd = topicVal != 0 ? 1 : 0;  // P4 can only come from a validator's rejection
  x.anyBehave = behaveAll != 0;
  x.behave = nullptr;
  x.cSpam[0] = x.cSpam[1] = nullptr;
  x.pmaskRow = nullptr;
  x.pmask = nullptr;
  x.spamRow = nullptr;
  x.spamCnt = nullptr;
  x.pflag[0] = x.pflag[1] = nullptr;
  x.cNSrv[0] = x.cNSrv[1] = nullptr;
  if (behaveAll) {
    uint8_t* b = dalloc<uint8_t>(N); chk(b);
    if (b) HIPCHECK(hipMemcpyAsync(b, behaveH.data(), N, hipMemcpyHostToDevice, stream));
    x.behave = b;
    if (behaveAll & GS_BEHAVE_IWANT_SPAM) {
      for (int k = 0; k < 2; ++k) {
        x.cSpam[k] = ralloc<int64_t>(0xFF); chk(x.cSpam[k]);
        x.cNSrv[k] = ralloc<uint8_t>(); chk(x.cNSrv[k]);
      }
      std::vector<int32_t> row(N, -1);
      int nsp = 0;
      for (int v = n0; v < n1; ++v)  // drec.peers rows of the owned spammers
        if (behaveH[v] & GS_BEHAVE_IWANT_SPAM) row[v] = nsp++;
      x.pmaskRow = dalloc<int32_t>(N); chk(x.pmaskRow);
      x.pmask = dalloc<uint64_t>((size_t)nsp * S); chk(x.pmask);
      if (ok) HIPCHECK(hipMemcpyAsync(x.pmaskRow, row.data(), (size_t)N * 4, hipMemcpyHostToDevice, stream));
      // peertx counts of the owned edges whose peer is an IWANT spammer
      spamRowH.assign((size_t)E, -1);
      int64_t nrow = 0;
      for (int64_t ee = e0; ee < e1; ++ee)
        if (behaveH[col[ee]] & GS_BEHAVE_IWANT_SPAM) spamRowH[ee] = (int32_t)nrow++;
      if (nrow > INT32_MAX) { gs_set_error("too many IWANT-spammer edges"); return GS_ECAPACITY; }
      x.spamRow = ealloc<int32_t>(); chk(x.spamRow);
      for (int k = 0; k < 2; ++k) { x.pflag[k] = dalloc<uint8_t>((size_t)poolSeg * world); chk(x.pflag[k]); }
      if (gp.GossipRetransmission >= 14) {  // spam_incr's nibble peaks at GossipRetransmission + 2
        gs_set_error("IWANT spammers need GossipRetransmission < 14 in this build");
        return GS_EUNSUPPORTED;
      }
      x.spamCnt = dalloc<uint32_t>((size_t)std::max<int64_t>(nrow, 1) * (S / 8)); chk(x.spamCnt);
      if (ok)
        HIPCHECK(hipMemcpyAsync(x.spamRow + e0, spamRowH.data() + e0, (size_t)eOwn * 4, hipMemcpyHostToDevice, stream));
      // `row` is pageable and dies with this block: the copy must have read it
      HIPCHECK(hipStreamSynchronize(stream));
    }
  }
  x.gater = gaterOn ? 1 : 0;
  x.gValidate = x.gThrottle = nullptr;
  x.gLast = nullptr;
  x.gSt = nullptr;
  x.gGrp = nullptr;
  x.gConn = nullptr;
  x.gExp = nullptr;
  x.gRetain = gaterP.RetainStats;
  x.lastRefresh = INT64_MIN;
  if (gaterOn) {
    x.gThreshold = gaterP.Threshold; x.gGlobalDecay = gaterP.GlobalDecay; x.gSourceDecay = gaterP.SourceDecay;
    x.gDecayToZero = gaterP.DecayToZero; x.gDupW = gaterP.DuplicateWeight; x.gIgnW = gaterP.IgnoreWeight;
    x.gRejW = gaterP.RejectWeight; x.gQuiet = gaterP.Quiet;
    x.gValidate = dalloc<double>(N); x.gThrottle = dalloc<double>(N); x.gLast = dalloc<int64_t>(N);
    // gSt: [4][eOwn] through the e0-shifted base, stat k of edge e at k * eOwn + e
    x.gSt = dalloc<double>(4 * (size_t)std::max<int64_t>(eOwn, 1));
    if (x.gSt) x.gSt -= e0;
    x.gGrp = ealloc<uint8_t>();
    x.gConn = ealloc<int32_t>(); x.gExp = ealloc<int64_t>();
    chk(x.gValidate); chk(x.gThrottle); chk(x.gLast); chk(x.gSt); chk(x.gGrp); chk(x.gConn); chk(x.gExp);
    if (ok) {
      // peers of one IP share a stats object (peer_gater.go:262-280); getIP = ipv4, 0 = "<unknown>"
      std::vector<uint8_t> grp(E);
      for (int u = 0; u < N; ++u)
        for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
          const uint32_t ip = ipv4.empty() ? 0u : ipv4[col[e]];
          int64_t f = rowptr[u];
          while ((ipv4.empty() ? 0u : ipv4[col[f]]) != ip) ++f;
          grp[e] = (uint8_t)(f - rowptr[u]);
        }
      std::vector<int64_t> never(N, INT64_MIN);
      // connected peers per stats object (AddPeer of every connection up at the start)
      std::vector<int32_t> conn((size_t)E, 0);
      for (int u = 0; u < N; ++u)
        for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
          if (!isDown(e)) conn[rowptr[u] + grp[e]]++;
      HIPCHECK(hipMemcpyAsync(x.gConn + e0, conn.data() + e0, (size_t)eOwn * 4, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipMemcpyAsync(x.gGrp + e0, grp.data() + e0, (size_t)eOwn, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipMemcpyAsync(x.gLast, never.data(), (size_t)N * 8, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipStreamSynchronize(stream));
    }
  }
#ifdef GS_STAMPS
  x.stamps = dalloc<unsigned long long>((size_t)(N / 1024 + 1) * 24);  // phase A | phase B | heartbeat
#endif
  x.pad = dalloc<double>(256 * 64 * 2); chk(x.pad);
  x.ctr = dalloc<unsigned long long>((size_t)C_NCOUNTERS * GS_CTR_SPREAD); x.err = dalloc<int32_t>(1);
  chk(x.ctr); chk(x.err);
  dScoreTmp = ealloc<double>(); chk(dScoreTmp);
  dHopOut = dalloc<int32_t>(N); dFromOut = dalloc<int32_t>(N); chk(dHopOut); chk(dFromOut);
  x.xmark = nullptr;
  x.nodeRank = nullptr;
  x.traced = nullptr;
  x.trace = nullptr;
  x.traceN = nullptr;
  x.traceCap = 0;
  x.traceRpc = traceRpc && !traceMask.empty();
  if (!traceMask.empty()) {
    uint8_t* tm = dalloc<uint8_t>(N); chk(tm);
    x.trace = dalloc<gs_trace_event>((size_t)traceCap); chk(x.trace);
    x.traceN = dalloc<unsigned long long>(1); chk(x.traceN);
    x.traceCap = traceCap;
    if (ok) {
      HIPCHECK(hipMemcpyAsync(tm, traceMask.data(), N, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipStreamSynchronize(stream));
    }
    x.traced = tm;
    // AddPeer (gossipsub.go:507, floodsub.go:45) and Join (gossipsub.go:1018,
    // floodsub.go:103) of the traced hosts at time 0, recorded on the host
    for (int u = n0; u < n1; ++u) {
      if (!traceMask[u]) continue;
      auto up = [&](int64_t e) { return !dormant.count({std::min(u, col[e]), std::max(u, col[e])}); };
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        if (up(e))  // the connection's protocol in `reason` on a mixed network
          tracePending.push_back(gs_trace_event{0, -1, GS_TRACE_ADD_PEER, u, col[e], -1, 0, mixed ? protoH[e] : (uint8_t)0});
      for (int t = 0; t < T; ++t)
        if ((sub[u] >> t) & 1) tracePending.push_back(gs_trace_event{0, -1, GS_TRACE_JOIN, u, -1, (int16_t)t, 0, 0});
      // the hello packet of every peer (pubsub.go:495; its RecvRPC at time 0)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        if (up(e)) hostRpc(GS_TRACE_RECV_RPC, u, col[e], 0, GS_RPC_ORD(0, GS_RPC_O_HELLO), -1, sub[col[e]], 1);
    }
  }
  if (world > 1) {
    x.xmark = ealloc<uint8_t>(); chk(x.xmark);
    uint8_t* nr = dalloc<uint8_t>(N); chk(nr);
    xCnt = dalloc<unsigned long long>(2 * world + 1); chk(xCnt);
    xOff = dalloc<int64_t>(world); chk(xOff);
    xpCnt = dalloc<unsigned long long>(4 * world); chk(xpCnt);
    xpOff = dalloc<int64_t>(2 * world); chk(xpOff);
    if (ok) {
      std::vector<uint8_t> h(N);
      for (int r = 0; r < world; ++r)
        for (int v = part[r]; v < part[r + 1]; ++v) h[v] = (uint8_t)r;
      HIPCHECK(hipMemcpyAsync(nr, h.data(), N, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipStreamSynchronize(stream));
    }
    x.nodeRank = nr;
    HIPCHECK(hipHostMalloc((void**)&xHost, (size_t)(3 * world + 4) * 8, hipHostMallocDefault));
  }
  if (!ok) {
    gs_set_error("device allocation failed (state); reduce num_nodes or slots_per_topic");
    return GS_ENOMEM;
  }
  {
    std::vector<int64_t> lp((size_t)N * T, INT64_MIN);
    HIPCHECK(hipMemcpyAsync(x.lastpub, lp.data(), lp.size() * 8, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
  }
  if (!events.empty() || doPX || !dormant.empty()) {
    const int rc = enableChurn();
    if (rc) return rc;
  }
  if (!dormant.empty()) {  // gs_set_dormant: these connections start down, without a score record
    std::vector<uint8_t> al((size_t)E, 1);
    for (int64_t e = 0; e < E; ++e)
      if (downH[e]) al[e] = aliveH[e] = 0;
    HIPCHECK(hipMemcpyAsync(d.alive, al.data(), (size_t)E, hipMemcpyHostToDevice, stream));
    if (d.rstate) HIPCHECK(hipMemcpyAsync(d.rstate, al.data(), (size_t)E, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));  // al is pageable
  }
  x.rpcB = x.rpcN = nullptr;
  x.acc = nullptr;
  if (acctOn) {
    // partitioned: every RPC is counted by its sender's rank, on the sender's
    // (owned) edge; gs_read_rpc_bytes returns the owned edges
    x.rpcB = ealloc<unsigned long long>(); x.rpcN = ealloc<unsigned long long>();
    AcctT* ac = dalloc<AcctT>(T);
    chk(x.rpcB); chk(x.rpcN); chk(ac);
    if (!ok) { gs_set_error("device allocation failed (RPC accounting)"); return GS_ENOMEM; }
    const uint64_t bo = (uint64_t)(gp.PruneBackoff / kSec);
    std::vector<AcctT> ah(T);
    for (int t = 0; t < T; ++t) {
      ah[t].msgF = (int32_t)gs_pb_field(acctMsg[t]);
      ah[t].graftEnt = (int32_t)gs_pb_field(gs_pb_graft(acctTl[t]));
      ah[t].pruneBody = (int32_t)gs_pb_prune(acctTl[t], bo);
      ah[t].pruneEnt10 = (int32_t)gs_pb_field(gs_pb_prune_v10(acctTl[t]));
      ah[t].ihaveHead = (int32_t)gs_pb_field(acctTl[t]);
    }
    x.acctIdF = (int32_t)gs_pb_field(acctIdLen);
    x.acctPiF = (int32_t)gs_pb_field(gs_pb_peerinfo(acctPidLen, acctRecLen));
    // the hello packet of every connection present at the start (pubsub.go:495)
    std::vector<unsigned long long> hb((size_t)E), hn((size_t)E, 1ull);
    for (int u = 0; u < N; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
        hb[e] = isDown(e) ? 0ull : (unsigned long long)helloBytes(sub[u]);
        hn[e] = isDown(e) ? 0ull : 1ull;
      }
    HIPCHECK(hipMemcpyAsync(ac, ah.data(), (size_t)T * sizeof(AcctT), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(x.rpcB + e0, hb.data() + e0, (size_t)eOwn * 8, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipMemcpyAsync(x.rpcN + e0, hn.data() + e0, (size_t)eOwn * 8, hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));  // pageable sources
    x.acc = ac;
  }
  started = true;
  return uploadMessages();
}

// host-side RPCs of this hop (hello packets, subscription announcements): one
// (edge, bytes) pair each, added on the device
int gs_engine::flushAcct() {
  if (world > 1) {  // a partitioned rank counts what its own nodes send
    size_t k = 0;
    for (size_t i = 0; i + 1 < acctPend.size(); i += 2)
      if (acctPend[i] >= e0 && acctPend[i] < e1) {
        acctPend[k++] = acctPend[i];
        acctPend[k++] = acctPend[i + 1];
      }
    acctPend.resize(k);
  }
  if (acctPend.empty()) return GS_OK;
  if ((int64_t)acctPend.size() > acctPendCap) {
    int64_t* p = nullptr;
    HIPCHECK(hipMalloc(&p, acctPend.size() * 2 * 8));
    allocs.push_back(p);
    dAcctPend = p;
    acctPendCap = (int64_t)acctPend.size() * 2;
  }
  HIPCHECK(hipMemcpyAsync(dAcctPend, acctPend.data(), acctPend.size() * 8, hipMemcpyHostToDevice, stream));
  const int n = (int)(acctPend.size() / 2);
  k_acct_add<<<nblk(n, 256), 256, 0, stream>>>(d, dAcctPend, n);
  HIPCHECK(hipStreamSynchronize(stream));  // acctPend is pageable
  acctPend.clear();
  return GS_OK;
}

int gs_engine::uploadMessages() {
  if (!started) return GS_OK;
  const size_t n = mSrc.size();
  if (n == uploaded) return GS_OK;
  if (n > msgCap) {
    size_t cap = std::max<size_t>(1024, n * 2);
    int32_t *s = nullptr, *t = nullptr, *sl = nullptr;
    int64_t* id = nullptr;
    uint8_t* kd = nullptr;
    HIPCHECK(hipMalloc(&kd, cap));
    allocs.push_back(kd);
    d.mKind = kd;
    HIPCHECK(hipMalloc(&s, cap * 4));
    HIPCHECK(hipMalloc(&t, cap * 4));
    HIPCHECK(hipMalloc(&sl, cap * 4));
    HIPCHECK(hipMalloc(&id, cap * 8));
    allocs.push_back(s); allocs.push_back(t); allocs.push_back(sl); allocs.push_back(id);
    d.mSrc = s; d.mTopic = t; d.mSlot = sl; d.mId = id;
    msgCap = cap;
    uploaded = 0;
  }
  const size_t k = n - uploaded;
  HIPCHECK(hipMemcpyAsync((void*)(d.mSrc + uploaded), mSrc.data() + uploaded, k * 4, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync((void*)(d.mTopic + uploaded), mTopic.data() + uploaded, k * 4, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync((void*)(d.mSlot + uploaded), mSlot.data() + uploaded, k * 4, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync((void*)(d.mId + uploaded), mId.data() + uploaded, k * 8, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync((void*)(d.mKind + uploaded), mKind.data() + uploaded, k, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipStreamSynchronize(stream));
  uploaded = n;
  return GS_OK;
}

template <class F>
static void launch_wpl(int W, F f) {
  const int wpl = (W + 63) / 64;
  switch (wpl) {
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    default: f(std::integral_constant<int, 4>()); break;
  }
}

// Connection churn state (gs_schedule_events): connection flags, score-record
// states and the P6 inputs, allocated on the first scheduled event.
int gs_engine::enableChurn() {
  if (churnOn) return GS_OK;
  if (denseFlood) {  // (its frontiers carry no per-copy lists to replay a lost connection from)
    gs_set_error("floodsub connection churn must be scheduled before the first step");
    return GS_EUNSUPPORTED;
  }
  auto* al = dalloc<uint8_t>(E);
  auto* rs = scoring ? dalloc<uint8_t>(E) : nullptr;
  auto* rx = scoring ? dalloc<int64_t>(E) : nullptr;
  auto* ip = dalloc<uint32_t>(N);
  auto* wl = dalloc<uint8_t>(N);
  if (!al || (scoring && (!rs || !rx)) || !ip || !wl) { gs_set_error("device allocation failed (churn state)"); return GS_ENOMEM; }
  HIPCHECK(hipMemsetAsync(al, 1, (size_t)E, stream));
  if (rs) HIPCHECK(hipMemsetAsync(rs, 1, (size_t)E, stream));
  std::vector<uint32_t> iph(N, 0);
  std::vector<uint8_t> wlh(N, 0);
  for (int v = 0; v < N; ++v) {
    iph[v] = ipv4.empty() ? 0u : ipv4[v];
    for (auto& nm : whitelist)
      if ((iph[v] & nm.second) == (nm.first & nm.second)) { wlh[v] = 1; break; }
  }
  HIPCHECK(hipMemcpyAsync(ip, iph.data(), (size_t)N * 4, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipMemcpyAsync(wl, wlh.data(), (size_t)N, hipMemcpyHostToDevice, stream));
  HIPCHECK(hipStreamSynchronize(stream));  // iph / wlh are pageable
  d.alive = al; d.rstate = rs; d.rexpire = rx; d.ipv4 = ip; d.ipWL = wl;
  aliveH.assign((size_t)E, 1);
  churnOn = true;
  return GS_OK;
}

// The peer-exchange dial requests of this hop (v << 32 | peer), for the next
// hop's applyEvents.
int gs_engine::readPx() {
  unsigned long long n = 0;
  HIPCHECK(hipMemcpyAsync(&n, d.pxqN, 8, hipMemcpyDeviceToHost, stream));
  HIPCHECK(hipStreamSynchronize(stream));
  n = std::min<unsigned long long>(n, (unsigned long long)d.pxqCap);
  if (n) {
    pxqH.resize(n);
    HIPCHECK(hipMemcpyAsync(pxqH.data(), d.pxq, n * 8, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipMemsetAsync(d.pxqN, 0, 8, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    for (unsigned long long x : pxqH) {
      const int a = (int)(x >> 32), b = (int)(x & 0xFFFFFFFFu);
      pxPend.push_back({std::min(a, b), std::max(a, b)});
    }
  }
  return GS_OK;
}

int gs_engine::uploadList(const std::vector<int32_t>& v) {
  if ((int64_t)v.size() > evCap) {
    int32_t* p = nullptr;
    const int64_t cap = std::max<int64_t>(1024, 2 * (int64_t)v.size());
    HIPCHECK(hipMalloc(&p, (size_t)cap * 4));
    allocs.push_back(p);
    dEv = p;
    evCap = cap;
  }
  return upload(dEv, v.data(), v.size() * 4);
}

// The events of hop h, at its start (the oracle's Sim::applyEvents): the
// announcements of hop h - 1 reach the peers, then every disconnect, connect,
// leave and join of hop h in that order.
int gs_engine::applyEvents(int64_t h) {
  const int64_t now = h * cfg.hop_ns;
  const int cur = (int)(h & 1), prv = cur ^ 1;
  bool subAChanged = false, subChanged = false, recChanged = false;
  for (const Ann& an : pendAnn) {
    if (traceRpc)  // RecvRPC of the announcement at every still-connected peer
      for (int64_t e = rowptr[an.node]; e < rowptr[an.node + 1]; ++e)
        if (aliveH[e])
          hostRpc(GS_TRACE_RECV_RPC, col[e], an.node, h, GS_RPC_ORD(0, GS_RPC_O_ANNOUNCE + an.topic), an.topic, 0,
                  an.sub ? 1 : 0);
    const uint64_t bit = 1ull << an.topic;
    subA[an.node] = an.sub ? (subA[an.node] | bit) : (subA[an.node] & ~bit);
    subAChanged = true;
  }
  pendAnn.clear();
  size_t end = nextEv;
  while (end < events.size() && events[end].hop == h) end++;
  std::vector<int32_t> down, up, leave, join;
  std::map<int, uint64_t> leaveM, joinM;
  auto edgeOf = [&](int a, int b) -> int64_t {
    auto bgn = col.begin() + rowptr[a], fin = col.begin() + rowptr[a + 1];
    auto it = std::lower_bound(bgn, fin, b);
    return (int64_t)(it - col.begin());
  };
  for (int pass = GS_EV_DISCONNECT; pass <= GS_EV_JOIN; ++pass) {
    if (pass == GS_EV_LEAVE && (doPX || !directPairs.empty())) {
      // the connector's dials of the previous hop (peer exchange, direct
      // peers) complete after this hop's scheduled disconnects and connects:
      // each pair once, ascending
      std::sort(pxPend.begin(), pxPend.end());
      pxPend.erase(std::unique(pxPend.begin(), pxPend.end()), pxPend.end());
      for (auto& pr : pxPend) {
        const int64_t ab = edgeOf(pr.first, pr.second), ba = edgeOf(pr.second, pr.first);
        if (aliveH[ab]) continue;
        aliveH[ab] = aliveH[ba] = 1;
        if (world == 1 || (ab >= e0 && ab < e1) || (ba >= e0 && ba < e1)) {
          up.push_back((int32_t)ab);
          up.push_back((int32_t)ba);
        }
        if (acctOn)  // hello packets both ways (pubsub.go:534)
          acctPend.insert(acctPend.end(), {ab, helloBytes(sub[pr.first]), ba, helloBytes(sub[pr.second])});
        if (traceRpc) {
          hostRpc(GS_TRACE_RECV_RPC, pr.first, pr.second, h, GS_RPC_ORD(0, GS_RPC_O_HELLO), -1, sub[pr.second], 1);
          hostRpc(GS_TRACE_RECV_RPC, pr.second, pr.first, h, GS_RPC_ORD(0, GS_RPC_O_HELLO), -1, sub[pr.first], 1);
        }
      }
      pxPend.clear();
    }
    for (size_t k = nextEv; k < end; ++k) {
      const Event& ev = events[k];
      if (ev.kind != pass) continue;
      if (pass <= GS_EV_CONNECT) {
        const int64_t ab = edgeOf(ev.a, ev.b), ba = edgeOf(ev.b, ev.a);
        const uint8_t want = pass == GS_EV_CONNECT ? 1 : 0;
        if (aliveH[ab] == want) continue;
        aliveH[ab] = aliveH[ba] = want;
        auto& lst = pass == GS_EV_CONNECT ? up : down;
        // a partitioned rank launches the pairs with a side it owns (the
        // kernels do only that side)
        if (world == 1 || (ab >= e0 && ab < e1) || (ba >= e0 && ba < e1)) {
          lst.push_back((int32_t)ab);
          lst.push_back((int32_t)ba);
        }
        if (acctOn && want) {  // hello packets both ways (pubsub.go:534)
          acctPend.insert(acctPend.end(), {ab, helloBytes(sub[ev.a]), ba, helloBytes(sub[ev.b])});
        }
        if (traceRpc && want) {  // the hellos' RecvRPC
          hostRpc(GS_TRACE_RECV_RPC, ev.a, ev.b, h, GS_RPC_ORD(0, GS_RPC_O_HELLO), -1, sub[ev.b], 1);
          hostRpc(GS_TRACE_RECV_RPC, ev.b, ev.a, h, GS_RPC_ORD(0, GS_RPC_O_HELLO), -1, sub[ev.a], 1);
        }
        if (traceRpc && !want) {  // RPCs in flight on the connection are lost
          rpcDowns.push_back({h, ev.a, ev.b});
          rpcDowns.push_back({h, ev.b, ev.a});
        }
      } else {
        const uint64_t bit = 1ull << ev.b;
        const bool joinEv = pass == GS_EV_JOIN;
        if (((sub[ev.a] & bit) != 0) == joinEv) continue;
        if (acctOn)  // announce (pubsub.go:775-792) to every connected peer
          for (int64_t e = rowptr[ev.a]; e < rowptr[ev.a + 1]; ++e)
            if (aliveH[e]) acctPend.insert(acctPend.end(), {e, gs_pb_field(gs_pb_subopts(acctTl[ev.b]))});
        if (traceRpc)
          for (int64_t e = rowptr[ev.a]; e < rowptr[ev.a + 1]; ++e)
            if (aliveH[e])
              hostRpc(GS_TRACE_SEND_RPC, ev.a, col[e], h, GS_RPC_ORD(0, GS_RPC_O_ANNOUNCE + ev.b), ev.b, 0,
                      joinEv ? 1 : 0);
        sub[ev.a] = joinEv ? (sub[ev.a] | bit) : (sub[ev.a] & ~bit);
        subChanged = true;
        pendAnn.push_back({ev.a, ev.b, joinEv});
        (joinEv ? joinM : leaveM)[ev.a] |= bit;
      }
    }
  }
  nextEv = end;
  // one item per node: node, topic mask (lo, hi) — its topics run in one wave
  // (a partitioned rank: its own nodes)
  for (auto* pr : {&leaveM, &joinM}) {
    auto& lst = pr == &leaveM ? leave : join;
    for (auto& kv : *pr) {
      if (kv.first < n0 || kv.first >= n1) continue;
      lst.push_back(kv.first);
      lst.push_back((int32_t)(uint32_t)kv.second);
      lst.push_back((int32_t)(uint32_t)(kv.second >> 32));
    }
  }
  if (acctOn) {
    const int rc = flushAcct();
    if (rc) return rc;
  }
  if (subAChanged) {
    const int rc = upload(dSubA, subA.data(), (size_t)N * 8);
    if (rc) return rc;
  }
  if (subChanged) {
    const int rc = upload(dSubOwn, sub.data(), (size_t)N * 8);
    if (rc) return rc;
  }
  if (!down.empty()) {
    int rc = uploadList(down);
    if (rc) return rc;
    k_edge_down<<<(unsigned)down.size(), 64, 0, stream>>>(d, dEv, h, now, prv);
    recChanged = true;
  }
  if (!up.empty()) {
    int rc = uploadList(up);
    if (rc) return rc;
    k_edge_up<<<nblk((int64_t)up.size(), 256), 256, 0, stream>>>(d, dEv, (int)up.size(), h);
    recChanged = true;
  }
  if (recChanged && p6Live() && n1 > n0) k_p6<<<n1 - n0, 64, 0, stream>>>(d, dP6w);
  if (!leave.empty()) {
    int rc = uploadList(leave);
    if (rc) return rc;
    k_leave<<<(unsigned)(leave.size() / 3), 64, 0, stream>>>(d, dEv, h, cur);
  }
  if (!join.empty()) {
    int rc = uploadList(join);
    if (rc) return rc;
    k_join_pairs<<<(unsigned)(join.size() / 3), 64, 0, stream>>>(d, dEv, h, now, cur);
  }
  HIPCHECK(hipGetLastError());
  return GS_OK;
}

int gs_engine::stepOne() {
  const int64_t h = hop;
  const int64_t now = h * cfg.hop_ns;
  const int cur = (int)(h & 1);
  if (churnOn) {
    const int rc = applyEvents(h);
    if (rc) return rc;
    if (h == directInitHop) directConnect();  // after DirectConnectInitialDelay (gossipsub.go:492-502)
  }
  const bool gossip = cfg.router == GS_ROUTER_GOSSIPSUB;
  // this hop's local publishes [b, e)
  size_t b = nextMsg, e = b;
  while (e < mHop.size() && mHop[e] == h) e++;
  nextMsg = e;
  const int n = (int)(e - b);
  // active word windows: amW = words of messages published in [h - maxAge, h]
  // (what this hop's frontier may hold), amR = the previous hop's (what the
  // senders' frontiers hold)
  WMask amR{}, amW{};
  // phase A's young slots (the messages of amR): per amR word (by rank) the
  // slot mask, then the number of young slots in the words before it
  yWord.assign((size_t)W, 0);
  yTabH.assign(2 * (size_t)W, 0);
  int nY = 0;
  {
    auto build = [&](int64_t lo, int64_t hi, WMask& m, bool young) {
      auto it = std::lower_bound(mHop.begin(), mHop.end(), lo);
      for (size_t k = (size_t)(it - mHop.begin()); k < mHop.size() && mHop[k] <= hi; ++k) {
        const int w = mSlot[k] >> 6;
        m.m[w >> 6] |= 1ull << (w & 63);
        if (young) yWord[w] |= 1ull << (mSlot[k] & 63);
      }
    };
    build(h - 1 - maxAge, h - 1, amR, true);
    build(h - maxAge, h, amW, false);
    int rk = 0;
    for (int w = 0; w < W; ++w) {
      if (!((amR.m[w >> 6] >> (w & 63)) & 1)) continue;
      yTabH[rk] = yWord[w];
      yTabH[(size_t)W + rk] = (uint64_t)nY | ((uint64_t)w << 32);  // (the word, for k_phase_a DENSE)
      nY += __builtin_popcountll(yWord[w]);
      ++rk;
    }
    if (rk) {
      const int rc = upload(d.yTab, yTabH.data(), yTabH.size() * 8);
      if (rc) return rc;
    }
  }
  std::vector<int32_t> retireWords;
  WMask amP{};  // words of the slots published this hop (phase A clears their old seen bits)
  for (size_t k = b; k < e; ++k) {
    const int w = mSlot[k] >> 6;
    amP.m[w >> 6] |= 1ull << (w & 63);
    if (std::find(retireWords.begin(), retireWords.end(), w) == retireWords.end()) retireWords.push_back(w);
  }
  HIPCHECK(hipMemsetAsync(d.pubmask[cur], 0, (size_t)W * 8, stream));
  HIPCHECK(hipMemsetAsync(d.poolCnt + (size_t)cur * d.poolSub * 16, 0, (size_t)d.poolSub * 16 * 8, stream));
  const int nOwn = n1 - n0;
  const int64_t eOwn = e1 - e0;
  const unsigned eb = nblk(eOwn, 256);
  const unsigned pb = nblk(eOwn * T, 256);
  if (scoring && narrowDlt && narrowFoldDue(h)) {
    // this hop's counts could take a 16-bit pending word past 255 per field:
    // fold what has accumulated since foldStart first
    if (eOwn) k_fold_all<<<pb, 256, 0, stream>>>(d);
    foldStart = h;
  }
  if (scoring) TIMED(this, GS_K_SCORE, (score_rows<1>(d, eOwn, T, nullptr, stream)));
  if (h == 0 && gossip && nOwn) TIMED(this, GS_K_JOIN, (k_join<<<nOwn, 64, 0, stream>>>(d, h, now, cur)));
  if (gossip && !floodPublish && n > 0) {
    // Publish to a topic we have not joined: fanout (gossipsub.go:977-994)
    std::vector<int32_t> pairs;
    std::vector<uint64_t> seenPair;
    for (size_t i = b; i < e; ++i) {
      const int src = mSrc[i], t = mTopic[i];
      if (src < n0 || src >= n1) continue;  // another rank's publisher
      if (routerOf(src) != GS_ROUTER_GOSSIPSUB) continue;  // floodsub / randomsub hosts keep no fanout
      if ((sub[src] >> t) & 1) continue;
      const uint64_t key = ((uint64_t)src << 6) | (uint64_t)t;
      if (std::find(seenPair.begin(), seenPair.end(), key) != seenPair.end()) continue;
      seenPair.push_back(key);
      pairs.push_back(src);
      pairs.push_back(t);
    }
    if (!pairs.empty()) {
      const int np = (int)pairs.size() / 2;
      if (np > pairCap) {
        int32_t* p = nullptr;
        HIPCHECK(hipMalloc(&p, (size_t)np * 2 * 4 * 2));
        allocs.push_back(p);
        dPairs = p;
        pairCap = np * 2;
      }
      const int rc = upload(dPairs, pairs.data(), pairs.size() * 4);
      if (rc) return rc;
      TIMED(this, GS_K_FANOUT, (k_fanout_pub<<<np, 64, 0, stream>>>(d, dPairs, np, h, now)));
    }
  }
  if (eOwn && !denseFlood) TIMED(this, GS_K_FWD, (k_fwd<<<eb, 256, 0, stream>>>(d, cur)));
  if (n > 0) k_pubmask<<<nblk(n, 256), 256, 0, stream>>>(d, (int)b, n, cur);
  k_oldmask<<<nblk(S, 256), 256, 0, stream>>>(d, h);
  {
    const int nR = __builtin_popcountll(amR.m[0]) + __builtin_popcountll(amR.m[1]) +
                   __builtin_popcountll(amR.m[2]) + __builtin_popcountll(amR.m[3]);
    // 8-bit (sender, topic) counters when no topic has more than 255 live
    // message slots: a sender delivers each message at most once per hop
    // (E_DOUBLE), so it cannot deliver more copies of one topic than that
    bool narrow = true;
    {
      auto it = std::lower_bound(mHop.begin(), mHop.end(), h - retireHops);
      std::fill(topicLive.begin(), topicLive.end(), 0);
      for (size_t k = (size_t)(it - mHop.begin()); k < mHop.size() && mHop[k] <= h; ++k)
        if (++topicLive[mTopic[k]] > 255) { narrow = false; break; }
    }
    if (narrowDlt && !narrow) {  // St <= 254 bounds a topic's live slots by 255: cannot happen
      gs_set_error("internal: 16-bit pending counts without narrow phase-A counters");
      return GS_EDEVICE;
    }
    const size_t nCnt = ((size_t)T * d.maxDeg + 7) & ~(size_t)7;
    const int nYp = (nY + 15) & ~15;
    // the adversarial model (validators, gater, attackers) has its own
    // instantiation: the honest path keeps its LDS budget and code
    const bool adv = topicVal != 0 || gaterOn || behaveAll != 0;
    const bool hasUnc = d.needAge || (adv && d.pmaskRow != nullptr);
    size_t lds = (narrow ? 2 : 4) * nCnt + 16 * (size_t)nR + ((2 * ((size_t)W + nR) + 15) & ~(size_t)15) +
                 (size_t)nYp + (hasUnc ? 4 * nCnt : 0);
    if (adv) lds += 4 * nCnt + 4 * 64 * 4 + 8 * 64 + 8 * (size_t)nR;
    if (nOwn) {
      const int rc = upload(dDev, &d, sizeof(Dev));
      if (rc) return rc;
    }
    // denseGossip: the words v's fb row of this parity is written over (this
    // hop's window, and what the row held two hops ago)
    WMask amF{};
    for (int k = 0; k < GS_MAX_WPL; ++k) amF.m[k] = amR.m[k] | amW.m[k] | amWPar[cur].m[k];
    amWPar[cur] = amW;
    TIMED(this, GS_K_PHASE_A, launch_wpl(W, [&](auto w) {
            if (!nOwn) return;
            constexpr int WV = decltype(w)::value;
            if (denseFlood) {
              k_flood_a<WV><<<nOwn, 64, 0, stream>>>(d, h, cur, amR, amW, amP);
            } else if (adv) {
              if (narrow)
                k_phase_a<WV, true, true><<<nOwn, 64, lds, stream>>>(dDev, h, cur, head, amR, amW, amP, amF, nR, nYp);
              else
                k_phase_a<WV, false, true><<<nOwn, 64, lds, stream>>>(dDev, h, cur, head, amR, amW, amP, amF, nR, nYp);
            } else if (denseGossip) {
              if (narrow)
                k_phase_a<WV, true, false, true><<<nOwn, 64, lds, stream>>>(d, h, cur, head, amR, amW, amP, amF, nR, nYp);
              else
                k_phase_a<WV, false, false, true><<<nOwn, 64, lds, stream>>>(d, h, cur, head, amR, amW, amP, amF, nR, nYp);
            } else if (narrow) {
              k_phase_a<WV, true, false><<<nOwn, 64, lds, stream>>>(d, h, cur, head, amR, amW, amP, amF, nR, nYp);
            } else {
              k_phase_a<WV, false, false><<<nOwn, 64, lds, stream>>>(d, h, cur, head, amR, amW, amP, amF, nR, nYp);
            }
          }));
  }
  if (!retireWords.empty()) {
    if ((int)retireWords.size() > retireCap) {
      int32_t* p = nullptr;
      HIPCHECK(hipMalloc(&p, retireWords.size() * 2 * 4));
      allocs.push_back(p);
      dRetire = p;
      retireCap = (int)retireWords.size() * 2;
    }
    const int rc = upload(dRetire, retireWords.data(), retireWords.size() * 4);
    if (rc) return rc;
    const int nw = (int)retireWords.size();
    if (nOwn && (d.spamRow != nullptr || d.pmaskRow != nullptr))
      k_retire<<<nblk((int64_t)nOwn * nw, 256), 256, 0, stream>>>(d, cur, dRetire, nw);
  }
  if (n > 0) {
    TIMED(this, GS_K_PUBLISH, (k_publish<<<nblk(n, 256), 256, 0, stream>>>(d, (int)b, n, h, cur, head)));
    if (!denseFlood) k_publist<<<nblk(n, 256), 256, 0, stream>>>(d, (int)b, n, cur);
    if (d.sel) k_publish_rs<<<n, 64, 0, stream>>>(d, (int)b);
  }
  // the copies the owned senders send next hop, per edge (phase A reads them)
  if (d.pushOvf) HIPCHECK(hipMemsetAsync(d.pushOvf, 0, 4, stream));
  if (nOwn && pushOn) TIMED(this, GS_K_PUSH, (k_push<<<nOwn, 64, 0, stream>>>(d, cur)));
  if (gossip) {
    if (scoring) TIMED(this, GS_K_SCORE, (score_rows<2>(d, eOwn, T, nullptr, stream)));
    // MaxIHaveLength cuts are possible only if the messages (phantom ids
    // included) that can sit in one gossip window outnumber MaxIHaveLength:
    // published within HistoryGossip + 1 heartbeats plus the delivery age bound
    // Bit 0: one topic's ids may exceed it (emitGossip's cut of a sender's
    // item); bit 1: a sender's ids over all topics may (handleIHave's iask
    // cut of its wants).  Both run in either phase-B instantiation.
    int cutMode = 0;
    {
      const int64_t lo = h - (int64_t)(gp.HistoryGossip + 1) * H - maxAge - 2;
      const auto a = std::lower_bound(mHop.begin(), mHop.end(), lo);
      const auto b2 = std::upper_bound(mHop.begin(), mHop.end(), h);
      if ((int64_t)(b2 - a) > (int64_t)gp.MaxIHaveLength) {
        cutMode |= 2;
        std::vector<int64_t> perT((size_t)T, 0);
        for (auto it = a; it != b2; ++it) perT[(size_t)mTopic[(size_t)(it - mHop.begin())]]++;
        for (int t = 0; t < T; ++t)
          if (perT[(size_t)t] > (int64_t)gp.MaxIHaveLength) cutMode |= 1;
      }
    }
    const size_t ldsB = cutMode ? GS_CUTLDS : 0;
    if (cutMode & 1) HIPCHECK(hipMemsetAsync(d.cutSpN, 0, 8, stream));
    if (nOwn) {
      const int rc = upload(dDev, &d, sizeof(Dev));
      if (rc) return rc;
    }
    TIMED(this, GS_K_PHASE_B,
          launch_wpl(W, [&](auto wpl) {
            constexpr int WV = decltype(wpl)::value;
            if (!nOwn) return;
            if (topicVal != 0 || gaterOn || behaveAll != 0 || anyPhantom)
              k_phase_b<WV, true><<<nOwn, 64, ldsB, stream>>>(dDev, h, now, cur, head, cutMode);
            else
              k_phase_b<WV, false><<<nOwn, 64, ldsB, stream>>>(dDev, h, now, cur, head, cutMode);
          }));
  }
  if (refreshDue(now)) {
    const unsigned rb = nblk(eOwn, GS_RP / T);
    const bool laneT = (64 % T) == 0;  // a lane keeps one topic
    auto refresh = [&](auto churnC, auto laneC, auto ndltC) {
      TIMED(this, GS_K_REFRESH,
            (k_refresh_rows<decltype(churnC)::value, decltype(laneC)::value, decltype(ndltC)::value>
             <<<rb, 64, 0, stream>>>(d, now)));
    };
    using TT = std::true_type;
    using FF = std::false_type;
    if (narrowDlt) {  // (St <= 254 and T even)
      if (churnOn && laneT) refresh(TT{}, TT{}, TT{});
      else if (churnOn) refresh(TT{}, FF{}, TT{});
      else if (laneT) refresh(FF{}, TT{}, TT{});
      else refresh(FF{}, FF{}, TT{});
    } else {
      if (churnOn && laneT) refresh(TT{}, TT{}, FF{});
      else if (churnOn) refresh(TT{}, FF{}, FF{});
      else if (laneT) refresh(FF{}, TT{}, FF{});
      else refresh(FF{}, FF{}, FF{});
    }
    if (churnOn && p6Live() && nOwn) k_p6<<<nOwn, 64, 0, stream>>>(d, dP6w);  // expired records
    refreshedHop = h;
    d.lastRefresh = now;  // the kernels launched from here on derive mesh pairs' meshTime from it
    hopsSinceFold = 0;
    foldStart = h + 1;
  } else if (scoring && !narrowDlt && ++hopsSinceFold >= foldEvery) {
    // pending delivery counts are 16-bit: fold them before they can overflow
    k_fold_all<<<pb, 256, 0, stream>>>(d);
    hopsSinceFold = 0;
  }
  if (gaterDecayDue(now)) {  // peerGater.background ticker (peer_gater.go:204-217)
    const int64_t nth = std::max<int64_t>(nOwn, eOwn);
    if (nth) k_gater_decay<<<nblk(nth, 256), 256, 0, stream>>>(d, now);
  }
  if (heartbeatDue(now)) {
    ticks++;
    if (!directPairs.empty() && ticks % gp.DirectConnectTicks == 0) directConnect();  // gossipsub.go:1318
    // right after a refresh S0 holds exact scores: recompute only what hb_pre
    // dirtied; opportunistic grafting (every OGT ticks) ranks every mesh
    // score, so it gets the full exact pass; otherwise the threshold-exact
    // memo pass (k_score_rows<4>), with the Dhi ranking's mesh members marked
    // by hb_pre so it computes their exact scores too
    const bool exactPass = scoring && (refreshedHop == h || ticks % (uint64_t)d.OGT == 0);
    if (nOwn)
      TIMED(this, GS_K_HB_PRE, (k_hb_pre<<<nOwn, 64, 0, stream>>>(d, now, ticks, scoring && !exactPass ? 1 : 0)));
    int allExact = 1;
    if (scoring && refreshedHop == h)
      TIMED(this, GS_K_SCORE, (score_rows<3>(d, eOwn, T, nullptr, stream)));
    else if (scoring && ticks % (uint64_t)d.OGT == 0)
      TIMED(this, GS_K_SCORE, (score_rows<0>(d, eOwn, T, d.score1, stream)));
    else if (scoring)
      TIMED(this, GS_K_SCORE, (score_rows<4>(d, eOwn, T, nullptr, stream)));
    const int newhead = (head + R - 1) % R;
    // nodes of degree <= 32: two topics per wave (one per half-wave)
    if (nOwn && d.maxDeg <= 32)
      TIMED(this, GS_K_HEARTBEAT,
            (k_heartbeat<true><<<nOwn, 64, 0, stream>>>(d, h, now, ticks, cur, head, newhead, allExact)));
    else if (nOwn)
      TIMED(this, GS_K_HEARTBEAT,
            (k_heartbeat<false><<<nOwn, 64, 0, stream>>>(d, h, now, ticks, cur, head, newhead, allExact)));
    // the peertx counters of the window that left the cache (pre-shift HL - 1)
    if (nOwn && gossip) {
      k_ptx_rebuild<<<nOwn, 64, (size_t)4 << d.ptxBits, stream>>>(d, (head + d.HL - 1) % R);
      const int64_t nO = (int64_t)1 << d.ptxOBits;  // (a table without entries returns at once)
      k_ptxo_collect<<<nblk(nO, 256), 256, 0, stream>>>(d, (head + d.HL - 1) % R);
      k_ptxo_reinsert<<<nblk(nO, 256), 256, 0, stream>>>(d);
      k_ptxo_fin<<<1, 1, 0, stream>>>(d);
    }
    head = newhead;
    heartbeats++;
  }
  // RPC accounting: this hop's forwarded and published messages, one RPC each
  if (acctOn && nOwn) k_acct_payload<<<nOwn, 64, 0, stream>>>(d, cur);
  if (traceRpc && nOwn) k_trace_payload<<<nOwn, 64, 0, stream>>>(d, cur, h);
  if (doPX) {
    const int rc = readPx();
    if (rc) return rc;
  }
  HIPCHECK(hipGetLastError());
  if (world > 1) {
    const int rc = exchange(cur, heartbeatDue(now));
    if (rc) return rc;
  }
  hop++;
  return GS_OK;
}

int gs_engine::checkDeviceError() {
  HIPCHECK(hipStreamSynchronize(stream));
  resolveTimings();
  int32_t err = 0;
  HIPCHECK(hipMemcpy(&err, d.err, 4, hipMemcpyDeviceToHost));
  return deviceErrorText(err, -1);
}

// Waits for the last n hops (first one = firstHop) and reports the first whose
// device error flag is set.
int gs_engine::drainErrors(int64_t firstHop, int n) {
  HIPCHECK(hipStreamSynchronize(stream));
  resolveTimings();
  for (int i = 0; i < n; ++i)
    if (errRing[i]) return deviceErrorText(errRing[i], firstHop + i);
  return GS_OK;
}

int gs_engine::deviceErrorText(int32_t err, int64_t atHop) {
  const int rc = deviceErrorCode(err);
  if (rc != GS_OK && atHop >= 0) {
    g_err = "hop " + std::to_string(atHop) + ": " + g_err;
    stickyRc = rc;
    stickyMsg = g_err;
  }
  return rc;
}

int gs_engine::deviceErrorCode(int32_t err) {
  switch (err) {
    case E_NONE: return GS_OK;
    case E_POOL: gs_set_error("IWANT payload arena overflow (max(2^24 / ranks, 4 x owned edges) ids per rank per hop)"); return GS_ECAPACITY;
    case E_PROMISES:
      gs_set_error("per-node promise table overflow (sized degree x (IWantFollowupTime / HeartbeatInterval + 2) "
                   "entries)");
      return GS_ECAPACITY;
    case E_PEERTX:
      gs_set_error("IWANT retransmission overflow table full (gs_set_peertx_capacity: 2^16 entries per rank "
                   "by default, 2^20 with IWANT spammers)");
      return GS_ECAPACITY;
    case E_LATE:
      gs_set_error("a message was first delivered later than the message window allows; raise slots_per_topic");
      return GS_ECAPACITY;
    case E_TRUNCATE:
      gs_set_error("the MaxIHaveLength cut table overflowed (more than 64 over-length IHAVE items at a node "
                   "spill into 2^20 entries per rank per hop), or a sender cut arose outside cut mode");
      return GS_ECAPACITY;
    case E_FCAP:
      gs_set_error("more first deliveries (plus own publishes) at one node in one hop than its "
                   "frontier list holds (min(slots + 64, 2^31 / num_nodes) entries)");
      return GS_ECAPACITY;
    case E_DELTA:
      gs_set_error("pending delivery count of one (edge, topic) overflowed 65535 (255 in the 16-bit layout) "
                   "between two folds");
      return GS_ECAPACITY;
    case E_TRACE:
      gs_set_error("more trace events between two gs_trace_read calls than the capacity given to gs_set_trace");
      return GS_ECAPACITY;
    case E_DOUBLE:
      gs_set_error("a peer sent the same message twice in one hop (outside the canonical model)");
      return GS_EUNSUPPORTED;
    case E_STAMP:
      gs_set_error("debug cycle stamp index outside its buffer (GS_STAMPS build)");
      return GS_EDEVICE;
    default: gs_set_error("unknown device error"); return GS_EDEVICE;
  }
}

// Grows a device buffer to `need` bytes, keeping its first `keep` bytes.
int gs_engine::growDev(uint8_t*& p, size_t& cap, size_t need, size_t keep) {
  if (need <= cap) return GS_OK;
  uint8_t* q = nullptr;
  const size_t ncap = std::max<size_t>(need + need / 4, 1 << 20);
  if (hipMalloc(&q, ncap) != hipSuccess) {
    gs_set_error("device allocation failed (exchange buffer)");
    return GS_ENOMEM;
  }
  if (p && keep) HIPCHECK(hipMemcpyAsync(q, p, std::min(keep, cap), hipMemcpyDeviceToDevice, stream));
  if (p) {
    HIPCHECK(hipStreamSynchronize(stream));
    HIPCHECK(hipFree(p));
  }
  p = q;
  cap = ncap;
  return GS_OK;
}

static inline size_t align8(size_t x) { return (x + 7) & ~(size_t)7; }

// End-of-hop exchange of a partitioned engine (gs_exchange.h): pack what this
// rank's nodes sent in hop h, hand it to the host transport, unpack what the
// other ranks' nodes sent to ours.
int gs_engine::exchange(int cur, bool hb) {
  const int nOwn = n1 - n0;
  const int64_t eOwn = e1 - e0;
  const size_t hdrBytes = align8((size_t)nOwn * 8);
  unsigned long long* cnt = xCnt;             // [world]
  unsigned long long* cursor = xCnt + world;  // [world]
  unsigned long long* bump = xCnt + 2 * world;
  // 1. counts + lists (into a buffer that usually suffices; re-packed if not)
  HIPCHECK(hipMemsetAsync(xCnt, 0, (size_t)(2 * world + 1) * 8, stream));
  if (eOwn) k_x_count<<<nblk(eOwn, 256), 256, 0, stream>>>(d, cur, cnt);
  const bool xpush = d.ibxRec[0] != nullptr;  // k_push ran: cross-rank edges' segments travel too
  if (xpush) {
    HIPCHECK(hipMemsetAsync(xpCnt, 0, (size_t)4 * world * 8, stream));
    if (eOwn) k_xp_count<<<nblk(eOwn, 256), 256, 0, stream>>>(d, cur, xpCnt);
    HIPCHECK(hipMemcpyAsync(xHost + world + 3, xpCnt, (size_t)2 * world * 8, hipMemcpyDeviceToHost, stream));
  }
  if (xSendCap < hdrBytes + (16u << 20)) {
    int rc = growDev(xSend, xSendCap, hdrBytes + (16u << 20));
    if (rc) return rc;
  }
  // A receiver reads this rank's frontier lists only where it walks them:
  // without push (T < 4), for an IWANT spammer's re-requests, or for a sender
  // whose copies overflowed its push region (record -1).  Otherwise every
  // cross-rank edge's copies travel as pushed segments (2b below) and the
  // lists stay home.
  // With push and no IWANT spammers the lists travel only if some sender's
  // push overflowed: that flag rides in the count readback below (one host
  // round trip per hop), and the lists are packed after it when needed.
  bool shipLists = true;
  const bool deferLists = xpush && d.cSpam[cur] == nullptr;
  if (deferLists) {
    xHost[world + 3 + 2 * world] = 0;
    HIPCHECK(hipMemcpyAsync(&xHost[world + 3 + 2 * world], d.pushOvf, 4, hipMemcpyDeviceToHost, stream));
  }
  auto packLists = [&]() {
    const int64_t capEnt = (int64_t)((xSendCap - hdrBytes) / 4);
    if (nOwn && shipLists)
      k_x_lists<<<nOwn, 64, 0, stream>>>(d, cur, bump, (int64_t*)xSend, (uint32_t*)(xSend + hdrBytes), capEnt);
  };
  if (!deferLists) packLists();
  HIPCHECK(hipMemcpyAsync(xHost, xCnt, (size_t)world * 8, hipMemcpyDeviceToHost, stream));
  HIPCHECK(hipMemcpyAsync(xHost + world, bump, 8, hipMemcpyDeviceToHost, stream));
  HIPCHECK(hipMemcpyAsync(xHost + world + 1, d.poolCnt + (size_t)cur * d.poolSub * 16, 8, hipMemcpyDeviceToHost,
                          stream));  // (poolSub == 1 when partitioned)
  // this rank's device error word travels with the sizes below, so every rank
  // stops at the same hop (a rank returning alone would leave the others
  // waiting in the next hop's collectives)
  xHost[world + 2] = 0;
  HIPCHECK(hipMemcpyAsync(xHost + world + 2, d.err, 4, hipMemcpyDeviceToHost, stream));
  HIPCHECK(hipStreamSynchronize(stream));
  if (deferLists) {
    shipLists = (int32_t)(xHost[world + 3 + 2 * world] & 0xFFFFFFFFu) != 0;
    if (shipLists) {  // (rare: a sender's copies overflowed its push region)
      packLists();
      HIPCHECK(hipMemcpyAsync(xHost + world, bump, 8, hipMemcpyDeviceToHost, stream));
      HIPCHECK(hipStreamSynchronize(stream));
    }
  }
  const size_t hdrB = shipLists ? hdrBytes : 0;
  const int32_t myErr = (int32_t)xHost[world + 2];
  const int64_t nEnt = (int64_t)xHost[world];
  const int64_t poolBase = (int64_t)rank * poolSeg;
  const int64_t nPool = std::min<int64_t>((int64_t)xHost[world + 1], poolSeg);
  const size_t entBytes = align8((size_t)nEnt * 4), poolBytes = align8((size_t)nPool * 4);
  const size_t gwBytes = hb ? (size_t)nOwn * W * 8 : 0;
  // randomsub hosts' target masks ride with their list entries (a receiver
  // walking a remote randomsub sender's list filters by them)
  const size_t selBytes = (shipLists && d.sel != nullptr) ? (size_t)nEnt * 8 : 0;
  const size_t bcast = hdrB + entBytes + selBytes + poolBytes + gwBytes;
  if (bcast > xSendCap) {  // grow (keeps nothing) and pack the lists again
    int rc = growDev(xSend, xSendCap, bcast);
    if (rc) return rc;
    HIPCHECK(hipMemsetAsync(bump, 0, 8, stream));
    packLists();
  }
  if (selBytes && nOwn)
    k_x_sel<<<nOwn, 64, 0, stream>>>(d, (const int64_t*)xSend, (const uint32_t*)(xSend + hdrBytes),
                                     (uint64_t*)(xSend + hdrB + entBytes));
  if (nPool)
    HIPCHECK(hipMemcpyAsync(xSend + hdrB + entBytes + selBytes, d.pool[cur] + poolBase, (size_t)nPool * 4,
                            hipMemcpyDeviceToDevice, stream));
  if (gwBytes)
    HIPCHECK(hipMemcpyAsync(xSend + hdrB + entBytes + selBytes + poolBytes, d.gw + (size_t)n0 * W, gwBytes,
                            hipMemcpyDeviceToDevice, stream));
  // 2. edge records, one block per destination rank
  std::vector<int64_t> sendRec(world), sendOff(world);
  int64_t totRec = 0;
  for (int r = 0; r < world; ++r) {
    sendRec[r] = (int64_t)xHost[r];
    sendOff[r] = totRec;
    totRec += sendRec[r];
  }
  {
    int rc = growDev(xSendE, xSendECap, (size_t)std::max<int64_t>(totRec, 1) * sizeof(XRec));
    if (rc) return rc;
  }
  if (totRec) {
    HIPCHECK(hipMemcpyAsync(xOff, sendOff.data(), (size_t)world * 8, hipMemcpyHostToDevice, stream));
    k_x_pack<<<nblk(eOwn, 256), 256, 0, stream>>>(d, cur, xOff, cursor, (XRec*)xSendE);
  }
  // 2b. pushed segments of cross-rank edges, one block per destination rank:
  //     [PRec x records][slots]
  std::vector<int64_t> pRec(world, 0), pSlots(world, 0), pBytes(world, 0), pOff(world, 0);
  if (xpush) {
    int64_t tot = 0;
    for (int r = 0; r < world; ++r) {
      pRec[r] = (int64_t)xHost[world + 3 + r];
      pSlots[r] = (int64_t)xHost[world + 3 + world + r];
      pBytes[r] = 16 * pRec[r] + 2 * pSlots[r];
      pOff[r] = tot;
      tot += pBytes[r];
    }
    int rc = growDev(xSendP, xSendPCap, (size_t)std::max<int64_t>(tot, 16));
    if (rc) return rc;
    if (tot) {
      std::vector<int64_t> offRec(2 * (size_t)world);
      for (int r = 0; r < world; ++r) {
        offRec[(size_t)r] = pOff[r];
        offRec[(size_t)world + r] = pRec[r];
      }
      HIPCHECK(hipMemcpyAsync(xpOff, offRec.data(), (size_t)2 * world * 8, hipMemcpyHostToDevice, stream));
      HIPCHECK(hipMemsetAsync(xpCnt + 2 * world, 0, (size_t)2 * world * 8, stream));
      k_xp_pack<<<nblk(eOwn, 256), 256, 0, stream>>>(d, cur, xpOff, xpOff + world, xpCnt + 2 * world, xSendP);
    }
  }
  HIPCHECK(hipStreamSynchronize(stream));  // sendOff is pageable; the transport reads the buffers
  // 3. sizes of every rank: [bcast bytes, list entries, arena ids, gw rows?,
  //    records to rank 0..world-1, device error word, dials, push records to
  //    rank 0..world-1, push slots to rank 0..world-1]
  // the connector's dials of this hop (peer exchange): every rank applies all
  // of them at the next hop's start (each launching the sides it owns)
  const int nS = 6 + 3 * world;
  std::vector<int64_t> mine(nS), all((size_t)nS * world);
  mine[5 + world] = (int64_t)pxPend.size();
  mine[0] = (int64_t)bcast; mine[1] = nEnt; mine[2] = nPool; mine[3] = (hb ? 1 : 0) | (shipLists ? 2 : 0);
  for (int r = 0; r < world; ++r) mine[4 + r] = sendRec[r];
  mine[4 + world] = myErr;
  for (int r = 0; r < world; ++r) {
    mine[6 + world + r] = pRec[r];
    mine[6 + 2 * world + r] = pSlots[r];
  }
  const auto t0 = std::chrono::steady_clock::now();
  if (tr.allgather_i64(tr.user, mine.data(), nS, all.data()) != 0) {
    gs_set_error("transport allgather_i64 failed");
    return GS_EDEVICE;
  }
  if (myErr) return deviceErrorText(myErr, hop);
  for (int r = 0; r < world; ++r) {
    const int32_t err = (int32_t)all[(size_t)r * nS + 4 + world];
    if (!err) continue;
    const int rc = deviceErrorCode(err);  // the failing rank's code and text
    g_err = "hop " + std::to_string(hop) + ": rank " + std::to_string(r) + ": " + g_err;
    stickyRc = rc;
    stickyMsg = g_err;
    return rc;
  }
  int64_t chunk = 8;
  for (int r = 0; r < world; ++r) chunk = std::max<int64_t>(chunk, all[(size_t)r * nS]);
  chunk = (int64_t)align8((size_t)chunk);
  {
    int rc = growDev(xSend, xSendCap, (size_t)chunk, bcast);  // the transport reads `chunk` bytes
    if (rc) return rc;
    rc = growDev(xRecv, xRecvCap, (size_t)chunk * world);
    if (rc) return rc;
  }
  if (tr.allgather(tr.user, xSend, xRecv, chunk) != 0) {
    gs_set_error("transport allgather failed");
    return GS_EDEVICE;
  }
  {
    int64_t maxD = 0;
    for (int r = 0; r < world; ++r) maxD = std::max<int64_t>(maxD, all[(size_t)r * nS + 5 + world]);
    if (maxD > 0) {
      std::vector<int64_t> dm((size_t)maxD, -1), da((size_t)maxD * world);
      for (size_t i = 0; i < pxPend.size(); ++i)
        dm[i] = ((int64_t)pxPend[i].first << 32) | (int64_t)(uint32_t)pxPend[i].second;
      if (tr.allgather_i64(tr.user, dm.data(), (int32_t)maxD, da.data()) != 0) {
        gs_set_error("transport allgather_i64 failed (dials)");
        return GS_EDEVICE;
      }
      pxPend.clear();
      for (int64_t x : da)
        if (x >= 0) pxPend.push_back({(int)(x >> 32), (int)(uint32_t)x});
    }
  }
  std::vector<int64_t> sendB(world), recvB(world);
  int64_t totIn = 0;
  for (int r = 0; r < world; ++r) {
    sendB[r] = sendRec[r] * (int64_t)sizeof(XRec);
    recvB[r] = all[(size_t)r * nS + 4 + rank] * (int64_t)sizeof(XRec);
    totIn += recvB[r];
  }
  {
    int rc = growDev(xRecvE, xRecvECap, (size_t)std::max<int64_t>(totIn, 1));
    if (rc) return rc;
  }
  if (tr.alltoallv(tr.user, xSendE, sendB.data(), xRecvE, recvB.data()) != 0) {
    gs_set_error("transport alltoallv failed");
    return GS_EDEVICE;
  }
  // the pushed segments land behind the owned senders' regions of ibx[cur]
  std::vector<int64_t> pInRec(world, 0), pInOff(world, 0);
  int64_t pIn = 0;
  if (xpush) {
    std::vector<int64_t> pInB(world, 0);
    for (int r = 0; r < world; ++r) {
      pInRec[r] = all[(size_t)r * nS + 6 + world + rank];
      pInB[r] = 16 * pInRec[r] + 2 * all[(size_t)r * nS + 6 + 2 * world + rank];
      pInOff[r] = pIn;
      pIn += pInB[r];
    }
    const size_t own = (size_t)ibxOwnSlots * 2;
    if (own + (size_t)pIn > ibxCapB[cur]) {
      // grow this parity's buffer, keeping the owned regions (this hop's
      // segments for local receivers)
      uint8_t* p = reinterpret_cast<uint8_t*>(d.ibx[cur]);
      const uint8_t* old = p;
      int rc = growDev(p, ibxCapB[cur], own + (size_t)pIn, own);
      if (rc) return rc;
      for (void*& a : allocs)
        if (a == old) a = nullptr;  // freed by growDev
      allocs.push_back(p);
      d.ibx[cur] = reinterpret_cast<uint16_t*>(p);
    }
    if (tr.alltoallv(tr.user, xSendP, pBytes.data(), reinterpret_cast<uint8_t*>(d.ibx[cur]) + own, pInB.data()) != 0) {
      gs_set_error("transport alltoallv failed (pushed segments)");
      return GS_EDEVICE;
    }
    xBytes += pIn;
  }
  xMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // 4. unpack the other ranks' parts into the mirrors
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    const int nr = part[r + 1] - part[r];
    const int64_t* a = &all[(size_t)r * nS];
    const bool lists = (a[3] & 2) != 0;  // rank r shipped its frontier lists
    const size_t hB = lists ? align8((size_t)nr * 8) : 0, eB = align8((size_t)a[1] * 4), pB = align8((size_t)a[2] * 4);
    const size_t sB = (lists && d.sel != nullptr) ? (size_t)a[1] * 8 : 0;  // the entries' randomsub masks
    const uint8_t* c = xRecv + (size_t)r * chunk;
    xBytes += a[0];
    if (nr && lists)
      k_x_unlists<<<nr, 64, 0, stream>>>(d, cur, (const int64_t*)c, (const uint32_t*)(c + hB),
                                         sB ? (const uint64_t*)(c + hB + eB) : nullptr, part[r]);
    if (a[2])
      HIPCHECK(hipMemcpyAsync(d.pool[cur] + (size_t)r * poolSeg, c + hB + eB + sB, (size_t)a[2] * 4,
                              hipMemcpyDeviceToDevice, stream));
    if ((a[3] & 1) && nr)
      HIPCHECK(hipMemcpyAsync(d.gw + (size_t)part[r] * W, c + hB + eB + sB + pB, (size_t)nr * W * 8,
                              hipMemcpyDeviceToDevice, stream));
  }
  xBytes += totIn;
  if (totIn) {
    const int64_t n = totIn / (int64_t)sizeof(XRec);
    k_x_unpack<<<nblk(n, 256), 256, 0, stream>>>(d, cur, (const XRec*)xRecvE, n);
  }
  for (int r = 0; r < world; ++r) {
    if (!pInRec[r]) continue;
    const uint8_t* blk = reinterpret_cast<const uint8_t*>(d.ibx[cur]) + (size_t)ibxOwnSlots * 2 + pInOff[r];
    const int64_t slotBase = ibxOwnSlots + (pInOff[r] + 16 * pInRec[r]) / 2;
    k_xp_unpack<<<nblk(pInRec[r], 256), 256, 0, stream>>>(d, cur, (const PRec*)blk, pInRec[r], slotBase);
  }
  HIPCHECK(hipGetLastError());
  return GS_OK;
}

// Moves the device's trace records to tracePending in canonical order.  The
// kernels record every delivered copy (GS_TRACE_COPY); the copy from the
// first deliverer of a fresh message is its DeliverMessage, every other copy
// a DuplicateMessage (pubsub.go:1010-1013).
int gs_engine::drainTrace() {
  if (!started || !d.traceN) return GS_OK;
  unsigned long long cnt = 0;
  HIPCHECK(hipStreamSynchronize(stream));
  HIPCHECK(hipMemcpy(&cnt, d.traceN, 8, hipMemcpyDeviceToHost));
  const int64_t k = std::min<int64_t>((int64_t)cnt, traceCap);
  std::vector<gs_trace_event> ev((size_t)k);
  if (k) HIPCHECK(hipMemcpy(ev.data(), d.trace, (size_t)k * sizeof(gs_trace_event), hipMemcpyDeviceToHost));
  // on the engine's stream: the next hop's appends are queued there too, and a
  // null-stream memset is not ordered against a non-blocking stream
  HIPCHECK(hipMemsetAsync(d.traceN, 0, 8, stream));
  struct Key {
    int64_t hop, msg;
    int32_t node, peer;
    bool operator<(const Key& o) const {
      return std::tie(hop, msg, node, peer) < std::tie(o.hop, o.msg, o.node, o.peer);
    }
  };
  // a copy is the delivering one (DeliverMessage), a rejected first copy or a
  // copy dropped by a full validation queue (RejectMessage), or else a duplicate
  std::vector<Key> delivered;
  for (const auto& e : ev)
    if ((e.type == GS_TRACE_DELIVER_MESSAGE || e.type == GS_TRACE_REJECT_MESSAGE) && e.phase == 2)
      delivered.push_back(Key{e.hop, e.msg, e.node, e.peer});
  std::sort(delivered.begin(), delivered.end());
  std::vector<gs_trace_event> keep(tracePending.begin() + traceOut, tracePending.end());
  std::vector<gs_trace_event> all;
  all.swap(traceFuture);
  for (auto e : ev) {
    if (e.type == GS_TRACE_COPY) {
      if (std::binary_search(delivered.begin(), delivered.end(), Key{e.hop, e.msg, e.node, e.peer})) continue;
      e.type = GS_TRACE_DUPLICATE_MESSAGE;
    }
    all.push_back(e);
  }
  // RPC blocks: a RECV stamped with a hop that has not run yet waits for it;
  // one whose connection closed at the start of its hop was lost in flight
  for (size_t i = 0; i < all.size();) {
    size_t j = i + 1;
    if (gs_trace_is_rpc(all[i]))
      while (j < all.size() && all[j].type == GS_TRACE_RPC_ITEM) ++j;
    const gs_trace_event& hd = all[i];
    bool drop = false;
    if (hd.hop >= hop) {
      traceFuture.insert(traceFuture.end(), all.begin() + i, all.begin() + j);
      drop = true;
    } else if (hd.type == GS_TRACE_RECV_RPC) {
      const std::array<int64_t, 3> k{hd.hop, hd.node, hd.peer};
      drop = std::find(rpcDowns.begin(), rpcDowns.end(), k) != rpcDowns.end();
    }
    if (!drop) keep.insert(keep.end(), all.begin() + i, all.begin() + j);
    i = j;
  }
  gs_trace_canonical(keep, cfg.seed, gp.MaxIHaveLength);
  tracePending.swap(keep);
  traceOut = 0;
  return GS_OK;
}

// Per-(edge, topic) arrays are edge-major rows [e*T + t] on the device (tix
// in gs_device.h); readbacks return them topic-major [t*E + e].
template <class X>
static int copy_back_pairs(gs_engine* g, X* dst, const X* src) {
  const size_t E = (size_t)g->E, T = (size_t)g->T;
  if (!g->started) {
    std::memset(dst, 0, T * E * sizeof(X));
    return GS_OK;
  }
  // only the owned edges [e0, e1) have per-(edge, topic) state on this rank
  const size_t e0 = (size_t)g->e0, e1 = (size_t)g->e1;
  std::vector<X> tmp(T * (e1 - e0));
  HIPCHECK(hipStreamSynchronize(g->stream));
  HIPCHECK(hipMemcpy(tmp.data(), src + e0 * T, tmp.size() * sizeof(X), hipMemcpyDeviceToHost));
  std::memset(dst, 0, T * E * sizeof(X));
  for (size_t e = e0; e < e1; ++e)
    for (size_t t = 0; t < T; ++t) dst[t * E + e] = tmp[(e - e0) * T + t];
  return GS_OK;
}
extern "C" {

const char* gs_last_error(void) { return g_err.c_str(); }

int gs_engine_create(const gs_config* cfg, const gs_gossipsub_params* gsp, const gs_peer_score_params* psp,
                     const gs_topic_score_params* topics, const uint8_t* topic_scored,
                     const gs_peer_score_thresholds* thr, const gs_peer_gater_params* gater, gs_engine** out) {
  if (!cfg || !out) { gs_set_error("null argument"); return GS_EINVAL; }
  if (cfg->num_nodes <= 0 || cfg->num_topics <= 0 || cfg->num_topics > 64 || cfg->hop_ns <= 0) {
    gs_set_error("invalid config: num_nodes > 0, 1 <= num_topics <= 64, hop_ns > 0 required");
    return GS_EINVAL;
  }
  if (cfg->router < 0 || cfg->router > 2) { gs_set_error("unknown router"); return GS_EINVAL; }
  if (cfg->slots_per_topic <= 0 || cfg->slots_per_topic % 64 != 0) {
    gs_set_error("slots_per_topic must be a positive multiple of 64");
    return GS_EINVAL;
  }
  if (gater) {
    if (cfg->router != GS_ROUTER_GOSSIPSUB) { gs_set_error("pubsub router is not gossipsub"); return GS_EINVAL; }
    int rc = gs_validate_peer_gater_params(gater);
    if (rc) return rc;
    if (gater->DecayInterval % cfg->hop_ns != 0) {
      gs_set_error("gater DecayInterval must be a multiple of hop_ns");
      return GS_EUNSUPPORTED;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gs_set_error("no HIP device available: the gossip engine needs an MI355X (gfx950)");
    return GS_EDEVICE;
  }
  if (cfg->device < 0 || cfg->device >= ndev) { gs_set_error("bad device ordinal"); return GS_EINVAL; }
  std::unique_ptr<gs_engine> g(new gs_engine());
  g->cfg = *cfg;
  if (gater) {
    g->gaterOn = true;
    g->gaterP = *gater;
  }
  g->N = cfg->num_nodes;
  g->T = cfg->num_topics;
  g->St = cfg->slots_per_topic;
  g->Wt = g->St / 64;
  g->W = g->T * g->Wt;
  g->S = g->T * g->St;
  if (g->W > 64 * GS_MAX_WPL) {
    gs_set_error("num_topics * slots_per_topic must be <= 16384 in this build");
    return GS_EUNSUPPORTED;
  }
  if (gsp) g->gp = *gsp; else gs_default_gossipsub_params(&g->gp);
  g->scoring = (cfg->flags & GS_FLAG_SCORING) != 0 && cfg->router == GS_ROUTER_GOSSIPSUB;
  g->floodPublish = (cfg->flags & GS_FLAG_FLOOD_PUBLISH) != 0;
  g->doPX = (cfg->flags & GS_FLAG_PEER_EXCHANGE) != 0 && cfg->router == GS_ROUTER_GOSSIPSUB;
  g->record = (cfg->flags & GS_FLAG_RECORD_DELIVERIES) != 0;
  g->tps.assign(g->T, gs_topic_score_params{});
  g->tscored.assign(g->T, 0);
  if (cfg->router == GS_ROUTER_GOSSIPSUB) {
    const gs_gossipsub_params& p = g->gp;
    if (p.HistoryGossip > p.HistoryLength || p.HistoryLength < 1) {
      gs_set_error("invalid parameters for message cache; gossip slots cannot be larger than history slots");
      return GS_EINVAL;
    }
    if (p.HeartbeatInterval % cfg->hop_ns != 0 || p.HeartbeatInterval < 2 * cfg->hop_ns ||
        p.HeartbeatInitialDelay % cfg->hop_ns != 0 || p.HeartbeatInitialDelay < cfg->hop_ns) {
      gs_set_error("HeartbeatInterval must be a multiple of hop_ns and >= 2 hops; "
                   "HeartbeatInitialDelay a multiple of hop_ns and >= 1 hop");
      return GS_EUNSUPPORTED;
    }
    if (p.DirectConnectTicks == 0) {  // heartbeatTicks % DirectConnectTicks (gossipsub.go:1597)
      gs_set_error("DirectConnectTicks must be > 0");
      return GS_EINVAL;
    }
    if (p.GossipRetransmission < 0 || p.MaxIHaveMessages < 0 || p.D < 0 || p.Dhi < 0 || p.Dscore < 0 ||
        p.Dscore > p.D || p.D > p.Dhi) {
      gs_set_error("invalid gossipsub degree parameters");
      return GS_EINVAL;
    }
    g->H = (int)(p.HeartbeatInterval / cfg->hop_ns);
    g->R = p.HistoryLength + 1;  // + the ghost slot holding the just-shifted window
  } else {
    g->R = 1;
  }
  g->setWindow();
  if (g->maxAge > 30000) { gs_set_error("heartbeat interval too long in hops"); return GS_EUNSUPPORTED; }
  if (g->scoring) {
    if (!psp || !topics || !topic_scored || !thr) {
      gs_set_error("scoring needs score params and thresholds");
      return GS_EINVAL;
    }
    int rc = gs_validate_peer_score_params(psp, topics, topic_scored, g->T);
    if (rc) return rc;
    rc = gs_validate_thresholds(thr);
    if (rc) return rc;
    if (psp->DecayInterval % cfg->hop_ns != 0) {
      gs_set_error("DecayInterval must be a multiple of hop_ns");
      return GS_EUNSUPPORTED;
    }
    g->sp = *psp;
    g->thr = *thr;
    for (int t = 0; t < g->T; ++t) { g->tps[t] = topics[t]; g->tscored[t] = topic_scored[t]; }
  }
  g->topicCounter.assign(g->T, 0);
  g->topicLive.assign(g->T, 0);
  g->slotOwnerHop.assign(g->S, INT64_MIN);
  g->slotOwnerId.assign(g->S, -1);
  *out = g.release();
  return GS_OK;
}

int gs_engine_destroy(gs_engine* eng) {
  delete eng;
  return GS_OK;
}

int gs_set_graph(gs_engine* g, const int64_t* rowptr, const int32_t* col, const uint8_t* outbound,
                 const uint8_t* direct) {
  return gs_set_graph_ex(g, rowptr, col, outbound, direct, nullptr);
}

int gs_set_routers(gs_engine* g, const uint8_t* router) {
  if (g->started) { gs_set_error("routers must be set before the first step"); return GS_ESTATE; }
  g->routerH.clear();
  if (router) {
    for (int u = 0; u < g->N; ++u)
      if (router[u] > GS_ROUTER_GOSSIPSUB_V10) { gs_set_error("unknown router"); return GS_EINVAL; }
    g->routerH.assign(router, router + g->N);
  }
  return GS_OK;
}

int gs_set_graph_ex(gs_engine* g, const int64_t* rowptr, const int32_t* col, const uint8_t* outbound,
                    const uint8_t* direct, const uint8_t* proto) {
  if (g->started) { gs_set_error("graph must be set before the first step"); return GS_ESTATE; }
  g->rowptr.assign(rowptr, rowptr + g->N + 1);
  g->E = g->rowptr[g->N];
  g->col.assign(col, col + g->E);
  for (int u = 0; u < g->N; ++u)
    for (int64_t e = g->rowptr[u]; e < g->rowptr[u + 1]; ++e) {
      const int v = g->col[e];
      if (v < 0 || v >= g->N || v == u || (e > g->rowptr[u] && g->col[e - 1] >= v)) {
        gs_set_error("graph rows must hold strictly ascending neighbour ids != self");
        return GS_EINVAL;
      }
    }
  g->outbound.assign(g->E, 0);
  g->direct.assign(g->E, 0);
  if (outbound) g->outbound.assign(outbound, outbound + g->E);
  if (direct) g->direct.assign(direct, direct + g->E);
  g->protoH.clear();
  if (proto) {
    for (int64_t e = 0; e < g->E; ++e)
      if (proto[e] > GS_PROTO_GOSSIPSUB_V11) { gs_set_error("unknown protocol"); return GS_EINVAL; }
    g->protoH.assign(proto, proto + g->E);
  }
  g->graphSet = true;
  return GS_OK;
}

int gs_set_subscriptions(gs_engine* g, const uint64_t* sub_mask) {
  if (g->started) { gs_set_error("subscriptions must be set before the first step"); return GS_ESTATE; }
  g->sub.assign(sub_mask, sub_mask + g->N);
  return GS_OK;
}

int gs_set_peer_attrs(gs_engine* g, const double* app_score, const uint32_t* ipv4) {
  if (g->started) { gs_set_error("peer attributes must be set before the first step"); return GS_ESTATE; }
  if (app_score) g->app.assign(app_score, app_score + g->N);
  if (ipv4) g->ipv4.assign(ipv4, ipv4 + g->N);
  return GS_OK;
}

int gs_set_ip_whitelist(gs_engine* g, int32_t n, const uint32_t* net, const uint32_t* mask) {
  if (g->started) { gs_set_error("whitelist must be set before the first step"); return GS_ESTATE; }
  g->whitelist.clear();
  for (int i = 0; i < n; ++i) g->whitelist.push_back({net[i], mask[i]});
  return GS_OK;
}

int gs_publish(gs_engine* g, int32_t n, const int32_t* src, const int32_t* topic, const int64_t* hop,
               int64_t* ids_out) {
  return gs_publish_ex(g, n, src, topic, hop, nullptr, ids_out);
}

int gs_publish_ex(gs_engine* g, int32_t n, const int32_t* src, const int32_t* topic, const int64_t* hop,
                  const uint8_t* kind, int64_t* ids_out) {
  int64_t last = g->mHop.empty() ? g->hop : std::max(g->hop, g->mHop.back());
  for (int i = 0; i < n; ++i) {
    if (src[i] < 0 || src[i] >= g->N || topic[i] < 0 || topic[i] >= g->T || hop[i] < last ||
        (kind && kind[i] > GS_MSG_PHANTOM)) {
      gs_set_error("publish: bad src/topic/kind or hop not non-decreasing from the current hop");
      return GS_EINVAL;
    }
    last = hop[i];
  }
  // assign message-window slots; a slot is recycled only after retireHops
  std::vector<int64_t> cnt = g->topicCounter, owner = g->slotOwnerHop;
  std::vector<int32_t> slots(n);
  for (int i = 0; i < n; ++i) {
    const int t = topic[i];
    const int slot = t * g->St + (int)(cnt[t] % g->St);
    cnt[t]++;
    if (owner[slot] != INT64_MIN && hop[i] - owner[slot] < g->retireHops) {
      gs_set_error("message window too small: more than slots_per_topic messages of one topic within " +
                   std::to_string(g->retireHops) + " hops");
      return GS_ECAPACITY;
    }
    owner[slot] = hop[i];
    slots[i] = slot;
    if (kind && kind[i] == GS_MSG_PHANTOM) g->anyPhantom = true;
  }
  g->topicCounter = cnt;
  g->slotOwnerHop = owner;
  for (int i = 0; i < n; ++i) {
    const int64_t id = (int64_t)g->mSrc.size();
    g->mSrc.push_back(src[i]);
    g->mTopic.push_back(topic[i]);
    g->mSlot.push_back(slots[i]);
    g->mId.push_back(id);
    g->mHop.push_back(hop[i]);
    g->mKind.push_back(kind ? kind[i] : (uint8_t)GS_MSG_VALID);
    g->slotOwnerId[slots[i]] = id;
    if (ids_out) ids_out[i] = id;
  }
  return g->uploadMessages();
}

int gs_set_validation(gs_engine* g, const uint8_t* topic_validator, int32_t queue_per_hop) {
  if (g->started || !g->mId.empty()) {
    gs_set_error("validation must be set before the first publish");
    return GS_ESTATE;
  }
  if (queue_per_hop < 0) { gs_set_error("queue_per_hop must be >= 0"); return GS_EINVAL; }
  g->topicVal = 0;
  if (topic_validator)
    for (int t = 0; t < g->T; ++t)
      if (topic_validator[t]) g->topicVal |= 1ull << t;
  g->valQueue = queue_per_hop;
  g->setWindow();
  return GS_OK;
}

int gs_schedule_events(gs_engine* g, int32_t n, const int32_t* kind, const int32_t* a, const int32_t* b,
                       const int64_t* hop) {
  if (n < 0 || (n > 0 && (!kind || !a || !b || !hop))) { gs_set_error("gs_schedule_events: bad arguments"); return GS_EINVAL; }
  if (!g->graphSet) { gs_set_error("graph not set"); return GS_ESTATE; }
  if (n > 0 && !g->churnWindow && !g->mId.empty()) {
    // late joiners catch up through gossip: the wide message window is chosen
    // when the first churn is scheduled, and it cannot change once messages
    // hold slots (gs_set_behaviour / gs_set_validation have the same rule)
    gs_set_error("connection churn must first be scheduled before the first publish");
    return GS_ESTATE;
  }
  int64_t last = g->events.empty() ? std::max<int64_t>(1, g->hop) : std::max(g->hop, g->events.back().hop);
  auto isEdge = [&](int x, int y) {
    auto bgn = g->col.begin() + g->rowptr[x], fin = g->col.begin() + g->rowptr[x + 1];
    auto it = std::lower_bound(bgn, fin, y);
    return it != fin && *it == y;
  };
  for (int32_t i = 0; i < n; ++i) {
    bool ok = hop[i] >= last && hop[i] >= 1 && kind[i] >= GS_EV_DISCONNECT && kind[i] <= GS_EV_JOIN &&
              a[i] >= 0 && a[i] < g->N;
    if (ok && kind[i] <= GS_EV_CONNECT) ok = b[i] >= 0 && b[i] < g->N && isEdge(a[i], b[i]);
    if (ok && kind[i] >= GS_EV_LEAVE) ok = b[i] >= 0 && b[i] < g->T;
    if (!ok) { gs_set_error("gs_schedule_events: bad event (kind, nodes, topic or hop order)"); return GS_EINVAL; }
    last = hop[i];
  }
  for (int32_t i = 0; i < n; ++i) g->events.push_back({hop[i], kind[i], a[i], b[i]});
  if (n > 0 && !g->started && g->mId.empty()) {
    g->churnWindow = true;  // late joiners catch up through gossip: the wide message window
    g->setWindow();
  }
  if (g->started && n > 0) return g->enableChurn();
  return GS_OK;
}

int gs_set_behaviour(gs_engine* g, const uint8_t* behaviour) {
  if (g->started || !g->mId.empty()) {
    gs_set_error("behaviours must be set before the first publish");
    return GS_ESTATE;
  }
  g->behaveH.clear();
  g->behaveAll = 0;
  if (behaviour) {
    g->behaveH.assign(behaviour, behaviour + g->N);
    for (uint8_t b : g->behaveH) g->behaveAll |= b;
    if (g->behaveAll & ~(uint8_t)(GS_BEHAVE_NO_FORWARD | GS_BEHAVE_IWANT_SPAM | GS_BEHAVE_GRAFT_SPAM |
                                  GS_BEHAVE_IHAVE_SPAM)) {
      gs_set_error("unknown behaviour bit");
      return GS_EINVAL;
    }
  }
  g->setWindow();
  return GS_OK;
}

int gs_step(gs_engine* g, int64_t hops) {
  if (!g->graphSet) { gs_set_error("graph not set"); return GS_ESTATE; }
  if (!g->started) {
    int rc = g->start();
    if (rc) return rc;
  }
  if (g->stickyRc) {
    gs_set_error(g->stickyMsg);
    return g->stickyRc;
  }
  if (!g->errRing)
    HIPCHECK(hipHostMalloc((void**)&g->errRing, gs_engine::kErrRing * sizeof(int32_t), hipHostMallocDefault));
  int64_t first = g->hop;
  int n = 0;
  for (int64_t i = 0; i < hops; ++i) {
    int rc = g->stepOne();
    if (rc) return rc;
    HIPCHECK(hipMemcpyAsync(g->errRing + n, g->d.err, 4, hipMemcpyDeviceToHost, g->stream));
    if (++n == gs_engine::kErrRing || g->pendKid.size() > 4096) {
      rc = g->drainErrors(first, n);
      if (rc) return rc;
      first = g->hop;
      n = 0;
    }
  }
  return g->drainErrors(first, n);
}

int gs_sync(gs_engine* g) {
  if (!g->started) return GS_OK;
  HIPCHECK(hipStreamSynchronize(g->stream));
  return GS_OK;
}

int gs_set_topic_score_params(gs_engine* g, int32_t topic, const gs_topic_score_params* p) {
  if (topic < 0 || topic >= g->T) { gs_set_error("bad topic"); return GS_EINVAL; }
  int rc = gs_validate_topic_score_params(p);
  if (rc) return rc;
  if (g->started && g->scoring && !g->d.needAge &&
      p->MeshMessageDeliveriesWindow < g->retireHops * g->cfg.hop_ns) {
    gs_set_error("MeshMessageDeliveriesWindow shorter than the message lifetime can only be set "
                 "before the first step (per-message first-delivery hops are not kept)");
    return GS_EUNSUPPORTED;
  }
  const bool existed = g->tscored[topic] != 0;
  const gs_topic_score_params old = g->tps[topic];
  g->tps[topic] = *p;
  g->tscored[topic] = 1;
  if (!g->started) return GS_OK;
  TopicP tp = to_dev(*p, g->scoring);
  if (g->scoring) k_fold<<<nblk(g->E, 256), 256, 0, g->stream>>>(g->d, topic);  // with the old caps
  HIPCHECK(hipMemcpyAsync(g->dTp + topic, &tp, sizeof(TopicP), hipMemcpyHostToDevice, g->stream));
  HIPCHECK(hipMemsetAsync(g->d.sdirty + g->e0, 1, (size_t)g->eOwn, g->stream));  // every score may have changed
  if (existed && g->scoring &&
      (p->FirstMessageDeliveriesCap < old.FirstMessageDeliveriesCap ||
       p->MeshMessageDeliveriesCap < old.MeshMessageDeliveriesCap))
    k_recap<<<nblk(g->E, 256), 256, 0, g->stream>>>(g->d, topic, p->FirstMessageDeliveriesCap,
                                                    p->MeshMessageDeliveriesCap);
  HIPCHECK(hipStreamSynchronize(g->stream));
  return GS_OK;
}

int gs_set_partition(gs_engine* g, int32_t rank, int32_t world, const gs_transport* tr) {
  if (g->started) { gs_set_error("the partition must be set before the first step"); return GS_ESTATE; }
  if (world < 1 || world > 255 || rank < 0 || rank >= world) { gs_set_error("bad rank / world"); return GS_EINVAL; }
  if (world > 1 && (!tr || !tr->allgather_i64 || !tr->allgather || !tr->alltoallv)) {
    gs_set_error("a partitioned engine needs a transport with allgather_i64, allgather and alltoallv");
    return GS_EINVAL;
  }
  g->rank = rank;
  g->world = world;
  if (tr) g->tr = *tr;
  return GS_OK;
}

int gs_partition_range(const gs_engine* g, int32_t* node_begin, int32_t* node_end) {
  if (!g->graphSet) { gs_set_error("graph not set"); return GS_ESTATE; }
  const std::vector<int32_t> part = partition_bounds(g->rowptr, g->N, g->world);
  *node_begin = part[g->rank];
  *node_end = part[g->rank + 1];
  return GS_OK;
}

int gs_set_rpc_accounting(gs_engine* g, const int32_t* msg_size, int32_t id_len, const int32_t* topic_len) {
  if (g->started) { gs_set_error("gs_set_rpc_accounting: before the first step"); return GS_ESTATE; }
  if (!msg_size || !topic_len || id_len < 0) { gs_set_error("gs_set_rpc_accounting: bad arguments"); return GS_EINVAL; }
  for (int t = 0; t < g->T; ++t)
    if (msg_size[t] < 0 || topic_len[t] < 0) { gs_set_error("gs_set_rpc_accounting: negative size"); return GS_EINVAL; }
  g->acctOn = true;
  g->acctMsg.assign(msg_size, msg_size + g->T);
  g->acctTl.assign(topic_len, topic_len + g->T);
  g->acctIdLen = id_len;
  return GS_OK;
}

int gs_set_rpc_px_sizes(gs_engine* g, int32_t peer_id_len, int32_t record_len) {
  if (g->started) { gs_set_error("gs_set_rpc_px_sizes: before the first step"); return GS_ESTATE; }
  if (peer_id_len < 0 || record_len < 0) { gs_set_error("gs_set_rpc_px_sizes: negative size"); return GS_EINVAL; }
  g->acctPidLen = peer_id_len;
  g->acctRecLen = record_len;
  return GS_OK;
}

int gs_read_rpc_bytes(gs_engine* g, int64_t* bytes, int64_t* rpcs) {
  if (!g->acctOn) { gs_set_error("gs_read_rpc_bytes: accounting is off"); return GS_ESTATE; }
  const int64_t E = g->E;
  if (!g->started) {
    for (int64_t e = 0; e < E; ++e) {
      if (bytes) bytes[e] = 0;
      if (rpcs) rpcs[e] = 0;
    }
    return GS_OK;
  }
  std::vector<unsigned long long> b(E), n(E);
  HIPCHECK(hipStreamSynchronize(g->stream));
  // (owned edges only on the device, Dev::rxi)
  HIPCHECK(hipMemcpy(b.data() + g->e0, g->d.rpcB + g->e0, (size_t)g->eOwn * 8, hipMemcpyDeviceToHost));
  HIPCHECK(hipMemcpy(n.data() + g->e0, g->d.rpcN + g->e0, (size_t)g->eOwn * 8, hipMemcpyDeviceToHost));
  for (int64_t e = 0; e < E; ++e) {
    const bool own = e >= g->e0 && e < g->e1;  // a partitioned rank reports its own edges
    if (bytes) bytes[e] = own ? (int64_t)b[e] : 0;
    if (rpcs) rpcs[e] = own ? (int64_t)n[e] : 0;
  }
  return GS_OK;
}

int gs_set_trace(gs_engine* g, const uint8_t* node_mask, int64_t capacity) {
  if (g->started) { gs_set_error("tracing must be set before the first step"); return GS_ESTATE; }
  if (node_mask && capacity <= 0) { gs_set_error("trace capacity must be positive"); return GS_EINVAL; }
  if (node_mask) g->traceMask.assign(node_mask, node_mask + g->N);
  else g->traceMask.clear();
  g->traceCap = capacity;
  return GS_OK;
}

int gs_set_dormant(gs_engine* g, int32_t n, const int32_t* a, const int32_t* b) {
  if (g->started) { gs_set_error("gs_set_dormant: before the first step"); return GS_ESTATE; }
  if (!g->graphSet) { gs_set_error("graph not set"); return GS_ESTATE; }
  if (n < 0 || (n > 0 && (!a || !b))) { gs_set_error("gs_set_dormant: bad arguments"); return GS_EINVAL; }
  for (int32_t i = 0; i < n; ++i) {
    bool ok = a[i] >= 0 && a[i] < g->N && b[i] >= 0 && b[i] < g->N;
    if (ok) {
      auto bgn = g->col.begin() + g->rowptr[a[i]], fin = g->col.begin() + g->rowptr[a[i] + 1];
      auto it = std::lower_bound(bgn, fin, b[i]);
      ok = it != fin && *it == b[i];
    }
    if (!ok) { gs_set_error("gs_set_dormant: not an edge of the graph"); return GS_EINVAL; }
    g->dormant.insert({std::min(a[i], b[i]), std::max(a[i], b[i])});
  }
  return GS_OK;
}

int gs_set_peertx_capacity(gs_engine* g, int32_t home_bits, int32_t overflow_bits) {
  if (g->started) { gs_set_error("the peertx capacity must be set before the first step"); return GS_ESTATE; }
  if (home_bits < 2 || home_bits > 16 || overflow_bits < 8 || overflow_bits > 30) {
    gs_set_error("gs_set_peertx_capacity: home_bits in [2, 16], overflow_bits in [8, 30]");
    return GS_EINVAL;
  }
  g->ptxHomeBits = home_bits;
  g->ptxOvfBits = overflow_bits;
  return GS_OK;
}

int gs_set_frontier_mode(gs_engine* g, int32_t mode) {
  if (g->started) { gs_set_error("the frontier mode must be set before the first step"); return GS_ESTATE; }
  if (mode != GS_FRONTIER_AUTO && mode != GS_FRONTIER_LISTS && mode != GS_FRONTIER_BITMAPS) {
    gs_set_error("gs_set_frontier_mode: GS_FRONTIER_AUTO, GS_FRONTIER_LISTS or GS_FRONTIER_BITMAPS");
    return GS_EINVAL;
  }
  g->frontierMode = mode;
  return GS_OK;
}

int gs_frontier_dense(const gs_engine* g) { return g->started && (g->denseFlood || g->denseGossip) ? 1 : 0; }

int gs_set_trace_rpc(gs_engine* g, int32_t on) {
  if (g->started) { gs_set_error("tracing must be set before the first step"); return GS_ESTATE; }
  g->traceRpc = on != 0;
  return GS_OK;
}

int gs_trace_read(gs_engine* g, gs_trace_event* out, int64_t cap, int64_t* n) {
  *n = 0;
  if (g->traceOut == 0 || g->traceOut == g->tracePending.size()) {
    int rc = g->drainTrace();
    if (rc) return rc;
  }
  const int64_t k = std::min<int64_t>(cap, (int64_t)(g->tracePending.size() - g->traceOut));
  std::copy(g->tracePending.begin() + g->traceOut, g->tracePending.begin() + g->traceOut + k, out);
  g->traceOut += (size_t)k;
  if (g->traceOut == g->tracePending.size()) {
    g->tracePending.clear();
    g->traceOut = 0;
  }
  *n = k;
  return GS_OK;
}

int gs_read_exchange_stats(gs_engine* g, double* host_ms, int64_t* bytes_in) {
  *host_ms = g->xMs;
  *bytes_in = g->xBytes;
  return GS_OK;
}

int64_t gs_num_edges(const gs_engine* g) { return g->E; }
int64_t gs_current_hop(const gs_engine* g) { return g->hop; }

int gs_read_counters(gs_engine* g, gs_counters* out) {
  std::memset(out, 0, sizeof(*out));
  if (g->started) {
    std::vector<unsigned long long> all((size_t)C_NCOUNTERS * GS_CTR_SPREAD);
    HIPCHECK(hipStreamSynchronize(g->stream));
    HIPCHECK(hipMemcpy(all.data(), g->d.ctr, all.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long c[C_NCOUNTERS] = {};
    for (int s = 0; s < GS_CTR_SPREAD; ++s)
      for (int k = 0; k < C_NCOUNTERS; ++k) c[k] += all[(size_t)s * C_NCOUNTERS + k];
    out->published = (int64_t)c[C_PUBLISHED];
    out->deliveries = (int64_t)c[C_DELIVERIES];
    out->duplicates = (int64_t)c[C_DUPLICATES];
    out->transmissions = (int64_t)c[C_TRANSMISSIONS];
    out->grafts_sent = (int64_t)c[C_GRAFTS];
    out->prunes_sent = (int64_t)c[C_PRUNES];
    out->ihave_sent = (int64_t)c[C_IHAVE];
    out->iwant_sent = (int64_t)c[C_IWANT_SENT];
    out->iwant_served = (int64_t)c[C_IWANT_SERVED];
    out->promises_broken = (int64_t)c[C_PROMISES_BROKEN];
    out->graylisted = (int64_t)c[C_GRAYLISTED];
    out->rejected = (int64_t)c[C_REJECTED];
    out->throttled = (int64_t)c[C_THROTTLED];
    out->gated = (int64_t)c[C_GATED];
  }
  out->hops = g->hop;
  out->heartbeats = g->heartbeats;
  return GS_OK;
}

#define NEED_STARTED(g)                        \
  do {                                         \
    if (!(g)->started) {                       \
      int _rc = (g)->start();                  \
      if (_rc) return _rc;                     \
    }                                          \
  } while (0)

int gs_read_scores(gs_engine* g, double* score) {
  if (!g->graphSet) { gs_set_error("graph not set"); return GS_ESTATE; }
  NEED_STARTED(g);
  score_rows<0>(g->d, g->eOwn, g->d.T, g->dScoreTmp, g->stream);
  // the owned edges (a partitioned rank's others read 0)
  std::memset(score, 0, (size_t)g->E * 8);
  HIPCHECK(hipMemcpyAsync(score + g->e0, g->dScoreTmp + g->e0, (size_t)g->eOwn * 8, hipMemcpyDeviceToHost, g->stream));
  HIPCHECK(hipStreamSynchronize(g->stream));
  if (g->mixed)  // only gossipsub hosts keep a peerScore (floodsub / randomsub: none, score 0)
    for (int u = 0; u < g->N; ++u)
      if (g->routerOf(u) != GS_ROUTER_GOSSIPSUB)
        for (int64_t e = g->rowptr[u]; e < g->rowptr[u + 1]; ++e) score[e] = 0.0;
  return GS_OK;
}

// A per-edge array (owned edges [e0, e1) on the device, Dev::rxi) into a
// host array of E entries; a partitioned rank's other entries read 0.
}  // extern "C"
template <class X>
static int copy_back_edges(gs_engine* g, X* dst, const X* src) {
  std::memset(dst, 0, (size_t)g->E * sizeof(X));
  if (!g->started) return GS_OK;
  HIPCHECK(hipStreamSynchronize(g->stream));
  HIPCHECK(hipMemcpy(dst + g->e0, src + g->e0, (size_t)g->eOwn * sizeof(X), hipMemcpyDeviceToHost));
  return GS_OK;
}
extern "C" {

int gs_read_mesh(gs_engine* g, uint64_t* mesh) { return copy_back_edges(g, mesh, g->d.mesh); }
int gs_read_fanout(gs_engine* g, uint64_t* fanout) { return copy_back_edges(g, fanout, g->d.fanout); }
int gs_read_backoff(gs_engine* g, int64_t* expire) { return copy_back_pairs(g, expire, g->d.backoff); }
int gs_read_topic_stats(gs_engine* g, double* fmd, double* mmd, double* mfp, double* imd, int64_t* mesh_time,
                        int64_t* graft_time, uint8_t* flags) {
  int rc;
  if (g->started && g->scoring) k_fold_all<<<nblk((int64_t)g->E * g->T, 256), 256, 0, g->stream>>>(g->d);
  if ((rc = copy_back_pairs(g, fmd, g->d.fmd))) return rc;
  if ((rc = copy_back_pairs(g, mmd, g->d.mmd))) return rc;
  if ((rc = copy_back_pairs(g, mfp, g->d.mfp))) return rc;
  if ((rc = copy_back_pairs(g, imd, g->d.imd))) return rc;
  if ((rc = copy_back_pairs(g, mesh_time, (const int64_t*)g->d.meshTime))) return rc;
  if ((rc = copy_back_pairs(g, graft_time, (const int64_t*)g->d.graftTime))) return rc;
  if ((rc = copy_back_pairs(g, flags, (const uint8_t*)g->d.flags))) return rc;
  // a mesh pair's meshTime is derived (mesh_time_of, gs_device.h)
  const int64_t lr = g->d.lastRefresh;
  for (int64_t i = 0; i < (int64_t)g->E * g->T; ++i)
    if (flags[i] & 1) mesh_time[i] = graft_time[i] <= lr ? lr - graft_time[i] : 0;
  return GS_OK;
}
int gs_read_behaviour_penalty(gs_engine* g, double* bp) { return copy_back_edges(g, bp, g->d.bp); }

// PubSubRouter.EnoughPeers of every owned host (gossip_engine.h), on the host
// from the mesh readback and the host mirrors of the announced subscriptions
// (subA), the connection states (aliveH) and the protocols.  A topic no peer
// announced counts as empty (the reference's missing p.topics entry).
int gs_enough_peers(gs_engine* g, int32_t topic, int32_t suggested, uint8_t* out) {
  if (topic < 0 || topic >= g->T || suggested < 0 || !out) { gs_set_error("gs_enough_peers: bad arguments"); return GS_EINVAL; }
  if (!g->started) { gs_set_error("gs_enough_peers: no state before the first step"); return GS_ESTATE; }
  std::vector<uint64_t> mesh((size_t)g->E);
  int rc = copy_back_edges(g, mesh.data(), g->d.mesh);
  if (rc) return rc;
  const uint64_t bit = 1ull << topic;
  std::memset(out, 0, (size_t)g->N);
  for (int u = g->n0; u < g->n1; ++u) {
    int fs = 0, rs = 0, gsn = 0, any = 0;
    for (int64_t e = g->rowptr[u]; e < g->rowptr[u + 1]; ++e) {
      if (!g->aliveH.empty() && !g->aliveH[e]) continue;
      if (!(g->subA[g->col[e]] & bit)) continue;
      const int pr = g->protoH[e];
      any++;
      fs += pr == GS_PROTO_FLOODSUB;
      rs += pr == GS_PROTO_RANDOMSUB;
      gsn += (mesh[e] & bit) != 0;
    }
    bool ok;
    switch (g->routerOf(u)) {
      case GS_ROUTER_GOSSIPSUB:  // gossipsub.go:549-576: floodsub peers = not mesh-capable
        ok = (fs + rs) + gsn >= (suggested ? suggested : g->gp.Dlo) || gsn >= g->gp.Dhi;
        break;
      case GS_ROUTER_RANDOMSUB:  // randomsub.go:59-89 (RandomSubD = 6)
        ok = fs + rs >= (suggested ? suggested : 6) || rs >= 6;
        break;
      default:  // floodsub.go:52-66 (FloodSubTopicSearchSize = 5)
        ok = any >= (suggested ? suggested : 5);
        break;
    }
    out[u] = ok ? 1 : 0;
  }
  return GS_OK;
}

int gs_read_topic_stats_edges(gs_engine* g, int64_t n, const int64_t* edges, double* fmd, double* mmd,
                              double* mfp, double* imd, int64_t* mesh_time, int64_t* graft_time,
                              uint8_t* flags) {
  if (n < 0 || (n > 0 && (!edges || !fmd || !mmd || !mfp || !imd || !mesh_time || !graft_time || !flags))) {
    gs_set_error("gs_read_topic_stats_edges: bad arguments");
    return GS_EINVAL;
  }
  for (int64_t i = 0; i < n; ++i)
    if (edges[i] < 0 || edges[i] >= g->E) { gs_set_error("gs_read_topic_stats_edges: edge out of range"); return GS_EINVAL; }
  const int64_t nk = n * g->T;
  if (!g->started || nk == 0) {
    std::fill(fmd, fmd + nk, 0.0); std::fill(mmd, mmd + nk, 0.0);
    std::fill(mfp, mfp + nk, 0.0); std::fill(imd, imd + nk, 0.0);
    std::fill(mesh_time, mesh_time + nk, 0); std::fill(graft_time, graft_time + nk, 0);
    std::fill(flags, flags + nk, 0);
    return GS_OK;
  }
  int64_t* dE = nullptr;
  uint8_t* dOut = nullptr;
  HIPCHECK(hipMalloc(&dE, (size_t)n * 8));
  if (hipMalloc(&dOut, (size_t)nk * 49) != hipSuccess) {
    (void)hipFree(dE);
    gs_set_error("device allocation failed (gs_read_topic_stats_edges)");
    return GS_ENOMEM;
  }
  std::vector<uint8_t> h((size_t)nk * 49);
  hipError_t rc = hipMemcpyAsync(dE, edges, (size_t)n * 8, hipMemcpyHostToDevice, g->stream);
  if (rc == hipSuccess) {
    k_gather_pairs<<<nblk(nk, 256), 256, 0, g->stream>>>(g->d, dE, n, dOut);
    rc = hipMemcpyAsync(h.data(), dOut, h.size(), hipMemcpyDeviceToHost, g->stream);
  }
  if (rc == hipSuccess) rc = hipStreamSynchronize(g->stream);
  (void)hipFree(dE);
  (void)hipFree(dOut);
  if (rc != hipSuccess) {
    gs_set_error(std::string("HIP error: ") + hipGetErrorString(rc) + " (gs_read_topic_stats_edges)");
    return GS_EDEVICE;
  }
  const size_t b8 = (size_t)nk * 8;
  std::memcpy(fmd, h.data(), b8);
  std::memcpy(mmd, h.data() + b8, b8);
  std::memcpy(mfp, h.data() + 2 * b8, b8);
  std::memcpy(imd, h.data() + 3 * b8, b8);
  std::memcpy(mesh_time, h.data() + 4 * b8, b8);
  std::memcpy(graft_time, h.data() + 5 * b8, b8);
  std::memcpy(flags, h.data() + 6 * b8, (size_t)nk);
  return GS_OK;
}

int gs_read_backoff_edges(gs_engine* g, int64_t n, const int64_t* edges, int64_t* expire) {
  if (n < 0 || (n > 0 && (!edges || !expire))) { gs_set_error("gs_read_backoff_edges: bad arguments"); return GS_EINVAL; }
  for (int64_t i = 0; i < n; ++i)
    if (edges[i] < 0 || edges[i] >= g->E) { gs_set_error("gs_read_backoff_edges: edge out of range"); return GS_EINVAL; }
  const int64_t nk = n * g->T;
  if (!g->started || nk == 0) {
    std::fill(expire, expire + nk, 0);
    return GS_OK;
  }
  int64_t* dE = nullptr;
  int64_t* dOut = nullptr;
  HIPCHECK(hipMalloc(&dE, (size_t)n * 8));
  if (hipMalloc(&dOut, (size_t)nk * 8) != hipSuccess) {
    (void)hipFree(dE);
    gs_set_error("device allocation failed (gs_read_backoff_edges)");
    return GS_ENOMEM;
  }
  hipError_t rc = hipMemcpyAsync(dE, edges, (size_t)n * 8, hipMemcpyHostToDevice, g->stream);
  if (rc == hipSuccess) {
    k_gather_backoff<<<nblk(nk, 256), 256, 0, g->stream>>>(g->d, dE, n, dOut);
    rc = hipMemcpyAsync(expire, dOut, (size_t)nk * 8, hipMemcpyDeviceToHost, g->stream);
  }
  if (rc == hipSuccess) rc = hipStreamSynchronize(g->stream);
  (void)hipFree(dE);
  (void)hipFree(dOut);
  if (rc != hipSuccess) {
    gs_set_error(std::string("HIP error: ") + hipGetErrorString(rc) + " (gs_read_backoff_edges)");
    return GS_EDEVICE;
  }
  return GS_OK;
}

int gs_read_deliveries(gs_engine* g, int64_t id, int32_t* hop, int32_t* from) {
  if (!g->record) { gs_set_error("GS_FLAG_RECORD_DELIVERIES not set"); return GS_ESTATE; }
  if (id < 0 || id >= (int64_t)g->mId.size()) { gs_set_error("unknown message id"); return GS_EINVAL; }
  const int slot = g->mSlot[id];
  if (g->slotOwnerId[slot] != id) {
    gs_set_error("message slot already recycled (window moved on)");
    return GS_ESTATE;
  }
  if (!g->started || g->mHop[id] >= g->hop) {
    for (int v = 0; v < g->N; ++v) { hop[v] = -1; from[v] = -1; }
    return GS_OK;
  }
  k_read_deliv<<<nblk(g->N, 256), 256, 0, g->stream>>>(g->d, slot, g->mHop[id], g->dHopOut, g->dFromOut);
  HIPCHECK(hipMemcpyAsync(hop, g->dHopOut, (size_t)g->N * 4, hipMemcpyDeviceToHost, g->stream));
  HIPCHECK(hipMemcpyAsync(from, g->dFromOut, (size_t)g->N * 4, hipMemcpyDeviceToHost, g->stream));
  HIPCHECK(hipStreamSynchronize(g->stream));
  return GS_OK;
}

#ifdef GS_STAMPS
// Debug build: phase-A cycle stamps of the sampled nodes of the last hop.
int gs_debug_stamps(gs_engine* g, unsigned long long* out, int n) {
  HIPCHECK(hipStreamSynchronize(g->stream));
  HIPCHECK(hipMemcpy(out, g->d.stamps, (size_t)n * 8, hipMemcpyDeviceToHost));
  return GS_OK;
}
// Debug build: the peertx entry count of every owned node.
int gs_debug_ptxn(gs_engine* g, int32_t* out, int n) {
  HIPCHECK(hipStreamSynchronize(g->stream));
  HIPCHECK(hipMemcpy(out, g->d.ptxN + g->n0, (size_t)n * 4, hipMemcpyDeviceToHost));
  return GS_OK;
}
#endif

int gs_set_profiling(gs_engine* g, int on) {
  if (g->started) {
    HIPCHECK(hipStreamSynchronize(g->stream));
    g->resolveTimings();
  }
  g->profiling = on != 0;
  for (int i = 0; i < GS_NUM_KERNELS; ++i) { g->kMs[i] = 0; g->kLaunches[i] = 0; }
  return GS_OK;
}

int gs_read_kernel_stats(gs_engine* g, double* total_ms, int64_t* launches) {
  if (g->started) {
    HIPCHECK(hipStreamSynchronize(g->stream));
    g->resolveTimings();
  }
  for (int i = 0; i < GS_NUM_KERNELS; ++i) { total_ms[i] = g->kMs[i]; launches[i] = g->kLaunches[i]; }
  return GS_OK;
}

}  // extern "C"
