// oracle_sim.cpp — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
//
// Lock-step CPU restatement of N go-libp2p-pubsub routers exchanging RPCs
// over a static graph; exports include/gossip_engine.h so tests drive the
// oracle and the HIP engine through identical calls.  Per-node code follows
// the reference line by line (citations inline).  The round schedule
// (DESIGN.md "Canonical round") is:
//   hop h, now = h*hop_ns:
//     [h==0] Join(t) for every subscribed topic (gossipsub.go:1011-1060)
//     score memo S0 of every neighbour (used by AcceptFrom and Publish filters)
//     local publishes of hop h (topic.go:207 -> publishMessage, pubsub.go:1056)
//     phase A: every node handles the payload messages of the RPCs sent to it
//              in hop h-1, senders ascending, RPCs in send order
//              (handleIncomingRPC pubsub.go:902-967, pushMsg :978-1022)
//     phase B: every node handles the control of those RPCs, per RPC, senders
//              ascending (HandleRPC gossipsub.go:591-608)
//     refreshScores if a DecayInterval tick falls on `now` (score.go:495)
//     heartbeat if a heartbeat tick falls on `now` (gossipsub.go:1299-1552)
//   RPCs produced during hop h are delivered in hop h+1.
#include <algorithm>
#include <cstdio>
#include <memory>
#include <omp.h>
#include <unordered_map>

#include "oracle_core.hpp"
#include "../include/gs_trace.h"
#include "../include/gs_rpcsize.h"
#include "../include/gs_proto.h"

namespace oracle {

static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }

struct IHaveEntry { int topic; std::vector<int64_t> mids; };
struct PruneEntry { int topic; uint64_t backoff; bool hasBackoff; std::vector<int> px; };
struct Control {
  std::vector<IHaveEntry> ihave;
  std::vector<int64_t> iwant;
  std::vector<int> graft;
  std::vector<PruneEntry> prune;
};
struct RPC {
  std::vector<int64_t> publish;
  bool hasCtl = false;
  Control ctl;
  // trace ordinal (include/gs_trace.h): the send phase and its position there
  int sp = 0;
  int64_t ord = 0;
};

// Peer-gater view of one node at hop start (AcceptFrom, peer_gater.go:320-363):
// every AcceptFrom of the hop decides on this snapshot, as the score filters
// decide on the S0 memo.
struct GateSnap {
  bool active = false;          // quiet period, throttle and ratio checks passed
  std::map<int, double> thr;    // (1 + deliver) / (1 + total) per peer; absent = AcceptAll
};

struct Sim;

struct Node {
  Sim* sim = nullptr;
  int id = 0;
  std::vector<int> nbrs;                 // ascending
  std::map<int, bool> outbound;          // gs.outbound
  std::set<int> direct;                  // gs.direct
  std::map<int, std::set<int>> topics;   // p.topics (static subscriptions of peers)
  uint64_t mySubs = 0;                   // p.mySubs
  std::unordered_set<int64_t> seen;      // p.seenMessages (timecache, no expiry in-window; never iterated)
  std::set<int> dead;                    // neighbours whose connection is down (not in p.peers)
  // gossipsub router state — gossipsub.go:400-457
  std::map<int, std::set<int>> mesh, fanout;
  std::map<int, int64_t> lastpub;
  std::map<int, std::vector<IHaveEntry>> gossip;  // pending gossip (gs.gossip)
  std::map<int, int> peerhave, iasked;
  std::map<int, std::map<int, int64_t>> backoff;
  MessageCache mcache;
  PeerScore score;
  GossipTracer gtracer;
  uint64_t heartbeatTicks = 0;
  std::map<int, double> memo;            // S0: hop-start score snapshot
  std::map<int, std::vector<RPC>> out;   // RPCs sent during this hop, per destination
  std::map<int, int> acceptStatus;       // AcceptFrom result per sender this hop
  gs_counters ctr{};                     // this node's event counters (summed by gs_read_counters)
  PeerGater gater;                       // gs.gate (WithPeerGater), when sim->gaterOn
  GateSnap gsnap;
  int valUsed = 0;                       // validation-queue entries used this hop
  uint8_t behave = 0;                    // GS_BEHAVE_* bits
  // mixed networks (gs_set_routers / gs_set_graph_ex): this host's router and
  // the protocol.ID of each of its connections (gs.peers / rs.peers,
  // gossipsub.go:505-508, randomsub.go:48-51)
  int router = GS_ROUTER_GOSSIPSUB;
  std::map<int, int> proto;
  bool isGossip() const { return router == GS_ROUTER_GOSSIPSUB; }
  // gs.feature(GossipSubFeatureMesh / GossipSubFeaturePX, gs.peers[p]) (gossipsub_feat.go:27-38)
  bool meshCap(int p) const;
  bool pxCap(int p) const;
  bool scored() const;                   // a peerScore exists (WithPeerScore on a gossipsub host)
  bool gatered() const;                  // a peerGater exists (WithPeerGater on a gossipsub host)
  int acceptFrom(int s, uint32_t draw);  // AcceptFrom incl. the gater, per RPC
  std::vector<gs_trace_event> ev;        // this node's trace events (it is the tracing host)

  double Score(int p);                   // gs.score.Score (0 when scoring is off)
  void sendRPC(int p, RPC rpc);
  void localPublish(const Msg& m);
  void handleMessage(int from, const Msg& m);
  void routerPublish(const Msg& m, int from);
  void gsPublish(const Msg& m, int from);
  std::vector<int> getPeers(int topic, int count, int site, const std::function<bool(int)>& filter);
  void join(int topic);
  void handleRPC(int from, const RPC& in);
  std::vector<int64_t> handleIHave(int p, const Control& ctl);
  std::vector<int64_t> handleIWant(int p, const Control& ctl);
  std::vector<PruneEntry> handleGraft(int p, const Control& ctl);
  void handlePrune(int p, const Control& ctl);
  void addBackoff(int p, int topic);
  void doAddBackoff(int p, int topic, int64_t interval);
  PruneEntry makePrune(int p, int topic, bool doPX);
  void pxConnect(std::vector<int> px);   // gossipsub.go:856-905
  std::vector<int> pxReq;                // peers to dial (connected at the next hop's start)
  void directConnect();
  void heartbeat();
  void emitGossip(int topic, const std::set<int>& exclude);
  void removePeer(int p);                // handleDeadPeers + RemovePeer
  void addPeer(int p);                   // newPeerStream -> AddPeer + hello
  void leaveTopic(int topic);            // handleRemoveSubscription -> Leave
  void joinTopic(int topic);             // handleAddSubscription -> Join
  void applyIwantPenalties();
  void clearBackoff();
};

struct Sim {
  gs_config cfg{};
  gs_gossipsub_params gp{};
  gs_peer_score_params sp{};
  std::vector<gs_topic_score_params> tparams;
  std::vector<uint8_t> tscored;
  gs_peer_score_thresholds thr{};
  bool scoring = false, floodPublish = false, record = false;
  bool doPX = false;                                    // WithPeerExchange
  bool hasDirect = false;                               // some host has direct peers (the connector dials them)
  int64_t directInitHop = 0;                            // DirectConnectInitialDelay in hops
  std::set<std::pair<int, int>> dormant;               // gs_set_dormant: connections down at the start
  bool gaterOn = false;
  // Reference order (gs_oracle_reference_order): each RPC is
  // handled whole, in arrival order — AcceptFrom on the live score and gater,
  // its messages, then its control (pubsub.go:946-969) — and the Publish
  // filters read the live score.  Off: the engine's canonical schedule
  // (hop-start memo S0, every payload of the hop before any control).
  bool refOrder = false;
  bool liveScore = false;  // AcceptFrom / Publish filters on the live score (refOrder implies it)
  gs_peer_gater_params gaterParams{};
  std::vector<uint8_t> topicVal;   // RegisterTopicValidator per topic
  int32_t valQueue = 0;            // validation queue entries per node per hop (0 = unlimited)
  std::vector<uint8_t> behave;     // GS_BEHAVE_* per node
  // mixed networks: router per host (gs_set_routers, empty: cfg.router) and
  // protocol per connection (gs_set_graph_ex, empty: negotiated at start)
  std::vector<uint8_t> nodeRouter, protoE;
  bool mixed = false;              // some host or connection differs from cfg.router's own
  int validateMixed();             // the gs_set_routers / gs_set_graph_ex rules (gossip_engine.h)
  std::vector<uint8_t> msgKind;    // GS_MSG_* per message id
  // churn / subscription events (gs_schedule_events), by hop
  struct Event { int64_t hop; int32_t kind, a, b; };
  std::vector<Event> sched;
  size_t nextEvent = 0;
  struct Ann { int node, topic; bool sub; };
  std::vector<Ann> pendingAnn;     // subscription announcements arriving next hop
  int N = 0, T = 0;
  int64_t E = 0;
  std::vector<int64_t> rowptr;
  std::vector<int32_t> col;
  std::vector<uint8_t> outboundE, directE;
  std::vector<uint64_t> subs;
  std::vector<double> appScore;
  std::vector<uint32_t> ipv4;
  std::vector<std::pair<uint32_t, uint32_t>> whitelist;
  std::vector<Node> nodes;
  // gs_oracle_replay: one host simulated alone, its inbox taken from a trace
  // (nodes stays empty; its events go to its own buffer)
  Node* solo = nullptr;
  std::vector<gs_trace_event>& evbuf(int node) { return !nodes.empty() ? nodes[node].ev : solo ? solo->ev : events; }
  bool graphSet = false, started = false;
  bool mixedChecked = false;  // validateMixed() ran (it negotiates protoE once)
  int64_t hop = 0;
  // messages
  std::vector<Msg> msgs;           // by id
  std::vector<int64_t> msgHop;     // scheduled publish hop
  size_t nextPub = 0;
  std::vector<std::unordered_map<int64_t, std::pair<int32_t, int32_t>>> deliv;  // per node
  gs_counters ctr{};
  int64_t now() const { return hop * cfg.hop_ns; }
  // EventTracer (trace.go:61-499) of the hosts with traced[u] != 0
  std::vector<uint8_t> traced;
  std::vector<gs_trace_event> events;  // drained from the nodes' buffers by gs_trace_read
  bool traceRpc = false;               // gs_set_trace_rpc: RECV_RPC / SEND_RPC with their items
  // one RPC event of `node` and its traceRPCMeta items (gossip_engine.h);
  // subs: the RPC's subscriptions (topic, subscribe)
  void emitRpc(int type, int node, int peer, int phase, int64_t ord, const RPC* r,
               const std::vector<std::pair<int, int>>& subs = {});
  void traceHello(int node, int from);  // RECV of from's hello packet (pubsub.go:495)
  // RPC byte accounting (gs_set_rpc_accounting): RPC.Size() and count of every
  // RPC a host sends, per directed edge (the sender's row)
  bool acct = false;
  std::vector<int32_t> acctMsg, acctTl;
  int32_t acctId = 0;
  int32_t acctPid = 38, acctRec = 0;  // PX PeerInfo: peer id and signed record lengths
  std::vector<int64_t> rpcBytes, rpcCount;
  void account(int u, int p, int64_t bytes) {
    if (!acct) return;
    const int e = edgeIndex(u, p);
    rpcBytes[e] += bytes;  // edges of u: only u's own (parallel) node loop writes them
    rpcCount[e] += 1;
  }
  int64_t rpcSize(const RPC& r) const;    // pb/rpc.pb.go Size() of r
  int64_t helloSize(uint64_t subs) const;
  size_t traceRead = 0;
  // Events go to the tracing host's own buffer, so nodes run in parallel
  // (OpenMP over nodes in every per-node phase; the canonical event order
  // of gs_trace.h is keyed by host, so the merge order does not matter).
  void emit(int type, int node, int peer, int topic, int64_t msg, int phase, int reason = 0);
  gs_counters total() const;

  int edgeIndex(int u, int v) const {
    auto b = col.begin() + rowptr[u], e = col.begin() + rowptr[u + 1];
    auto it = std::lower_bound(b, e, v);
    if (it == e || *it != v) return -1;
    return (int)(it - col.begin());
  }
  bool heartbeatDue(int64_t t) const {
    if (cfg.router != GS_ROUTER_GOSSIPSUB) return false;
    if (t < gp.HeartbeatInitialDelay) return false;
    return (t - gp.HeartbeatInitialDelay) % gp.HeartbeatInterval == 0;
  }
  bool refreshDue(int64_t t) const { return scoring && t > 0 && t % sp.DecayInterval == 0; }
  bool gaterDecayDue(int64_t t) const { return gaterOn && t > 0 && t % gaterParams.DecayInterval == 0; }
  int kindOf(const Msg& m) const {  // verdict of m's topic validator (GS_MSG_VALID without one)
    const int k = msgKind[m.id];
    if (k == GS_MSG_PHANTOM) return k;
    return topicVal[m.topic] ? k : GS_MSG_VALID;
  }
  void start();
  void initNode(Node& nd, int u);  // start()'s per-host part: router state, AddPeer of every connection
  void step();
  // the per-host bodies of step()'s phases (also run alone by gs_oracle_replay)
  void nodeMemo(Node& nd, int64_t t);
  void nodePhaseA(Node& nd, const std::map<int, std::vector<RPC>>& in);
  void nodePhaseB(Node& nd, const std::map<int, std::vector<RPC>>& in);
  void nodeRefOrder(Node& nd, const std::map<int, std::vector<RPC>>& in);
  void applyEvents(std::vector<std::map<int, std::vector<RPC>>>& inbox);
  // RecvRPC (pubsub.go:903) of every RPC in node u's inbox: before AcceptFrom,
  // so graylisted and gated RPCs are traced too
  void traceRecv(int u, const std::map<int, std::vector<RPC>>& in) {
    if (!traceRpc || traced.empty() || !traced[u]) return;
    for (auto& kv : in)
      for (const RPC& r : kv.second)
        emitRpc(GS_TRACE_RECV_RPC, u, kv.first, r.publish.empty() ? 3 : 2, GS_RPC_ORD(r.sp, r.ord), &r);
  }
  void announce(int a, int topic, bool sub);
};

void Sim::emit(int type, int node, int peer, int topic, int64_t msg, int phase, int reason) {
  if (traced.empty() || !traced[node]) return;
  gs_trace_event e;
  e.hop = hop; e.msg = msg; e.type = type; e.node = node; e.peer = peer;
  e.topic = (int16_t)topic; e.phase = (uint8_t)phase; e.reason = (uint8_t)reason;
  evbuf(node).push_back(e);
}

void Sim::emitRpc(int type, int node, int peer, int phase, int64_t ord, const RPC* r,
                  const std::vector<std::pair<int, int>>& subs) {
  if (!traceRpc || traced.empty() || !traced[node]) return;
  std::vector<gs_trace_event>& buf = evbuf(node);
  buf.push_back(gs_trace_event{hop, ord, type, node, peer, -1, (uint8_t)phase, 0});
  auto item = [&](int kind, int topic, int64_t msg) {
    buf.push_back(gs_trace_event{hop, msg, GS_TRACE_RPC_ITEM, node, peer, (int16_t)topic, (uint8_t)phase, (uint8_t)kind});
  };
  if (r) {  // traceRPCMeta (trace.go:310-383)
    for (int64_t mid : r->publish) item(GS_RPC_ITEM_MSG, msgs[mid].topic, mid);
    if (r->hasCtl) {
      item(GS_RPC_ITEM_CTL, -1, -1);
      for (const IHaveEntry& ih : r->ctl.ihave)
        for (int64_t mid : ih.mids) item(GS_RPC_ITEM_IHAVE, ih.topic, mid);
      for (int64_t mid : r->ctl.iwant) item(GS_RPC_ITEM_IWANT, -1, mid);
      for (int t : r->ctl.graft) item(GS_RPC_ITEM_GRAFT, t, -1);
      for (const PruneEntry& pe : r->ctl.prune) {
        item(GS_RPC_ITEM_PRUNE, pe.topic, -1);
        for (int q : pe.px) item(GS_RPC_ITEM_PX, pe.topic, q);
      }
    }
  }
  for (auto& st : subs) item(GS_RPC_ITEM_SUB, st.first, st.second);
}

void Sim::traceHello(int node, int from) {
  if (!traceRpc || traced.empty() || !traced[node]) return;
  std::vector<std::pair<int, int>> items;
  const uint64_t m = !nodes.empty() ? nodes[from].mySubs : this->subs.empty() ? 0 : this->subs[from];
  for (int t = 0; t < T; ++t)
    if ((m >> t) & 1) items.push_back({t, 1});
  emitRpc(GS_TRACE_RECV_RPC, node, from, 0, GS_RPC_ORD(0, GS_RPC_O_HELLO), nullptr, items);
}

gs_counters Sim::total() const {
  gs_counters c = ctr;
  for (const Node& nd : nodes) {
    c.published += nd.ctr.published; c.deliveries += nd.ctr.deliveries; c.duplicates += nd.ctr.duplicates;
    c.transmissions += nd.ctr.transmissions; c.grafts_sent += nd.ctr.grafts_sent;
    c.prunes_sent += nd.ctr.prunes_sent; c.ihave_sent += nd.ctr.ihave_sent; c.iwant_sent += nd.ctr.iwant_sent;
    c.iwant_served += nd.ctr.iwant_served; c.promises_broken += nd.ctr.promises_broken;
    c.graylisted += nd.ctr.graylisted; c.rejected += nd.ctr.rejected; c.throttled += nd.ctr.throttled;
    c.gated += nd.ctr.gated;
  }
  return c;
}

// RPC.Size() (include/gs_rpcsize.h): publish entries, then the control message
// when the RPC carries one (rpcWithControl always does).
int64_t Sim::rpcSize(const RPC& r) const {
  int64_t s = 0;
  for (int64_t mid : r.publish) s += gs_pb_field(acctMsg[msgs[mid].topic]);
  if (r.hasCtl) {
    int64_t c = 0;
    for (const IHaveEntry& ih : r.ctl.ihave) c += gs_pb_field(gs_pb_ihave(acctTl[ih.topic], (int64_t)ih.mids.size(), acctId));
    if (!r.ctl.iwant.empty()) c += gs_pb_field(gs_pb_iwant((int64_t)r.ctl.iwant.size(), acctId));
    for (int t : r.ctl.graft) c += gs_pb_field(gs_pb_graft(acctTl[t]));
    for (const PruneEntry& pe : r.ctl.prune)
      c += gs_pb_field(pe.hasBackoff ? gs_pb_prune_px(acctTl[pe.topic], pe.backoff, (int64_t)pe.px.size(),
                                                      gs_pb_peerinfo(acctPid, acctRec))
                                     : gs_pb_prune_v10(acctTl[pe.topic]));
    s += gs_pb_field(c);
  }
  return s;
}
// getHelloPacket (pubsub.go:853-866 area): one SubOpts per subscribed topic
int64_t Sim::helloSize(uint64_t subs) const {
  int64_t s = 0;
  for (int t = 0; t < T; ++t)
    if ((subs >> t) & 1) s += gs_pb_field(gs_pb_subopts(acctTl[t]));
  return s;
}

bool Node::scored() const { return sim->scoring && isGossip(); }
// a single-router engine's connections all run the router's own protocol
bool Node::meshCap(int p) const {
  if (!sim->mixed) return true;
  auto it = proto.find(p);
  return it != proto.end() && it->second >= GS_PROTO_GOSSIPSUB_V10;
}
bool Node::pxCap(int p) const {
  if (!sim->mixed) return true;
  auto it = proto.find(p);
  return it != proto.end() && it->second == GS_PROTO_GOSSIPSUB_V11;
}
bool Node::gatered() const { return sim->gaterOn && isGossip(); }
double Node::Score(int p) { return scored() ? score.score(p) : 0.0; }

// sendRPC / doSendRPC — gossipsub.go:1092-1156 (queues never drop in the
// simulator; pending gossip is piggybacked exactly as sendRPC does).
void Node::sendRPC(int p, RPC rpc) {
  if ((behave & GS_BEHAVE_NO_FORWARD) && rpc.hasCtl) return;  // a squatter sends no control at all
  if (dead.count(p)) return;  // gossipsub.go:1101-1104: no outbound queue for p
  auto g = gossip.find(p);
  if (g != gossip.end()) {  // piggybackGossip gossipsub.go:1736-1744
    rpc.hasCtl = true;
    rpc.ctl.ihave = g->second;
    gossip.erase(g);
  }
  sim->account(id, p, sim->acct ? sim->rpcSize(rpc) : 0);
  sim->emitRpc(GS_TRACE_SEND_RPC, id, p, rpc.sp, GS_RPC_ORD(rpc.sp, rpc.ord), &rpc);  // gossipsub.go:1152
  ctr.grafts_sent += (int64_t)rpc.ctl.graft.size();
  ctr.prunes_sent += (int64_t)rpc.ctl.prune.size();
  ctr.ihave_sent += (int64_t)rpc.ctl.ihave.size();
  ctr.iwant_sent += (int64_t)rpc.ctl.iwant.size();
  out[p].push_back(std::move(rpc));
}

// getPeers — gossipsub.go:1841-1861 with the keyed shuffle (gs_rng.h).
std::vector<int> Node::getPeers(int topic, int count, int site, const std::function<bool(int)>& filter) {
  auto tm = topics.find(topic);
  if (tm == topics.end()) return {};
  std::vector<std::pair<uint64_t, int>> peers;
  for (int p : tm->second)  // mesh-capable peers only (gossipsub.go:1849)
    if (meshCap(p) && filter(p))
      peers.push_back({gs_key64(sim->cfg.seed, site, id, (uint32_t)sim->hop, p, topic), p});
  std::sort(peers.begin(), peers.end());
  std::vector<int> res;
  for (auto& kp : peers) res.push_back(kp.second);
  if (count > 0 && (int)res.size() > count) res.resize(count);
  return res;
}

// Join — gossipsub.go:1011-1060 (router); floodsub/randomsub Join only trace.
void Node::join(int topic) {
  if (!isGossip()) return;
  if (mesh.count(topic)) return;
  std::set<int> gmap;
  auto fo = fanout.find(topic);
  if (fo != fanout.end()) {
    gmap = fo->second;
    for (auto it = gmap.begin(); it != gmap.end();) {
      if (Score(*it) < 0) it = gmap.erase(it); else ++it;
    }
    if ((int)gmap.size() < sim->gp.D) {
      auto more = getPeers(topic, sim->gp.D - (int)gmap.size(), GS_SITE_GP_JOIN, [&](int p) {
        return !gmap.count(p) && !direct.count(p) && Score(p) >= 0;
      });
      for (int p : more) gmap.insert(p);
    }
    fanout.erase(topic);
    lastpub.erase(topic);
  } else {
    auto peers = getPeers(topic, sim->gp.D, GS_SITE_GP_JOIN, [&](int p) {
      return !direct.count(p) && Score(p) >= 0;
    });
    gmap.insert(peers.begin(), peers.end());
  }
  mesh[topic] = gmap;
  for (int p : gmap) {
    sim->emit(GS_TRACE_GRAFT, id, p, topic, -1, 0);        // tracer.Graft gossipsub.go:1057
    if (sim->scoring) score.Graft(p, topic, sim->now());  // tracer.Graft
    RPC r; r.hasCtl = true; r.ctl.graft.push_back(topic);  // sendGraft gossipsub.go:1080
    r.sp = 0; r.ord = topic;
    sendRPC(p, std::move(r));
  }
}

// Topic.Publish -> PushLocal -> validate(sync) -> markSeen -> publishMessage
// (topic.go:207-245, validation.go:216-226, pubsub.go:1056-1060).  Raw tracers
// skip self-originated messages (trace.go:89,101,132,162).
void Node::localPublish(const Msg& m) {
  if (sim->msgKind[m.id] == GS_MSG_PHANTOM) {
    // an advertised-only id: in the author's mcache (so emitGossip lists it)
    // and seen set, never sent (IHAVE spam, gossipsub_spam_test.go:196-203)
    seen.insert(m.id);
    if (isGossip()) mcache.Put(m);
    return;
  }
  sim->emit(GS_TRACE_PUBLISH_MESSAGE, id, -1, m.topic, m.id, 1);  // validation.go:217
  sim->emit(GS_TRACE_DELIVER_MESSAGE, id, id, m.topic, m.id, 1);  // pubsub.go:1057
  seen.insert(m.id);
  ctr.published++;
  if (sim->record) sim->deliv[id][m.id] = {(int32_t)sim->hop, -1};
  routerPublish(m, id);
}

// pushMsg — pubsub.go:978-1022, then the validation pipeline (validation.go:
// 230-351) with instantaneous validators: Push queues a message of a topic with
// a validator (dropped with RejectValidationQueueFull when this hop's queue
// entries are used up), validate() marks it seen, traces ValidateMessage and
// applies the verdict; an accepted message is published (publishMessage).
void Node::handleMessage(int from, const Msg& m) {
  if (!((mySubs >> m.topic) & 1)) return;  // subscribedToMsg / canRelayMsg (pubsub.go:959)
  const int64_t now = sim->now();
  if (m.from == id && from != id) {         // self-origin rejection (pubsub.go:1001-1006)
    if (scored()) score.RejectMessage(m, from, RejectSelfOrigin, now);
    if (gatered()) gater.RejectMessage(from, RejectSelfOrigin, now);
    return;
  }
  if (seen.count(m.id)) {                   // duplicate (pubsub.go:1010-1013)
    sim->emit(GS_TRACE_DUPLICATE_MESSAGE, id, from, m.topic, m.id, 2);
    ctr.duplicates++;
    if (scored()) score.DuplicateMessage(m, from, now);
    if (gatered()) gater.DuplicateMessage(from);
    return;
  }
  if (sim->topicVal[m.topic]) {             // val.Push: a validator applies (validation.go:230-243)
    if (sim->valQueue > 0 && valUsed >= sim->valQueue) {
      // RejectValidationQueueFull: not marked seen, a later copy may validate
      sim->emit(GS_TRACE_REJECT_MESSAGE, id, from, m.topic, m.id, 2, GS_REJECT_QUEUE_FULL);
      ctr.throttled++;
      if (scored()) gtracer.RejectMessage(m.id, RejectValidationQueueFull);  // peerScore ignores it
      if (gatered()) gater.RejectMessage(from, RejectValidationQueueFull, now);
      return;
    }
    valUsed++;
    seen.insert(m.id);                      // validate(): markSeen, then ValidateMessage
    if (scored()) { score.ValidateMessage(m, now); gtracer.ValidateMessage(m.id); }
    if (gatered()) gater.ValidateMessage();
    const int kind = sim->kindOf(m);
    if (kind == GS_MSG_REJECT || kind == GS_MSG_IGNORE) {  // validation.go:331-336, 349-352
      const int reason = kind == GS_MSG_REJECT ? RejectValidationFailed : RejectValidationIgnored;
      sim->emit(GS_TRACE_REJECT_MESSAGE, id, from, m.topic, m.id, 2,
                kind == GS_MSG_REJECT ? GS_REJECT_VALIDATION_FAILED : GS_REJECT_VALIDATION_IGNORED);
      ctr.rejected++;
      if (scored()) { score.RejectMessage(m, from, reason, now); gtracer.RejectMessage(m.id, reason); }
      if (gatered()) gater.RejectMessage(from, reason, now);
      return;
    }
  } else {
    seen.insert(m.id);                      // markSeen
  }
  sim->emit(GS_TRACE_DELIVER_MESSAGE, id, from, m.topic, m.id, 2);
  ctr.deliveries++;
  if (sim->record) sim->deliv[id][m.id] = {(int32_t)sim->hop, from};
  if (scored()) {                       // tracer.DeliverMessage -> raw tracers
    score.DeliverMessage(m, from, now);
    gtracer.DeliverMessage(m.id);
  }
  if (gatered()) gater.DeliverMessage(from);
  if (behave & GS_BEHAVE_NO_FORWARD) return;  // a squatter relays nothing
  routerPublish(m, from);
}

// AcceptFrom — gossipsub.go:578-589, then peerGater.AcceptFrom (peer_gater.go:
// 320-363) on the hop-start snapshot; `draw` names the RPC (the message id of a
// payload RPC, 0xFFFFFFFF for the sender's control RPCs of this hop).
int Node::acceptFrom(int s, uint32_t draw) {
  if (!isGossip()) return PeerGater::AcceptAll;  // floodsub.go:68, randomsub.go:91
  if (direct.count(s)) return PeerGater::AcceptAll;
  if (sim->liveScore) {  // gossipsub.go:578-589 on the live score, then peer_gater.go:320-363 live
    if (scored() && Score(s) < sim->thr.GraylistThreshold) return PeerGater::AcceptNone;
    if (!gatered()) return PeerGater::AcceptAll;
    const double u = gs_key_to_unit(gs_key64(sim->cfg.seed, GS_SITE_GATER, id, s, (uint32_t)sim->hop, draw));
    return gater.AcceptFrom(s, sim->now(), u);
  }
  if (scored() && memo[s] < sim->thr.GraylistThreshold) return PeerGater::AcceptNone;
  if (!gatered() || !gsnap.active) return PeerGater::AcceptAll;
  auto it = gsnap.thr.find(s);
  if (it == gsnap.thr.end()) return PeerGater::AcceptAll;  // total == 0
  const double u = gs_key_to_unit(gs_key64(sim->cfg.seed, GS_SITE_GATER, id, s, (uint32_t)sim->hop, draw));
  return u < it->second ? PeerGater::AcceptAll : PeerGater::AcceptControl;
}

void Node::routerPublish(const Msg& m, int from) {
  if (router == GS_ROUTER_FLOODSUB) {  // FloodSubRouter.Publish floodsub.go:76-100
    auto tm = topics.find(m.topic);
    if (tm == topics.end()) return;
    for (int pid : tm->second) {
      if (pid == from || pid == m.from) continue;
      RPC r; r.publish.push_back(m.id);
      r.sp = from == id ? 1 : 2; r.ord = m.id;
      sendRPC(pid, std::move(r));
    }
    return;
  }
  if (router == GS_ROUTER_RANDOMSUB) {  // RandomSubRouter.Publish randomsub.go:99-160
    auto tm = topics.find(m.topic);
    if (tm == topics.end()) return;
    std::set<int> tosend;
    std::vector<int> rspeers;
    for (int p : tm->second) {
      if (p == from || p == m.from) continue;
      if (sim->mixed && proto[p] == GS_PROTO_FLOODSUB) tosend.insert(p);  // floodsub peers: always (randomsub.go:117-118)
      else rspeers.push_back(p);
    }
    const int RandomSubD = 6;  // randomsub.go:17
    if ((int)rspeers.size() > RandomSubD) {
      int target = RandomSubD;
      int sq = (int)std::ceil(std::sqrt((double)sim->cfg.randomsub_size));
      if (sq > target) target = sq;
      if (target > (int)rspeers.size()) target = (int)rspeers.size();
      std::vector<std::pair<uint64_t, int>> keyed;
      for (int p : rspeers)
        keyed.push_back({gs_key64(sim->cfg.seed, GS_SITE_RANDOMSUB, id, (uint32_t)m.id, p, 0), p});
      std::sort(keyed.begin(), keyed.end());
      for (int i = 0; i < target; ++i) tosend.insert(keyed[i].second);
    } else {
      tosend.insert(rspeers.begin(), rspeers.end());
    }
    for (int p : tosend) {
      RPC r; r.publish.push_back(m.id);
      r.sp = from == id ? 1 : 2; r.ord = m.id;
      sendRPC(p, std::move(r));
    }
    return;
  }
  gsPublish(m, from);
}

// GossipSubRouter.Publish — gossipsub.go:939-1009.  Score filters read the
// hop-start memo S0 (forwarding decisions inside a hop).
void Node::gsPublish(const Msg& m, int from) {
  mcache.Put(m);
  int topic = m.topic;
  std::set<int> tosend;
  auto tm = topics.find(topic);
  if (tm == topics.end()) return;
  auto s0 = [&](int p) { return scored() ? (sim->liveScore ? Score(p) : memo[p]) : 0.0; };
  if (sim->floodPublish && from == id) {
    for (int p : tm->second)
      if (direct.count(p) || s0(p) >= sim->thr.PublishThreshold) tosend.insert(p);
  } else {
    for (int p : direct)
      if (tm->second.count(p)) tosend.insert(p);
    // floodsub peers (gossipsub.go:969-975): not mesh-capable, score >= publishThreshold
    for (int p : tm->second)
      if (!meshCap(p) && s0(p) >= sim->thr.PublishThreshold) tosend.insert(p);
    auto gm = mesh.find(topic);
    std::set<int> gmap;
    if (gm == mesh.end()) {
      auto fo = fanout.find(topic);
      if (fo == fanout.end() || fo->second.empty()) {
        auto peers = getPeers(topic, sim->gp.D, GS_SITE_GP_FANOUT_PUB, [&](int p) {
          return !direct.count(p) && s0(p) >= sim->thr.PublishThreshold;
        });
        if (!peers.empty()) fanout[topic] = std::set<int>(peers.begin(), peers.end());
      }
      fo = fanout.find(topic);
      if (fo != fanout.end()) gmap = fo->second;
      lastpub[topic] = sim->now();
    } else {
      gmap = gm->second;
    }
    tosend.insert(gmap.begin(), gmap.end());
  }
  for (int pid : tosend) {
    if (pid == from || pid == m.from) continue;
    RPC r; r.publish.push_back(m.id);
    r.sp = from == id ? 1 : 2; r.ord = m.id;
    sendRPC(pid, std::move(r));
  }
}

// HandleRPC — gossipsub.go:591-608 (one call per control-carrying RPC).
void Node::handleRPC(int from, const RPC& in) {
  const Control& ctl = in.ctl;
  auto iwant = handleIHave(from, ctl);
  auto ihave = handleIWant(from, ctl);
  auto prune = handleGraft(from, ctl);
  handlePrune(from, ctl);
  if (iwant.empty() && ihave.empty() && prune.empty()) return;
  RPC r;
  r.hasCtl = true;
  r.publish = ihave;
  if (!iwant.empty()) r.ctl.iwant = iwant;
  r.ctl.prune = prune;
  ctr.iwant_served += (int64_t)ihave.size();
  // the reply's ordinal names the RPC it answers (include/gs_trace.h)
  r.sp = 3;
  r.ord = in.sp == 0 ? in.ord : in.sp == 2 ? GS_RPC_O_ANS_SPAM : in.sp == 3 ? GS_RPC_O_ANS_REPLY : GS_RPC_O_ANS_HB;
  sendRPC(from, std::move(r));
}

// handleIHave — gossipsub.go:610-672.  The iwant set is shuffled by key
// (GS_SITE_IWANT) and the promise taken on the first element (the uniform
// rand.Intn(len) pick of gossip_tracer.go:53 on a uniformly shuffled list).
std::vector<int64_t> Node::handleIHave(int p, const Control& ctl) {
  double sc = Score(p);
  if (sc < sim->thr.GossipThreshold) return {};
  peerhave[p]++;
  if (peerhave[p] > sim->gp.MaxIHaveMessages) return {};
  if (iasked[p] >= sim->gp.MaxIHaveLength) return {};
  std::set<int64_t> iwant;
  for (const IHaveEntry& ih : ctl.ihave) {
    if (!mesh.count(ih.topic)) continue;
    for (int64_t mid : ih.mids) {
      if (seen.count(mid)) continue;
      iwant.insert(mid);
    }
  }
  if (iwant.empty()) return {};
  int iask = (int)iwant.size();
  if (iask + iasked[p] > sim->gp.MaxIHaveLength) iask = sim->gp.MaxIHaveLength - iasked[p];
  std::vector<std::pair<uint64_t, int64_t>> keyed;
  for (int64_t mid : iwant)
    keyed.push_back({gs_key64_mid(sim->cfg.seed, GS_SITE_IWANT, id, p, (uint32_t)mid, (uint32_t)sim->hop), mid});
  std::sort(keyed.begin(), keyed.end());
  std::vector<int64_t> lst;
  for (int i = 0; i < iask; ++i) lst.push_back(keyed[i].second);
  iasked[p] += iask;
  if (sim->scoring) gtracer.AddPromise(p, lst, 0, sim->now());
  return lst;
}

// handleIWant — gossipsub.go:674-711 (served in ascending message id).
std::vector<int64_t> Node::handleIWant(int p, const Control& ctl) {
  double sc = Score(p);
  if (sc < sim->thr.GossipThreshold) return {};
  if (behave & GS_BEHAVE_NO_FORWARD) return {};  // a squatter serves nothing
  std::set<int64_t> ihave;
  for (int64_t mid : ctl.iwant) {
    if (sim->msgKind[mid] == GS_MSG_PHANTOM) continue;  // advertised, never served
    int count = 0;
    if (!mcache.GetForPeer(mid, p, nullptr, &count)) continue;
    if (count > sim->gp.GossipRetransmission) continue;
    ihave.insert(mid);
  }
  return std::vector<int64_t>(ihave.begin(), ihave.end());
}

// handleGraft — gossipsub.go:713-804 (no PX records are produced: doPX off).
std::vector<PruneEntry> Node::handleGraft(int p, const Control& ctl) {
  std::vector<int> prune;
  double sc = Score(p);
  int64_t now = sim->now();
  bool doPX = sim->doPX;  // cleared by any GRAFT of the RPC that must not leak peers (:716-775)
  for (int topic : ctl.graft) {
    auto pm = mesh.find(topic);
    if (pm == mesh.end()) { doPX = false; continue; }
    std::set<int>& peers = pm->second;
    if (peers.count(p)) continue;
    if (direct.count(p)) { prune.push_back(topic); doPX = false; continue; }
    auto bt = backoff.find(topic);
    if (bt != backoff.end()) {
      auto be = bt->second.find(p);
      if (be != bt->second.end() && now < be->second) {
        if (sim->scoring) score.AddPenalty(p, 1);
        doPX = false;
        int64_t floodCutoff = be->second + (sim->gp.GraftFloodThreshold - sim->gp.PruneBackoff);
        if (now < floodCutoff && sim->scoring) score.AddPenalty(p, 1);
        addBackoff(p, topic);
        prune.push_back(topic);
        continue;
      }
    }
    if (sc < 0) { prune.push_back(topic); doPX = false; addBackoff(p, topic); continue; }
    if ((int)peers.size() >= sim->gp.Dhi && !outbound[p]) {
      prune.push_back(topic);
      addBackoff(p, topic);
      continue;
    }
    sim->emit(GS_TRACE_GRAFT, id, p, topic, -1, 3);  // gossipsub.go:790
    if (sim->scoring) score.Graft(p, topic, now);
    peers.insert(p);
  }
  std::vector<PruneEntry> res;
  for (int t : prune) res.push_back(makePrune(p, t, doPX));
  return res;
}

// handlePrune — gossipsub.go:806-838 (PX ignored: no peer records).
void Node::handlePrune(int p, const Control& ctl) {
  if (ctl.prune.empty()) return;
  const double sc = Score(p);  // :807, before any of the RPC's prunes
  for (const PruneEntry& pr : ctl.prune) {
    auto pm = mesh.find(pr.topic);
    if (pm == mesh.end()) continue;
    sim->emit(GS_TRACE_PRUNE, id, p, pr.topic, -1, 3);  // gossipsub.go:817
    if (sim->scoring) score.Prune(p, pr.topic);
    pm->second.erase(p);
    if (pr.hasBackoff && pr.backoff > 0)
      doAddBackoff(p, pr.topic, (int64_t)pr.backoff * kSecond);
    else
      addBackoff(p, pr.topic);
    // PX from peers with insufficient score is ignored (:827-836)
    if (!pr.px.empty() && !(sc < sim->thr.AcceptPXThreshold)) pxConnect(pr.px);
  }
}

// pxConnect — gossipsub.go:856-905: at most PrunePeers suggestions (shuffled
// then truncated), the ones not connected yet are dialled.  A dial needs a slot
// in the simulated graph (a connection that is down); it completes at the
// start of the next hop (the connector goroutine, :907-937).
void Node::pxConnect(std::vector<int> px) {
  if ((int)px.size() > sim->gp.PrunePeers) {
    std::vector<std::pair<uint64_t, int>> keyed;
    for (int q : px) keyed.push_back({gs_key64(sim->cfg.seed, GS_SITE_PX_CONNECT, id, (uint32_t)sim->hop, q, 0), q});
    std::sort(keyed.begin(), keyed.end());
    px.clear();
    for (int i = 0; i < sim->gp.PrunePeers; ++i) px.push_back(keyed[i].second);
  }
  for (int q : px) {
    if (q == id || sim->edgeIndex(id, q) < 0) continue;  // no slot for this connection
    if (!dead.count(q)) continue;                        // connected already
    pxReq.push_back(q);
  }
}

void Node::addBackoff(int p, int topic) { doAddBackoff(p, topic, sim->gp.PruneBackoff); }  // :840
void Node::doAddBackoff(int p, int topic, int64_t interval) {  // :844-854
  auto& b = backoff[topic];
  int64_t expire = sim->now() + interval;
  auto it = b.find(p);
  int64_t cur = it == b.end() ? kTimeZero : it->second;
  if (cur < expire) b[p] = expire;
}
// makePrune — gossipsub.go:1803-1839 (v1.1 peers: backoff in whole seconds;
// with PX, up to PrunePeers other topic peers of non-negative score)
PruneEntry Node::makePrune(int p, int topic, bool doPX) {
  PruneEntry e;
  e.topic = topic;
  if (!pxCap(p)) {  // gossipsub v1.0 peer: neither PX nor a backoff (gossipsub.go:1804-1807)
    e.hasBackoff = false;
    e.backoff = 0;
    return e;
  }
  e.hasBackoff = true;
  e.backoff = (uint64_t)(sim->gp.PruneBackoff / kSecond);
  if (doPX) {  // getPeers(topic, PrunePeers, xp != p && Score(xp) >= 0), its own shuffle per PRUNE
    auto tm = topics.find(topic);
    std::vector<std::pair<uint64_t, int>> keyed;
    if (tm != topics.end())
      for (int xp : tm->second)
        if (meshCap(xp) && xp != p && Score(xp) >= 0)  // getPeers' mesh filter (:1849)
          keyed.push_back({gs_key64(sim->cfg.seed, GS_SITE_PX, id, (uint32_t)sim->hop, xp,
                                    ((uint32_t)p << 6) | (uint32_t)topic), xp});
    std::sort(keyed.begin(), keyed.end());
    for (size_t i = 0; i < keyed.size() && (int)i < sim->gp.PrunePeers; ++i) e.px.push_back(keyed[i].second);
  }
  return e;
}

// clearBackoff — gossipsub.go:1573-1592 (slack uses the package var, 1s)
void Node::clearBackoff() {
  if (heartbeatTicks % 15 != 0) return;
  int64_t now = sim->now();
  for (auto it = backoff.begin(); it != backoff.end();) {
    for (auto jt = it->second.begin(); jt != it->second.end();) {
      if (jt->second + 2 * kSecond < now) jt = it->second.erase(jt); else ++jt;
    }
    if (it->second.empty()) it = backoff.erase(it); else ++it;
  }
}

void Node::applyIwantPenalties() {  // gossipsub.go:1566-1571
  if (!sim->scoring) return;
  auto broken = gtracer.GetBrokenPromises(sim->now());
  for (auto& kv : broken) {
    score.AddPenalty(kv.first, kv.second);
    ctr.promises_broken += kv.second;
  }
}

// emitGossip — gossipsub.go:1658-1712
void Node::emitGossip(int topic, const std::set<int>& exclude) {
  if (behave & GS_BEHAVE_NO_FORWARD) return;  // a squatter emits no gossip
  std::vector<int64_t> mids = mcache.GetGossipIDs(topic);
  if (mids.empty()) return;
  const bool spam = (behave & GS_BEHAVE_IHAVE_SPAM) != 0;  // IHAVE to every topic peer
  std::vector<int> peers;
  auto tm = topics.find(topic);
  if (tm != topics.end())
    for (int p : tm->second)
      if (meshCap(p) && (spam || (!exclude.count(p) && !direct.count(p) && Score(p) >= sim->thr.GossipThreshold)))
        peers.push_back(p);
  int target = sim->gp.Dlazy;
  int factor = (int)(sim->gp.GossipFactor * (double)peers.size());
  if (factor > target) target = factor;
  if (spam) target = (int)peers.size();
  if (target >= (int)peers.size()) {
    target = (int)peers.size();
  } else {
    std::vector<std::pair<uint64_t, int>> keyed;
    for (int p : peers)
      keyed.push_back({gs_key64(sim->cfg.seed, GS_SITE_EMIT_PEERS, id, (uint32_t)sim->hop, p, topic), p});
    std::sort(keyed.begin(), keyed.end());
    peers.clear();
    for (auto& kp : keyed) peers.push_back(kp.second);
  }
  peers.resize(target);
  std::sort(mids.begin(), mids.end());  // the IHAVE payload is a set of ids
  for (int p : peers) {
    IHaveEntry e;
    e.topic = topic;
    if ((int)mids.size() > sim->gp.MaxIHaveLength) {
      std::vector<std::pair<uint64_t, int64_t>> keyed;
      for (int64_t mid : mids)
        keyed.push_back({gs_key64_mid(sim->cfg.seed, GS_SITE_EMIT_MIDS, id, p, (uint32_t)mid, (uint32_t)sim->hop), mid});
      std::sort(keyed.begin(), keyed.end());
      for (int i = 0; i < sim->gp.MaxIHaveLength; ++i) e.mids.push_back(keyed[i].second);
    } else {
      e.mids = mids;
    }
    gossip[p].push_back(std::move(e));  // enqueueGossip
  }
}

// directConnect — gossipsub.go:1594-1616 (and the initial dial of :492-502):
// every direct peer that is not connected is dialled; the connector's dials
// complete at the next hop's start (Sim::applyEvents).
void Node::directConnect() {
  for (int p : direct)
    if (dead.count(p)) pxReq.push_back(p);
}

// heartbeat — gossipsub.go:1299-1552
void Node::heartbeat() {
  const gs_gossipsub_params& gp = sim->gp;
  const int64_t now = sim->now();
  const uint32_t hopw = (uint32_t)sim->hop;
  heartbeatTicks++;
  std::map<int, std::vector<int>> tograft, toprune;
  std::map<int, bool> noPX;
  clearBackoff();
  peerhave.clear();  // clearIHaveCounters
  iasked.clear();
  applyIwantPenalties();
  if (heartbeatTicks % gp.DirectConnectTicks == 0) directConnect();
  std::map<int, double> scores;  // score memo
  auto score = [&](int p) {
    auto it = scores.find(p);
    if (it != scores.end()) return it->second;
    double s = Score(p);
    scores[p] = s;
    return s;
  };
  for (auto& mt : mesh) {
    const int topic = mt.first;
    std::set<int>& peers = mt.second;
    auto prunePeer = [&](int p) {
      sim->emit(GS_TRACE_PRUNE, id, p, topic, -1, 4);  // gossipsub.go:1334
      if (sim->scoring) this->score.Prune(p, topic);
      peers.erase(p);
      addBackoff(p, topic);
      toprune[p].push_back(topic);
    };
    auto graftPeer = [&](int p) {
      sim->emit(GS_TRACE_GRAFT, id, p, topic, -1, 4);  // gossipsub.go:1343
      if (sim->scoring) this->score.Graft(p, topic, now);
      peers.insert(p);
      tograft[p].push_back(topic);
    };
    // drop all peers with negative score, without PX
    std::vector<int> cur(peers.begin(), peers.end());
    for (int p : cur)
      if (score(p) < 0) { prunePeer(p); noPX[p] = true; }
    // a GRAFT spammer first leaves the mesh (PRUNE with backoff), then re-GRAFTs
    // during the backoff (gossipsub_spam_test.go:428-446)
    if ((behave & GS_BEHAVE_GRAFT_SPAM) && heartbeatTicks == 1) {
      std::vector<int> all(peers.begin(), peers.end());
      for (int p : all) prunePeer(p);
    }
    // do we have enough peers?
    if ((int)peers.size() < gp.Dlo) {
      auto& bo = backoff[topic];
      int ineed = gp.D - (int)peers.size();
      auto plst = getPeers(topic, ineed, GS_SITE_GP_DLO, [&](int p) {
        return !peers.count(p) && !bo.count(p) && !direct.count(p) && score(p) >= 0;
      });
      for (int p : plst) graftPeer(p);
      if (bo.empty()) backoff.erase(topic);
    }
    // do we have too many peers?
    if ((int)peers.size() > gp.Dhi) {
      // shuffle then sort by score desc == sort by (score desc, key asc)
      std::vector<std::pair<double, std::pair<uint64_t, int>>> ks;
      for (int p : peers)
        ks.push_back({score(p), {gs_key64(sim->cfg.seed, GS_SITE_DHI_SHUFFLE, id, hopw, p, topic), p}});
      std::sort(ks.begin(), ks.end(), [](const auto& a, const auto& b) {
        if (a.first != b.first) return a.first > b.first;
        return a.second < b.second;
      });
      std::vector<int> plst;
      for (auto& k : ks) plst.push_back(k.second.second);
      // shuffle the tail [Dscore:]
      {
        std::vector<std::pair<uint64_t, int>> tail;
        for (size_t i = gp.Dscore; i < plst.size(); ++i)
          tail.push_back({gs_key64(sim->cfg.seed, GS_SITE_DHI_TAIL, id, hopw, plst[i], topic), plst[i]});
        std::sort(tail.begin(), tail.end());
        for (size_t i = 0; i < tail.size(); ++i) plst[gp.Dscore + i] = tail[i].second;
      }
      int outb = 0;
      for (int i = 0; i < gp.D; ++i) if (outbound[plst[i]]) outb++;
      if (outb < gp.Dout) {
        auto rotate = [&](int i) {
          int p = plst[i];
          for (int j = i; j > 0; --j) plst[j] = plst[j - 1];
          plst[0] = p;
        };
        if (outb > 0) {
          int ih = outb;
          for (int i = 1; i < gp.D && ih > 0; ++i)
            if (outbound[plst[i]]) { rotate(i); ih--; }
        }
        int ineed = gp.Dout - outb;
        for (int i = gp.D; i < (int)plst.size() && ineed > 0; ++i)
          if (outbound[plst[i]]) { rotate(i); ineed--; }
      }
      for (size_t i = gp.D; i < plst.size(); ++i) prunePeer(plst[i]);
    }
    // do we have enough outbound peers?
    if ((int)peers.size() >= gp.Dlo) {
      int outb = 0;
      for (int p : peers) if (outbound[p]) outb++;
      if (outb < gp.Dout) {
        int ineed = gp.Dout - outb;
        auto& bo = backoff[topic];
        auto plst = getPeers(topic, ineed, GS_SITE_GP_DOUT, [&](int p) {
          return !peers.count(p) && !bo.count(p) && !direct.count(p) && outbound[p] && score(p) >= 0;
        });
        for (int p : plst) graftPeer(p);
        if (bo.empty()) backoff.erase(topic);
      }
    }
    // opportunistic grafting
    if (heartbeatTicks % gp.OpportunisticGraftTicks == 0 && peers.size() > 1) {
      std::vector<double> sc;
      for (int p : peers) sc.push_back(score(p));
      std::sort(sc.begin(), sc.end());
      double medianScore = sc[peers.size() / 2];
      if (medianScore < sim->thr.OpportunisticGraftThreshold) {
        auto& bo = backoff[topic];
        auto plst = getPeers(topic, gp.OpportunisticGraftPeers, GS_SITE_GP_OPPORTUNISTIC, [&](int p) {
          return !peers.count(p) && !bo.count(p) && !direct.count(p) && score(p) > medianScore;
        });
        for (int p : plst) graftPeer(p);
        if (bo.empty()) backoff.erase(topic);
      }
    }
    if ((behave & GS_BEHAVE_GRAFT_SPAM) && heartbeatTicks > 1) {
      // GRAFT during backoff (gossipsub_spam_test.go:428-500): every topic peer we
      // are in backoff with gets a GRAFT; our own mesh is left as it is
      auto bt = backoff.find(topic);
      auto tm = topics.find(topic);
      if (bt != backoff.end() && tm != topics.end())
        for (auto& be : bt->second)
          if (be.second > now && !peers.count(be.first) && tm->second.count(be.first))
            tograft[be.first].push_back(topic);
    }
    emitGossip(topic, peers);
  }
  // expire fanout for topics we haven't published to in a while
  for (auto it = lastpub.begin(); it != lastpub.end();) {
    if (it->second + gp.FanoutTTL < now) {
      fanout.erase(it->first);
      it = lastpub.erase(it);
    } else {
      ++it;
    }
  }
  // maintain our fanout for topics we are publishing but we have not joined
  for (auto& ft : fanout) {
    const int topic = ft.first;
    std::set<int>& peers = ft.second;
    for (auto it = peers.begin(); it != peers.end();) {
      bool inTopic = topics.count(topic) && topics[topic].count(*it);
      if (!inTopic || score(*it) < sim->thr.PublishThreshold) it = peers.erase(it); else ++it;
    }
    if ((int)peers.size() < gp.D) {
      int ineed = gp.D - (int)peers.size();
      auto plst = getPeers(topic, ineed, GS_SITE_GP_FANOUT_HB, [&](int p) {
        return !peers.count(p) && !direct.count(p) && score(p) >= sim->thr.PublishThreshold;
      });
      for (int p : plst) peers.insert(p);
    }
    emitGossip(topic, peers);
  }
  // sendGraftPrune — gossipsub.go:1618-1654
  for (auto& kv : tograft) {
    int p = kv.first;
    RPC r;
    r.hasCtl = true;
    r.ctl.graft = kv.second;
    auto pr = toprune.find(p);
    if (pr != toprune.end()) {
      for (int topic : pr->second) r.ctl.prune.push_back(makePrune(p, topic, sim->doPX && !noPX[p]));
      toprune.erase(pr);
    }
    r.sp = 4;
    sendRPC(p, std::move(r));
  }
  for (auto& kv : toprune) {
    RPC r;
    r.hasCtl = true;
    for (int topic : kv.second) r.ctl.prune.push_back(makePrune(kv.first, topic, sim->doPX && !noPX[kv.first]));
    r.sp = 4;
    sendRPC(kv.first, std::move(r));
  }
  // flush — gossipsub.go:1714-1728
  std::vector<int> gpeers;
  for (auto& kv : gossip) gpeers.push_back(kv.first);
  for (int p : gpeers) {
    RPC r;
    r.hasCtl = true;
    r.sp = 4;
    sendRPC(p, std::move(r));  // sendRPC piggybacks the pending IHAVE
  }
  mcache.Shift();
}

// handleDeadPeers (pubsub.go:521-551): the peer leaves every topic map, then
// GossipSubRouter.RemovePeer (gossipsub.go:534-547) with tracer.RemovePeer
// (trace.go:215) -> peerScore.RemovePeer (score.go:602-635), peerGater.RemovePeer.
void Node::removePeer(int p) {
  if (dead.count(p)) return;
  dead.insert(p);
  for (auto& kv : topics) kv.second.erase(p);
  sim->emit(GS_TRACE_REMOVE_PEER, id, p, -1, -1, 0);
  for (auto& kv : mesh) kv.second.erase(p);
  for (auto& kv : fanout) kv.second.erase(p);
  gossip.erase(p);
  if (scored()) score.RemovePeer(p, sim->now());
  if (gatered()) gater.RemovePeer(p, sim->now());
}

// A new stream from p (pubsub.go:499-515): AddPeer (gossipsub.go:505-532,
// tracer.AddPeer -> peerScore.AddPeer score.go:586-600, peerGater.AddPeer);
// the hello packet's subscriptions (pubsub.go:495-497) are applied at once.
void Node::addPeer(int p) {
  if (!dead.count(p)) return;
  dead.erase(p);
  sim->emit(GS_TRACE_ADD_PEER, id, p, -1, -1, 0, sim->mixed ? proto[p] : 0);
  const int64_t e = sim->edgeIndex(id, p);
  outbound[p] = sim->outboundE.empty() ? false : sim->outboundE[e] != 0;
  if (scored()) {
    std::vector<uint32_t> ips;
    if (!sim->ipv4.empty() && sim->ipv4[p] != 0) ips.push_back(sim->ipv4[p]);
    score.AddPeer(p, ips);
  }
  if (gatered()) gater.AddPeer(p);
  for (int t = 0; t < sim->T; ++t)
    if ((sim->nodes[p].mySubs >> t) & 1) topics[t].insert(p);
}

// handleRemoveSubscription (pubsub.go:665-686): announce(topic, false), then
// the router's Leave: gossipsub.go:1062-1078 (tracer.Leave, PRUNE to every mesh
// peer), floodsub.go:106-108, randomsub.go:166-168 (which traces a Join).
void Node::leaveTopic(int topic) {
  const uint64_t bit = 1ull << topic;
  if (!(mySubs & bit)) return;
  mySubs &= ~bit;
  if (router == GS_ROUTER_RANDOMSUB) { sim->emit(GS_TRACE_JOIN, id, -1, topic, -1, 0); return; }
  if (router == GS_ROUTER_FLOODSUB) { sim->emit(GS_TRACE_LEAVE, id, -1, topic, -1, 0); return; }
  auto gm = mesh.find(topic);
  if (gm == mesh.end()) return;
  sim->emit(GS_TRACE_LEAVE, id, -1, topic, -1, 0);
  std::set<int> gmap = gm->second;
  mesh.erase(gm);
  for (int p : gmap) {
    sim->emit(GS_TRACE_PRUNE, id, p, topic, -1, 0);  // tracer.Prune (gossipsub.go:1075)
    if (scored()) score.Prune(p, topic);
    RPC r;  // sendPrune (gossipsub.go:1093-1097)
    r.hasCtl = true;
    r.ctl.prune.push_back(makePrune(p, topic, sim->doPX));  // sendPrune: gs.doPX (:1087)
    r.sp = 0; r.ord = GS_RPC_O_LEAVE + topic;
    sendRPC(p, std::move(r));
  }
}

// handleAddSubscription (pubsub.go:692-713): announce(topic, true), then Join.
void Node::joinTopic(int topic) {
  const uint64_t bit = 1ull << topic;
  if (mySubs & bit) return;
  mySubs |= bit;
  sim->emit(GS_TRACE_JOIN, id, -1, topic, -1, 0);  // tracer.Join gossipsub.go:1018, floodsub.go:103
  join(topic);
}

// The events of this hop, at its start: first the subscription announcements
// sent during the previous hop reach the peers that are still connected
// (handleIncomingRPC processes subscriptions first, pubsub.go:915-941), then
// the scheduled events: every disconnect, every connect, every leave, every
// join (canonical order); disconnects and connects in schedule order, leaves
// and joins by (node, topic).  A lost connection drops what was in flight.
// announce (pubsub.go:775-792): one SubOpts RPC to every connected peer
void Sim::announce(int a, int topic, bool sub) {
  for (int p : nodes[a].nbrs)
    if (!nodes[a].dead.count(p)) {
      if (acct) account(a, p, gs_pb_field(gs_pb_subopts(acctTl[topic])));
      emitRpc(GS_TRACE_SEND_RPC, a, p, 0, GS_RPC_ORD(0, GS_RPC_O_ANNOUNCE + topic), nullptr,
              {{topic, sub ? 1 : 0}});  // pubsub.go:785
    }
}

void Sim::applyEvents(std::vector<std::map<int, std::vector<RPC>>>& inbox) {
  for (const Ann& an : pendingAnn)
    for (int p : nodes[an.node].nbrs) {
      Node& np = nodes[p];
      if (np.dead.count(an.node)) continue;
      if (an.sub) np.topics[an.topic].insert(an.node); else np.topics[an.topic].erase(an.node);
      emitRpc(GS_TRACE_RECV_RPC, p, an.node, 0, GS_RPC_ORD(0, GS_RPC_O_ANNOUNCE + an.topic), nullptr,
              {{an.topic, an.sub ? 1 : 0}});
    }
  pendingAnn.clear();
  // one hop's events in four passes (disconnects, connects, leaves, joins),
  // each in schedule order
  size_t end = nextEvent;
  while (end < sched.size() && sched[end].hop == hop) end++;
  for (int pass = GS_EV_DISCONNECT; pass <= GS_EV_JOIN; ++pass) {
  if (pass == GS_EV_LEAVE && (doPX || hasDirect)) {
    // the connector's dials of the previous hop (peer exchange, direct peers)
    // complete after this hop's scheduled disconnects and connects: each pair
    // once, ascending
    std::set<std::pair<int, int>> px;
    for (Node& nd : nodes) {
      for (int q : nd.pxReq) px.insert({std::min(nd.id, q), std::max(nd.id, q)});
      nd.pxReq.clear();
    }
    for (auto& pr : px) {
      if (!nodes[pr.first].dead.count(pr.second)) continue;
      nodes[pr.first].addPeer(pr.second);
      nodes[pr.second].addPeer(pr.first);
      traceHello(pr.first, pr.second);
      traceHello(pr.second, pr.first);
      account(pr.first, pr.second, acct ? helloSize(nodes[pr.first].mySubs) : 0);
      account(pr.second, pr.first, acct ? helloSize(nodes[pr.second].mySubs) : 0);
    }
  }
  std::vector<Event> evs;
  for (size_t k = nextEvent; k < end; ++k)
    if (sched[k].kind == pass) evs.push_back(sched[k]);
  if (pass >= GS_EV_LEAVE)  // leaves and joins of one hop in (node, topic) order
    std::stable_sort(evs.begin(), evs.end(), [](const Event& x, const Event& y) {
      return x.a != y.a ? x.a < y.a : x.b < y.b;
    });
  for (const Event& ev : evs) {
    switch (ev.kind) {
      case GS_EV_DISCONNECT:
        if (nodes[ev.a].dead.count(ev.b)) break;
        nodes[ev.a].removePeer(ev.b);
        nodes[ev.b].removePeer(ev.a);
        inbox[ev.a].erase(ev.b);
        inbox[ev.b].erase(ev.a);
        break;
      case GS_EV_CONNECT:
        if (!nodes[ev.a].dead.count(ev.b)) break;
        nodes[ev.a].addPeer(ev.b);
        nodes[ev.b].addPeer(ev.a);
        traceHello(ev.a, ev.b);
        traceHello(ev.b, ev.a);
        account(ev.a, ev.b, acct ? helloSize(nodes[ev.a].mySubs) : 0);  // hello packets (pubsub.go:534)
        account(ev.b, ev.a, acct ? helloSize(nodes[ev.b].mySubs) : 0);
        break;
      case GS_EV_LEAVE:
        if (!((nodes[ev.a].mySubs >> ev.b) & 1)) break;
        announce(ev.a, ev.b, false);
        nodes[ev.a].leaveTopic(ev.b);
        pendingAnn.push_back({ev.a, ev.b, false});
        break;
      case GS_EV_JOIN:
        if ((nodes[ev.a].mySubs >> ev.b) & 1) break;
        announce(ev.a, ev.b, true);
        nodes[ev.a].joinTopic(ev.b);
        pendingAnn.push_back({ev.a, ev.b, true});
        break;
    }
  }
  }
  nextEvent = end;
}

// protocol negotiation: include/gs_proto.h (shared with the product)
static int negotiate(int ra, int rb) { return gs_negotiate(ra, rb); }
static bool speaks(int r, int proto) { return gs_router_speaks(r, proto) != 0; }

int Sim::validateMixed() {
  auto rt = [&](int u) { return nodeRouter.empty() ? cfg.router : (int)nodeRouter[u]; };
  mixed = !nodeRouter.empty() || !protoE.empty();
  const bool given = !protoE.empty();
  if (!given) protoE.assign((size_t)E, 0);
  for (int u = 0; u < N; ++u) {
    const int ru = rt(u);
    if ((ru == GS_ROUTER_GOSSIPSUB || ru == GS_ROUTER_GOSSIPSUB_V10) && cfg.router != GS_ROUTER_GOSSIPSUB) {
      set_error("gossipsub hosts need cfg.router == GS_ROUTER_GOSSIPSUB (their params come from the engine)");
      return GS_EINVAL;
    }
    const bool gsHost = ru == GS_ROUTER_GOSSIPSUB || ru == GS_ROUTER_GOSSIPSUB_V10;
    if (!behave.empty() && behave[u] && !gsHost) { set_error("attacker behaviours need gossipsub hosts"); return GS_EINVAL; }
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
      const int v = col[e], rv = rt(v);
      if (!gsHost && !directE.empty() && directE[e]) { set_error("direct peers need a gossipsub host"); return GS_EINVAL; }
      if (!given) {
        protoE[e] = (uint8_t)negotiate(ru, rv);
      } else {
        const int pr = protoE[e] == GS_PROTO_DEFAULT ? negotiate(ru, rv) : protoE[e];
        const int pb = protoE[edgeIndex(v, u)] == GS_PROTO_DEFAULT ? negotiate(rv, ru) : protoE[edgeIndex(v, u)];
        if (pr != pb || !speaks(ru, pr) || !speaks(rv, pr)) {
          set_error("proto[e] must be a protocol both hosts speak, equal on both directions of the connection");
          return GS_EINVAL;
        }
      }
    }
  }
  if (given)
    for (int u = 0; u < N; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
        if (protoE[e] == GS_PROTO_DEFAULT) protoE[e] = (uint8_t)negotiate(rt(u), rt(col[e]));
  return GS_OK;
}

void Sim::initNode(Node& nd, int u) {
  nd.sim = this;
  nd.id = u;
  nd.mySubs = subs.empty() ? 0 : subs[u];
  nd.mcache.init(gp.HistoryGossip, gp.HistoryLength);
  nd.score.params = sp;
  for (int t = 0; t < T; ++t)
    if (tscored[t]) nd.score.topics[t] = tparams[t];
  nd.score.appSpecificScore = [this](int p) { return appScore.empty() ? 0.0 : appScore[p]; };
  nd.score.whitelist = whitelist;
  nd.gtracer.followUpTime = gp.IWantFollowupTime;
  nd.behave = behave.empty() ? 0 : behave[u];
  nd.router = nodeRouter.empty() ? cfg.router
              : nodeRouter[u] == GS_ROUTER_GOSSIPSUB_V10 ? GS_ROUTER_GOSSIPSUB : nodeRouter[u];
  if (gaterOn) {
    nd.gater.params = gaterParams;
    nd.gater.getIP = [this](int p) { return ipv4.empty() ? 0u : ipv4[p]; };  // 0 = "<unknown>"
  }
  for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
    int v = col[e];
    nd.nbrs.push_back(v);
    nd.proto[v] = protoE[e];
    if (dormant.count({std::min(u, v), std::max(u, v)})) {  // gs_set_dormant: not connected yet
      nd.dead.insert(v);
      nd.outbound[v] = outboundE.empty() ? false : outboundE[e] != 0;
      if (!directE.empty() && directE[e]) nd.direct.insert(v);
      continue;
    }
    emit(GS_TRACE_ADD_PEER, u, v, -1, -1, 0, mixed ? protoE[e] : 0);  // AddPeer gossipsub.go:507, floodsub.go:45
    nd.outbound[v] = outboundE.empty() ? false : outboundE[e] != 0;  // AddPeer gossipsub.go:505-532
    if (!directE.empty() && directE[e]) nd.direct.insert(v);
    std::vector<uint32_t> ips;
    if (!ipv4.empty() && ipv4[v] != 0) ips.push_back(ipv4[v]);
    if (nd.scored()) nd.score.AddPeer(v, ips);
    if (nd.gatered()) nd.gater.AddPeer(v);  // tracer.AddPeer -> peerGater.AddPeer (peer_gater.go:366-372)
    for (int t = 0; t < T; ++t)
      if (!subs.empty() && ((subs[v] >> t) & 1)) nd.topics[t].insert(v);
  }
}

void Sim::start() {
  nodes.assign(N, Node());
  if (record) deliv.assign(N, {});
  for (int u = 0; u < N; ++u) initNode(nodes[u], u);
  hasDirect = false;
  for (const Node& nd : nodes) hasDirect = hasDirect || (nd.isGossip() && !nd.direct.empty());
  hasDirect = hasDirect && cfg.router == GS_ROUTER_GOSSIPSUB;
  directInitHop = gp.DirectConnectInitialDelay <= 0 ? 0 : (gp.DirectConnectInitialDelay + cfg.hop_ns - 1) / cfg.hop_ns;
  auto up = [&](int u, int v) { return !dormant.count({std::min(u, v), std::max(u, v)}); };
  for (int u = 0; u < N; ++u)  // the hello packet of every connection (pubsub.go:495)
    for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e)
      if (up(u, col[e])) traceHello(u, col[e]);
  if (acct) {  // the hello packet of every connection (pubsub.go:495)
    rpcBytes.assign(E, 0);
    rpcCount.assign(E, 0);
    for (int u = 0; u < N; ++u)
      for (int64_t e = rowptr[u]; e < rowptr[u + 1]; ++e) {
        if (!up(u, col[e])) continue;
        rpcBytes[e] += helloSize(subs.empty() ? 0 : subs[u]);
        rpcCount[e] += 1;
      }
  }
  started = true;
}

// S0 memo and the gater snapshot of one host at the start of hop t
void Sim::nodeMemo(Node& nd, int64_t t) {
  nd.memo.clear();
  if (nd.scored())
    for (int v : nd.nbrs) nd.memo[v] = nd.score.score(v);
  if (nd.gatered()) {
    PeerGater& g = nd.gater;
    nd.gsnap.thr.clear();
    nd.gsnap.active = !(g.lastThrottle == kTimeZero || t - g.lastThrottle > g.params.Quiet) &&
                      g.throttle != 0 && !(g.validate != 0 && g.throttle / g.validate < g.params.Threshold);
    if (nd.gsnap.active)
      for (int v : nd.nbrs) {
        const double th = g.acceptThreshold(v);
        if (th >= 0) nd.gsnap.thr[v] = th;
      }
  }
}

// handleIncomingRPC per RPC, senders ascending, RPCs in send order
void Sim::nodeRefOrder(Node& nd, const std::map<int, std::vector<RPC>>& in) {
  nd.valUsed = 0;
  traceRecv(nd.id, in);
  for (auto& kv : in) {
    const int s = kv.first;
    std::vector<int64_t> got;  // accepted payload (the IWANT spammer re-requests it)
    for (const RPC& r : kv.second) {
      nd.ctr.transmissions += (int64_t)r.publish.size();
      const int st = nd.acceptFrom(s, r.hasCtl ? 0xFFFFFFFFu : (uint32_t)r.publish[0]);
      if (st == PeerGater::AcceptNone) { nd.ctr.graylisted++; continue; }  // pubsub.go:947-949
      if (st == PeerGater::AcceptControl) {                                // pubsub.go:951-955
        if (!r.publish.empty()) nd.ctr.gated++;
        if (nd.scored()) nd.gtracer.ThrottlePeer(s);
      } else {
        for (int64_t mid : r.publish) nd.handleMessage(s, msgs[mid]);
        got.insert(got.end(), r.publish.begin(), r.publish.end());
      }
      if (r.hasCtl && nd.isGossip()) nd.handleRPC(s, r);  // pubsub.go:969
    }
    if ((nd.behave & GS_BEHAVE_IWANT_SPAM) && !got.empty() && nd.isGossip() && nd.meshCap(s)) {
      std::sort(got.begin(), got.end());
      RPC r;
      r.hasCtl = true;
      r.ctl.iwant = got;
      r.sp = 2; r.ord = GS_RPC_O_SPAM;
      nd.sendRPC(s, std::move(r));
    }
  }
}

// phase A: payload messages, senders ascending; a sender's messages in
// ascending id (their order only matters for the validation queue)
void Sim::nodePhaseA(Node& nd, const std::map<int, std::vector<RPC>>& in) {
  nd.acceptStatus.clear();
  nd.valUsed = 0;
  traceRecv(nd.id, in);
  for (auto& kv : in) {
    int s = kv.first;
    bool anyCtl = false;
    for (const RPC& r : kv.second) anyCtl |= r.hasCtl;
    // one AcceptFrom per RPC; a sender's control RPCs of one hop share one draw
    const int ctlSt = anyCtl ? nd.acceptFrom(s, 0xFFFFFFFFu) : PeerGater::AcceptAll;
    nd.acceptStatus[s] = ctlSt;
    for (const RPC& r : kv.second) nd.ctr.transmissions += (int64_t)r.publish.size();  // copies on the wire
    bool throttledPeer = anyCtl && ctlSt == PeerGater::AcceptControl;
    std::vector<int64_t> mids;
    int64_t gray = 0;
    for (const RPC& r : kv.second) {
      const int st = r.hasCtl ? ctlSt : nd.acceptFrom(s, (uint32_t)r.publish[0]);
      if (st == PeerGater::AcceptNone) { gray++; continue; }          // pubsub.go:947-949
      if (st == PeerGater::AcceptControl) {                            // pubsub.go:951-955
        throttledPeer = true;
        if (!r.publish.empty()) nd.ctr.gated++;
        continue;
      }
      mids.insert(mids.end(), r.publish.begin(), r.publish.end());
    }
    nd.ctr.graylisted += gray;
    if (gray) continue;  // AcceptNone is per sender and hop (the S0 memo)
    // tracer.ThrottlePeer -> gossipTracer.ThrottlePeer (gossip_tracer.go:163-181)
    if (throttledPeer && nd.scored()) nd.gtracer.ThrottlePeer(s);
    std::sort(mids.begin(), mids.end());
    for (int64_t mid : mids) nd.handleMessage(s, msgs[mid]);
    if ((nd.behave & GS_BEHAVE_IWANT_SPAM) && !mids.empty() && nd.isGossip() && nd.meshCap(s)) {
      // re-request every message received from s (gossipsub_spam_test.go:113-128)
      RPC r;
      r.hasCtl = true;
      r.ctl.iwant = mids;
      r.sp = 2; r.ord = GS_RPC_O_SPAM;
      nd.sendRPC(s, std::move(r));
    }
  }
}

// phase B: control, per RPC, senders ascending
void Sim::nodePhaseB(Node& nd, const std::map<int, std::vector<RPC>>& in) {
  if (!nd.isGossip()) return;  // FloodSubRouter / RandomSubRouter.HandleRPC: no-ops
  for (auto& kv : in) {
    int s = kv.first;
    if (nd.acceptStatus[s] == PeerGater::AcceptNone) continue;
    for (const RPC& r : kv.second)
      if (r.hasCtl) nd.handleRPC(s, r);
  }
}

void Sim::step() {
  const int64_t t = now();
  // the RPCs sent during hop h-1 are this hop's inbox
  std::vector<std::map<int, std::vector<RPC>>> inbox(N);
  for (Node& nd : nodes) {
    for (auto& kv : nd.out) inbox[kv.first][nd.id] = std::move(kv.second);
    nd.out.clear();
  }
  // Every per-node phase below touches only the node's own state (its router
  // maps, peerScore, mcache, outbox, counters and trace buffer) and reads
  // shared immutable data, so nodes run in parallel; the phase order is kept.
  applyEvents(inbox);
  if (hasDirect && hop == directInitHop)  // connect to direct peers after DirectConnectInitialDelay (:492-502)
    for (Node& nd : nodes) nd.directConnect();
  if (hop == 0) {  // Join: the GRAFTs it sends arrive in hop 1
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u)
      for (int tp = 0; tp < T; ++tp)
        if ((nodes[u].mySubs >> tp) & 1) {
          emit(GS_TRACE_JOIN, u, -1, tp, -1, 0);  // tracer.Join gossipsub.go:1018, floodsub.go:103
          nodes[u].join(tp);
        }
  }
  // S0 memo and the gater snapshot
  if (scoring || gaterOn) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodeMemo(nodes[u], t);
  }
  // local publishes of this hop
  while (nextPub < msgs.size() && msgHop[nextPub] == hop) {
    const Msg& m = msgs[nextPub];
    nodes[m.from].localPublish(m);
    nextPub++;
  }
  if (refOrder) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodeRefOrder(nodes[u], inbox[u]);
  } else {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodePhaseA(nodes[u], inbox[u]);
  }
  if (cfg.router == GS_ROUTER_GOSSIPSUB && !refOrder) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodePhaseB(nodes[u], inbox[u]);
  }
  if (refreshDue(t)) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodes[u].score.refreshScores(t);
  }
  if (gaterDecayDue(t)) {  // peerGater.background ticker (peer_gater.go:204-217)
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodes[u].gater.decayStats(t);
  }
  if (scoring && t > 0 && t % (60 * kSecond) == 0) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u) nodes[u].score.gc(t);
  }
  if (heartbeatDue(t)) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int u = 0; u < N; ++u)
      if (nodes[u].isGossip()) nodes[u].heartbeat();
    ctr.heartbeats++;
  }
  ctr.hops++;
  hop++;
}


// ---------------------------------------------------------------- replay
// gs_oracle_replay_* (test infrastructure): one host of a simulation run on
// its own, its inbox taken from the RecvRPC blocks of an event trace (the
// reference's EventTracer view of everything a host receives, trace.go:241-
// 383).  A host's state is a function of its inbox, its own publishes and the
// static shared inputs (graph, subscriptions, peer attributes, the publish
// schedule), so the replay runs exactly the per-host phase bodies Sim::step
// runs for every host (nodeMemo, nodePhaseA, nodePhaseB, refreshScores,
// heartbeat), hop by hop, and its events and final router / score state must
// equal the full run's for that host.  The full-size GPU tests replay sampled
// hosts of the 1M-peer runs from the engine's own trace this way.
struct Replay {
  Sim* sim = nullptr;
  Node nd;
  int64_t hop = 0;
  std::vector<int64_t> myPubs;  // ids of the messages this host publishes, ascending
  size_t nextPub = 0;
  // hop -> sender -> (ordinal, RPC), sorted by ordinal before the hop runs
  std::map<int64_t, std::map<int, std::vector<std::pair<int64_t, RPC>>>> inbox;
  std::vector<gs_trace_event> pend;
  size_t pendOut = 0;
};

static int replay_parse(Replay& r, const gs_trace_event* ev, int64_t n) {
  Sim& s = *r.sim;
  const int u = r.nd.id;
  for (int64_t i = 0; i < n;) {
    int64_t j = i + 1;
    if (gs_trace_is_rpc(ev[i]))
      while (j < n && ev[j].type == GS_TRACE_RPC_ITEM) ++j;
    const gs_trace_event& hd = ev[i];
    if (hd.type == GS_TRACE_RECV_RPC && hd.node == u) {
      const int64_t sp = hd.msg >> 40, ord = hd.msg & (((int64_t)1 << 40) - 1);
      if (hd.hop < r.hop) { set_error("gs_oracle_replay_run: an RPC for a hop already replayed"); return GS_EINVAL; }
      if (!(sp == 0 && ord >= GS_RPC_O_ANNOUNCE)) {  // hellos / announcements: the static topic maps
        RPC rpc;
        rpc.sp = (int)sp;
        rpc.ord = ord;
        const int from = hd.peer;
        for (int64_t k = i + 1; k < j; ++k) {
          const gs_trace_event& x = ev[k];
          switch (x.reason) {
            case GS_RPC_ITEM_MSG: rpc.publish.push_back(x.msg); break;
            case GS_RPC_ITEM_CTL: rpc.hasCtl = true; break;
            case GS_RPC_ITEM_IHAVE:
              if (rpc.ctl.ihave.empty() || rpc.ctl.ihave.back().topic != x.topic)
                rpc.ctl.ihave.push_back(IHaveEntry{x.topic, {}});
              rpc.ctl.ihave.back().mids.push_back(x.msg);
              break;
            case GS_RPC_ITEM_IWANT: rpc.ctl.iwant.push_back(x.msg); break;
            case GS_RPC_ITEM_GRAFT: rpc.ctl.graft.push_back(x.topic); break;
            case GS_RPC_ITEM_PRUNE: {  // makePrune (gossipsub.go:1803-1839): the sender's PruneBackoff
              PruneEntry pe;
              pe.topic = x.topic;
              pe.hasBackoff = r.nd.pxCap(from);
              pe.backoff = pe.hasBackoff ? (uint64_t)(s.gp.PruneBackoff / kSecond) : 0;
              rpc.ctl.prune.push_back(pe);
              break;
            }
            case GS_RPC_ITEM_PX:
              for (auto it = rpc.ctl.prune.rbegin(); it != rpc.ctl.prune.rend(); ++it)
                if (it->topic == x.topic) { it->px.push_back((int)x.msg); break; }
              break;
            default: break;
          }
        }
        r.inbox[hd.hop][from].push_back({hd.msg, std::move(rpc)});
      }
    }
    i = j;
  }
  return GS_OK;
}

static void replay_hop(Replay& r) {
  Sim& s = *r.sim;
  Node& nd = r.nd;
  s.solo = &nd;
  s.hop = r.hop;
  const int64_t t = s.now();
  nd.out.clear();  // sent last hop (their SendRPC events are recorded)
  std::map<int, std::vector<RPC>> in;
  auto ih = r.inbox.find(r.hop);
  if (ih != r.inbox.end()) {
    for (auto& kv : ih->second) {
      auto& v = kv.second;
      std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      auto& dst = in[kv.first];
      for (auto& pr : v) dst.push_back(std::move(pr.second));
    }
    r.inbox.erase(ih);
  }
  if (r.hop == 0)
    for (int tp = 0; tp < s.T; ++tp)
      if ((nd.mySubs >> tp) & 1) {
        s.emit(GS_TRACE_JOIN, nd.id, -1, tp, -1, 0);
        nd.join(tp);
      }
  if (s.scoring || s.gaterOn) s.nodeMemo(nd, t);
  while (r.nextPub < r.myPubs.size() && s.msgHop[(size_t)r.myPubs[r.nextPub]] <= r.hop) {
    const int64_t id = r.myPubs[r.nextPub++];
    if (s.msgHop[(size_t)id] == r.hop) nd.localPublish(s.msgs[(size_t)id]);
  }
  if (s.refOrder) {
    s.nodeRefOrder(nd, in);
  } else {
    s.nodePhaseA(nd, in);
    if (s.cfg.router == GS_ROUTER_GOSSIPSUB) s.nodePhaseB(nd, in);
  }
  if (s.refreshDue(t)) nd.score.refreshScores(t);
  if (s.gaterDecayDue(t)) nd.gater.decayStats(t);
  if (s.scoring && t > 0 && t % (60 * kSecond) == 0) nd.score.gc(t);
  if (s.heartbeatDue(t) && nd.isGossip()) nd.heartbeat();
  r.hop++;
}


}  // namespace oracle

using namespace oracle;

struct gs_engine {
  Sim sim;
};

extern "C" {

int gs_abi_version(void) { return GS_ABI_VERSION; }
const char* gs_last_error(void) { return g_err.c_str(); }
void gs_default_gossipsub_params(gs_gossipsub_params* out) { defaultGossipSubParams(out); }
void gs_default_peer_gater_params(gs_peer_gater_params* out) { defaultPeerGaterParams(out); }
double gs_score_parameter_decay_with_base(int64_t decay, int64_t base, double dtz) {
  return scoreParameterDecayWithBase(decay, base, dtz);
}
double gs_score_parameter_decay(int64_t decay) { return scoreParameterDecayWithBase(decay, kSecond, 0.01); }
int gs_validate_thresholds(const gs_peer_score_thresholds* p) { return validateThresholds(p); }
int gs_validate_peer_score_params(const gs_peer_score_params* p, const gs_topic_score_params* topics,
                                  const uint8_t* scored, int32_t T) {
  return validatePeerScoreParams(p, topics, scored, T);
}
int gs_validate_topic_score_params(const gs_topic_score_params* p) { return validateTopicParams(p); }
int gs_validate_peer_gater_params(const gs_peer_gater_params* p) { return validateGaterParams(p); }

int gs_engine_create(const gs_config* cfg, const gs_gossipsub_params* gsp, const gs_peer_score_params* psp,
                     const gs_topic_score_params* topics, const uint8_t* topic_scored,
                     const gs_peer_score_thresholds* thr, const gs_peer_gater_params* gater, gs_engine** out) {
  if (!cfg || !out) { set_error("null argument"); return GS_EINVAL; }
  if (cfg->num_nodes <= 0 || cfg->num_topics <= 0 || cfg->num_topics > 64 || cfg->hop_ns <= 0) {
    set_error("invalid config: num_nodes > 0, 1 <= num_topics <= 64, hop_ns > 0 required");
    return GS_EINVAL;
  }
  if (cfg->router < 0 || cfg->router > 2) { set_error("unknown router"); return GS_EINVAL; }
  std::unique_ptr<gs_engine> eng(new gs_engine());
  Sim& s = eng->sim;
  s.cfg = *cfg;
  s.N = cfg->num_nodes;
  s.T = cfg->num_topics;
  if (gsp) s.gp = *gsp; else defaultGossipSubParams(&s.gp);
  s.scoring = (cfg->flags & GS_FLAG_SCORING) != 0 && cfg->router == GS_ROUTER_GOSSIPSUB;
  s.floodPublish = (cfg->flags & GS_FLAG_FLOOD_PUBLISH) != 0;
  s.doPX = (cfg->flags & GS_FLAG_PEER_EXCHANGE) != 0 && cfg->router == GS_ROUTER_GOSSIPSUB;
  s.record = (cfg->flags & GS_FLAG_RECORD_DELIVERIES) != 0;
  s.tparams.assign(s.T, gs_topic_score_params{});
  s.tscored.assign(s.T, 0);
  s.topicVal.assign(s.T, 0);
  if (gater) {
    if (cfg->router != GS_ROUTER_GOSSIPSUB) { set_error("pubsub router is not gossipsub"); return GS_EINVAL; }
    int rc = validateGaterParams(gater);
    if (rc) return rc;
    if (gater->DecayInterval % cfg->hop_ns != 0) { set_error("gater DecayInterval must be a multiple of hop_ns"); return GS_EUNSUPPORTED; }
    s.gaterOn = true;
    s.gaterParams = *gater;
  }
  if (cfg->router == GS_ROUTER_GOSSIPSUB) {
    if (s.gp.HistoryGossip > s.gp.HistoryLength) {
      set_error("invalid parameters for message cache; gossip slots cannot be larger than history slots");
      return GS_EINVAL;
    }
    if (s.gp.HeartbeatInterval <= 0 || s.gp.HeartbeatInterval % cfg->hop_ns != 0 ||
        s.gp.HeartbeatInitialDelay < 0 || s.gp.HeartbeatInitialDelay % cfg->hop_ns != 0) {
      set_error("HeartbeatInterval and HeartbeatInitialDelay must be multiples of hop_ns");
      return GS_EUNSUPPORTED;
    }
    if (s.gp.DirectConnectTicks == 0) {  // heartbeatTicks % DirectConnectTicks (gossipsub.go:1597)
      set_error("DirectConnectTicks must be > 0");
      return GS_EINVAL;
    }
  }
  if (s.scoring) {
    if (!psp || !topics || !topic_scored || !thr) { set_error("scoring needs score params and thresholds"); return GS_EINVAL; }
    int rc = validatePeerScoreParams(psp, topics, topic_scored, s.T);
    if (rc) return rc;
    rc = validateThresholds(thr);
    if (rc) return rc;
    if (psp->DecayInterval % cfg->hop_ns != 0) { set_error("DecayInterval must be a multiple of hop_ns"); return GS_EUNSUPPORTED; }
    s.sp = *psp;
    s.thr = *thr;
    for (int t = 0; t < s.T; ++t) { s.tparams[t] = topics[t]; s.tscored[t] = topic_scored[t]; }
  }
  *out = eng.release();
  return GS_OK;
}

int gs_engine_destroy(gs_engine* eng) { delete eng; return GS_OK; }
// Oracle-only switch (tests/test_oracle_schedule.py): the reference's per-RPC
// order with live scores instead of the engine's canonical schedule.
int gs_oracle_reference_order(gs_engine* eng, int32_t on) {
  if (eng->sim.hop != 0) { set_error("gs_oracle_reference_order: set before the first step"); return GS_EINVAL; }
  // 1: per-RPC order + live scores; 2: the canonical phase split with live scores
  eng->sim.refOrder = on == 1;
  eng->sim.liveScore = on != 0;
  return GS_OK;
}

int gs_set_graph(gs_engine* eng, const int64_t* rowptr, const int32_t* col, const uint8_t* outbound,
                 const uint8_t* direct) {
  return gs_set_graph_ex(eng, rowptr, col, outbound, direct, nullptr);
}

int gs_set_graph_ex(gs_engine* eng, const int64_t* rowptr, const int32_t* col, const uint8_t* outbound,
                    const uint8_t* direct, const uint8_t* proto) {
  Sim& s = eng->sim;
  if (s.started) { set_error("graph must be set before the first step"); return GS_ESTATE; }
  s.rowptr.assign(rowptr, rowptr + s.N + 1);
  s.E = s.rowptr[s.N];
  s.col.assign(col, col + s.E);
  for (int u = 0; u < s.N; ++u)
    for (int64_t e = s.rowptr[u]; e < s.rowptr[u + 1]; ++e) {
      int v = s.col[e];
      if (v < 0 || v >= s.N || v == u || (e > s.rowptr[u] && s.col[e - 1] >= v)) {
        set_error("graph rows must hold strictly ascending neighbour ids != self"); return GS_EINVAL; }
    }
  for (int u = 0; u < s.N; ++u)
    for (int64_t e = s.rowptr[u]; e < s.rowptr[u + 1]; ++e)
      if (s.edgeIndex(s.col[e], u) < 0) { set_error("graph must be symmetric"); return GS_EINVAL; }
  s.outboundE.assign(s.E, 0);
  s.directE.assign(s.E, 0);
  if (outbound) s.outboundE.assign(outbound, outbound + s.E);
  if (direct) s.directE.assign(direct, direct + s.E);
  s.protoE.clear();
  if (proto) {
    for (int64_t e = 0; e < s.E; ++e)
      if (proto[e] > GS_PROTO_GOSSIPSUB_V11) { set_error("unknown protocol"); return GS_EINVAL; }
    s.protoE.assign(proto, proto + s.E);
  }
  s.graphSet = true;
  return GS_OK;
}

int gs_set_routers(gs_engine* eng, const uint8_t* router) {
  Sim& s = eng->sim;
  if (s.started) { set_error("routers must be set before the first step"); return GS_ESTATE; }
  s.nodeRouter.clear();
  if (router) {
    for (int u = 0; u < s.N; ++u)
      if (router[u] > GS_ROUTER_GOSSIPSUB_V10) { set_error("unknown router"); return GS_EINVAL; }
    s.nodeRouter.assign(router, router + s.N);
  }
  return GS_OK;
}

// PubSubRouter.EnoughPeers per host (gossip_engine.h).  A topic no peer of the
// host announced counts as an empty one.
int gs_enough_peers(gs_engine* eng, int32_t topic, int32_t suggested, uint8_t* out) {
  Sim& s = eng->sim;
  if (topic < 0 || topic >= s.T || suggested < 0 || !out) { set_error("gs_enough_peers: bad arguments"); return GS_EINVAL; }
  if (!s.started) { set_error("gs_enough_peers: no state before the first step"); return GS_ESTATE; }
  for (int u = 0; u < s.N; ++u) {
    Node& nd = s.nodes[u];
    auto tm = nd.topics.find(topic);
    const std::set<int> none;
    const std::set<int>& tmap = tm == nd.topics.end() ? none : tm->second;
    bool ok = false;
    if (nd.router == GS_ROUTER_GOSSIPSUB) {  // gossipsub.go:549-576
      int fs = 0;
      for (int p : tmap) fs += nd.meshCap(p) ? 0 : 1;
      auto gm = nd.mesh.find(topic);
      const int gsn = gm == nd.mesh.end() ? 0 : (int)gm->second.size();
      const int sg = suggested == 0 ? s.gp.Dlo : suggested;
      ok = fs + gsn >= sg || gsn >= s.gp.Dhi;
    } else if (nd.router == GS_ROUTER_RANDOMSUB) {  // randomsub.go:59-89
      int fs = 0, rs = 0;
      for (int p : tmap) {
        fs += nd.proto[p] == GS_PROTO_FLOODSUB;
        rs += nd.proto[p] == GS_PROTO_RANDOMSUB;
      }
      const int sg = suggested == 0 ? 6 : suggested;  // RandomSubD
      ok = fs + rs >= sg || rs >= 6;
    } else {  // floodsub.go:52-66
      const int sg = suggested == 0 ? 5 : suggested;  // FloodSubTopicSearchSize
      ok = (int)tmap.size() >= sg;
    }
    out[u] = ok ? 1 : 0;
  }
  return GS_OK;
}

int gs_set_subscriptions(gs_engine* eng, const uint64_t* sub_mask) {
  Sim& s = eng->sim;
  if (s.started) { set_error("subscriptions must be set before the first step"); return GS_ESTATE; }
  s.subs.assign(sub_mask, sub_mask + s.N);
  return GS_OK;
}

int gs_set_peer_attrs(gs_engine* eng, const double* app_score, const uint32_t* ipv4) {
  Sim& s = eng->sim;
  if (s.started) { set_error("peer attributes must be set before the first step"); return GS_ESTATE; }
  if (app_score) s.appScore.assign(app_score, app_score + s.N);
  if (ipv4) s.ipv4.assign(ipv4, ipv4 + s.N);
  return GS_OK;
}

int gs_set_ip_whitelist(gs_engine* eng, int32_t n, const uint32_t* net, const uint32_t* mask) {
  Sim& s = eng->sim;
  if (s.started) { set_error("whitelist must be set before the first step"); return GS_ESTATE; }
  s.whitelist.clear();
  for (int i = 0; i < n; ++i) s.whitelist.push_back({net[i], mask[i]});
  return GS_OK;
}

int gs_publish_ex(gs_engine* eng, int32_t n, const int32_t* src, const int32_t* topic, const int64_t* hop,
                  const uint8_t* kind, int64_t* ids_out) {
  Sim& s = eng->sim;
  int64_t last = s.msgHop.empty() ? s.hop : std::max(s.hop, s.msgHop.back());
  for (int i = 0; i < n; ++i) {
    if (src[i] < 0 || src[i] >= s.N || topic[i] < 0 || topic[i] >= s.T || hop[i] < last ||
        (kind && kind[i] > GS_MSG_PHANTOM)) {
      set_error("publish: bad src/topic/kind or hop not non-decreasing from the current hop"); return GS_EINVAL; }
    last = hop[i];
  }
  for (int i = 0; i < n; ++i) {
    int64_t id = (int64_t)s.msgs.size();
    s.msgs.push_back(Msg{id, topic[i], src[i]});
    s.msgHop.push_back(hop[i]);
    s.msgKind.push_back(kind ? kind[i] : (uint8_t)GS_MSG_VALID);
    if (ids_out) ids_out[i] = id;
  }
  return GS_OK;
}

int gs_publish(gs_engine* eng, int32_t n, const int32_t* src, const int32_t* topic, const int64_t* hop,
               int64_t* ids_out) {
  return gs_publish_ex(eng, n, src, topic, hop, nullptr, ids_out);
}

int gs_set_validation(gs_engine* eng, const uint8_t* topic_validator, int32_t queue_per_hop) {
  Sim& s = eng->sim;
  if (s.started) { set_error("validation must be set before the first step"); return GS_ESTATE; }
  if (queue_per_hop < 0) { set_error("queue_per_hop must be >= 0"); return GS_EINVAL; }
  s.topicVal.assign(s.T, 0);
  if (topic_validator) s.topicVal.assign(topic_validator, topic_validator + s.T);
  s.valQueue = queue_per_hop;
  return GS_OK;
}

int gs_set_behaviour(gs_engine* eng, const uint8_t* behaviour) {
  Sim& s = eng->sim;
  if (s.started) { set_error("behaviours must be set before the first step"); return GS_ESTATE; }
  s.behave.clear();
  if (behaviour) s.behave.assign(behaviour, behaviour + s.N);
  return GS_OK;
}

int gs_schedule_events(gs_engine* eng, int32_t n, const int32_t* kind, const int32_t* a, const int32_t* b,
                       const int64_t* hop) {
  Sim& s = eng->sim;
  if (n < 0 || (n > 0 && (!kind || !a || !b || !hop))) { set_error("gs_schedule_events: bad arguments"); return GS_EINVAL; }
  if (!s.graphSet) { set_error("graph not set"); return GS_ESTATE; }
  int64_t last = s.sched.empty() ? std::max<int64_t>(1, s.hop) : std::max(s.hop, s.sched.back().hop);
  for (int32_t i = 0; i < n; ++i) {
    bool ok = hop[i] >= last && hop[i] >= 1 && kind[i] >= GS_EV_DISCONNECT && kind[i] <= GS_EV_JOIN &&
              a[i] >= 0 && a[i] < s.N;
    if (ok && kind[i] <= GS_EV_CONNECT) ok = b[i] >= 0 && b[i] < s.N && s.edgeIndex(a[i], b[i]) >= 0;
    if (ok && kind[i] >= GS_EV_LEAVE) ok = b[i] >= 0 && b[i] < s.T;
    if (!ok) { set_error("gs_schedule_events: bad event (kind, nodes, topic or hop order)"); return GS_EINVAL; }
    last = hop[i];
  }
  for (int32_t i = 0; i < n; ++i) s.sched.push_back({hop[i], kind[i], a[i], b[i]});
  return GS_OK;
}

int gs_step(gs_engine* eng, int64_t hops) {
  Sim& s = eng->sim;
  if (!s.graphSet) { set_error("graph not set"); return GS_ESTATE; }
  if (!s.started) {
    if (!s.mixedChecked) {
      const int rc = s.validateMixed();
      if (rc) return rc;
      s.mixedChecked = true;
    }
    s.start();
  }
  for (int64_t i = 0; i < hops; ++i) s.step();
  return GS_OK;
}
int gs_sync(gs_engine*) { return GS_OK; }

int gs_set_topic_score_params(gs_engine* eng, int32_t topic, const gs_topic_score_params* p) {
  Sim& s = eng->sim;
  if (topic < 0 || topic >= s.T) { set_error("bad topic"); return GS_EINVAL; }
  int rc = validateTopicParams(p);
  if (rc) return rc;
  s.tparams[topic] = *p;
  s.tscored[topic] = 1;
  for (Node& nd : s.nodes) nd.score.SetTopicScoreParams(topic, *p);
  return GS_OK;
}

int64_t gs_num_edges(const gs_engine* eng) { return eng->sim.E; }
int64_t gs_current_hop(const gs_engine* eng) { return eng->sim.hop; }
int gs_read_counters(gs_engine* eng, gs_counters* out) { *out = eng->sim.total(); return GS_OK; }

int gs_read_scores(gs_engine* eng, double* score) {
  Sim& s = eng->sim;
  if (!s.started) s.start();
  for (int u = 0; u < s.N; ++u)
    for (int64_t e = s.rowptr[u]; e < s.rowptr[u + 1]; ++e)
      score[e] = s.nodes[u].Score(s.col[e]);
  return GS_OK;
}

int gs_read_mesh(gs_engine* eng, uint64_t* mesh) {
  Sim& s = eng->sim;
  std::fill(mesh, mesh + s.E, 0);
  if (!s.started) return GS_OK;
  for (int u = 0; u < s.N; ++u)
    for (auto& kv : s.nodes[u].mesh)
      for (int p : kv.second) mesh[s.edgeIndex(u, p)] |= 1ull << kv.first;
  return GS_OK;
}

int gs_read_fanout(gs_engine* eng, uint64_t* fanout) {
  Sim& s = eng->sim;
  std::fill(fanout, fanout + s.E, 0);
  if (!s.started) return GS_OK;
  for (int u = 0; u < s.N; ++u)
    for (auto& kv : s.nodes[u].fanout)
      for (int p : kv.second) fanout[s.edgeIndex(u, p)] |= 1ull << kv.first;
  return GS_OK;
}

int gs_read_backoff(gs_engine* eng, int64_t* expire) {
  Sim& s = eng->sim;
  std::fill(expire, expire + s.E * s.T, 0);
  if (!s.started) return GS_OK;
  for (int u = 0; u < s.N; ++u)
    for (auto& kv : s.nodes[u].backoff)
      for (auto& pe : kv.second) expire[(int64_t)kv.first * s.E + s.edgeIndex(u, pe.first)] = pe.second;
  return GS_OK;
}

int gs_read_topic_stats(gs_engine* eng, double* fmd, double* mmd, double* mfp, double* imd, int64_t* mesh_time,
                        int64_t* graft_time, uint8_t* flags) {
  Sim& s = eng->sim;
  const int64_t n = s.E * s.T;
  std::fill(fmd, fmd + n, 0.0); std::fill(mmd, mmd + n, 0.0);
  std::fill(mfp, mfp + n, 0.0); std::fill(imd, imd + n, 0.0);
  std::fill(mesh_time, mesh_time + n, 0); std::fill(graft_time, graft_time + n, 0);
  std::fill(flags, flags + n, 0);
  if (!s.started) return GS_OK;
  for (int u = 0; u < s.N; ++u)
    for (auto& ps : s.nodes[u].score.peerStats) {
      int64_t e = s.edgeIndex(u, ps.first);
      for (auto& ts : ps.second.topics) {
        int64_t i = (int64_t)ts.first * s.E + e;
        fmd[i] = ts.second.firstMessageDeliveries;
        mmd[i] = ts.second.meshMessageDeliveries;
        mfp[i] = ts.second.meshFailurePenalty;
        imd[i] = ts.second.invalidMessageDeliveries;
        mesh_time[i] = ts.second.meshTime;
        graft_time[i] = ts.second.graftTime;
        flags[i] = (ts.second.inMesh ? 1 : 0) | (ts.second.meshMessageDeliveriesActive ? 2 : 0);
      }
    }
  return GS_OK;
}

int gs_read_topic_stats_edges(gs_engine* eng, int64_t n, const int64_t* edges, double* fmd, double* mmd,
                              double* mfp, double* imd, int64_t* mesh_time, int64_t* graft_time, uint8_t* flags) {
  Sim& s = eng->sim;
  if (n < 0 || (n > 0 && (!edges || !fmd || !mmd || !mfp || !imd || !mesh_time || !graft_time || !flags))) {
    set_error("gs_read_topic_stats_edges: bad arguments");
    return GS_EINVAL;
  }
  for (int64_t i = 0; i < n; ++i)
    if (edges[i] < 0 || edges[i] >= s.E) { set_error("gs_read_topic_stats_edges: edge out of range"); return GS_EINVAL; }
  const int64_t nk = n * s.T;
  std::fill(fmd, fmd + nk, 0.0); std::fill(mmd, mmd + nk, 0.0);
  std::fill(mfp, mfp + nk, 0.0); std::fill(imd, imd + nk, 0.0);
  std::fill(mesh_time, mesh_time + nk, 0); std::fill(graft_time, graft_time + nk, 0);
  std::fill(flags, flags + nk, 0);
  if (!s.started) return GS_OK;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t e = edges[i];
    const int u = (int)(std::upper_bound(s.rowptr.begin(), s.rowptr.end(), e) - s.rowptr.begin()) - 1;
    auto ps = s.nodes[u].score.peerStats.find(s.col[e]);
    if (ps == s.nodes[u].score.peerStats.end()) continue;
    for (auto& ts : ps->second.topics) {
      const int64_t k = i * s.T + ts.first;
      fmd[k] = ts.second.firstMessageDeliveries;
      mmd[k] = ts.second.meshMessageDeliveries;
      mfp[k] = ts.second.meshFailurePenalty;
      imd[k] = ts.second.invalidMessageDeliveries;
      mesh_time[k] = ts.second.meshTime;
      graft_time[k] = ts.second.graftTime;
      flags[k] = (ts.second.inMesh ? 1 : 0) | (ts.second.meshMessageDeliveriesActive ? 2 : 0);
    }
  }
  return GS_OK;
}

int gs_read_backoff_edges(gs_engine* eng, int64_t n, const int64_t* edges, int64_t* expire) {
  Sim& s = eng->sim;
  if (n < 0 || (n > 0 && (!edges || !expire))) { set_error("gs_read_backoff_edges: bad arguments"); return GS_EINVAL; }
  for (int64_t i = 0; i < n; ++i)
    if (edges[i] < 0 || edges[i] >= s.E) { set_error("gs_read_backoff_edges: edge out of range"); return GS_EINVAL; }
  std::fill(expire, expire + n * s.T, 0);
  if (!s.started) return GS_OK;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t e = edges[i];
    const int u = (int)(std::upper_bound(s.rowptr.begin(), s.rowptr.end(), e) - s.rowptr.begin()) - 1;
    for (auto& kv : s.nodes[u].backoff) {
      auto be = kv.second.find(s.col[e]);
      if (be != kv.second.end()) expire[i * s.T + kv.first] = be->second;
    }
  }
  return GS_OK;
}

int gs_read_behaviour_penalty(gs_engine* eng, double* bp) {
  Sim& s = eng->sim;
  std::fill(bp, bp + s.E, 0.0);
  if (!s.started) return GS_OK;
  for (int u = 0; u < s.N; ++u)
    for (auto& ps : s.nodes[u].score.peerStats) bp[s.edgeIndex(u, ps.first)] = ps.second.behaviourPenalty;
  return GS_OK;
}

int gs_read_deliveries(gs_engine* eng, int64_t id, int32_t* hop, int32_t* from) {
  Sim& s = eng->sim;
  if (!s.record) { set_error("GS_FLAG_RECORD_DELIVERIES not set"); return GS_ESTATE; }
  if (id < 0 || id >= (int64_t)s.msgs.size()) { set_error("unknown message id"); return GS_EINVAL; }
  for (int u = 0; u < s.N; ++u) {
    hop[u] = -1; from[u] = -1;
    if (!s.started) continue;
    auto it = s.deliv[u].find(id);
    if (it != s.deliv[u].end()) { hop[u] = it->second.first; from[u] = it->second.second; }
  }
  return GS_OK;
}

int gs_set_profiling(gs_engine*, int) { return GS_OK; }
int gs_read_kernel_stats(gs_engine*, double* total_ms, int64_t* launches) {
  for (int i = 0; i < GS_NUM_KERNELS; ++i) { total_ms[i] = 0; launches[i] = 0; }
  return GS_OK;
}

// The oracle simulates the whole graph: world == 1 only (gossip_engine.h).
int gs_set_partition(gs_engine*, int32_t rank, int32_t world, const gs_transport*) {
  if (world == 1 && rank == 0) return GS_OK;
  return GS_EUNSUPPORTED;
}
int gs_partition_range(const gs_engine* g, int32_t* node_begin, int32_t* node_end) {
  *node_begin = 0;
  *node_end = g->sim.N;
  return GS_OK;
}
int gs_set_dormant(gs_engine* g, int32_t n, const int32_t* a, const int32_t* b) {
  Sim& s = g->sim;
  if (s.started) { set_error("gs_set_dormant: before the first step"); return GS_ESTATE; }
  if (!s.graphSet) { set_error("graph not set"); return GS_ESTATE; }
  if (n < 0 || (n > 0 && (!a || !b))) { set_error("gs_set_dormant: bad arguments"); return GS_EINVAL; }
  for (int32_t i = 0; i < n; ++i) {
    if (a[i] < 0 || a[i] >= s.N || b[i] < 0 || b[i] >= s.N || s.edgeIndex(a[i], b[i]) < 0) {
      set_error("gs_set_dormant: not an edge of the graph");
      return GS_EINVAL;
    }
    s.dormant.insert({std::min(a[i], b[i]), std::max(a[i], b[i])});
  }
  return GS_OK;
}

int gs_set_rpc_accounting(gs_engine* g, const int32_t* msg_size, int32_t id_len, const int32_t* topic_len) {
  Sim& sim = g->sim;
  if (sim.started) { set_error("gs_set_rpc_accounting: before the first step"); return GS_ESTATE; }
  if (!msg_size || !topic_len || id_len < 0) { set_error("gs_set_rpc_accounting: bad arguments"); return GS_EINVAL; }
  for (int t = 0; t < sim.T; ++t)
    if (msg_size[t] < 0 || topic_len[t] < 0) { set_error("gs_set_rpc_accounting: negative size"); return GS_EINVAL; }
  sim.acct = true;
  sim.acctMsg.assign(msg_size, msg_size + sim.T);
  sim.acctTl.assign(topic_len, topic_len + sim.T);
  sim.acctId = id_len;
  return GS_OK;
}

// makePrune's PX PeerInfo sizes (gossipsub.go:1820-1833): peer id bytes and
// signed-peer-record bytes (0: the peerstore has no certified address book)
int gs_set_rpc_px_sizes(gs_engine* g, int32_t peer_id_len, int32_t record_len) {
  Sim& sim = g->sim;
  if (sim.started) { set_error("gs_set_rpc_px_sizes: before the first step"); return GS_ESTATE; }
  if (peer_id_len < 0 || record_len < 0) { set_error("gs_set_rpc_px_sizes: negative size"); return GS_EINVAL; }
  sim.acctPid = peer_id_len;
  sim.acctRec = record_len;
  return GS_OK;
}

int gs_read_rpc_bytes(gs_engine* g, int64_t* bytes, int64_t* rpcs) {
  Sim& sim = g->sim;
  if (!sim.acct) { set_error("gs_read_rpc_bytes: accounting is off"); return GS_ESTATE; }
  for (int64_t e = 0; e < sim.E; ++e) {
    if (bytes) bytes[e] = sim.started ? sim.rpcBytes[e] : 0;
    if (rpcs) rpcs[e] = sim.started ? sim.rpcCount[e] : 0;
  }
  return GS_OK;
}

int gs_set_trace(gs_engine* g, const uint8_t* node_mask, int64_t capacity) {
  (void)capacity;  // the oracle keeps every event
  if (g->sim.started) { set_error("tracing must be set before the first step"); return GS_ESTATE; }
  if (node_mask) g->sim.traced.assign(node_mask, node_mask + g->sim.N);
  else g->sim.traced.clear();
  return GS_OK;
}
int gs_set_peertx_capacity(gs_engine* g, int32_t home_bits, int32_t overflow_bits) {
  // mcache.peertx is a map here (mcache.go:66-80): no capacity to set
  if (g->sim.started) { set_error("the peertx capacity must be set before the first step"); return GS_ESTATE; }
  if (home_bits < 2 || home_bits > 16 || overflow_bits < 8 || overflow_bits > 30) {
    set_error("gs_set_peertx_capacity: home_bits in [2, 16], overflow_bits in [8, 30]");
    return GS_EINVAL;
  }
  return GS_OK;
}
int gs_set_frontier_mode(gs_engine* g, int32_t mode) {
  // the oracle walks every copy: no strategy to choose
  if (g->sim.started) { set_error("the frontier mode must be set before the first step"); return GS_ESTATE; }
  if (mode != GS_FRONTIER_AUTO && mode != GS_FRONTIER_LISTS && mode != GS_FRONTIER_BITMAPS) {
    set_error("gs_set_frontier_mode: GS_FRONTIER_AUTO, GS_FRONTIER_LISTS or GS_FRONTIER_BITMAPS");
    return GS_EINVAL;
  }
  return GS_OK;
}
int gs_frontier_dense(const gs_engine*) { return 0; }
int gs_set_trace_rpc(gs_engine* g, int32_t on) {
  if (g->sim.started) { set_error("tracing must be set before the first step"); return GS_ESTATE; }
  g->sim.traceRpc = on != 0;
  return GS_OK;
}
int gs_trace_read(gs_engine* g, gs_trace_event* out, int64_t cap, int64_t* n) {
  Sim& s = g->sim;
  if (s.traceRead == 0) {
    for (Node& nd : s.nodes) {
      s.events.insert(s.events.end(), nd.ev.begin(), nd.ev.end());
      nd.ev.clear();
    }
    gs_trace_canonical(s.events, s.cfg.seed, s.gp.MaxIHaveLength);
  }
  const int64_t k = std::min<int64_t>(cap, (int64_t)(s.events.size() - s.traceRead));
  for (int64_t i = 0; i < k; ++i) out[i] = s.events[s.traceRead + i];
  s.traceRead += (size_t)k;
  if (s.traceRead == s.events.size()) { s.events.clear(); s.traceRead = 0; }
  *n = k;
  return GS_OK;
}
int gs_trace_encode(const gs_trace_event*, int64_t, int32_t, int64_t, const char* const*, const char*, uint8_t*,
                    int64_t, int64_t* written) {
  *written = 0;
  set_error("gs_trace_encode is in the product library");
  return GS_EUNSUPPORTED;
}
// ---- gs_oracle_replay: one host replayed from its RecvRPC trace (see Replay)
int gs_oracle_replay_new(gs_engine* eng, int32_t node, void** out) {
  Sim& s = eng->sim;
  if (!out) { set_error("null argument"); return GS_EINVAL; }
  if (!s.graphSet || s.started) { set_error("gs_oracle_replay_new: set the graph, and do not step the engine"); return GS_ESTATE; }
  if (node < 0 || node >= s.N) { set_error("gs_oracle_replay_new: bad node"); return GS_EINVAL; }
  if (!s.sched.empty() || s.doPX || !s.dormant.empty() || s.acct) {
    set_error("gs_oracle_replay_new: churn, peer exchange, dormant slots and RPC accounting are not replayed");
    return GS_EUNSUPPORTED;
  }
  for (uint8_t d : s.directE)
    if (d) { set_error("gs_oracle_replay_new: direct peers are not replayed"); return GS_EUNSUPPORTED; }
  if (!s.mixedChecked) {
    const int rc = s.validateMixed();
    if (rc) return rc;
    s.mixedChecked = true;
  }
  if (s.traced.size() != (size_t)s.N) s.traced.assign((size_t)s.N, 0);
  s.traced[(size_t)node] = 1;
  s.traceRpc = true;
  s.record = false;  // the replayed host's deliveries are its DeliverMessage events
  std::unique_ptr<Replay> r(new Replay());
  r->sim = &eng->sim;
  s.solo = &r->nd;
  s.hop = 0;
  s.initNode(r->nd, node);
  for (int64_t e = s.rowptr[node]; e < s.rowptr[node + 1]; ++e) s.traceHello(node, s.col[e]);
  for (size_t k = 0; k < s.msgs.size(); ++k)
    if (s.msgs[k].from == node) r->myPubs.push_back((int64_t)k);
  *out = r.release();
  return GS_OK;
}

int gs_oracle_replay_run(void* h, int64_t hops, const gs_trace_event* ev, int64_t n) {
  Replay& r = *(Replay*)h;
  if (hops < 0 || n < 0 || (n > 0 && !ev)) { set_error("gs_oracle_replay_run: bad arguments"); return GS_EINVAL; }
  const int rc = replay_parse(r, ev, n);
  if (rc) return rc;
  for (int64_t i = 0; i < hops; ++i) replay_hop(r);
  return GS_OK;
}

// The replayed host's events since the last call, in canonical order.
int gs_oracle_replay_events(void* h, gs_trace_event* out, int64_t cap, int64_t* n) {
  Replay& r = *(Replay*)h;
  Sim& s = *r.sim;
  if (r.pendOut == 0) {
    r.pend.insert(r.pend.end(), r.nd.ev.begin(), r.nd.ev.end());
    r.nd.ev.clear();
    gs_trace_canonical(r.pend, s.cfg.seed, s.gp.MaxIHaveLength);
  }
  const int64_t k = std::min<int64_t>(cap, (int64_t)(r.pend.size() - r.pendOut));
  for (int64_t i = 0; i < k; ++i) out[i] = r.pend[r.pendOut + (size_t)i];
  r.pendOut += (size_t)k;
  if (r.pendOut == r.pend.size()) { r.pend.clear(); r.pendOut = 0; }
  *n = k;
  return GS_OK;
}

// The replayed host's router and score state per out-edge (CSR order of its
// row), per-topic arrays [edge * T + topic]; null pointers are skipped.
// Backoff reads 0 where the reference's map has no entry.
int gs_oracle_replay_state(void* h, uint64_t* mesh, uint64_t* fanout, int64_t* backoff, double* score, double* bp,
                           double* fmd, double* mmd, double* mfp, double* imd, int64_t* mesh_time,
                           int64_t* graft_time, uint8_t* flags) {
  Replay& r = *(Replay*)h;
  Sim& s = *r.sim;
  Node& nd = r.nd;
  const int T = s.T;
  const int deg = (int)nd.nbrs.size();
  for (int k = 0; k < deg; ++k) {
    const int p = nd.nbrs[(size_t)k];
    uint64_t m = 0, f = 0;
    for (auto& kv : nd.mesh) if (kv.second.count(p)) m |= 1ull << kv.first;
    for (auto& kv : nd.fanout) if (kv.second.count(p)) f |= 1ull << kv.first;
    if (mesh) mesh[k] = m;
    if (fanout) fanout[k] = f;
    if (score) score[k] = nd.Score(p);
    auto ps = nd.score.peerStats.find(p);
    if (bp) bp[k] = ps == nd.score.peerStats.end() ? 0.0 : ps->second.behaviourPenalty;
    for (int t = 0; t < T; ++t) {
      const size_t i = (size_t)k * T + t;
      if (backoff) {
        auto bt = nd.backoff.find(t);
        int64_t x = 0;
        if (bt != nd.backoff.end()) {
          auto be = bt->second.find(p);
          if (be != bt->second.end()) x = be->second;
        }
        backoff[i] = x;
      }
      TopicStats ts;
      if (ps != nd.score.peerStats.end()) {
        auto it = ps->second.topics.find(t);
        if (it != ps->second.topics.end()) ts = it->second;
      }
      if (fmd) fmd[i] = ts.firstMessageDeliveries;
      if (mmd) mmd[i] = ts.meshMessageDeliveries;
      if (mfp) mfp[i] = ts.meshFailurePenalty;
      if (imd) imd[i] = ts.invalidMessageDeliveries;
      if (mesh_time) mesh_time[i] = ts.meshTime;
      if (graft_time) graft_time[i] = ts.graftTime;
      if (flags) flags[i] = (uint8_t)((ts.inMesh ? 1 : 0) | (ts.meshMessageDeliveriesActive ? 2 : 0));
    }
  }
  return GS_OK;
}

void gs_oracle_replay_free(void* h) {
  Replay* r = (Replay*)h;
  if (!r) return;
  if (r->sim->solo == &r->nd) r->sim->solo = nullptr;
  delete r;
}

// Oracle-only: OpenMP threads the per-node phases use (bench.py's cpu_baseline).
int gs_oracle_threads(void) {
  int n = 1;
#pragma omp parallel
  {
#pragma omp single
    n = omp_get_num_threads();
  }
  return n;
}

// Oracle-only: sets the OpenMP threads of the per-node phases (bench.py's
// cpu_baseline times the sample at 1 thread and at the box's CPU share).
void gs_oracle_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

int gs_read_exchange_stats(gs_engine*, double* host_ms, int64_t* bytes_in) {
  *host_ms = 0;
  *bytes_in = 0;
  return GS_OK;
}

}  // extern "C"
