// oracle_objects.cpp — TEST INFRASTRUCTURE ONLY.
//
// Flat C exports of the single-router objects in oracle_core.hpp so the
// reference's own known-answer unit tests (score_test.go, mcache_test.go,
// gossip_tracer_test.go, peer_gater_test.go) can be restated in pytest
// against exactly the code the simulator runs.  Peer ids are small ints
// ("A" = 0, "B" = 1, ...); message ids are ints; time is explicit (ns).
#include "oracle_core.hpp"

using namespace oracle;

struct ops_obj {
  PeerScore ps;
  std::vector<double> app;  // AppSpecificScore(p) values
};

extern "C" {

// ---- peerScore ----
ops_obj* ops_new(const gs_peer_score_params* p) {
  ops_obj* o = new ops_obj();
  o->ps.params = *p;
  o->app.assign(64, 0.0);
  o->ps.appSpecificScore = [o](int peer) { return o->app[peer]; };
  return o;
}
void ops_free(ops_obj* o) { delete o; }
void ops_set_app_score(ops_obj* o, int p, double v) {
  if (p >= (int)o->app.size()) o->app.resize((size_t)p + 1, 0.0);
  o->app[p] = v;
}
// State injection (tests/test_fullsize_gpu.py): the engine's counters of one
// (edge, topic) become peer p's TopicStats, so score() (score.go:256-333) is
// recomputed by the oracle's own code from state the oracle cannot simulate
// at full size.  flags: bit0 inMesh, bit1 meshMessageDeliveriesActive.
void ops_set_stats(ops_obj* o, int p, int topic, int flags, int64_t graft_time, int64_t mesh_time, double fmd,
                   double mmd, double mfp, double imd) {
  TopicStats& ts = o->ps.peerStats[p].topics[topic];
  ts.inMesh = (flags & 1) != 0;
  ts.meshMessageDeliveriesActive = (flags & 2) != 0;
  ts.graftTime = graft_time;
  ts.meshTime = mesh_time;
  ts.firstMessageDeliveries = fmd;
  ts.meshMessageDeliveries = mmd;
  ts.meshFailurePenalty = mfp;
  ts.invalidMessageDeliveries = imd;
}
void ops_set_behaviour_penalty(ops_obj* o, int p, double bp) { o->ps.peerStats[p].behaviourPenalty = bp; }
void ops_set_topic(ops_obj* o, int topic, const gs_topic_score_params* tp) { o->ps.topics[topic] = *tp; }
void ops_set_topic_score_params(ops_obj* o, int topic, const gs_topic_score_params* tp) {
  o->ps.SetTopicScoreParams(topic, *tp);
}
void ops_add_whitelist(ops_obj* o, uint32_t net, uint32_t mask) { o->ps.whitelist.push_back({net, mask}); }
void ops_add_peer(ops_obj* o, int p) { o->ps.AddPeer(p, {}); }
void ops_remove_peer(ops_obj* o, int p, int64_t now) { o->ps.RemovePeer(p, now); }
// setIPsForPeer (score_test.go:1073-1080): setIPs(p, ips, {}) then pstats.ips = ips
void ops_set_ips(ops_obj* o, int p, int n, const uint32_t* ips) {
  std::vector<uint32_t> v(ips, ips + n);
  o->ps.setIPs(p, v, {});
  auto it = o->ps.peerStats.find(p);
  if (it != o->ps.peerStats.end()) it->second.ips = v;
}
double ops_score(ops_obj* o, int p) { return o->ps.score(p); }
void ops_graft(ops_obj* o, int p, int topic, int64_t now) { o->ps.Graft(p, topic, now); }
void ops_prune(ops_obj* o, int p, int topic) { o->ps.Prune(p, topic); }
void ops_add_penalty(ops_obj* o, int p, int count) { o->ps.AddPenalty(p, count); }
void ops_refresh(ops_obj* o, int64_t now) { o->ps.refreshScores(now); }
void ops_validate(ops_obj* o, int64_t mid, int topic, int from, int64_t now) {
  o->ps.ValidateMessage(Msg{mid, topic, -1}, now); (void)from;
}
void ops_deliver(ops_obj* o, int64_t mid, int topic, int from, int64_t now) {
  o->ps.DeliverMessage(Msg{mid, topic, -1}, from, now);
}
void ops_duplicate(ops_obj* o, int64_t mid, int topic, int from, int64_t now) {
  o->ps.DuplicateMessage(Msg{mid, topic, -1}, from, now);
}
void ops_reject(ops_obj* o, int64_t mid, int topic, int from, int reason, int64_t now) {
  o->ps.RejectMessage(Msg{mid, topic, -1}, from, reason, now);
}
void ops_gc(ops_obj* o, int64_t now) { o->ps.gc(now); }
void ops_expire_head(ops_obj* o, int64_t t) { o->ps.expireHead(t); }
int ops_topic_stats(ops_obj* o, int p, int topic, double* out4) {
  auto it = o->ps.peerStats.find(p);
  if (it == o->ps.peerStats.end()) return -1;
  auto ts = it->second.topics.find(topic);
  if (ts == it->second.topics.end()) return -1;
  out4[0] = ts->second.firstMessageDeliveries;
  out4[1] = ts->second.meshMessageDeliveries;
  out4[2] = ts->second.meshFailurePenalty;
  out4[3] = ts->second.invalidMessageDeliveries;
  return 0;
}

// ---- MessageCache ----
MessageCache* omc_new(int gossip, int history) {
  MessageCache* m = new MessageCache();
  if (!m->init(gossip, history)) { delete m; return nullptr; }
  return m;
}
void omc_free(MessageCache* m) { delete m; }
void omc_put(MessageCache* m, int64_t mid, int topic) { m->Put(Msg{mid, topic, -1}); }
int omc_get(MessageCache* m, int64_t mid) { return m->Get(mid) ? 1 : 0; }
int omc_get_for_peer(MessageCache* m, int64_t mid, int p) {
  int c = 0;
  return m->GetForPeer(mid, p, nullptr, &c) ? c : -1;
}
int omc_gossip_ids(MessageCache* m, int topic, int64_t* out, int cap) {
  auto v = m->GetGossipIDs(topic);
  int n = (int)v.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = v[i];
  return n;
}
int omc_len(MessageCache* m) { return (int)m->msgs.size(); }
void omc_shift(MessageCache* m) { m->Shift(); }

// ---- gossipTracer ----
GossipTracer* ogt_new(int64_t follow_up) {
  GossipTracer* g = new GossipTracer();
  g->followUpTime = follow_up;
  return g;
}
void ogt_free(GossipTracer* g) { delete g; }
void ogt_add_promise(GossipTracer* g, int p, int n, const int64_t* mids, int idx, int64_t now) {
  g->AddPromise(p, std::vector<int64_t>(mids, mids + n), (size_t)idx, now);
}
// writes (peer, count) pairs; returns number of peers with broken promises
int ogt_broken(GossipTracer* g, int64_t now, int* peers, int* counts, int cap) {
  auto r = g->GetBrokenPromises(now);
  int i = 0;
  for (auto& kv : r) { if (i < cap) { peers[i] = kv.first; counts[i] = kv.second; } ++i; }
  return i;
}
void ogt_deliver(GossipTracer* g, int64_t mid) { g->DeliverMessage(mid); }
void ogt_throttle(GossipTracer* g, int p) { g->ThrottlePeer(p); }

// ---- peerGater ----
PeerGater* opg_new(const gs_peer_gater_params* p, const uint32_t* ip_of_peer, int npeers) {
  PeerGater* g = new PeerGater();
  g->params = *p;
  std::vector<uint32_t> ips(ip_of_peer, ip_of_peer + npeers);
  g->getIP = [ips](int peer) { return peer < (int)ips.size() ? ips[peer] : 0xFFFFFFFFu; };
  return g;
}
void opg_free(PeerGater* g) { delete g; }
void opg_add_peer(PeerGater* g, int p) { g->AddPeer(p); }
void opg_remove_peer(PeerGater* g, int p, int64_t now) { g->RemovePeer(p, now); }
int opg_accept_from(PeerGater* g, int p, int64_t now, double u) { return g->AcceptFrom(p, now, u); }
void opg_validate(PeerGater* g) { g->ValidateMessage(); }
void opg_deliver(PeerGater* g, int p) { g->DeliverMessage(p); }
void opg_duplicate(PeerGater* g, int p) { g->DuplicateMessage(p); }
void opg_reject(PeerGater* g, int p, int reason, int64_t now) { g->RejectMessage(p, reason, now); }
void opg_decay(PeerGater* g, int64_t now) { g->decayStats(now); }
int opg_has_peer_stats(PeerGater* g, int p) { return g->peerStats.count(p) ? 1 : 0; }
int opg_has_ip_stats(PeerGater* g, uint32_t ip) { return g->ipStats.count(ip) ? 1 : 0; }
void opg_set_ip_expire(PeerGater* g, uint32_t ip, int64_t t) { g->ipStats[ip].expire = t; }

// ---- RNG ----
uint64_t orng_key64(uint32_t seed, uint32_t site, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return gs_key64(seed, site, a, b, c, d);
}
uint64_t orng_key64_mid(uint32_t seed, uint32_t site, uint32_t a, uint32_t b, uint32_t mid, uint32_t d) {
  return gs_key64_mid(seed, site, a, b, mid, d);
}
void orng_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) { gs_philox4x32_10(ctr, key, out); }

}  // extern "C"
