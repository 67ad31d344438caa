// oracle_core.hpp — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
//
// CPU restatement of the reference's per-router objects, following the Go
// source line by line with three canonicalisations:
//   * virtual clock: every time.Now() becomes an explicit `now` (int64 ns);
//   * map iteration in ascending key order (std::map / std::set);
//   * math/rand replaced by the keyed Philox stream of include/gs_rng.h.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load the oracle library.  Pinned by the reference's own known-answer tests
// (score_test.go, score_params_test.go, mcache_test.go, gossip_tracer_test.go,
// peer_gater_test.go) restated in tests/test_oracle_*.py.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/gossip_engine.h"
#include "../include/gs_rng.h"

namespace oracle {

static const int64_t kSecond = 1000000000LL;
static const int64_t kMillisecond = 1000000LL;
static const int64_t kTimeZero = INT64_MIN;  // Go's time.Time{} (IsZero)
static const int64_t kTimeCacheDuration = 120 * kSecond;  // pubsub.go:30

void set_error(const std::string& s);

inline bool isInvalidNumber(double x) { return std::isnan(x) || std::isinf(x); }  // score_params.go:291

// ---------------------------------------------------------------- params
inline void defaultGossipSubParams(gs_gossipsub_params* p) {  // gossipsub.go:226-255 (+ vars 32-59)
  p->D = 6; p->Dlo = 5; p->Dhi = 12; p->Dscore = 4; p->Dout = 2;
  p->HistoryLength = 5;
  p->HistoryGossip = 5;  // fork quirk: HistoryGossip = GossipSubHistoryLength (gossipsub.go:234)
  p->Dlazy = 6; p->GossipFactor = 0.25; p->GossipRetransmission = 3;
  p->HeartbeatInitialDelay = 100 * kMillisecond; p->HeartbeatInterval = 1 * kSecond;
  p->FanoutTTL = 60 * kSecond; p->PrunePeers = 16; p->PruneBackoff = 60 * kSecond;
  p->Connectors = 8; p->MaxPendingConnections = 128; p->ConnectionTimeout = 30 * kSecond;
  p->DirectConnectTicks = 300; p->DirectConnectInitialDelay = kSecond;
  p->OpportunisticGraftTicks = 60; p->OpportunisticGraftPeers = 2;
  p->GraftFloodThreshold = 10 * kSecond; p->MaxIHaveLength = 5000; p->MaxIHaveMessages = 10;
  p->IWantFollowupTime = 3 * kSecond;
}

// ScoreParameterDecayWithBase — score_params.go:282-287
inline double scoreParameterDecayWithBase(int64_t decay, int64_t base, double decayToZero) {
  double ticks = (double)(decay / base);
  return std::pow(decayToZero, 1 / ticks);
}

inline void defaultPeerGaterParams(gs_peer_gater_params* p) {  // peer_gater.go:19-28, 97-116
  p->Threshold = 0.33;
  p->GlobalDecay = scoreParameterDecayWithBase(2 * 60 * kSecond, kSecond, 0.01);
  p->SourceDecay = scoreParameterDecayWithBase(3600 * kSecond, kSecond, 0.01);
  p->DecayToZero = 0.01; p->DecayInterval = kSecond; p->RetainStats = 6 * 3600 * kSecond;
  p->Quiet = 60 * kSecond; p->DuplicateWeight = 0.125; p->IgnoreWeight = 1.0; p->RejectWeight = 16.0;
}

// PeerScoreThresholds.validate — score_params.go:34-51
inline int validateThresholds(const gs_peer_score_thresholds* p) {
  if (p->GossipThreshold > 0 || isInvalidNumber(p->GossipThreshold)) {
    set_error("invalid gossip threshold; it must be <= 0 and a valid number"); return GS_EINVAL; }
  if (p->PublishThreshold > 0 || p->PublishThreshold > p->GossipThreshold || isInvalidNumber(p->PublishThreshold)) {
    set_error("invalid publish threshold; it must be <= 0 and <= gossip threshold and a valid number"); return GS_EINVAL; }
  if (p->GraylistThreshold > 0 || p->GraylistThreshold > p->PublishThreshold || isInvalidNumber(p->GraylistThreshold)) {
    set_error("invalid graylist threshold; it must be <= 0 and <= publish threshold and a valid number"); return GS_EINVAL; }
  if (p->AcceptPXThreshold < 0 || isInvalidNumber(p->AcceptPXThreshold)) {
    set_error("invalid accept PX threshold; it must be >= 0 and a valid number"); return GS_EINVAL; }
  if (p->OpportunisticGraftThreshold < 0 || isInvalidNumber(p->OpportunisticGraftThreshold)) {
    set_error("invalid opportunistic grafting threshold; it must be >= 0 and a valid number"); return GS_EINVAL; }
  return GS_OK;
}

// TopicScoreParams.validate — score_params.go:200-268
inline int validateTopicParams(const gs_topic_score_params* p) {
#define TV(cond, msg) if (cond) { set_error(msg); return GS_EINVAL; }
  TV(p->TopicWeight < 0 || isInvalidNumber(p->TopicWeight), "invalid topic weight; must be >= 0 and a valid number");
  TV(p->TimeInMeshQuantum == 0, "invalid TimeInMeshQuantum; must be non zero");
  TV(p->TimeInMeshWeight < 0 || isInvalidNumber(p->TimeInMeshWeight), "invalid TimeInMeshWeight; must be positive (or 0 to disable) and a valid number");
  TV(p->TimeInMeshWeight != 0 && p->TimeInMeshQuantum <= 0, "invalid TimeInMeshQuantum; must be positive");
  TV(p->TimeInMeshWeight != 0 && (p->TimeInMeshCap <= 0 || isInvalidNumber(p->TimeInMeshCap)), "invalid TimeInMeshCap; must be positive and a valid number");
  TV(p->FirstMessageDeliveriesWeight < 0 || isInvalidNumber(p->FirstMessageDeliveriesWeight), "invallid FirstMessageDeliveriesWeight; must be positive (or 0 to disable) and a valid number");
  TV(p->FirstMessageDeliveriesWeight != 0 && (p->FirstMessageDeliveriesDecay <= 0 || p->FirstMessageDeliveriesDecay >= 1 || isInvalidNumber(p->FirstMessageDeliveriesDecay)), "invalid FirstMessageDeliveriesDecay; must be between 0 and 1");
  TV(p->FirstMessageDeliveriesWeight != 0 && (p->FirstMessageDeliveriesCap <= 0 || isInvalidNumber(p->FirstMessageDeliveriesCap)), "invalid FirstMessageDeliveriesCap; must be positive and a valid number");
  TV(p->MeshMessageDeliveriesWeight > 0 || isInvalidNumber(p->MeshMessageDeliveriesWeight), "invalid MeshMessageDeliveriesWeight; must be negative (or 0 to disable) and a valid number");
  TV(p->MeshMessageDeliveriesWeight != 0 && (p->MeshMessageDeliveriesDecay <= 0 || p->MeshMessageDeliveriesDecay >= 1 || isInvalidNumber(p->MeshMessageDeliveriesDecay)), "invalid MeshMessageDeliveriesDecay; must be between 0 and 1");
  TV(p->MeshMessageDeliveriesWeight != 0 && (p->MeshMessageDeliveriesCap <= 0 || isInvalidNumber(p->MeshMessageDeliveriesCap)), "invalid MeshMessageDeliveriesCap; must be positive and a valid number");
  TV(p->MeshMessageDeliveriesWeight != 0 && (p->MeshMessageDeliveriesThreshold <= 0 || isInvalidNumber(p->MeshMessageDeliveriesThreshold)), "invalid MeshMessageDeliveriesThreshold; must be positive and a valid number");
  TV(p->MeshMessageDeliveriesWindow < 0, "invalid MeshMessageDeliveriesWindow; must be non-negative");
  TV(p->MeshMessageDeliveriesWeight != 0 && p->MeshMessageDeliveriesActivation < kSecond, "invalid MeshMessageDeliveriesActivation; must be at least 1s");
  TV(p->MeshFailurePenaltyWeight > 0 || isInvalidNumber(p->MeshFailurePenaltyWeight), "invalid MeshFailurePenaltyWeight; must be negative (or 0 to disable) and a valid number");
  TV(p->MeshFailurePenaltyWeight != 0 && (isInvalidNumber(p->MeshFailurePenaltyDecay) || p->MeshFailurePenaltyDecay <= 0 || p->MeshFailurePenaltyDecay >= 1), "invalid MeshFailurePenaltyDecay; must be between 0 and 1");
  TV(p->InvalidMessageDeliveriesWeight > 0 || isInvalidNumber(p->InvalidMessageDeliveriesWeight), "invalid InvalidMessageDeliveriesWeight; must be negative (or 0 to disable) and a valid number");
  TV(p->InvalidMessageDeliveriesDecay <= 0 || p->InvalidMessageDeliveriesDecay >= 1 || isInvalidNumber(p->InvalidMessageDeliveriesDecay), "invalid InvalidMessageDeliveriesDecay; must be between 0 and 1");
  return GS_OK;
}

// PeerScoreParams.validate — score_params.go:151-198 (topics first, ascending)
inline int validatePeerScoreParams(const gs_peer_score_params* p, const gs_topic_score_params* topics,
                                   const uint8_t* scored, int T) {
  for (int t = 0; t < T; ++t) {
    if (scored && scored[t]) {
      int rc = validateTopicParams(&topics[t]);
      if (rc) return rc;
    }
  }
  TV(p->TopicScoreCap < 0 || isInvalidNumber(p->TopicScoreCap), "invalid topic score cap; must be positive (or 0 for no cap) and a valid number");
  TV(!p->AppSpecificScorePresent, "missing application specific score function");
  TV(p->IPColocationFactorWeight > 0 || isInvalidNumber(p->IPColocationFactorWeight), "invalid IPColocationFactorWeight; must be negative (or 0 to disable) and a valid number");
  TV(p->IPColocationFactorWeight != 0 && p->IPColocationFactorThreshold < 1, "invalid IPColocationFactorThreshold; must be at least 1");
  TV(p->BehaviourPenaltyWeight > 0 || isInvalidNumber(p->BehaviourPenaltyWeight), "invalid BehaviourPenaltyWeight; must be negative (or 0 to disable) and a valid number");
  TV(p->BehaviourPenaltyWeight != 0 && (p->BehaviourPenaltyDecay <= 0 || p->BehaviourPenaltyDecay >= 1 || isInvalidNumber(p->BehaviourPenaltyDecay)), "invalid BehaviourPenaltyDecay; must be between 0 and 1");
  TV(p->BehaviourPenaltyThreshold < 0 || isInvalidNumber(p->BehaviourPenaltyThreshold), "invalid BehaviourPenaltyThreshold; must be >= 0 and a valid number");
  TV(p->DecayInterval < kSecond, "invalid DecayInterval; must be at least 1s");
  TV(p->DecayToZero <= 0 || p->DecayToZero >= 1 || isInvalidNumber(p->DecayToZero), "invalid DecayToZero; must be between 0 and 1");
  return GS_OK;
}

// PeerGaterParams.validate — peer_gater.go:57-88
inline int validateGaterParams(const gs_peer_gater_params* p) {
  TV(p->Threshold <= 0, "invalid Threshold; must be > 0");
  TV(p->GlobalDecay <= 0 || p->GlobalDecay >= 1, "invalid GlobalDecay; must be between 0 and 1");
  TV(p->SourceDecay <= 0 || p->SourceDecay >= 1, "invalid SourceDecay; must be between 0 and 1");
  TV(p->DecayInterval < kSecond, "invalid DecayInterval; must be at least 1s");
  TV(p->DecayToZero <= 0 || p->DecayToZero >= 1, "invalid DecayToZero; must be between 0 and 1");
  TV(p->Quiet < kSecond, "invalud Quiet interval; must be at least 1s");
  TV(p->DuplicateWeight <= 0, "invalid DuplicateWeight; must be > 0");
  TV(p->IgnoreWeight < 1, "invalid IgnoreWeight; must be >= 1");
  TV(p->RejectWeight < 1, "invalud RejectWeight; must be >= 1");
#undef TV
  return GS_OK;
}

// ---------------------------------------------------------------- peerScore
// delivery record status — score.go:112-118
enum { deliveryUnknown = 0, deliveryValid, deliveryInvalid, deliveryIgnored, deliveryThrottled };

// reject reasons — tracer.go:28-38
enum RejectReason {
  RejectBlacklstedPeer = 0, RejectBlacklistedSource, RejectMissingSignature, RejectUnexpectedSignature,
  RejectUnexpectedAuthInfo, RejectInvalidSignature, RejectValidationQueueFull, RejectValidationThrottled,
  RejectValidationFailed, RejectValidationIgnored, RejectSelfOrigin
};

struct TopicStats {  // score.go:37-62
  bool inMesh = false;
  int64_t graftTime = 0;
  int64_t meshTime = 0;
  double firstMessageDeliveries = 0;
  double meshMessageDeliveries = 0;
  bool meshMessageDeliveriesActive = false;
  double meshFailurePenalty = 0;
  double invalidMessageDeliveries = 0;
};

struct PeerStats {  // score.go:17-35
  bool connected = false;
  int64_t expire = 0;
  std::map<int, TopicStats> topics;
  std::vector<uint32_t> ips;
  std::map<uint32_t, bool> ipWhitelist;
  double behaviourPenalty = 0;
};

// drec.peers (a Go map[peer.ID]struct{}): a sorted vector, iterated ascending
// like the std::set it replaces (a few peers per record; a tree node per peer
// made the mid-size goldens' millions of records the oracle's memory bound).
struct PeerSet {
  std::vector<int> v;
  size_t count(int p) const { return std::binary_search(v.begin(), v.end(), p) ? 1 : 0; }
  void insert(int p) {
    auto it = std::lower_bound(v.begin(), v.end(), p);
    if (it == v.end() || *it != p) v.insert(it, p);
  }
  void clear() { std::vector<int>().swap(v); }
  std::vector<int>::const_iterator begin() const { return v.begin(); }
  std::vector<int>::const_iterator end() const { return v.end(); }
};
struct DeliveryRecord {  // score.go:98-103
  int status = deliveryUnknown;
  int64_t firstSeen = 0;
  int64_t validated = kTimeZero;
  PeerSet peers;
};

struct Msg {  // the fields of pb.Message the hot path reads
  int64_t id;   // msgID (DefaultMsgIdFn(from || seqno), pubsub.go:973)
  int topic;    // GetTopic()
  int from;     // GetFrom(): the author (origin node), -1 = none
};

class PeerScore {
 public:
  gs_peer_score_params params{};
  std::map<int, gs_topic_score_params> topics;  // params.Topics
  std::map<int, PeerStats> peerStats;
  std::map<uint32_t, std::set<int>> peerIPs;
  std::unordered_map<int64_t, DeliveryRecord> records;  // messageDeliveries.records (never iterated)
  std::deque<std::pair<int64_t, int64_t>> gcQueue;  // (id, expire) head..tail
  std::function<double(int)> appSpecificScore = [](int) { return 0.0; };
  std::vector<std::pair<uint32_t, uint32_t>> whitelist;  // (net, mask)

  // SetTopicScoreParams — score.go:192-232
  void SetTopicScoreParams(int topic, const gs_topic_score_params& p) {
    auto it = topics.find(topic);
    bool exist = it != topics.end();
    gs_topic_score_params old{};
    if (exist) old = it->second;
    topics[topic] = p;
    if (!exist) return;
    bool recap = false;
    if (p.FirstMessageDeliveriesCap < old.FirstMessageDeliveriesCap) recap = true;
    if (p.MeshMessageDeliveriesCap < old.MeshMessageDeliveriesCap) recap = true;
    if (!recap) return;
    for (auto& kv : peerStats) {
      auto ts = kv.second.topics.find(topic);
      if (ts == kv.second.topics.end()) continue;
      if (ts->second.firstMessageDeliveries > p.FirstMessageDeliveriesCap)
        ts->second.firstMessageDeliveries = p.FirstMessageDeliveriesCap;
      if (ts->second.meshMessageDeliveries > p.MeshMessageDeliveriesCap)
        ts->second.meshMessageDeliveries = p.MeshMessageDeliveriesCap;
    }
  }

  // score — score.go:256-333 (topics summed in ascending topic order)
  double score(int p) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return 0;
    PeerStats& pstats = it->second;
    double score = 0;
    for (auto& kv : pstats.topics) {
      auto tp = topics.find(kv.first);
      if (tp == topics.end()) continue;
      const gs_topic_score_params& topicParams = tp->second;
      const TopicStats& tstats = kv.second;
      double topicScore = 0;
      if (tstats.inMesh) {  // P1
        double p1 = (double)(tstats.meshTime / topicParams.TimeInMeshQuantum);
        if (p1 > topicParams.TimeInMeshCap) p1 = topicParams.TimeInMeshCap;
        topicScore += p1 * topicParams.TimeInMeshWeight;
      }
      double p2 = tstats.firstMessageDeliveries;  // P2
      topicScore += p2 * topicParams.FirstMessageDeliveriesWeight;
      if (tstats.meshMessageDeliveriesActive) {  // P3
        if (tstats.meshMessageDeliveries < topicParams.MeshMessageDeliveriesThreshold) {
          double deficit = topicParams.MeshMessageDeliveriesThreshold - tstats.meshMessageDeliveries;
          double p3 = deficit * deficit;
          topicScore += p3 * topicParams.MeshMessageDeliveriesWeight;
        }
      }
      double p3b = tstats.meshFailurePenalty;  // P3b
      topicScore += p3b * topicParams.MeshFailurePenaltyWeight;
      double p4 = tstats.invalidMessageDeliveries * tstats.invalidMessageDeliveries;  // P4
      topicScore += p4 * topicParams.InvalidMessageDeliveriesWeight;
      score += topicScore * topicParams.TopicWeight;
    }
    if (params.TopicScoreCap > 0 && score > params.TopicScoreCap) score = params.TopicScoreCap;
    double p5 = appSpecificScore(p);  // P5
    score += p5 * params.AppSpecificWeight;
    double p6 = ipColocationFactor(p);  // P6
    score += p6 * params.IPColocationFactorWeight;
    if (pstats.behaviourPenalty > params.BehaviourPenaltyThreshold) {  // P7
      double excess = pstats.behaviourPenalty - params.BehaviourPenaltyThreshold;
      double p7 = excess * excess;
      score += p7 * params.BehaviourPenaltyWeight;
    }
    return score;
  }

  // ipColocationFactor — score.go:335-379 (IPv4 only; whitelist as net/mask)
  double ipColocationFactor(int p) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return 0;
    PeerStats& pstats = it->second;
    double result = 0;
    for (uint32_t ip : pstats.ips) {
      if (!whitelist.empty()) {
        auto w = pstats.ipWhitelist.find(ip);
        bool whitelisted;
        if (w == pstats.ipWhitelist.end()) {
          whitelisted = false;
          for (auto& nm : whitelist)
            if ((ip & nm.second) == (nm.first & nm.second)) { whitelisted = true; break; }
          pstats.ipWhitelist[ip] = whitelisted;
        } else {
          whitelisted = w->second;
        }
        if (whitelisted) continue;
      }
      int peersInIP = (int)peerIPs[ip].size();
      if (peersInIP > params.IPColocationFactorThreshold) {
        double surpluss = (double)(peersInIP - params.IPColocationFactorThreshold);
        result += surpluss * surpluss;
      }
    }
    return result;
  }

  // AddPenalty — score.go:382-396
  void AddPenalty(int p, int count) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    it->second.behaviourPenalty += (double)count;
  }

  // refreshScores — score.go:495-556
  void refreshScores(int64_t now) {
    for (auto it = peerStats.begin(); it != peerStats.end();) {
      PeerStats& pstats = it->second;
      if (!pstats.connected) {
        if (now > pstats.expire) {
          removeIPs(it->first, pstats.ips);
          it = peerStats.erase(it);
          continue;
        }
        ++it;
        continue;
      }
      for (auto& kv : pstats.topics) {
        auto tp = topics.find(kv.first);
        if (tp == topics.end()) continue;
        const gs_topic_score_params& topicParams = tp->second;
        TopicStats& tstats = kv.second;
        tstats.firstMessageDeliveries *= topicParams.FirstMessageDeliveriesDecay;
        if (tstats.firstMessageDeliveries < params.DecayToZero) tstats.firstMessageDeliveries = 0;
        tstats.meshMessageDeliveries *= topicParams.MeshMessageDeliveriesDecay;
        if (tstats.meshMessageDeliveries < params.DecayToZero) tstats.meshMessageDeliveries = 0;
        tstats.meshFailurePenalty *= topicParams.MeshFailurePenaltyDecay;
        if (tstats.meshFailurePenalty < params.DecayToZero) tstats.meshFailurePenalty = 0;
        tstats.invalidMessageDeliveries *= topicParams.InvalidMessageDeliveriesDecay;
        if (tstats.invalidMessageDeliveries < params.DecayToZero) tstats.invalidMessageDeliveries = 0;
        if (tstats.inMesh) {
          tstats.meshTime = now - tstats.graftTime;
          if (tstats.meshTime > topicParams.MeshMessageDeliveriesActivation)
            tstats.meshMessageDeliveriesActive = true;
        }
      }
      pstats.behaviourPenalty *= params.BehaviourPenaltyDecay;
      if (pstats.behaviourPenalty < params.DecayToZero) pstats.behaviourPenalty = 0;
      ++it;
    }
  }

  // AddPeer — score.go:586-600 (ips supplied by the caller instead of host.Network)
  void AddPeer(int p, const std::vector<uint32_t>& ips) {
    PeerStats& pstats = peerStats[p];
    pstats.connected = true;
    setIPs(p, ips, pstats.ips);
    pstats.ips = ips;
  }

  // RemovePeer — score.go:602-635
  void RemovePeer(int p, int64_t now) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    if (score(p) > 0) {
      removeIPs(p, it->second.ips);
      peerStats.erase(it);
      return;
    }
    PeerStats& pstats = it->second;
    for (auto& kv : pstats.topics) {
      TopicStats& tstats = kv.second;
      tstats.firstMessageDeliveries = 0;
      double threshold = topics[kv.first].MeshMessageDeliveriesThreshold;
      if (tstats.inMesh && tstats.meshMessageDeliveriesActive && tstats.meshMessageDeliveries < threshold) {
        double deficit = threshold - tstats.meshMessageDeliveries;
        tstats.meshFailurePenalty += deficit * deficit;
      }
      tstats.inMesh = false;
    }
    pstats.connected = false;
    pstats.expire = now + params.RetainScore;
  }

  TopicStats* getTopicStats(PeerStats& pstats, int topic) {  // score.go:865-880
    auto it = pstats.topics.find(topic);
    if (it != pstats.topics.end()) return &it->second;
    if (topics.find(topic) == topics.end()) return nullptr;
    return &pstats.topics[topic];
  }

  // Graft — score.go:640-658
  void Graft(int p, int topic, int64_t now) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    TopicStats* tstats = getTopicStats(it->second, topic);
    if (!tstats) return;
    tstats->inMesh = true;
    tstats->graftTime = now;
    tstats->meshTime = 0;
    tstats->meshMessageDeliveriesActive = false;
  }

  // Prune — score.go:660-682
  void Prune(int p, int topic) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    TopicStats* tstats = getTopicStats(it->second, topic);
    if (!tstats) return;
    double threshold = topics[topic].MeshMessageDeliveriesThreshold;
    if (tstats->meshMessageDeliveriesActive && tstats->meshMessageDeliveries < threshold) {
      double deficit = threshold - tstats->meshMessageDeliveries;
      tstats->meshFailurePenalty += deficit * deficit;
    }
    tstats->inMesh = false;
  }

  // ValidateMessage — score.go:684-691
  void ValidateMessage(const Msg& m, int64_t now) { (void)getRecord(m.id, now); }

  // DeliverMessage — score.go:693-717
  void DeliverMessage(const Msg& m, int receivedFrom, int64_t now) {
    markFirstMessageDelivery(receivedFrom, m);
    DeliveryRecord& drec = getRecord(m.id, now);
    if (drec.status != deliveryUnknown) return;
    drec.status = deliveryValid;
    drec.validated = now;
    for (int p : drec.peers)
      if (p != receivedFrom) markDuplicateMessageDelivery(p, m, kTimeZero, now);
  }

  // RejectMessage — score.go:719-784
  void RejectMessage(const Msg& m, int receivedFrom, int reason, int64_t now) {
    switch (reason) {
      case RejectMissingSignature: case RejectInvalidSignature: case RejectUnexpectedSignature:
      case RejectUnexpectedAuthInfo: case RejectSelfOrigin:
        markInvalidMessageDelivery(receivedFrom, m);
        return;
      case RejectBlacklstedPeer: case RejectBlacklistedSource: return;
      case RejectValidationQueueFull: return;
    }
    DeliveryRecord& drec = getRecord(m.id, now);
    if (drec.status != deliveryUnknown) return;
    switch (reason) {
      case RejectValidationThrottled: drec.status = deliveryThrottled; drec.peers.clear(); return;
      case RejectValidationIgnored: drec.status = deliveryIgnored; drec.peers.clear(); return;
    }
    drec.status = deliveryInvalid;
    markInvalidMessageDelivery(receivedFrom, m);
    for (int p : drec.peers) markInvalidMessageDelivery(p, m);
    drec.peers.clear();
  }

  // DuplicateMessage — score.go:786-818.  Returns true when the duplicate
  // was counted for the first time (used by the simulator's invariants).
  bool DuplicateMessage(const Msg& m, int receivedFrom, int64_t now) {
    DeliveryRecord& drec = getRecord(m.id, now);
    if (drec.peers.count(receivedFrom)) return false;
    switch (drec.status) {
      case deliveryUnknown: drec.peers.insert(receivedFrom); break;
      case deliveryValid:
        drec.peers.insert(receivedFrom);
        markDuplicateMessageDelivery(receivedFrom, m, drec.validated, now);
        break;
      case deliveryInvalid: markInvalidMessageDelivery(receivedFrom, m); break;
      default: break;
    }
    return true;
  }

  // getRecord — score.go:823-844
  DeliveryRecord& getRecord(int64_t id, int64_t now) {
    auto it = records.find(id);
    if (it != records.end()) return it->second;
    DeliveryRecord& rec = records[id];
    rec.firstSeen = now;
    gcQueue.emplace_back(id, now + kTimeCacheDuration);
    return rec;
  }

  // gc — score.go:846-860
  void gc(int64_t now) {
    while (!gcQueue.empty() && now > gcQueue.front().second) {
      records.erase(gcQueue.front().first);
      gcQueue.pop_front();
    }
  }
  void expireHead(int64_t t) { if (!gcQueue.empty()) gcQueue.front().second = t; }

  // markInvalidMessageDelivery — score.go:884-897
  void markInvalidMessageDelivery(int p, const Msg& m) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    TopicStats* tstats = getTopicStats(it->second, m.topic);
    if (!tstats) return;
    tstats->invalidMessageDeliveries += 1;
  }

  // markFirstMessageDelivery — score.go:902-929
  void markFirstMessageDelivery(int p, const Msg& m) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    TopicStats* tstats = getTopicStats(it->second, m.topic);
    if (!tstats) return;
    double cap = topics[m.topic].FirstMessageDeliveriesCap;
    tstats->firstMessageDeliveries += 1;
    if (tstats->firstMessageDeliveries > cap) tstats->firstMessageDeliveries = cap;
    if (!tstats->inMesh) return;
    cap = topics[m.topic].MeshMessageDeliveriesCap;
    tstats->meshMessageDeliveries += 1;
    if (tstats->meshMessageDeliveries > cap) tstats->meshMessageDeliveries = cap;
  }

  // markDuplicateMessageDelivery — score.go:934-964
  void markDuplicateMessageDelivery(int p, const Msg& m, int64_t validated, int64_t now) {
    auto it = peerStats.find(p);
    if (it == peerStats.end()) return;
    TopicStats* tstats = getTopicStats(it->second, m.topic);
    if (!tstats) return;
    if (!tstats->inMesh) return;
    const gs_topic_score_params& tparams = topics[m.topic];
    if (validated != kTimeZero && now - validated > tparams.MeshMessageDeliveriesWindow) return;
    double cap = tparams.MeshMessageDeliveriesCap;
    tstats->meshMessageDeliveries += 1;
    if (tstats->meshMessageDeliveries > cap) tstats->meshMessageDeliveries = cap;
  }

  // setIPs — score.go:1011-1049
  void setIPs(int p, const std::vector<uint32_t>& newips, const std::vector<uint32_t>& oldips) {
    for (uint32_t ip : newips) {
      bool inOld = false;
      for (uint32_t x : oldips) if (x == ip) { inOld = true; break; }
      if (inOld) continue;
      peerIPs[ip].insert(p);
    }
    for (uint32_t ip : oldips) {
      bool inNew = false;
      for (uint32_t x : newips) if (x == ip) { inNew = true; break; }
      if (inNew) continue;
      auto it = peerIPs.find(ip);
      if (it == peerIPs.end()) continue;
      it->second.erase(p);
      if (it->second.empty()) peerIPs.erase(it);
    }
  }

  // removeIPs — score.go:1052-1064
  void removeIPs(int p, const std::vector<uint32_t>& ips) {
    for (uint32_t ip : ips) {
      auto it = peerIPs.find(ip);
      if (it == peerIPs.end()) continue;
      it->second.erase(p);
      if (it->second.empty()) peerIPs.erase(it);
    }
  }
};

// ---------------------------------------------------------------- MessageCache
// mcache.go:23-104.  Messages are identified by id; the cache keeps (id, topic).
class MessageCache {
 public:
  struct Entry { int64_t mid; int topic; };
  std::map<int64_t, Msg> msgs;
  std::map<int64_t, std::map<int, int>> peertx;
  std::vector<std::vector<Entry>> history;
  int gossip = 0;

  MessageCache() {}
  MessageCache(int gossip_, int historyLen) { init(gossip_, historyLen); }
  bool init(int gossip_, int historyLen) {  // NewMessageCache — panics if gossip > history
    if (gossip_ > historyLen) {
      set_error("invalid parameters for message cache; gossip slots cannot be larger than history slots");
      return false;
    }
    history.assign(historyLen, {});
    gossip = gossip_;
    msgs.clear(); peertx.clear();
    return true;
  }
  void Put(const Msg& m) {  // mcache.go:55-59
    msgs[m.id] = m;
    history[0].push_back({m.id, m.topic});
  }
  bool Get(int64_t mid, Msg* out = nullptr) const {  // mcache.go:61-64
    auto it = msgs.find(mid);
    if (it == msgs.end()) return false;
    if (out) *out = it->second;
    return true;
  }
  bool GetForPeer(int64_t mid, int p, Msg* out, int* count) {  // mcache.go:66-80
    auto it = msgs.find(mid);
    if (it == msgs.end()) return false;
    int& c = peertx[mid][p];
    c++;
    if (out) *out = it->second;
    *count = c;
    return true;
  }
  std::vector<int64_t> GetGossipIDs(int topic) const {  // mcache.go:82-92
    std::vector<int64_t> mids;
    for (int i = 0; i < gossip; ++i)
      for (const Entry& e : history[i])
        if (e.topic == topic) mids.push_back(e.mid);
    return mids;
  }
  void Shift() {  // mcache.go:94-104
    for (const Entry& e : history.back()) { msgs.erase(e.mid); peertx.erase(e.mid); }
    for (int i = (int)history.size() - 2; i >= 0; --i) history[i + 1] = history[i];
    history[0].clear();
  }
};

// ---------------------------------------------------------------- gossipTracer
// gossip_tracer.go:15-181.  AddPromise's rand.Intn(len) index is supplied by
// the caller (the simulator passes 0 after a keyed shuffle).
class GossipTracer {
 public:
  int64_t followUpTime = 3 * kSecond;
  std::map<int64_t, std::map<int, int64_t>> promises;
  std::map<int, std::set<int64_t>> peerPromises;

  void AddPromise(int p, const std::vector<int64_t>& msgIDs, size_t idx, int64_t now) {  // :48-75
    int64_t mid = msgIDs[idx];
    auto& pr = promises[mid];
    if (!pr.count(p)) {
      pr[p] = now + followUpTime;
      peerPromises[p].insert(mid);
    }
  }
  std::map<int, int> GetBrokenPromises(int64_t now) {  // :79-115
    std::map<int, int> res;
    for (auto it = promises.begin(); it != promises.end();) {
      for (auto jt = it->second.begin(); jt != it->second.end();) {
        if (jt->second < now) {
          res[jt->first]++;
          auto pp = peerPromises.find(jt->first);
          if (pp != peerPromises.end()) {
            pp->second.erase(it->first);
            if (pp->second.empty()) peerPromises.erase(pp);
          }
          jt = it->second.erase(jt);
        } else {
          ++jt;
        }
      }
      if (it->second.empty()) it = promises.erase(it); else ++it;
    }
    return res;
  }
  void fulfillPromise(int64_t mid) { promises.erase(mid); }  // :119-126
  void DeliverMessage(int64_t mid) { fulfillPromise(mid); }
  void ValidateMessage(int64_t mid) { fulfillPromise(mid); }
  void RejectMessage(int64_t mid, int reason) {  // :133-146
    if (reason == RejectMissingSignature || reason == RejectInvalidSignature) return;
    fulfillPromise(mid);
  }
  void ThrottlePeer(int p) {  // :163-181
    auto pp = peerPromises.find(p);
    if (pp == peerPromises.end()) return;
    for (int64_t mid : pp->second) {
      auto it = promises.find(mid);
      if (it == promises.end()) continue;
      it->second.erase(p);
      if (it->second.empty()) promises.erase(it);
    }
    peerPromises.erase(pp);
  }
};

// ---------------------------------------------------------------- peerGater
// peer_gater.go:119-442.  getIP is supplied by the caller.
class PeerGater {
 public:
  enum { AcceptNone = 0, AcceptControl = 1, AcceptAll = 2 };  // pubsub.go:191-199 (values)
  struct Stats { int connected = 0; int64_t expire = 0; double deliver = 0, duplicate = 0, ignore = 0, reject = 0; };
  gs_peer_gater_params params{};
  double validate = 0, throttle = 0;
  int64_t lastThrottle = kTimeZero;
  std::map<int, uint32_t> peerStats;          // peer -> ip key (shared Stats per IP)
  std::map<uint32_t, Stats> ipStats;
  std::function<uint32_t(int)> getIP = [](int) { return 0u; };

  Stats& getPeerStats(int p) {  // :262-269
    auto it = peerStats.find(p);
    if (it == peerStats.end()) {
      uint32_t ip = getIP(p);
      peerStats[p] = ip;
      return ipStats[ip];
    }
    return ipStats[it->second];
  }
  void decayStats(int64_t now) {  // :219-260
    validate *= params.GlobalDecay;
    if (validate < params.DecayToZero) validate = 0;
    throttle *= params.GlobalDecay;
    if (throttle < params.DecayToZero) throttle = 0;
    for (auto it = ipStats.begin(); it != ipStats.end();) {
      Stats& st = it->second;
      if (st.connected > 0) {
        st.deliver *= params.SourceDecay; if (st.deliver < params.DecayToZero) st.deliver = 0;
        st.duplicate *= params.SourceDecay; if (st.duplicate < params.DecayToZero) st.duplicate = 0;
        st.ignore *= params.SourceDecay; if (st.ignore < params.DecayToZero) st.ignore = 0;
        st.reject *= params.SourceDecay; if (st.reject < params.DecayToZero) st.reject = 0;
      } else if (st.expire < now) {
        it = ipStats.erase(it);
        continue;
      }
      ++it;
    }
  }
  // The per-peer part of AcceptFrom (:340-357): (1 + deliver) / (1 + total),
  // or -1 when total == 0 (AcceptAll).
  double acceptThreshold(int p) {
    Stats& st = getPeerStats(p);
    double total = st.deliver + params.DuplicateWeight * st.duplicate + params.IgnoreWeight * st.ignore +
                   params.RejectWeight * st.reject;
    if (total == 0) return -1;
    return (1 + st.deliver) / (1 + total);
  }
  // AcceptFrom — :320-363.  `u` is the uniform draw replacing rand.Float64().
  int AcceptFrom(int p, int64_t now, double u) {
    if (lastThrottle == kTimeZero || now - lastThrottle > params.Quiet) return AcceptAll;
    if (throttle == 0) return AcceptAll;
    if (validate != 0 && throttle / validate < params.Threshold) return AcceptAll;
    Stats& st = getPeerStats(p);
    double total = st.deliver + params.DuplicateWeight * st.duplicate + params.IgnoreWeight * st.ignore +
                   params.RejectWeight * st.reject;
    if (total == 0) return AcceptAll;
    double threshold = (1 + st.deliver) / (1 + total);
    if (u < threshold) return AcceptAll;
    return AcceptControl;
  }
  void AddPeer(int p) { getPeerStats(p).connected++; }  // :366-372
  void RemovePeer(int p, int64_t now) {  // :374-383
    Stats& st = getPeerStats(p);
    st.connected--;
    st.expire = now + params.RetainStats;
    peerStats.erase(p);
  }
  void ValidateMessage() { validate++; }           // :390-395
  void DeliverMessage(int p) { getPeerStats(p).deliver += 1; }  // :397-411 (weight 1)
  void RejectMessage(int p, int reason, int64_t now) {  // :413-432
    switch (reason) {
      case RejectValidationQueueFull: case RejectValidationThrottled:
        lastThrottle = now; throttle++; break;
      case RejectValidationIgnored: getPeerStats(p).ignore++; break;
      default: getPeerStats(p).reject++; break;
    }
  }
  void DuplicateMessage(int p) { getPeerStats(p).duplicate++; }  // :434-440
};

}  // namespace oracle
