// gs_params.cpp — product-side parameter defaults and validation (host).
//
// Mirrors score_params.go:34-51 (PeerScoreThresholds.validate), :151-198
// (PeerScoreParams.validate), :200-268 (TopicScoreParams.validate), :277-287
// (ScoreParameterDecay*), gossipsub.go:226-255 (DefaultGossipSubParams) and
// peer_gater.go:57-116 (PeerGaterParams).  Error strings are the reference's.
#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/gossip_engine.h"
#include "gs_host.h"

static const int64_t kSec = 1000000000LL;
static const int64_t kMs = 1000000LL;

static bool invalid(double x) { return std::isnan(x) || std::isinf(x); }

#define CHECK(cond, msg)        \
  do {                          \
    if (cond) {                 \
      gs_set_error(msg);        \
      return GS_EINVAL;         \
    }                           \
  } while (0)

extern "C" {

int gs_abi_version(void) { return GS_ABI_VERSION; }

void gs_default_gossipsub_params(gs_gossipsub_params* p) {
  p->D = 6; p->Dlo = 5; p->Dhi = 12; p->Dscore = 4; p->Dout = 2;
  p->HistoryLength = 5;
  p->HistoryGossip = 5;  // = GossipSubHistoryLength (fork quirk, gossipsub.go:234)
  p->Dlazy = 6; p->GossipFactor = 0.25; p->GossipRetransmission = 3;
  p->HeartbeatInitialDelay = 100 * kMs; p->HeartbeatInterval = kSec; p->FanoutTTL = 60 * kSec;
  p->PrunePeers = 16; p->PruneBackoff = 60 * kSec; p->Connectors = 8; p->MaxPendingConnections = 128;
  p->ConnectionTimeout = 30 * kSec; p->DirectConnectTicks = 300; p->DirectConnectInitialDelay = kSec;
  p->OpportunisticGraftTicks = 60; p->OpportunisticGraftPeers = 2; p->GraftFloodThreshold = 10 * kSec;
  p->MaxIHaveLength = 5000; p->MaxIHaveMessages = 10; p->IWantFollowupTime = 3 * kSec;
}

double gs_score_parameter_decay_with_base(int64_t decay, int64_t base, double decayToZero) {
  double ticks = (double)(decay / base);
  return std::pow(decayToZero, 1 / ticks);
}

double gs_score_parameter_decay(int64_t decay) { return gs_score_parameter_decay_with_base(decay, kSec, 0.01); }

void gs_default_peer_gater_params(gs_peer_gater_params* p) {
  p->Threshold = 0.33;
  p->GlobalDecay = gs_score_parameter_decay(2 * 60 * kSec);
  p->SourceDecay = gs_score_parameter_decay(3600 * kSec);
  p->DecayInterval = kSec; p->DecayToZero = 0.01; p->RetainStats = 6 * 3600 * kSec; p->Quiet = 60 * kSec;
  p->DuplicateWeight = 0.125; p->IgnoreWeight = 1.0; p->RejectWeight = 16.0;
}

int gs_validate_thresholds(const gs_peer_score_thresholds* p) {
  CHECK(p->GossipThreshold > 0 || invalid(p->GossipThreshold),
        "invalid gossip threshold; it must be <= 0 and a valid number");
  CHECK(p->PublishThreshold > 0 || p->PublishThreshold > p->GossipThreshold || invalid(p->PublishThreshold),
        "invalid publish threshold; it must be <= 0 and <= gossip threshold and a valid number");
  CHECK(p->GraylistThreshold > 0 || p->GraylistThreshold > p->PublishThreshold || invalid(p->GraylistThreshold),
        "invalid graylist threshold; it must be <= 0 and <= publish threshold and a valid number");
  CHECK(p->AcceptPXThreshold < 0 || invalid(p->AcceptPXThreshold),
        "invalid accept PX threshold; it must be >= 0 and a valid number");
  CHECK(p->OpportunisticGraftThreshold < 0 || invalid(p->OpportunisticGraftThreshold),
        "invalid opportunistic grafting threshold; it must be >= 0 and a valid number");
  return GS_OK;
}

int gs_validate_topic_score_params(const gs_topic_score_params* p) {
  CHECK(p->TopicWeight < 0 || invalid(p->TopicWeight), "invalid topic weight; must be >= 0 and a valid number");
  CHECK(p->TimeInMeshQuantum == 0, "invalid TimeInMeshQuantum; must be non zero");
  CHECK(p->TimeInMeshWeight < 0 || invalid(p->TimeInMeshWeight),
        "invalid TimeInMeshWeight; must be positive (or 0 to disable) and a valid number");
  CHECK(p->TimeInMeshWeight != 0 && p->TimeInMeshQuantum <= 0, "invalid TimeInMeshQuantum; must be positive");
  CHECK(p->TimeInMeshWeight != 0 && (p->TimeInMeshCap <= 0 || invalid(p->TimeInMeshCap)),
        "invalid TimeInMeshCap; must be positive and a valid number");
  CHECK(p->FirstMessageDeliveriesWeight < 0 || invalid(p->FirstMessageDeliveriesWeight),
        "invallid FirstMessageDeliveriesWeight; must be positive (or 0 to disable) and a valid number");
  CHECK(p->FirstMessageDeliveriesWeight != 0 &&
            (p->FirstMessageDeliveriesDecay <= 0 || p->FirstMessageDeliveriesDecay >= 1 ||
             invalid(p->FirstMessageDeliveriesDecay)),
        "invalid FirstMessageDeliveriesDecay; must be between 0 and 1");
  CHECK(p->FirstMessageDeliveriesWeight != 0 &&
            (p->FirstMessageDeliveriesCap <= 0 || invalid(p->FirstMessageDeliveriesCap)),
        "invalid FirstMessageDeliveriesCap; must be positive and a valid number");
  CHECK(p->MeshMessageDeliveriesWeight > 0 || invalid(p->MeshMessageDeliveriesWeight),
        "invalid MeshMessageDeliveriesWeight; must be negative (or 0 to disable) and a valid number");
  CHECK(p->MeshMessageDeliveriesWeight != 0 &&
            (p->MeshMessageDeliveriesDecay <= 0 || p->MeshMessageDeliveriesDecay >= 1 ||
             invalid(p->MeshMessageDeliveriesDecay)),
        "invalid MeshMessageDeliveriesDecay; must be between 0 and 1");
  CHECK(p->MeshMessageDeliveriesWeight != 0 &&
            (p->MeshMessageDeliveriesCap <= 0 || invalid(p->MeshMessageDeliveriesCap)),
        "invalid MeshMessageDeliveriesCap; must be positive and a valid number");
  CHECK(p->MeshMessageDeliveriesWeight != 0 &&
            (p->MeshMessageDeliveriesThreshold <= 0 || invalid(p->MeshMessageDeliveriesThreshold)),
        "invalid MeshMessageDeliveriesThreshold; must be positive and a valid number");
  CHECK(p->MeshMessageDeliveriesWindow < 0, "invalid MeshMessageDeliveriesWindow; must be non-negative");
  CHECK(p->MeshMessageDeliveriesWeight != 0 && p->MeshMessageDeliveriesActivation < kSec,
        "invalid MeshMessageDeliveriesActivation; must be at least 1s");
  CHECK(p->MeshFailurePenaltyWeight > 0 || invalid(p->MeshFailurePenaltyWeight),
        "invalid MeshFailurePenaltyWeight; must be negative (or 0 to disable) and a valid number");
  CHECK(p->MeshFailurePenaltyWeight != 0 &&
            (invalid(p->MeshFailurePenaltyDecay) || p->MeshFailurePenaltyDecay <= 0 ||
             p->MeshFailurePenaltyDecay >= 1),
        "invalid MeshFailurePenaltyDecay; must be between 0 and 1");
  CHECK(p->InvalidMessageDeliveriesWeight > 0 || invalid(p->InvalidMessageDeliveriesWeight),
        "invalid InvalidMessageDeliveriesWeight; must be negative (or 0 to disable) and a valid number");
  CHECK(p->InvalidMessageDeliveriesDecay <= 0 || p->InvalidMessageDeliveriesDecay >= 1 ||
            invalid(p->InvalidMessageDeliveriesDecay),
        "invalid InvalidMessageDeliveriesDecay; must be between 0 and 1");
  return GS_OK;
}

int gs_validate_peer_score_params(const gs_peer_score_params* p, const gs_topic_score_params* topics,
                                  const uint8_t* scored, int32_t T) {
  for (int t = 0; t < T; ++t) {
    if (scored && scored[t]) {
      int rc = gs_validate_topic_score_params(&topics[t]);
      if (rc) return rc;
    }
  }
  CHECK(p->TopicScoreCap < 0 || invalid(p->TopicScoreCap),
        "invalid topic score cap; must be positive (or 0 for no cap) and a valid number");
  CHECK(!p->AppSpecificScorePresent, "missing application specific score function");
  CHECK(p->IPColocationFactorWeight > 0 || invalid(p->IPColocationFactorWeight),
        "invalid IPColocationFactorWeight; must be negative (or 0 to disable) and a valid number");
  CHECK(p->IPColocationFactorWeight != 0 && p->IPColocationFactorThreshold < 1,
        "invalid IPColocationFactorThreshold; must be at least 1");
  CHECK(p->BehaviourPenaltyWeight > 0 || invalid(p->BehaviourPenaltyWeight),
        "invalid BehaviourPenaltyWeight; must be negative (or 0 to disable) and a valid number");
  CHECK(p->BehaviourPenaltyWeight != 0 &&
            (p->BehaviourPenaltyDecay <= 0 || p->BehaviourPenaltyDecay >= 1 || invalid(p->BehaviourPenaltyDecay)),
        "invalid BehaviourPenaltyDecay; must be between 0 and 1");
  CHECK(p->BehaviourPenaltyThreshold < 0 || invalid(p->BehaviourPenaltyThreshold),
        "invalid BehaviourPenaltyThreshold; must be >= 0 and a valid number");
  CHECK(p->DecayInterval < kSec, "invalid DecayInterval; must be at least 1s");
  CHECK(p->DecayToZero <= 0 || p->DecayToZero >= 1 || invalid(p->DecayToZero),
        "invalid DecayToZero; must be between 0 and 1");
  return GS_OK;
}

int gs_validate_peer_gater_params(const gs_peer_gater_params* p) {
  CHECK(p->Threshold <= 0, "invalid Threshold; must be > 0");
  CHECK(p->GlobalDecay <= 0 || p->GlobalDecay >= 1, "invalid GlobalDecay; must be between 0 and 1");
  CHECK(p->SourceDecay <= 0 || p->SourceDecay >= 1, "invalid SourceDecay; must be between 0 and 1");
  CHECK(p->DecayInterval < kSec, "invalid DecayInterval; must be at least 1s");
  CHECK(p->DecayToZero <= 0 || p->DecayToZero >= 1, "invalid DecayToZero; must be between 0 and 1");
  CHECK(p->Quiet < kSec, "invalud Quiet interval; must be at least 1s");
  CHECK(p->DuplicateWeight <= 0, "invalid DuplicateWeight; must be > 0");
  CHECK(p->IgnoreWeight < 1, "invalid IgnoreWeight; must be >= 1");
  CHECK(p->RejectWeight < 1, "invalud RejectWeight; must be >= 1");
  return GS_OK;
}

}  // extern "C"
