/*
 * gossip_engine.h — C-ABI of the MI355X batched gossip engine.
 *
 * One engine handle simulates N go-libp2p-pubsub routers in lock step over a
 * static peer graph.  It is the drop-in boundary for the router hot path of
 * the reference (seveirbian/go-libp2p-pubsub, mounted at /root/reference):
 *
 *   PubSubRouter interface           pubsub.go:158-187
 *   FloodSubRouter.Publish           floodsub.go:76-100
 *   RandomSubRouter.Publish          randomsub.go:99-160
 *   GossipSubRouter (Publish, HandleRPC, heartbeat, emitGossip, Join)
 *                                    gossipsub.go:591-1078, 1299-1712
 *   MessageCache                     mcache.go:23-104
 *   peerScore (score, refreshScores, delivery hooks)
 *                                    score.go:256-964
 *   gossipTracer promises            gossip_tracer.go:48-126
 *
 * Every entry point takes plain host pointers and sizes (the caller owns all
 * host arrays; they are copied in and out).  The engine owns device memory.
 * Return value: GS_OK (0) or a negative GS_E* code; gs_last_error() returns a
 * thread-local message for the most recent failure.  A handle must not be
 * used concurrently (mirrors the single processLoop goroutine, pubsub.go:471).
 *
 * Durations are int64 nanoseconds (Go time.Duration).  Peers are int32 node
 * indices, topics are int32 indices in [0, num_topics), messages are int64
 * ids assigned by gs_publish in publish order.
 *
 * Two libraries export this ABI:
 *   libgossip_engine.so  — the product: HIP kernels for gfx950 (MI355X).
 *   oracle/_build/libgossip_oracle.so — the CPU restatement used ONLY by
 *                          tests/bench as the parity checker.
 */
#ifndef GOSSIP_ENGINE_H
#define GOSSIP_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 3

/* ---- error codes ------------------------------------------------------- */
#define GS_OK 0
#define GS_EINVAL (-1)       /* invalid argument / parameter validation failed */
#define GS_ESTATE (-2)       /* call not valid in the engine's current state */
#define GS_ENOMEM (-3)       /* host or device allocation failed */
#define GS_EDEVICE (-4)      /* HIP runtime error / no device */
#define GS_ECAPACITY (-5)    /* a bounded table or the message window overflowed */
#define GS_EUNSUPPORTED (-6) /* configuration outside what this build supports */

/* ---- router selection (NewFloodSub / NewRandomSub / NewGossipSub) ------ */
#define GS_ROUTER_FLOODSUB 0  /* floodsub.go:25  */
#define GS_ROUTER_RANDOMSUB 1 /* randomsub.go:21 */
#define GS_ROUTER_GOSSIPSUB 2 /* gossipsub.go:198 */

/* ---- engine flags ------------------------------------------------------ */
#define GS_FLAG_SCORING (1u << 0)       /* WithPeerScore (gossipsub.go:258)    */
#define GS_FLAG_FLOOD_PUBLISH (1u << 1) /* WithFloodPublish (gossipsub.go:304) */
#define GS_FLAG_PEER_EXCHANGE (1u << 3) /* WithPeerExchange (gossipsub.go:320): PRUNEs carry
                                           up to PrunePeers peers (makePrune :1803-1839); a
                                           pruned host connects to them (pxConnect :856-905)
                                           when the pruner's score is >= AcceptPXThreshold.
                                           A connection needs a slot in the graph: an edge of
                                           gs_set_graph that is down (gs_set_dormant, churn) */
#define GS_FLAG_RECORD_DELIVERIES (1u << 2) /* keep per-(node,message) first
                                               delivery hop/sender for readback */

/* GossipSubParams — gossipsub.go:62-195, defaults gossipsub.go:226-255. */
typedef struct gs_gossipsub_params {
  int32_t D, Dlo, Dhi, Dscore, Dout;
  int32_t HistoryLength, HistoryGossip;
  int32_t Dlazy;
  double GossipFactor;
  int32_t GossipRetransmission;
  int64_t HeartbeatInitialDelay;
  int64_t HeartbeatInterval;
  int64_t FanoutTTL;
  int32_t PrunePeers;
  int64_t PruneBackoff;
  int32_t Connectors;
  int32_t MaxPendingConnections;
  int64_t ConnectionTimeout;
  uint64_t DirectConnectTicks;
  int64_t DirectConnectInitialDelay;
  uint64_t OpportunisticGraftTicks;
  int32_t OpportunisticGraftPeers;
  int64_t GraftFloodThreshold;
  int32_t MaxIHaveLength;
  int32_t MaxIHaveMessages;
  int64_t IWantFollowupTime;
} gs_gossipsub_params;

/* PeerScoreParams — score_params.go:53-96.  AppSpecificScore (a Go func) is
 * replaced by a per-node array given to gs_set_peer_attrs; the flag below
 * says whether that function "is set" for validation (score_params.go:165). */
typedef struct gs_peer_score_params {
  double TopicScoreCap;
  int32_t AppSpecificScorePresent;
  double AppSpecificWeight;
  double IPColocationFactorWeight;
  int32_t IPColocationFactorThreshold;
  double BehaviourPenaltyWeight;
  double BehaviourPenaltyThreshold;
  double BehaviourPenaltyDecay;
  int64_t DecayInterval;
  double DecayToZero;
  int64_t RetainScore;
} gs_peer_score_params;

/* TopicScoreParams — score_params.go:98-148. */
typedef struct gs_topic_score_params {
  double TopicWeight;
  double TimeInMeshWeight;
  int64_t TimeInMeshQuantum;
  double TimeInMeshCap;
  double FirstMessageDeliveriesWeight;
  double FirstMessageDeliveriesDecay;
  double FirstMessageDeliveriesCap;
  double MeshMessageDeliveriesWeight;
  double MeshMessageDeliveriesDecay;
  double MeshMessageDeliveriesCap;
  double MeshMessageDeliveriesThreshold;
  int64_t MeshMessageDeliveriesWindow;
  int64_t MeshMessageDeliveriesActivation;
  double MeshFailurePenaltyWeight;
  double MeshFailurePenaltyDecay;
  double InvalidMessageDeliveriesWeight;
  double InvalidMessageDeliveriesDecay;
} gs_topic_score_params;

/* PeerScoreThresholds — score_params.go:12-32. */
typedef struct gs_peer_score_thresholds {
  double GossipThreshold;
  double PublishThreshold;
  double GraylistThreshold;
  double AcceptPXThreshold;
  double OpportunisticGraftThreshold;
} gs_peer_score_thresholds;

/* PeerGaterParams — peer_gater.go:31-55 (TopicDeliveryWeights omitted). */
typedef struct gs_peer_gater_params {
  double Threshold;
  double GlobalDecay;
  double SourceDecay;
  int64_t DecayInterval;
  double DecayToZero;
  int64_t RetainStats;
  int64_t Quiet;
  double DuplicateWeight;
  double IgnoreWeight;
  double RejectWeight;
} gs_peer_gater_params;

/* Engine configuration (not a reference struct: the simulator's own knobs). */
typedef struct gs_config {
  int32_t router;          /* GS_ROUTER_* */
  int32_t randomsub_size;  /* NewRandomSub(size) */
  int32_t num_nodes;       /* N */
  int32_t num_topics;      /* T, 1..64 */
  int32_t slots_per_topic; /* message window per topic, multiple of 64 */
  uint32_t seed;           /* counter-based RNG seed (replaces math/rand) */
  int64_t hop_ns;          /* virtual time per propagation hop */
  uint32_t flags;          /* GS_FLAG_* */
  int32_t device;          /* HIP device ordinal (product library only) */
} gs_config;

/* Aggregate counters since create (read with gs_read_counters). */
typedef struct gs_counters {
  int64_t hops;
  int64_t heartbeats;
  int64_t published;       /* local publishes (PublishMessage)               */
  int64_t deliveries;      /* first deliveries (DeliverMessage)              */
  int64_t duplicates;      /* duplicate receptions (DuplicateMessage)        */
  int64_t transmissions;   /* message copies delivered over edges (counted on arrival), dups included */
  int64_t grafts_sent;     /* GRAFT control entries sent                     */
  int64_t prunes_sent;     /* PRUNE control entries sent                     */
  int64_t ihave_sent;      /* IHAVE control entries sent (one per topic)     */
  int64_t iwant_sent;      /* message ids requested through IWANT            */
  int64_t iwant_served;    /* messages served in response to IWANT           */
  int64_t promises_broken; /* broken IWANT promises turned into P7 penalties */
  int64_t graylisted;      /* RPCs dropped by AcceptFrom == AcceptNone       */
  int64_t rejected;        /* messages rejected by validation (ValidationReject
                              / ValidationIgnore, validation.go:331-336)      */
  int64_t throttled;       /* copies dropped by a full validation queue
                              (RejectValidationQueueFull, validation.go:236-241) */
  int64_t gated;           /* payload RPCs dropped by the peer gater
                              (AcceptControl, pubsub.go:951-955)              */
} gs_counters;

/* ---- defaults / helpers ------------------------------------------------ */
int gs_abi_version(void);
const char* gs_last_error(void);
void gs_default_gossipsub_params(gs_gossipsub_params* out); /* gossipsub.go:226 */
void gs_default_peer_gater_params(gs_peer_gater_params* out); /* peer_gater.go:114 */
/* ScoreParameterDecayWithBase — score_params.go:282-287. */
double gs_score_parameter_decay_with_base(int64_t decay, int64_t base, double decay_to_zero);
double gs_score_parameter_decay(int64_t decay); /* score_params.go:277 */
/* validate() — score_params.go:34-51, 151-198, 200-268; peer_gater.go:57-88. */
int gs_validate_thresholds(const gs_peer_score_thresholds* p);
int gs_validate_peer_score_params(const gs_peer_score_params* p,
                                  const gs_topic_score_params* topics,
                                  const uint8_t* topic_scored, int32_t num_topics);
int gs_validate_topic_score_params(const gs_topic_score_params* p);
int gs_validate_peer_gater_params(const gs_peer_gater_params* p);

/* ---- engine lifecycle -------------------------------------------------- */
typedef struct gs_engine gs_engine;

/* Creates the engine.  gossipsub/score/threshold/gater params may be NULL
 * when unused by the router.  gater != NULL enables the peer gater
 * (WithPeerGater, peer_gater.go:164-191; gossipsub only).  topics[T] and topic_scored[T] give the
 * PeerScoreParams.Topics map (topic_scored[t] != 0 <=> key present). */
int gs_engine_create(const gs_config* cfg, const gs_gossipsub_params* gsp,
                     const gs_peer_score_params* psp,
                     const gs_topic_score_params* topics,
                     const uint8_t* topic_scored,
                     const gs_peer_score_thresholds* thr,
                     const gs_peer_gater_params* gater, gs_engine** out);
int gs_engine_destroy(gs_engine* eng);

/* Static symmetric graph in CSR: neighbours of node u are col[rowptr[u] ..
 * rowptr[u+1]), strictly ascending, each edge present in both directions.
 * outbound[e] != 0: u dialed col[e] (AddPeer direction, gossipsub.go:505-532).
 * direct[e]   != 0: col[e] is a direct peer of u (WithDirectPeers).  NULL = 0. */
int gs_set_graph(gs_engine* eng, const int64_t* rowptr, const int32_t* col,
                 const uint8_t* outbound, const uint8_t* direct);

/* ---- mixed networks: routers per host, protocols per connection -------- */
/* The protocol.ID a connection runs, as PubSubRouter.AddPeer(peer.ID,
 * protocol.ID) receives it (pubsub.go:165; gossipsub.go:505, randomsub.go:49,
 * floodsub.go:44).  Both hosts of a connection run the same protocol (the one
 * multistream-select negotiated: the first of the dialer's Protocols() the
 * listener supports, gossipsub.go:29-30 GossipSubDefaultProtocols). */
#define GS_PROTO_DEFAULT 0       /* the engine's own: the router of cfg.router     */
#define GS_PROTO_FLOODSUB 1      /* /floodsub/1.0.0   floodsub.go:12              */
#define GS_PROTO_RANDOMSUB 2     /* /randomsub/1.0.0  randomsub.go:13             */
#define GS_PROTO_GOSSIPSUB_V10 3 /* /meshsub/1.0.0    gossipsub.go:23: mesh, no PX */
#define GS_PROTO_GOSSIPSUB_V11 4 /* /meshsub/1.1.0    gossipsub.go:26: mesh + PX   */
/* gs_set_graph plus proto[e] (GS_PROTO_*, NULL: negotiated from the hosts'
 * routers, gs_set_routers).  proto[e] must be one both hosts speak and equal
 * on both directions of the connection (checked at the first step).  A
 * gossipsub host sends to a FLOODSUB / RANDOMSUB-protocol peer as to a
 * floodsub peer: it forwards every message of the peer's topics when the
 * peer's score >= PublishThreshold (gossipsub.go:969-975), never grafts it or
 * gossips to it (GossipSubFeatureMesh, gossipsub_feat.go:27-38, getPeers
 * :1849, emitGossip :1681) and counts it in EnoughPeers (:557-562); to a
 * GOSSIPSUB_V10 peer its PRUNEs carry neither PX nor a backoff (makePrune
 * :1804-1807).  A randomsub host always forwards to its FLOODSUB-protocol
 * peers and samples only its RANDOMSUB-protocol ones (randomsub.go:117-150). */
int gs_set_graph_ex(gs_engine* eng, const int64_t* rowptr, const int32_t* col,
                    const uint8_t* outbound, const uint8_t* direct, const uint8_t* proto);
/* The router each host runs (NewFloodSub / NewRandomSub / NewGossipSub):
 * router[u] = GS_ROUTER_FLOODSUB, GS_ROUTER_RANDOMSUB (NewRandomSub with
 * cfg.randomsub_size), GS_ROUTER_GOSSIPSUB (protocols v1.1, v1.0, floodsub)
 * or GS_ROUTER_GOSSIPSUB_V10 (a gossipsub host speaking only v1.0 and
 * floodsub: WithGossipSubProtocols, gossipsub_feat.go:41-56).  NULL: every
 * host runs cfg.router.  Gossipsub hosts need cfg.router == GS_ROUTER_GOSSIPSUB
 * (their params, scoring, peer gater and options come from the engine);
 * attacker behaviours (gs_set_behaviour) need gossipsub hosts.  Before the
 * first step. */
#define GS_ROUTER_GOSSIPSUB_V10 3
int gs_set_routers(gs_engine* eng, const uint8_t* router /*[N]*/);
/* PubSubRouter.EnoughPeers(topic, suggested) of every host (gossipsub.go:
 * 549-576, randomsub.go:59-89, floodsub.go:52-66) at the current state:
 * out[u] = 1 / 0 (a partitioned engine fills its own nodes, 0 elsewhere). */
int gs_enough_peers(gs_engine* eng, int32_t topic, int32_t suggested, uint8_t* out /*[N]*/);
/* Topic subscriptions (bit t of sub_mask[u]): Join(t) at hop 0. */
int gs_set_subscriptions(gs_engine* eng, const uint64_t* sub_mask);
/* Per-node attributes: app_score[N] (P5, AppSpecificScore), ipv4[N] (P6),
 * either may be NULL (zeros). */
int gs_set_peer_attrs(gs_engine* eng, const double* app_score, const uint32_t* ipv4);
/* IPColocationFactorWhitelist as IPv4 (net, mask) pairs. */
int gs_set_ip_whitelist(gs_engine* eng, int32_t n, const uint32_t* net, const uint32_t* mask);

/* Schedules n local publishes (Topic.Publish at node src[i] at hop hop[i]).
 * hop[] must be non-decreasing and >= the engine's current hop.  Message ids
 * are assigned in call order and written to ids_out (may be NULL). */
int gs_publish(gs_engine* eng, int32_t n, const int32_t* src, const int32_t* topic,
               const int64_t* hop, int64_t* ids_out);

/* ---- adversarial model ---------------------- */
/* Message kinds (gs_publish_ex).  REJECT / IGNORE are the verdict every
 * receiver's topic validator returns (RegisterTopicValidator, validation.go;
 * they apply on topics with a validator, gs_set_validation, else the message
 * is valid); the author forwards it without validating (an attacker).
 * PHANTOM: an id the author advertises in IHAVE (it sits in the author's
 * mcache) but never sends or serves — IHAVE spam of unpublished ids
 * (gossipsub_spam_test.go:135-270), whose IWANT promises break (P7). */
#define GS_MSG_VALID 0
#define GS_MSG_REJECT 1
#define GS_MSG_IGNORE 2
#define GS_MSG_PHANTOM 3
/* gs_publish with a kind per message (kind == NULL: all valid). */
int gs_publish_ex(gs_engine* eng, int32_t n, const int32_t* src, const int32_t* topic,
                  const int64_t* hop, const uint8_t* kind, int64_t* ids_out);
/* Topic validators (topic_validator[t] != 0: RegisterTopicValidator(t)) and
 * the validation queue: at most queue_per_hop received messages enter
 * validation per node per hop (0 = unlimited); later fresh copies are
 * dropped with RejectValidationQueueFull (validation.go:236-241), which is
 * what drives the peer gater (peer_gater.go:413-420).  Before the first step.
 * Signature policy: the model is StrictNoSign (unsigned messages).  Only topics
 * with a validator pass through the queue; under the reference's default
 * StrictSign every received message would (validation.Push, validation.go:233
 * queues when a topic has validators OR the message carries a signature), so
 * queue-full drops and the gater inputs they feed occur more often there. */
int gs_set_validation(gs_engine* eng, const uint8_t* topic_validator, int32_t queue_per_hop);
/* Per-node behaviour bits (simulated attackers, restating the reference's
 * attack mocks).  Before the first step; NULL = all honest. */
#define GS_BEHAVE_NO_FORWARD 1u /* sybilSquatter (gossipsub_test.go:1781-1815): relays
                                   nothing, serves no IWANT, emits no IHAVE */
#define GS_BEHAVE_IWANT_SPAM 2u /* re-requests every message it receives from its
                                   sender (gossipsub_spam_test.go:24-132)      */
#define GS_BEHAVE_GRAFT_SPAM 4u /* every heartbeat re-GRAFTs the topic peers it is
                                   in backoff with (gossipsub_spam_test.go:349-548) */
#define GS_BEHAVE_IHAVE_SPAM 8u /* emitGossip to every topic peer, mesh peers included
                                   (IHAVE spam, gossipsub_spam_test.go:196-222) */
int gs_set_behaviour(gs_engine* eng, const uint8_t* behaviour /*[N]*/);

/* Connection churn and subscription changes: a schedule of events, applied at
 * the start of their hop in the order given (hops non-decreasing across calls,
 * >= 1 and >= the current hop).
 *   GS_EV_DISCONNECT (a, b): the connection between nodes a and b (an edge
 *     pair of the graph) goes down.  Both hosts run handleDeadPeers
 *     (pubsub.go:521-551): the peer leaves every topic map, then
 *     GossipSubRouter.RemovePeer (gossipsub.go:534-547: mesh, fanout, pending
 *     gossip dropped, tracer.RemovePeer -> peerScore.RemovePeer score.go:602-635:
 *     a positive score is dropped, otherwise retained for RetainScore with
 *     firstMessageDeliveries reset and the mesh delivery penalty applied).  RPCs
 *     still in flight on the connection are lost.
 *   GS_EV_CONNECT (a, b): the connection comes back: AddPeer on both hosts
 *     (gossipsub.go:505-532, score.go:586-600 revives a retained record), the
 *     hello packet's subscriptions known at once (pubsub.go:495-497).
 *   GS_EV_LEAVE (a, topic b): node a unsubscribes (handleRemoveSubscription
 *     pubsub.go:665-686): announce (the peers update their topic maps when it
 *     arrives, next hop), then Leave (gossipsub.go:1062-1078: PRUNE every mesh
 *     peer).
 *   GS_EV_JOIN (a, topic b): node a subscribes (handleAddSubscription
 *     pubsub.go:692-713): announce, then Join (gossipsub.go:1011-1060).
 * An event that finds its state already (a connection down twice, a topic
 * left twice) does nothing.  With the peer gater, a disconnect is its
 * RemovePeer (the IP's stats expire RetainStats after its last peer left,
 * peer_gater.go:366-383) and a connect its AddPeer (a live stats object is
 * revived); a partitioned engine applies every event on every rank,
 * each rank launching the side of a connection it owns.
 * Direct peers (gs_set_graph's direct flags) that are not connected are
 * dialled by the connector at hop ceil(DirectConnectInitialDelay / hop_ns)
 * (gossipsub.go:492-502) and at every heartbeat whose tick count is a
 * multiple of DirectConnectTicks (directConnect, gossipsub.go:1594-1616); a
 * dial made during hop h connects at the start of hop h + 1, after that hop's
 * scheduled disconnects and connects (AddPeer both ways, hellos).
 * DirectConnectTicks = 0 is GS_EINVAL at creation (the reference divides by
 * it). */
/* Before the first step: the connections a[i]-b[i] (edges of the graph, both
 * directions) start down: no AddPeer, no hello, no score record.  A
 * GS_EV_CONNECT, a peer-exchange connect (GS_FLAG_PEER_EXCHANGE) or a direct
 * peer's dial brings one up.  A PX-suggested peer without such a slot cannot
 * be dialled (the reference's connector dials any peer; the simulated graph
 * is fixed). */
int gs_set_dormant(gs_engine* eng, int32_t n, const int32_t* a, const int32_t* b);
#define GS_EV_DISCONNECT 0
#define GS_EV_CONNECT 1
#define GS_EV_LEAVE 2
#define GS_EV_JOIN 3
int gs_schedule_events(gs_engine* eng, int32_t n, const int32_t* kind, const int32_t* a, const int32_t* b,
                       const int64_t* hop);

/* Advances the simulation by `hops` lock-step hops. */
/* Before the first step: the mcache.peertx tables (mcache.go:66-80, the
 * GossipRetransmission counts of handleIWant): 2^home_bits slots per node
 * (default 10; 12 with IWANT spammers, 2..16) and a per-rank overflow table of
 * 2^overflow_bits entries (default 16; 20 with IWANT spammers, 8..30) that takes
 * the keys of nodes whose own table is full.  Only a full overflow table is a
 * GS_ECAPACITY error of gs_step.  Replaces no reference call: the reference's
 * peertx is an unbounded Go map. */
int gs_set_peertx_capacity(gs_engine* eng, int32_t home_bits, int32_t overflow_bits);
/* Before the first step: how phase A reads what the senders forwarded.
 * GS_FRONTIER_AUTO (default): frontier bitmaps where they measured faster
 * (floodsub without per-copy records), per-copy lists elsewhere.
 * GS_FRONTIER_LISTS: lists everywhere.  GS_FRONTIER_BITMAPS: bitmaps wherever
 * the engine supports them (also gossipsub on one topic without the
 * adversarial model, churn, PX or a P3 window shorter than a message's
 * lifetime; one rank).  Results are identical; only speed differs.  Replaces
 * no reference call (an engine strategy knob).  gs_frontier_dense: 1 once
 * started if phase A reads bitmaps. */
#define GS_FRONTIER_AUTO 0
#define GS_FRONTIER_LISTS 1
#define GS_FRONTIER_BITMAPS 2
int gs_set_frontier_mode(gs_engine* eng, int32_t mode);
int gs_frontier_dense(const gs_engine* eng);
int gs_step(gs_engine* eng, int64_t hops);
/* Waits for all queued device work (no-op on the oracle). */
int gs_sync(gs_engine* eng);

/* Replaces topic score params at the current time (Topic.SetScoreParams ->
 * peerScore.SetTopicScoreParams, score.go:192-232, including the recap). */
int gs_set_topic_score_params(gs_engine* eng, int32_t topic, const gs_topic_score_params* p);

/* ---- partitioned engines: one rank per GPU ------------ */
/* The reference runs one router per host and its only cross-host traffic is
 * RPCs (handleIncomingRPC / sendRPC, pubsub.go:902-970, gossipsub.go:1092-
 * 1156).  A partitioned engine owns a contiguous node range (balanced by
 * edges, gs_partition_range) and simulates only those routers; at the end of
 * every hop the RPCs its nodes sent to other ranks' nodes are exchanged
 * through the host transport below (RCCL all-gather / all-to-all over xGMI in
 * the Python host; any transport with the same semantics works).  Every rank
 * must make the same sequence of set_graph / set_subscriptions / publish /
 * step calls.  Callbacks return 0 on success and are called from gs_step on
 * the calling thread, with no device work of the engine pending. */
typedef struct gs_transport {
  void* user;
  /* all[r*n + i] = rank r's mine[i] (host memory, n int64 per rank). */
  int (*allgather_i64)(void* user, const int64_t* mine, int32_t n, int64_t* all);
  /* Device buffers: recv[r*bytes .. (r+1)*bytes) = rank r's send[0..bytes). */
  int (*allgather)(void* user, const void* send, void* recv, int64_t bytes);
  /* Device buffers: send holds the blocks for ranks 0..world-1 back to back
   * (send_bytes[r] each); recv receives rank r's block for this rank at the
   * prefix offset of recv_bytes[0..r). */
  int (*alltoallv)(void* user, const void* send, const int64_t* send_bytes, void* recv,
                   const int64_t* recv_bytes);
} gs_transport;
/* Before the first step.  world == 1 (the default) simulates the whole graph;
 * the transport is copied (it may be NULL then).  The oracle supports
 * world == 1 only. */
int gs_set_partition(gs_engine* eng, int32_t rank, int32_t world, const gs_transport* tr);
/* A partitioned rank holds the state of its owned nodes and of their edges
 * [rowptr[node_begin], rowptr[node_end)) only: the per-edge readbacks
 * (gs_read_mesh, gs_read_fanout, gs_read_scores, gs_read_behaviour_penalty,
 * gs_read_backoff, gs_read_topic_stats, gs_read_rpc_bytes) fill the owned
 * edges and zero the rest, so the ranks' arrays together are the whole graph's. */
/* Nodes [node_begin, node_end) owned by this rank (after gs_set_graph). */
int gs_partition_range(const gs_engine* eng, int32_t* node_begin, int32_t* node_end);
/* Host time spent in the transport and bytes received from other ranks. */
int gs_read_exchange_stats(gs_engine* eng, double* host_ms, int64_t* bytes_in);

/* ---- RPC byte accounting ---------------------- */
/* The reference's sendRPC measures every outgoing RPC (out.Size(),
 * gossipsub.go:1121-1137); pubsub.go sends the hello packet (pubsub.go:495,
 * 534) and subscription announcements (pubsub.go:775-792).  With accounting
 * on, the engine sums the protobuf size (include/gs_rpcsize.h) and the count of
 * every RPC each host sends, per directed edge: forwarded and published
 * messages, GRAFT / PRUNE / IHAVE / IWANT control, IWANT replies, hellos (for
 * every connection at the start and on every reconnect) and announcements.
 * Sizes: a message of topic t is msg_size[t] bytes (its Message.Size()),
 * every message id id_len bytes, topic t's name topic_len[t] bytes.  Before
 * the first step.  A partitioned rank counts the RPCs its own nodes send. */
int gs_set_rpc_accounting(gs_engine* eng, const int32_t* msg_size /*[T]*/, int32_t id_len,
                          const int32_t* topic_len /*[T]*/);
/* Peer exchange under accounting: a PRUNE's PX entries (makePrune,
 * gossipsub.go:1811-1836) are PeerInfo{peerID, signedPeerRecord} of
 * peer_id_len and record_len bytes (record_len 0: no certified address book,
 * the record is nil and absent).  Defaults 38 (an Ed25519 peer id) and 0.
 * Before the first step. */
int gs_set_rpc_px_sizes(gs_engine* eng, int32_t peer_id_len, int32_t record_len);
/* bytes[e], rpcs[e]: totals sent by node u to col[e] (rowptr[u] <= e <
 * rowptr[u+1]) since the start (either array may be NULL); a partitioned rank
 * fills its own edges and zeroes the others. */
int gs_read_rpc_bytes(gs_engine* eng, int64_t* bytes /*[E]*/, int64_t* rpcs /*[E]*/);

/* ---- readbacks (host arrays sized by the caller) ----------------------- */
/* A partitioned engine reports its own nodes / edges only: counters count its
 * nodes' events, per-edge arrays are valid on its edges [rowptr[node_begin],
 * rowptr[node_end]) and zero elsewhere, per-node arrays on its nodes (-1
 * elsewhere). */
int64_t gs_num_edges(const gs_engine* eng);
int64_t gs_current_hop(const gs_engine* eng);
int gs_read_counters(gs_engine* eng, gs_counters* out);
/* Score(p) for every edge (observer u, neighbour col[e]) at the current state. */
int gs_read_scores(gs_engine* eng, double* score /*[E]*/);
/* mesh / fanout topic masks per edge (bit t: col[e] in mesh[t] of u). */
int gs_read_mesh(gs_engine* eng, uint64_t* mesh /*[E]*/);
int gs_read_fanout(gs_engine* eng, uint64_t* fanout /*[E]*/);
/* backoff expiry (ns) per [t*E + e]; 0 = no backoff entry. */
int gs_read_backoff(gs_engine* eng, int64_t* expire /*[T*E]*/);
/* peerStats topic counters per [t*E + e]; flags bit0 inMesh, bit1 P3 active. */
int gs_read_topic_stats(gs_engine* eng, double* fmd, double* mmd, double* mfp,
                        double* imd, int64_t* mesh_time, int64_t* graft_time,
                        uint8_t* flags);
int gs_read_behaviour_penalty(gs_engine* eng, double* bp /*[E]*/);
/* The same counters for n chosen edges only, edge-major: out[i*T + t] is
 * (edges[i], t).  For spot checks at sizes where the full T*E readback is too
 * large (1M peers x 64 topics = 2.05e9 pairs).  An edge outside this rank's
 * range (partitioned engine) reads 0; an edge outside [0, E) is GS_EINVAL. */
int gs_read_topic_stats_edges(gs_engine* eng, int64_t n, const int64_t* edges, double* fmd,
                              double* mmd, double* mfp, double* imd, int64_t* mesh_time,
                              int64_t* graft_time, uint8_t* flags);
/* Backoff expiries (ns, 0 = no entry) of n chosen edges, out[i*T + t]; the
 * edge-list form of gs_read_backoff for full-size spot checks. */
int gs_read_backoff_edges(gs_engine* eng, int64_t n, const int64_t* edges, int64_t* expire);
/* Per node: hop of first delivery of message `id` (-1: never) and the node it
 * was first received from (-1: origin or never).  Valid while the message's
 * slot has not been recycled. */
int gs_read_deliveries(gs_engine* eng, int64_t id, int32_t* hop /*[N]*/,
                       int32_t* from /*[N]*/);

/* ---- trace events (EventTracer, trace.go:61-499 + pb/trace.proto) ------ */
/* Event types: the values of pb.TraceEvent.Type (pb/trace.proto:28-42). */
#define GS_TRACE_PUBLISH_MESSAGE 0
#define GS_TRACE_REJECT_MESSAGE 1
#define GS_TRACE_DUPLICATE_MESSAGE 2
#define GS_TRACE_DELIVER_MESSAGE 3
#define GS_TRACE_ADD_PEER 4
#define GS_TRACE_REMOVE_PEER 5
#define GS_TRACE_RECV_RPC 6
#define GS_TRACE_SEND_RPC 7
#define GS_TRACE_DROP_RPC 8
#define GS_TRACE_JOIN 9
#define GS_TRACE_LEAVE 10
#define GS_TRACE_GRAFT 11
#define GS_TRACE_PRUNE 12
/* Not a pb.TraceEvent type: one entry of the RPCMeta of the RPC event before
 * it.  reason = GS_RPC_ITEM_*, msg = the message id (MSG, IHAVE, IWANT; SUB:
 * 1 = subscribe, 0 = unsubscribe), topic = the topic (-1 for IWANT / CTL). */
#define GS_TRACE_RPC_ITEM 32
#define GS_RPC_ITEM_MSG 0   /* RPCMeta.messages[]: MessageMeta{messageID, topic}          */
#define GS_RPC_ITEM_SUB 1   /* RPCMeta.subscription[]: SubMeta{subscribe, topic}          */
#define GS_RPC_ITEM_CTL 2   /* the RPC carries a ControlMessage (RPCMeta.control is set)  */
#define GS_RPC_ITEM_IHAVE 3 /* ControlMeta.ihave[topic].messageIDs[]                     */
#define GS_RPC_ITEM_IWANT 4 /* ControlMeta.iwant[0].messageIDs[]                         */
#define GS_RPC_ITEM_GRAFT 5 /* ControlMeta.graft[]: ControlGraftMeta{topic}               */
#define GS_RPC_ITEM_PRUNE 6 /* ControlMeta.prune[]: ControlPruneMeta{topic}              */
#define GS_RPC_ITEM_PX 7    /* ControlPruneMeta.peers[] of the PRUNE of `topic` (msg = the peer) */
/* One traced event of host `node` (32 bytes).  Recorded: PUBLISH_MESSAGE
 * (validation.go:217), DELIVER_MESSAGE / DUPLICATE_MESSAGE (pubsub.go:1011,
 * 1057; receivedFrom = peer), ADD_PEER (gossipsub.go:507, floodsub.go:45),
 * JOIN (gossipsub.go:1018, floodsub.go:103), GRAFT / PRUNE (gossipsub.go:790,
 * 817, 1057, 1334, 1343), and with gs_set_trace_rpc the RPC events RECV_RPC
 * (pubsub.go:903) and SEND_RPC (gossipsub.go:1152, floodsub.go:93,
 * randomsub.go:154, pubsub.go:785).  DROP_RPC is never recorded: outbound
 * queues never drop in this model (gossipsub.go:1149-1156 takes its send
 * branch), so the reference's drop path is unreachable.  `phase` orders the
 * events of one (hop, node): 0 connection and Join, 1 local publish, 2
 * received messages, 3 received control, 4 heartbeat; gs_trace_read returns
 * events in the canonical order of include/gs_trace.h.
 * An RPC event (type RECV_RPC / SEND_RPC) has peer = the sender / the
 * receiver and msg = the RPC's ordinal (gs_trace_rpc_ordinal); it is followed
 * by one GS_TRACE_RPC_ITEM event per entry of its traceRPCMeta (trace.go:
 * 310-383), in the order the encoders write them. */
typedef struct gs_trace_event {
  int64_t hop;    /* virtual time: timestamp = hop * hop_ns */
  int64_t msg;    /* message id, -1 = none */
  int32_t type;   /* GS_TRACE_* */
  int32_t node;   /* the tracing host */
  int32_t peer;   /* peer / receivedFrom, -1 = none */
  int16_t topic;  /* -1 = none */
  uint8_t phase;
  uint8_t reason; /* REJECT_MESSAGE: GS_REJECT_*; ADD_PEER: the connection's GS_PROTO_*
                     (0 on a single-router engine: gs_trace_encode's `proto`) */
} gs_trace_event;
/* RejectMessage reasons, in the order of tracer.go:27-38 (their strings are
 * what the encoders write). */
#define GS_REJECT_BLACKLISTED_PEER 0
#define GS_REJECT_BLACKLISTED_SOURCE 1
#define GS_REJECT_MISSING_SIGNATURE 2
#define GS_REJECT_UNEXPECTED_SIGNATURE 3
#define GS_REJECT_UNEXPECTED_AUTH_INFO 4
#define GS_REJECT_INVALID_SIGNATURE 5
#define GS_REJECT_QUEUE_FULL 6
#define GS_REJECT_VALIDATION_THROTTLED 7
#define GS_REJECT_VALIDATION_FAILED 8
#define GS_REJECT_VALIDATION_IGNORED 9
#define GS_REJECT_SELF_ORIGIN 10
/* Before the first step: trace the hosts with node_mask[u] != 0 (NULL: off),
 * keeping up to `capacity` events between two gs_trace_read calls (more is a
 * GS_ECAPACITY error of gs_step). */
int gs_set_trace(gs_engine* eng, const uint8_t* node_mask, int64_t capacity);
/* Before the first step: also record the RPC events of the traced hosts
 * (every RPC they send or receive, with its traceRPCMeta items).  The
 * product library records an RPC where it is sent: on a partitioned engine a
 * rank returns its own traced hosts' events plus the RECV_RPC blocks of the
 * RPCs its hosts sent to other ranks' traced hosts, so the union of every
 * rank's stream is the unpartitioned stream (each rank's in canonical order). */
int gs_set_trace_rpc(gs_engine* eng, int32_t on);
/* Moves up to `cap` recorded events, in canonical order, into out; *n = the
 * number written.  Call until *n < cap to drain. */
int gs_trace_read(gs_engine* eng, gs_trace_event* out, int64_t cap, int64_t* n);
#define GS_TRACE_FORMAT_PB 0   /* uvarint-delimited pb.TraceEvent (PBTracer, tracer.go:141-181) */
#define GS_TRACE_FORMAT_JSON 1 /* one JSON object per line (JSONTracer, tracer.go:79-139) */
/* Encodes events as the reference's tracers write them.  peerID bytes are
 * "n<index>", messageID bytes the decimal id, topic names topic_names[t]
 * (NULL: the decimal index), timestamp hop * hop_ns, AddPeer.proto `proto`.
 * Writes at most cap bytes; *written = bytes needed (GS_ECAPACITY if > cap).
 * Product library only (the oracle returns GS_EUNSUPPORTED). */
int gs_trace_encode(const gs_trace_event* ev, int64_t n, int32_t format, int64_t hop_ns,
                    const char* const* topic_names, const char* proto, uint8_t* buf, int64_t cap,
                    int64_t* written);

/* ---- kernel timing (HIP events on the engine's stream) ----------------- */
/* Kernel classes timed when profiling is on (gs_set_profiling(eng, 1)). */
#define GS_K_SCORE 0     /* peerScore.score over all edges              */
#define GS_K_REFRESH 1   /* refreshScores decay                          */
#define GS_K_JOIN 2      /* Join at hop 0                                */
#define GS_K_FANOUT 3    /* publish-time fanout creation                 */
#define GS_K_FWD 4       /* forwarding-target snapshot                   */
#define GS_K_PHASE_A 5   /* payload messages (propagation hop)           */
#define GS_K_PUBLISH 6   /* local publish bookkeeping                    */
#define GS_K_PHASE_B 7   /* HandleRPC control processing                 */
#define GS_K_HB_PRE 8    /* heartbeat prelude (backoff, penalties)       */
#define GS_K_HEARTBEAT 9 /* mesh maintenance + emitGossip + mcache shift */
#define GS_K_PUSH 10     /* per-edge copies for the next hop (k_push)    */
#define GS_NUM_KERNELS 11
/* Starts/stops per-kernel timing and clears the accumulators.  The oracle
 * accepts the call and reports zeros. */
int gs_set_profiling(gs_engine* eng, int on);
/* total_ms[GS_NUM_KERNELS], launches[GS_NUM_KERNELS] since gs_set_profiling(1). */
int gs_read_kernel_stats(gs_engine* eng, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_ENGINE_H */
