/*
 * gs_trace.h — canonical order of trace events (gossip_engine.h), shared by
 * the product library and the oracle so both return identical sequences.
 *
 * The reference emits events as its goroutines run; the simulator orders the
 * events of one hop per host by phase (connection/Join, local publish,
 * received messages, received control, heartbeat) and inside a phase by the
 * canonical order the round schedule already uses:
 *   phase 0  topic ascending; AddPeer (topic -1) first; Join before the
 *            Graft of its topic (gossipsub.go:1018 then :1057), peers ascending
 *   phase 1  message id, PublishMessage before DeliverMessage
 *   phase 2  sender ascending, then message id (pushMsg per RPC)
 *   phase 3  sender ascending, Graft before Prune (HandleRPC, gossipsub.go:
 *            597-600), topic ascending
 *   phase 4  topic ascending (the heartbeat's mesh loop), type, peer
 */
#ifndef GS_TRACE_H
#define GS_TRACE_H
#ifdef __cplusplus
#include <tuple>

#include "gossip_engine.h"

inline std::tuple<int64_t, int32_t, int32_t, int64_t, int64_t, int64_t, int64_t> gs_trace_key(const gs_trace_event& e) {
  int64_t a = 0, b = 0, c = 0, d = 0;
  switch (e.phase) {
    case 0: a = e.topic; b = e.type == GS_TRACE_JOIN ? -1 : e.peer; c = e.type; break;
    case 1: a = e.msg; b = e.type == GS_TRACE_PUBLISH_MESSAGE ? 0 : 1; break;
    case 2: a = e.peer; b = e.msg; c = e.type; break;
    case 3: a = e.peer; b = e.type; c = e.topic; break;
    default: a = e.topic; b = e.type; c = e.peer; break;
  }
  d = e.msg;
  return std::make_tuple(e.hop, e.node, (int32_t)e.phase, a, b, c, d);
}
inline bool gs_trace_less(const gs_trace_event& x, const gs_trace_event& y) { return gs_trace_key(x) < gs_trace_key(y); }
#endif
#endif
