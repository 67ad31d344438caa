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
 *
 * RPC events (RECV_RPC / SEND_RPC, gs_set_trace_rpc) carry their traceRPCMeta
 * as the GS_TRACE_RPC_ITEM events right after them; the RPC and its items
 * move as one block.  Inside its phase a host's RECV_RPCs come first (sender,
 * then ordinal: the order the sender sent them), its SEND_RPCs last (receiver,
 * ordinal).  A RECV_RPC is in phase 2 when the RPC carries messages, else 3;
 * hello packets and subscription announcements are received in phase 0.  The
 * ordinal of an RPC is GS_RPC_ORD(send phase, o):
 *   send phase 0: Join GRAFT (o = topic), Leave PRUNE (64 + topic), announcement
 *                 (128 + topic), hello packet (192)
 *   send phase 1: local publish (o = message id)
 *   send phase 2: forwarded message (o = message id), IWANT-spam request (GS_RPC_O_SPAM)
 *   send phase 3: HandleRPC reply, o = the RPC it answers: a Join GRAFT (topic),
 *                 an IWANT-spam request (96), a reply carrying IWANTs (97), the
 *                 heartbeat RPC (98)
 *   send phase 4: the heartbeat RPC (sendGraftPrune + gossip, 0)
 * Items are canonicalized: messages by id; IHAVE ids per topic ascending
 * (above MaxIHaveLength ids, emitGossip's keyed subset, gossipsub.go:1702-1709,
 * then ascending); IWANT ids in handleIHave's keyed order (gossipsub.go:663),
 * an IWANT-spam list ascending; GRAFT / PRUNE by topic.  The reference sends
 * shuffled lists (shuffleStrings), so any fixed order is one of its orders.
 */
#ifndef GS_TRACE_H
#define GS_TRACE_H
#include <stdint.h>
#define GS_RPC_ORD(sp, o) (((int64_t)(sp) << 40) | (int64_t)(o))
#define GS_RPC_O_SPAM (((int64_t)1 << 40) - 1)
#define GS_RPC_O_LEAVE 64
#define GS_RPC_O_ANNOUNCE 128
#define GS_RPC_O_HELLO 192
#define GS_RPC_O_ANS_SPAM 96
#define GS_RPC_O_ANS_REPLY 97
#define GS_RPC_O_ANS_HB 98
#ifdef __cplusplus
#include <algorithm>
#include <climits>
#include <tuple>
#include <utility>
#include <vector>

#include "gossip_engine.h"
#include "gs_rng.h"

inline bool gs_trace_is_rpc(const gs_trace_event& e) {
  return e.type == GS_TRACE_RECV_RPC || e.type == GS_TRACE_SEND_RPC;
}

inline std::tuple<int64_t, int32_t, int32_t, int64_t, int64_t, int64_t, int64_t> gs_trace_key(const gs_trace_event& e) {
  int64_t a = 0, b = 0, c = 0, d = 0;
  if (gs_trace_is_rpc(e))
    return std::make_tuple(e.hop, e.node, (int32_t)e.phase, e.type == GS_TRACE_RECV_RPC ? INT64_MIN : INT64_MAX,
                           (int64_t)e.peer, e.msg, (int64_t)0);
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

// The items of one RPC (it[0] is the RPC event) in canonical order.
inline void gs_trace_canon_items(gs_trace_event* it, size_t n, uint32_t seed, int maxIHaveLength) {
  if (n < 2) return;
  const gs_trace_event& r = it[0];
  const bool send = r.type == GS_TRACE_SEND_RPC;
  const uint32_t sender = (uint32_t)(send ? r.node : r.peer), receiver = (uint32_t)(send ? r.peer : r.node);
  const uint32_t hopSent = (uint32_t)(send ? r.hop : r.hop - 1);
  const bool spamList = (r.msg >> 40) == 2;  // an IWANT-spam request: ascending ids
  std::vector<std::pair<std::tuple<int, int, uint64_t, int64_t>, gs_trace_event>> v;
  bool ctl = false;
  for (size_t i = 1; i < n; ++i) {
    const gs_trace_event& x = it[i];
    if (x.reason == GS_RPC_ITEM_CTL) {
      if (ctl) continue;
      ctl = true;
    }
    uint64_t k = 0;
    if (x.reason == GS_RPC_ITEM_IHAVE)
      k = gs_key64_mid(seed, GS_SITE_EMIT_MIDS, sender, receiver, (uint32_t)x.msg, hopSent);
    else if (x.reason == GS_RPC_ITEM_IWANT && !spamList)
      k = gs_key64_mid(seed, GS_SITE_IWANT, sender, receiver, (uint32_t)x.msg, hopSent);
    v.push_back({std::make_tuple((int)x.reason, (int)x.topic, k, x.msg), x});
  }
  // IHAVE: ascending ids, or the MaxIHaveLength smallest keys in key order
  std::sort(v.begin(), v.end(), [](const auto& p, const auto& q) {
    const auto& a = p.first;
    const auto& b = q.first;
    if (std::get<0>(a) != std::get<0>(b)) return std::get<0>(a) < std::get<0>(b);
    if (std::get<1>(a) != std::get<1>(b)) return std::get<1>(a) < std::get<1>(b);
    if (std::get<0>(a) == GS_RPC_ITEM_IWANT && std::get<2>(a) != std::get<2>(b)) return std::get<2>(a) < std::get<2>(b);
    return std::get<3>(a) < std::get<3>(b);
  });
  std::vector<gs_trace_event> out;
  out.reserve(v.size());
  for (size_t i = 0; i < v.size();) {
    size_t j = i;
    while (j < v.size() && std::get<0>(v[j].first) == std::get<0>(v[i].first) &&
           std::get<1>(v[j].first) == std::get<1>(v[i].first))
      ++j;
    if (std::get<0>(v[i].first) == GS_RPC_ITEM_IHAVE && (int)(j - i) > maxIHaveLength) {
      // the keyed subset, then ascending ids like every other IHAVE
      std::sort(v.begin() + i, v.begin() + j, [](const auto& p, const auto& q) {
        return std::make_pair(std::get<2>(p.first), std::get<3>(p.first)) <
               std::make_pair(std::get<2>(q.first), std::get<3>(q.first));
      });
      std::sort(v.begin() + i, v.begin() + i + maxIHaveLength,
                [](const auto& p, const auto& q) { return std::get<3>(p.first) < std::get<3>(q.first); });
      for (size_t q = i; q < i + (size_t)maxIHaveLength; ++q) out.push_back(v[q].second);
    } else {
      for (size_t q = i; q < j; ++q) out.push_back(v[q].second);
    }
    i = j;
  }
  for (size_t q = 0; q < out.size(); ++q) it[1 + q] = out[q];
  for (size_t q = 1 + out.size(); q < n; ++q) it[q].type = -1;  // cut ids, removed below
}

// Canonical order of a drained event list: RPC events with their items as
// blocks (items canonicalized), every block sorted by its head's key.
inline void gs_trace_canonical(std::vector<gs_trace_event>& ev, uint32_t seed, int maxIHaveLength) {
  std::vector<std::pair<size_t, size_t>> blk;  // [begin, end)
  for (size_t i = 0; i < ev.size();) {
    size_t j = i + 1;
    if (gs_trace_is_rpc(ev[i]))
      while (j < ev.size() && ev[j].type == GS_TRACE_RPC_ITEM) ++j;
    blk.push_back({i, j});
    i = j;
  }
  for (auto& b : blk)
    if (gs_trace_is_rpc(ev[b.first])) gs_trace_canon_items(&ev[b.first], b.second - b.first, seed, maxIHaveLength);
  std::stable_sort(blk.begin(), blk.end(),
                   [&](const auto& x, const auto& y) { return gs_trace_less(ev[x.first], ev[y.first]); });
  std::vector<gs_trace_event> out;
  out.reserve(ev.size());
  for (auto& b : blk)
    for (size_t i = b.first; i < b.second; ++i)
      if (ev[i].type != -1) out.push_back(ev[i]);
  ev.swap(out);
}
#endif
#endif
