/* gs_rpcsize.h — protobuf sizes of the simulated RPCs (pb/rpc.proto, the
 * gogo-generated Size() of pb/rpc.pb.go), shared by the product kernels and
 * the oracle for the per-edge RPC byte accounting (SURVEY.md §8(f) rank 3:
 * sendRPC measures out.Size(), gossipsub.go:1121-1137).
 *
 * Every field of these messages has a number below 16, so a tag is one byte;
 * a length-delimited field costs 1 + varint(len) + len.  "body" is the size of
 * a message without its own tag and length (what Size() returns).
 *   RPC            subscriptions=1 (SubOpts), publish=2 (Message), control=3
 *   SubOpts        subscribe=1 (bool: tag + 1 byte), topicid=2
 *   ControlMessage ihave=1, iwant=2, graft=3, prune=4
 *   ControlIHave   topicID=1, messageIDs=2 (repeated string)
 *   ControlIWant   messageIDs=1
 *   ControlGraft   topicID=1
 *   ControlPrune   topicID=1, peers=2 (PeerInfo, PX on), backoff=3 (uint64 varint)
 *   PeerInfo       peerID=1, signedPeerRecord=2 (nil without a certified address book: absent)
 * rpcWithControl (comm.go:179-195) always sets Control, so a reply that only
 * carries messages still has an empty ControlMessage (2 bytes); rpcWithMessages
 * and rpcWithSubs (comm.go:167-177) set none.
 */
#ifndef GS_RPCSIZE_H
#define GS_RPCSIZE_H

#include <stdint.h>

#if defined(__HIPCC__)
#define GS_PBFN __host__ __device__ static inline
#else
#define GS_PBFN static inline
#endif

GS_PBFN int64_t gs_pb_vlen(uint64_t v) {
  int64_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
/* a length-delimited field holding `len` bytes */
GS_PBFN int64_t gs_pb_field(int64_t len) { return 1 + gs_pb_vlen((uint64_t)len) + len; }
/* SubOpts body: subscribe + topicid */
GS_PBFN int64_t gs_pb_subopts(int64_t topic_len) { return 2 + gs_pb_field(topic_len); }
/* ControlIHave body with n ids of id_len bytes */
GS_PBFN int64_t gs_pb_ihave(int64_t topic_len, int64_t n, int64_t id_len) {
  return gs_pb_field(topic_len) + n * gs_pb_field(id_len);
}
/* ControlIWant body */
GS_PBFN int64_t gs_pb_iwant(int64_t n, int64_t id_len) { return n * gs_pb_field(id_len); }
/* ControlGraft body */
GS_PBFN int64_t gs_pb_graft(int64_t topic_len) { return gs_pb_field(topic_len); }
/* ControlPrune body as makePrune builds it for a v1.1 peer without PX
 * (gossipsub.go:1803-1839): topicID and backoff seconds */
GS_PBFN int64_t gs_pb_prune(int64_t topic_len, uint64_t backoff_s) {
  return gs_pb_field(topic_len) + 1 + gs_pb_vlen(backoff_s);
}

/* PeerInfo body (makePrune's PX entry, gossipsub.go:1820-1833): the peer id
 * and, when the peerstore holds a signed peer record for it, the record */
GS_PBFN int64_t gs_pb_peerinfo(int64_t peer_id_len, int64_t record_len) {
  return gs_pb_field(peer_id_len) + (record_len > 0 ? gs_pb_field(record_len) : 0);
}
/* ControlPrune body for a v1.1 peer with npx PeerInfo entries of body pi */
GS_PBFN int64_t gs_pb_prune_px(int64_t topic_len, uint64_t backoff_s, int64_t npx, int64_t pi) {
  return gs_pb_prune(topic_len, backoff_s) + npx * gs_pb_field(pi);
}

/* ControlPrune body for a gossipsub v1.0 peer: topicID only (makePrune
 * gossipsub.go:1804-1807 sends neither PX nor a backoff to it) */
GS_PBFN int64_t gs_pb_prune_v10(int64_t topic_len) { return gs_pb_field(topic_len); }

#endif
