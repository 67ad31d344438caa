/* gs_rpc.h — RPC size accounting and fragmentation.
 *
 * Replaces the reference's fragmentRPC / fragmentMessageIds
 * (gossipsub.go:1158-1272), which sendRPC (gossipsub.go:1101-1156) calls when
 * an outgoing RPC reaches the stream's maximum message size.  Only the
 * encoded sizes of an RPC's parts decide how it is cut, so the boundary takes
 * the shape of the RPC (pb/rpc.proto) as sizes and returns, for every part,
 * the fragment it lands in.  Host code only (no device); exported by the
 * product library libgossip_engine.so.
 */
#ifndef GS_RPC_H
#define GS_RPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One RPC as fragmentRPC sees it.  Sizes are the gogo Size() of each part
 * (without its own tag and length prefix).  Message ids are given by length:
 * id_len holds the ids of ihave[0], ihave[1], ..., then those of iwant[0],
 * iwant[1], ... (ControlMessage field order). */
typedef struct gs_rpc_shape {
  int32_t n_sub;
  const int64_t* sub_size;         /* RPC_SubOpts.Size() */
  int32_t n_pub;
  const int64_t* pub_size;         /* Message.Size() */
  int32_t has_control;             /* rpc.Control != nil */
  int32_t n_ihave;
  const int64_t* ihave_topic_len;  /* len(TopicID), -1 when TopicID is nil */
  const int32_t* ihave_nids;       /* len(MessageIDs) of each ControlIHave */
  int32_t n_iwant;
  const int32_t* iwant_nids;       /* len(MessageIDs) of each ControlIWant */
  const int64_t* id_len;           /* len of every id, ihave ids first */
  int32_t n_graft;
  const int64_t* graft_size;       /* ControlGraft.Size() */
  int32_t n_prune;
  const int64_t* prune_size;       /* ControlPrune.Size() */
} gs_rpc_shape;

#define GS_RPC_IHAVE 0
#define GS_RPC_IWANT 1

/* Where fragmentRPC put every part.  Arrays are caller-owned, sized as noted.
 * A "bucket" is one ControlIHave / ControlIWant of the output: when the control
 * message is split, fragmentMessageIds cuts every IWANT then every IHAVE into
 * buckets (ids over the limit are dropped: id_bucket = -1) and each bucket is
 * a new entry without TopicID (gossipsub.go:1228-1245); otherwise every entry
 * is one bucket, kept whole. */
typedef struct gs_rpc_fragments {
  int32_t* sub_frag;     /* [n_sub] */
  int32_t* pub_frag;     /* [n_pub] */
  int32_t* graft_frag;   /* [n_graft] */
  int32_t* prune_frag;   /* [n_prune] */
  int32_t* id_bucket;    /* [total ids] bucket index or -1 */
  int32_t bucket_cap;    /* capacity of the three bucket arrays */
  int32_t* bucket_frag;  /* [bucket_cap] fragment holding the bucket */
  int32_t* bucket_kind;  /* [bucket_cap] GS_RPC_IHAVE / GS_RPC_IWANT */
  int32_t* bucket_src;   /* [bucket_cap] index of the input entry of that kind */
  int32_t frag_cap;      /* capacity of frag_size */
  int64_t* frag_size;    /* [frag_cap] RPC.Size() of each fragment */
  int32_t n_bucket;      /* out */
  int32_t n_frag;        /* out */
  int32_t control_whole; /* out: 1 when the control message went unaltered into the last fragment */
} gs_rpc_fragments;

/* RPC.Size() of the shape (gogo wire size, pb/rpc.pb.go). */
int64_t gs_rpc_size(const gs_rpc_shape* rpc);

/* fragmentRPC(rpc, limit) (gossipsub.go:1158).  Returns 0, GS_EINVAL (-1)
 * with gs_last_error() = "message with len=%d exceeds limit %d" when one
 * published message is over the limit (gossipsub.go:1191-1193), or
 * GS_ECAPACITY (-5) when frag_cap / bucket_cap is too small (n_frag and
 * n_bucket then hold the sizes needed). */
int gs_fragment_rpc(const gs_rpc_shape* rpc, int64_t limit, gs_rpc_fragments* out);

#ifdef __cplusplus
}
#endif
#endif /* GS_RPC_H */
