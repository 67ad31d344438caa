// gs_rpc.cpp — fragmentRPC / fragmentMessageIds (gossipsub.go:1158-1272) over
// the size shape of an RPC (include/gs_rpc.h).  Sizes follow the gogo
// generated Size() of pb/rpc.pb.go: every embedded message or bytes/string
// field costs tag (1 byte for these field numbers) + uvarint(len) + len.
// Host code only; no device involvement.
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/gossip_engine.h"
#include "../../include/gs_rpc.h"
#include "gs_host.h"

namespace {

int64_t sov(uint64_t v) {
  int64_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
// One length-delimited field of body size s.
int64_t field(int64_t s) { return 1 + sov((uint64_t)s) + s; }

struct Shape {
  const gs_rpc_shape* r;
  int64_t total_ids = 0;
  std::vector<int64_t> ihave_off, iwant_off;  // offsets into id_len

  explicit Shape(const gs_rpc_shape* rpc) : r(rpc) {
    for (int32_t i = 0; i < r->n_ihave; ++i) {
      ihave_off.push_back(total_ids);
      total_ids += r->ihave_nids[i];
    }
    for (int32_t i = 0; i < r->n_iwant; ++i) {
      iwant_off.push_back(total_ids);
      total_ids += r->iwant_nids[i];
    }
  }
  int64_t ids_size(int64_t off, int32_t n) const {
    int64_t s = 0;
    for (int32_t k = 0; k < n; ++k) s += field(r->id_len[off + k]);
    return s;
  }
  // ControlIHave.Size() / ControlIWant.Size() of the input entries.
  int64_t ihave_size(int32_t i) const {
    int64_t tl = r->ihave_topic_len ? r->ihave_topic_len[i] : -1;
    return (tl >= 0 ? field(tl) : 0) + ids_size(ihave_off[i], r->ihave_nids[i]);
  }
  int64_t iwant_size(int32_t i) const { return ids_size(iwant_off[i], r->iwant_nids[i]); }
  int64_t control_size() const {
    int64_t c = 0;
    for (int32_t i = 0; i < r->n_ihave; ++i) c += field(ihave_size(i));
    for (int32_t i = 0; i < r->n_iwant; ++i) c += field(iwant_size(i));
    for (int32_t i = 0; i < r->n_graft; ++i) c += field(r->graft_size[i]);
    for (int32_t i = 0; i < r->n_prune; ++i) c += field(r->prune_size[i]);
    return c;
  }
  int64_t rpc_size() const {
    int64_t s = 0;
    for (int32_t i = 0; i < r->n_sub; ++i) s += field(r->sub_size[i]);
    for (int32_t i = 0; i < r->n_pub; ++i) s += field(r->pub_size[i]);
    if (r->has_control) s += field(control_size());
    return s;
  }
};

// One output RPC: subscriptions + publish bytes, and an optional Control.
struct Frag {
  int64_t body = 0;  // fields 1 and 2
  bool ctl = false;
  int64_t ctl_body = 0;
  int64_t size() const { return body + (ctl ? field(ctl_body) : 0); }
};

struct Bucket {
  int32_t frag, kind, src;
};

bool check_shape(const gs_rpc_shape* r) {
  if (!r || r->n_sub < 0 || r->n_pub < 0 || r->n_ihave < 0 || r->n_iwant < 0 ||
      r->n_graft < 0 || r->n_prune < 0)
    return false;
  if ((r->n_sub && !r->sub_size) || (r->n_pub && !r->pub_size) ||
      (r->n_graft && !r->graft_size) || (r->n_prune && !r->prune_size) ||
      (r->n_ihave && !r->ihave_nids) || (r->n_iwant && !r->iwant_nids))
    return false;
  int64_t ids = 0;
  for (int32_t i = 0; i < r->n_ihave; ++i) {
    if (r->ihave_nids[i] < 0) return false;
    ids += r->ihave_nids[i];
  }
  for (int32_t i = 0; i < r->n_iwant; ++i) {
    if (r->iwant_nids[i] < 0) return false;
    ids += r->iwant_nids[i];
  }
  if (ids && !r->id_len) return false;
  // sizes are byte counts: never negative (a TopicID length may be -1 = nil)
  auto nonneg = [](const int64_t* a, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
      if (a[i] < 0) return false;
    return true;
  };
  if (!nonneg(r->sub_size, r->n_sub) || !nonneg(r->pub_size, r->n_pub) || !nonneg(r->graft_size, r->n_graft) ||
      !nonneg(r->prune_size, r->n_prune) || !nonneg(r->id_len, ids))
    return false;
  if (r->ihave_topic_len)
    for (int32_t i = 0; i < r->n_ihave; ++i)
      if (r->ihave_topic_len[i] < -1) return false;
  if (!r->has_control && (r->n_ihave || r->n_iwant || r->n_graft || r->n_prune)) return false;
  return true;
}

}  // namespace

extern "C" int64_t gs_rpc_size(const gs_rpc_shape* rpc) {
  if (!check_shape(rpc)) {
    gs_set_error("gs_rpc_size: bad shape");
    return GS_EINVAL;
  }
  return Shape(rpc).rpc_size();
}

extern "C" int gs_fragment_rpc(const gs_rpc_shape* rpc, int64_t limit, gs_rpc_fragments* out) {
  if (!check_shape(rpc) || !out || limit <= 0 || (rpc->n_sub && !out->sub_frag) ||
      (rpc->n_pub && !out->pub_frag) || (rpc->n_graft && !out->graft_frag) ||
      (rpc->n_prune && !out->prune_frag) || out->frag_cap < 0 || out->bucket_cap < 0 ||
      (out->frag_cap > 0 && !out->frag_size) ||
      (out->bucket_cap > 0 && (!out->bucket_frag || !out->bucket_kind || !out->bucket_src))) {
    gs_set_error("gs_fragment_rpc: bad arguments");
    return GS_EINVAL;
  }
  const Shape S(rpc);
  if (S.total_ids && !out->id_bucket) {
    gs_set_error("gs_fragment_rpc: id_bucket is NULL");
    return GS_EINVAL;
  }
  std::vector<Frag> frags;
  std::vector<Bucket> buckets;

  // gossipsub.go:1159-1161: small enough, the RPC goes out unaltered.
  const bool whole = S.rpc_size() < limit;
  out->control_whole = 0;
  if (whole) {
    Frag f;
    for (int32_t i = 0; i < rpc->n_sub; ++i) out->sub_frag[i] = 0, f.body += field(rpc->sub_size[i]);
    for (int32_t i = 0; i < rpc->n_pub; ++i) out->pub_frag[i] = 0, f.body += field(rpc->pub_size[i]);
    f.ctl = rpc->has_control != 0;
    if (f.ctl) f.ctl_body = S.control_size();
    frags.push_back(f);
  } else {
    frags.emplace_back();  // rpcs[0], gossipsub.go:1165
    // outRPC, gossipsub.go:1170-1186
    auto out_rpc = [&](int64_t add, bool with_ctl) -> int32_t {
      Frag& cur = frags.back();
      if (cur.size() + add + 1 < limit) {
        if (with_ctl && !cur.ctl) cur.ctl = true, cur.ctl_body = 0;
        return (int32_t)frags.size() - 1;
      }
      Frag next;
      next.ctl = with_ctl;
      frags.push_back(next);
      return (int32_t)frags.size() - 1;
    };
    for (int32_t i = 0; i < rpc->n_pub; ++i) {
      const int64_t s = rpc->pub_size[i];
      if (s > limit) {  // gossipsub.go:1191-1193
        gs_set_error("message with len=" + std::to_string(s) + " exceeds limit " +
                     std::to_string(limit));
        return GS_EINVAL;
      }
      const int32_t k = out_rpc(s, false);
      frags[k].body += field(s);
      out->pub_frag[i] = k;
    }
    for (int32_t i = 0; i < rpc->n_sub; ++i) {
      const int32_t k = out_rpc(rpc->sub_size[i], false);
      frags[k].body += field(rpc->sub_size[i]);
      out->sub_frag[i] = k;
    }
    if (rpc->has_control) {
      const int64_t csize = S.control_size();
      if (field(csize) < limit) {  // gossipsub.go:1209-1213
        Frag f;
        f.ctl = true;
        f.ctl_body = csize;
        frags.push_back(f);
        out->control_whole = 1;
      } else {
        auto add_ctl = [&](int64_t s) -> int32_t {
          const int32_t k = out_rpc(s, true);
          frags[k].ctl_body += field(s);
          return k;
        };
        for (int32_t i = 0; i < rpc->n_graft; ++i) out->graft_frag[i] = add_ctl(rpc->graft_size[i]);
        for (int32_t i = 0; i < rpc->n_prune; ++i) out->prune_frag[i] = add_ctl(rpc->prune_size[i]);
        // fragmentMessageIds (gossipsub.go:1249-1272) with limit - 6 (:1229, :1238);
        // every bucket becomes a fresh entry without TopicID.
        const int64_t lim = limit - 6;
        auto split = [&](int kind, int32_t src, int64_t off, int32_t n) {
          std::vector<int64_t> bsize(1, 0);  // ControlI*.Size() of each bucket
          std::vector<int32_t> ids;          // bucket of each kept id, relative
          int64_t blen = 0;
          int32_t cur = 0;
          for (int32_t m = 0; m < n; ++m) {
            const int64_t l = rpc->id_len[off + m];
            const int64_t sz = l + 2;
            if (sz > lim) {
              out->id_bucket[off + m] = -1;
              continue;
            }
            blen += sz;
            if (blen > lim) {
              bsize.push_back(0);
              ++cur;
              blen = sz;
            }
            bsize[cur] += field(l);
            out->id_bucket[off + m] = (int32_t)buckets.size() + cur;
          }
          for (size_t b = 0; b < bsize.size(); ++b)
            buckets.push_back({add_ctl(bsize[b]), kind, src});
        };
        for (int32_t i = 0; i < rpc->n_iwant; ++i)
          split(GS_RPC_IWANT, i, S.iwant_off[i], rpc->iwant_nids[i]);
        for (int32_t i = 0; i < rpc->n_ihave; ++i)
          split(GS_RPC_IHAVE, i, S.ihave_off[i], rpc->ihave_nids[i]);
      }
    }
  }
  if (whole || out->control_whole) {
    // Control entries unaltered, all in the last fragment; one bucket per entry.
    const int32_t last = (int32_t)frags.size() - 1;
    for (int32_t i = 0; i < rpc->n_graft; ++i) out->graft_frag[i] = last;
    for (int32_t i = 0; i < rpc->n_prune; ++i) out->prune_frag[i] = last;
    for (int32_t i = 0; i < rpc->n_ihave; ++i) {
      for (int32_t m = 0; m < rpc->ihave_nids[i]; ++m)
        out->id_bucket[S.ihave_off[i] + m] = (int32_t)buckets.size();
      buckets.push_back({last, GS_RPC_IHAVE, i});
    }
    for (int32_t i = 0; i < rpc->n_iwant; ++i) {
      for (int32_t m = 0; m < rpc->iwant_nids[i]; ++m)
        out->id_bucket[S.iwant_off[i] + m] = (int32_t)buckets.size();
      buckets.push_back({last, GS_RPC_IWANT, i});
    }
  }

  out->n_frag = (int32_t)frags.size();
  out->n_bucket = (int32_t)buckets.size();
  if (out->n_frag > out->frag_cap || out->n_bucket > out->bucket_cap) {
    gs_set_error("gs_fragment_rpc: frag_cap or bucket_cap too small (see n_frag, n_bucket)");
    return GS_ECAPACITY;
  }
  for (size_t k = 0; k < frags.size(); ++k) out->frag_size[k] = frags[k].size();
  for (size_t b = 0; b < buckets.size(); ++b) {
    out->bucket_frag[b] = buckets[b].frag;
    out->bucket_kind[b] = buckets[b].kind;
    out->bucket_src[b] = buckets[b].src;
  }
  return 0;
}
