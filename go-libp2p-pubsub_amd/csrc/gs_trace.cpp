// gs_trace.cpp — encodes gs_trace_event records as the reference's event
// tracers write pb.TraceEvent (pb/trace.proto, generated code pb/trace.pb.go):
//   GS_TRACE_FORMAT_PB    PBTracer (tracer.go:141-181): each event marshalled
//                         (gogo: fields in ascending field-number order, a
//                         sub-message as tag + length + body) and written
//                         through a uvarint-delimited protoio writer;
//   GS_TRACE_FORMAT_JSON  JSONTracer (tracer.go:79-139): encoding/json of the
//                         Go struct, one object + '\n' per event: struct field
//                         order, omitempty, []byte as padded standard base64,
//                         the enum Type as its number.
// Host code only; no device involvement.
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gossip_engine.h"
#include "gs_host.h"

namespace {

std::string peer_bytes(int32_t p) { return "n" + std::to_string(p); }
std::string msg_bytes(int64_t m) { return std::to_string(m); }

// ---- protobuf wire format
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
void put_bytes(std::string& o, int field, const std::string& b) {
  put_varint(o, ((uint64_t)field << 3) | 2);
  put_varint(o, b.size());
  o += b;
}
void put_int(std::string& o, int field, int64_t v) {
  put_varint(o, ((uint64_t)field << 3) | 0);
  put_varint(o, (uint64_t)v);  // int64 varint: two's complement for negatives
}

// ---- JSON
std::string b64(const std::string& s) {
  static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  size_t i = 0;
  for (; i + 2 < s.size(); i += 3) {
    const uint32_t x = ((uint8_t)s[i] << 16) | ((uint8_t)s[i + 1] << 8) | (uint8_t)s[i + 2];
    o += A[x >> 18]; o += A[(x >> 12) & 63]; o += A[(x >> 6) & 63]; o += A[x & 63];
  }
  if (i + 1 == s.size()) {
    const uint32_t x = (uint8_t)s[i] << 16;
    o += A[x >> 18]; o += A[(x >> 12) & 63]; o += "==";
  } else if (i + 2 == s.size()) {
    const uint32_t x = ((uint8_t)s[i] << 16) | ((uint8_t)s[i + 1] << 8);
    o += A[x >> 18]; o += A[(x >> 12) & 63]; o += A[(x >> 6) & 63]; o += '=';
  }
  return o;
}
// encoding/json's string encoder as of the reference's Go (1.13-1.15,
// encode.go encodeState.string with escapeHTML): \" \\ \n \r \t short
// escapes, other control bytes and < > & as \u00XX, U+2028 / U+2029 escaped,
// invalid UTF-8 replaced by \ufffd (one per bad byte, utf8.DecodeRuneInString).
std::string jstr(const std::string& s) {
  std::string o = "\"";
  const size_t n = s.size();
  for (size_t i = 0; i < n;) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
      else if (c == '\n') o += "\\n";
      else if (c == '\r') o += "\\r";
      else if (c == '\t') o += "\\t";
      else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
        char buf[8];
        std::snprintf(buf, sizeof buf, "\\u%04x", c);
        o += buf;
      } else o += (char)c;
      ++i;
      continue;
    }
    // decode one rune; width 0 = invalid
    uint32_t r = 0;
    size_t w = 0;
    auto cont = [&](size_t k) { return i + k < n && ((unsigned char)s[i + k] & 0xC0) == 0x80; };
    if (c >= 0xC2 && c <= 0xDF && cont(1)) {
      r = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F);
      w = 2;
    } else if (c >= 0xE0 && c <= 0xEF && cont(1) && cont(2)) {
      r = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
      if (r >= 0x800 && !(r >= 0xD800 && r <= 0xDFFF)) w = 3;
    } else if (c >= 0xF0 && c <= 0xF4 && cont(1) && cont(2) && cont(3)) {
      r = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
      if (r >= 0x10000 && r <= 0x10FFFF) w = 4;
    }
    if (w == 0) {
      o += "\\ufffd";
      ++i;
    } else if (r == 0x2028 || r == 0x2029) {
      o += r == 0x2028 ? "\\u2028" : "\\u2029";
      i += w;
    } else {
      o.append(s, i, w);
      i += w;
    }
  }
  return o + "\"";
}

struct Field {  // one field of a sub-message: bytes (base64 in JSON) or string
  int num;
  const char* name;
  std::string val;
  bool isBytes;
};

// rejection reasons, tracer.go:27-38 (GS_REJECT_* order)
const char* kReason[] = {"blacklisted peer", "blacklisted source", "missing signature", "unexpected signature",
                         "unexpected auth info", "invalid signature", "validation queue full",
                         "validation throttled", "validation failed", "validation ignored",
                         "self originated message"};
const int kNumReasons = 11;

// pb.TraceEvent field number / JSON name of the sub-message of each type
const int kSubField[13] = {4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const char* kSubName[13] = {"publishMessage", "rejectMessage", "duplicateMessage", "deliverMessage", "addPeer",
                            "removePeer", "recvRPC", "sendRPC", "dropRPC", "join", "leave", "graft", "prune"};

std::vector<Field> sub_fields(const gs_trace_event& e, const std::string& topic, const char* proto) {
  switch (e.type) {
    case GS_TRACE_PUBLISH_MESSAGE:  // trace.proto PublishMessage {messageID=1, topic=2}
      return {{1, "messageID", msg_bytes(e.msg), true}, {2, "topic", topic, false}};
    case GS_TRACE_REJECT_MESSAGE:  // {messageID=1, receivedFrom=2, reason=3, topic=4}
      return {{1, "messageID", msg_bytes(e.msg), true}, {2, "receivedFrom", peer_bytes(e.peer), true},
              {3, "reason", e.reason < kNumReasons ? kReason[e.reason] : "", false}, {4, "topic", topic, false}};
    case GS_TRACE_REMOVE_PEER:  // {peerID=1}
      return {{1, "peerID", peer_bytes(e.peer), true}};
    case GS_TRACE_LEAVE:  // {topic=2} (pb/trace.proto:99-101)
      return {{2, "topic", topic, false}};
    case GS_TRACE_DUPLICATE_MESSAGE:  // {messageID=1, receivedFrom=2, topic=3}
      return {{1, "messageID", msg_bytes(e.msg), true}, {2, "receivedFrom", peer_bytes(e.peer), true},
              {3, "topic", topic, false}};
    case GS_TRACE_DELIVER_MESSAGE:  // {messageID=1, topic=2, receivedFrom=3}
      return {{1, "messageID", msg_bytes(e.msg), true}, {2, "topic", topic, false},
              {3, "receivedFrom", peer_bytes(e.peer), true}};
    case GS_TRACE_ADD_PEER:  // {peerID=1, proto=2}
    {
      // the connection's protocol.ID (reason = GS_PROTO_*); 0: the caller's default
      static const char* const kProto[] = {nullptr, "/floodsub/1.0.0", "/randomsub/1.0.0", "/meshsub/1.0.0",
                                           "/meshsub/1.1.0"};
      const char* pr = e.reason >= 1 && e.reason <= 4 ? kProto[e.reason] : proto;
      return {{1, "peerID", peer_bytes(e.peer), true}, {2, "proto", pr ? pr : "", false}};
    }
    case GS_TRACE_JOIN:  // {topic=1}
      return {{1, "topic", topic, false}};
    case GS_TRACE_GRAFT:
    case GS_TRACE_PRUNE:  // {peerID=1, topic=2}
      return {{1, "peerID", peer_bytes(e.peer), true}, {2, "topic", topic, false}};
    default:
      return {};
  }
}

// ---- RPCMeta (trace.go:310-383, pb/trace.proto RPCMeta) of an RPC event's
// items ev[1..n): messages, subscriptions, then the control message when the
// RPC carries one (ihave per topic, one iwant entry, graft, prune).
struct Meta {
  std::vector<std::pair<int64_t, int>> msgs;  // (id, topic)
  std::vector<std::pair<int, bool>> subs;     // (topic, subscribe)
  bool ctl = false;
  std::vector<std::pair<int, std::vector<int64_t>>> ihave;
  std::vector<int64_t> iwant;
  std::vector<int> graft;
  std::vector<std::pair<int, std::vector<int>>> prune;  // (topic, PX peers)
};
Meta collect(const gs_trace_event* it, int64_t n) {
  Meta m;
  for (int64_t i = 0; i < n; ++i) {
    const gs_trace_event& x = it[i];
    switch (x.reason) {
      case GS_RPC_ITEM_MSG: m.msgs.push_back({x.msg, x.topic}); break;
      case GS_RPC_ITEM_SUB: m.subs.push_back({x.topic, x.msg != 0}); break;
      case GS_RPC_ITEM_CTL: m.ctl = true; break;
      case GS_RPC_ITEM_IHAVE:
        if (m.ihave.empty() || m.ihave.back().first != x.topic) m.ihave.push_back({x.topic, {}});
        m.ihave.back().second.push_back(x.msg);
        break;
      case GS_RPC_ITEM_IWANT: m.iwant.push_back(x.msg); break;
      case GS_RPC_ITEM_GRAFT: m.graft.push_back(x.topic); break;
      case GS_RPC_ITEM_PRUNE: m.prune.push_back({x.topic, {}}); break;
      case GS_RPC_ITEM_PX:
        for (auto& pr : m.prune)
          if (pr.first == x.topic) pr.second.push_back((int)x.msg);
        break;
      default: break;
    }
  }
  return m;
}
std::string meta_pb(const Meta& m, const std::function<std::string(int)>& tn) {
  std::string o;
  for (auto& mm : m.msgs) {  // MessageMeta{messageID=1, topic=2}
    std::string b;
    put_bytes(b, 1, msg_bytes(mm.first));
    put_bytes(b, 2, tn(mm.second));
    put_bytes(o, 1, b);
  }
  for (auto& sm : m.subs) {  // SubMeta{subscribe=1, topic=2}
    std::string b;
    put_int(b, 1, sm.second ? 1 : 0);
    put_bytes(b, 2, tn(sm.first));
    put_bytes(o, 2, b);
  }
  if (m.ctl) {  // ControlMeta{ihave=1, iwant=2, graft=3, prune=4}
    std::string c;
    for (auto& ih : m.ihave) {
      std::string b;
      put_bytes(b, 1, tn(ih.first));
      for (int64_t id : ih.second) put_bytes(b, 2, msg_bytes(id));
      put_bytes(c, 1, b);
    }
    if (!m.iwant.empty()) {
      std::string b;
      for (int64_t id : m.iwant) put_bytes(b, 1, msg_bytes(id));
      put_bytes(c, 2, b);
    }
    for (int t : m.graft) {
      std::string b;
      put_bytes(b, 1, tn(t));
      put_bytes(c, 3, b);
    }
    for (auto& pr : m.prune) {  // ControlPruneMeta{topic=1, peers=2}
      std::string b;
      put_bytes(b, 1, tn(pr.first));
      for (int q : pr.second) put_bytes(b, 2, peer_bytes(q));
      put_bytes(c, 4, b);
    }
    put_bytes(o, 3, c);
  }
  return o;
}
std::string meta_json(const Meta& m, const std::function<std::string(int)>& tn) {
  std::string o = "{";
  bool first = true;
  auto sep = [&]() {
    if (!first) o += ",";
    first = false;
  };
  auto ids = [&](const std::vector<int64_t>& v) {
    std::string a = "[";
    for (size_t i = 0; i < v.size(); ++i) a += (i ? ",\"" : "\"") + b64(msg_bytes(v[i])) + "\"";
    return a + "]";
  };
  if (!m.msgs.empty()) {
    sep();
    o += "\"messages\":[";
    for (size_t i = 0; i < m.msgs.size(); ++i)
      o += std::string(i ? "," : "") + "{\"messageID\":\"" + b64(msg_bytes(m.msgs[i].first)) + "\",\"topic\":" +
           jstr(tn(m.msgs[i].second)) + "}";
    o += "]";
  }
  if (!m.subs.empty()) {
    sep();
    o += "\"subscription\":[";
    for (size_t i = 0; i < m.subs.size(); ++i)
      o += std::string(i ? "," : "") + "{\"subscribe\":" + (m.subs[i].second ? "true" : "false") +
           ",\"topic\":" + jstr(tn(m.subs[i].first)) + "}";
    o += "]";
  }
  if (m.ctl) {
    sep();
    std::string c = "{";
    bool cf = true;
    auto csep = [&]() {
      if (!cf) c += ",";
      cf = false;
    };
    if (!m.ihave.empty()) {
      csep();
      c += "\"ihave\":[";
      for (size_t i = 0; i < m.ihave.size(); ++i)
        c += std::string(i ? "," : "") + "{\"topic\":" + jstr(tn(m.ihave[i].first)) +
             (m.ihave[i].second.empty() ? "" : ",\"messageIDs\":" + ids(m.ihave[i].second)) + "}";
      c += "]";
    }
    if (!m.iwant.empty()) {
      csep();
      c += "\"iwant\":[{\"messageIDs\":" + ids(m.iwant) + "}]";
    }
    if (!m.graft.empty()) {
      csep();
      c += "\"graft\":[";
      for (size_t i = 0; i < m.graft.size(); ++i) c += std::string(i ? "," : "") + "{\"topic\":" + jstr(tn(m.graft[i])) + "}";
      c += "]";
    }
    if (!m.prune.empty()) {
      csep();
      c += "\"prune\":[";
      for (size_t i = 0; i < m.prune.size(); ++i) {
        c += std::string(i ? "," : "") + "{\"topic\":" + jstr(tn(m.prune[i].first));
        if (!m.prune[i].second.empty()) {
          c += ",\"peers\":[";
          for (size_t k = 0; k < m.prune[i].second.size(); ++k)
            c += std::string(k ? "," : "") + "\"" + b64(peer_bytes(m.prune[i].second[k])) + "\"";
          c += "]";
        }
        c += "}";
      }
      c += "]";
    }
    o += "\"control\":" + c + "}";
  }
  return o + "}";
}

}  // namespace

extern "C" int gs_trace_encode(const gs_trace_event* ev, int64_t n, int32_t format, int64_t hop_ns,
                               const char* const* topic_names, const char* proto, uint8_t* buf, int64_t cap,
                               int64_t* written) {
  if (!written || n < 0 || (n > 0 && !ev) || (format != GS_TRACE_FORMAT_PB && format != GS_TRACE_FORMAT_JSON)) {
    gs_set_error("gs_trace_encode: bad arguments");
    return GS_EINVAL;
  }
  std::string out;
  auto tn = [&](int t) -> std::string {
    return t < 0 ? std::string() : (topic_names ? std::string(topic_names[t]) : std::to_string(t));
  };
  for (int64_t i = 0; i < n; ++i) {
    const gs_trace_event& e = ev[i];
    if (e.type < 0 || e.type > GS_TRACE_PRUNE) {
      gs_set_error(e.type == GS_TRACE_RPC_ITEM ? "gs_trace_encode: an RPC item without its RPC event"
                                               : "gs_trace_encode: unknown event type");
      return GS_EINVAL;
    }
    const std::string topic = tn(e.topic);
    const std::string peer = peer_bytes(e.node);
    const int64_t ts = e.hop * hop_ns;
    if (e.type == GS_TRACE_RECV_RPC || e.type == GS_TRACE_SEND_RPC || e.type == GS_TRACE_DROP_RPC) {
      // RecvRPC{receivedFrom=1, meta=2} / SendRPC, DropRPC{sendTo=1, meta=2}
      int64_t j = i + 1;
      while (j < n && ev[j].type == GS_TRACE_RPC_ITEM) ++j;
      const Meta m = collect(ev + i + 1, j - i - 1);
      const char* who = e.type == GS_TRACE_RECV_RPC ? "receivedFrom" : "sendTo";
      if (format == GS_TRACE_FORMAT_PB) {
        std::string body;
        put_bytes(body, 1, peer_bytes(e.peer));
        put_bytes(body, 2, meta_pb(m, tn));
        std::string msg;
        put_int(msg, 1, e.type);
        put_bytes(msg, 2, peer);
        put_int(msg, 3, ts);
        put_bytes(msg, kSubField[e.type], body);
        put_varint(out, msg.size());
        out += msg;
      } else {
        out += "{\"type\":" + std::to_string(e.type) + ",\"peerID\":\"" + b64(peer) + "\",\"timestamp\":" +
               std::to_string(ts) + ",\"" + kSubName[e.type] + "\":{\"" + who + "\":\"" + b64(peer_bytes(e.peer)) +
               "\",\"meta\":" + meta_json(m, tn) + "}}\n";
      }
      i = j - 1;
      continue;
    }
    const std::vector<Field> fs = sub_fields(e, topic, proto);
    if (format == GS_TRACE_FORMAT_PB) {
      std::string body;
      for (const Field& f : fs) put_bytes(body, f.num, f.val);  // trace.go sets every field
      std::string m;
      put_int(m, 1, e.type);
      put_bytes(m, 2, peer);
      put_int(m, 3, ts);
      put_bytes(m, kSubField[e.type], body);
      put_varint(out, m.size());
      out += m;
    } else {
      std::string j = "{\"type\":" + std::to_string(e.type) + ",\"peerID\":\"" + b64(peer) +
                      "\",\"timestamp\":" + std::to_string(ts) + ",\"" + kSubName[e.type] + "\":{";
      bool first = true;
      for (const Field& f : fs) {
        if (f.isBytes && f.val.empty()) continue;  // omitempty: nil/empty []byte (a *string is always set)
        if (!first) j += ",";
        first = false;
        j += "\"" + std::string(f.name) + "\":" + (f.isBytes ? "\"" + b64(f.val) + "\"" : jstr(f.val));
      }
      j += "}}\n";
      out += j;
    }
  }
  *written = (int64_t)out.size();
  if ((int64_t)out.size() > cap) {
    gs_set_error("gs_trace_encode: buffer too small (see *written)");
    return GS_ECAPACITY;
  }
  if (!out.empty()) std::memcpy(buf, out.data(), out.size());
  return GS_OK;
}
