/* gs_proto.h — protocol negotiation of mixed networks (gs_set_routers /
 * gs_set_graph_ex in gossip_engine.h), shared by the product library and the
 * oracle so both derive the same per-connection protocol.
 *
 * A pubsub stream is opened with the opener's Protocols() in preference order
 * (pubsub.go:499-515 newPeerStream -> host.NewStream(..., rt.Protocols()...));
 * multistream-select takes the first one the other host supports:
 *   FloodSubRouter.Protocols   [floodsub]                        floodsub.go:26
 *   RandomSubRouter.Protocols  [randomsub, floodsub]             randomsub.go:40
 *   GossipSubRouter.Protocols  [meshsub/1.1, meshsub/1.0, floodsub]
 *                              (GossipSubDefaultProtocols, gossipsub_feat.go:24)
 *   a v1.0-only gossipsub host [meshsub/1.0, floodsub] (WithGossipSubProtocols :41-56)
 * Every pair of these lists agrees on the same protocol whichever host opens
 * the stream, so both directions of a connection run one protocol. */
#ifndef GS_PROTO_H
#define GS_PROTO_H

#include "gossip_engine.h"

static inline int gs_router_protocols(int router, int out[3]) {
  switch (router) {
    case GS_ROUTER_FLOODSUB: out[0] = GS_PROTO_FLOODSUB; return 1;
    case GS_ROUTER_RANDOMSUB: out[0] = GS_PROTO_RANDOMSUB; out[1] = GS_PROTO_FLOODSUB; return 2;
    case GS_ROUTER_GOSSIPSUB_V10: out[0] = GS_PROTO_GOSSIPSUB_V10; out[1] = GS_PROTO_FLOODSUB; return 2;
    default:
      out[0] = GS_PROTO_GOSSIPSUB_V11; out[1] = GS_PROTO_GOSSIPSUB_V10; out[2] = GS_PROTO_FLOODSUB;
      return 3;
  }
}
/* does a host running `router` speak `proto`? */
static inline int gs_router_speaks(int router, int proto) {
  int p[3];
  const int n = gs_router_protocols(router, p);
  for (int i = 0; i < n; ++i)
    if (p[i] == proto) return 1;
  return 0;
}
/* the protocol a stream between hosts running routers a and b settles on */
static inline int gs_negotiate(int a, int b) {
  int pa[3];
  const int na = gs_router_protocols(a, pa);
  for (int i = 0; i < na; ++i)
    if (gs_router_speaks(b, pa[i])) return pa[i];
  return GS_PROTO_FLOODSUB;
}

#endif
