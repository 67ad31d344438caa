/* gs_transport.h — native RCCL transport for a partitioned engine
 * (SURVEY.md §8(b), §8(e)).
 *
 * In the reference every host runs its own router and the only traffic
 * between hosts is RPCs over per-peer streams (comm.go handleNewStream /
 * handleSendingMessages; pubsub.go:902-970 handleIncomingRPC, gossipsub.go:
 * 1092-1156 sendRPC).  A partitioned engine (gs_set_partition) simulates one
 * contiguous node range per GPU and hands the RPCs its nodes sent to other
 * ranks' nodes to a gs_transport at the end of every hop.  This file gives a
 * C / cgo host that transport without Python: RCCL collectives (over xGMI
 * between the GPUs of one node) directly on the engine's device buffers —
 *   allgather_i64  ncclAllGather of a few int64 per rank (staged through a
 *                  small device buffer);
 *   allgather      ncclAllGather of the equal-size per-rank chunks;
 *   alltoallv      grouped ncclSend / ncclRecv, one pair per peer rank with a
 *                  non-empty block (the rank's own block is a device copy).
 * Same semantics as pubsub_amd.transport.TorchTransport (torch.distributed
 * "nccl" backend), so the two are interchangeable.  Product library only.
 */
#ifndef GS_TRANSPORT_H
#define GS_TRANSPORT_H

#include <stdint.h>

#include "gossip_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GS_RCCL_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */

typedef struct gs_rccl gs_rccl;

/* On ONE rank (rank 0): a fresh communicator id; the host sends the bytes to
 * every other rank over any channel (the reference's hosts have their own). */
int gs_rccl_get_unique_id(uint8_t id[GS_RCCL_ID_BYTES]);
/* Every rank, collectively (blocks until all `world` ranks joined): the
 * communicator of `rank` on HIP device `device`, with its own stream. */
int gs_rccl_create(int32_t rank, int32_t world, const uint8_t id[GS_RCCL_ID_BYTES], int32_t device,
                   gs_rccl** out);
/* The gs_transport callbacks over this communicator (pass to
 * gs_set_partition; `out->user` is the communicator). */
int gs_rccl_transport(gs_rccl* comm, gs_transport* out);
/* Collective calls made and bytes this rank received from other ranks. */
int gs_rccl_stats(const gs_rccl* comm, int64_t* calls, int64_t* bytes_in);
int gs_rccl_destroy(gs_rccl* comm);

#ifdef __cplusplus
}
#endif
#endif
