// gs_transport_rccl.cpp — the native RCCL gs_transport (include/gs_transport.h).
//
// One communicator and one HIP stream per rank.  Every callback enqueues its
// collective on that stream and waits for it before returning: the engine
// calls the transport between hops with none of its own device work pending
// (gossip_engine.h), and reads the received buffers right after.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/gs_transport.h"
#include "gs_host.h"

struct gs_rccl {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int rank = 0, world = 1, device = 0;
  int64_t* scratch = nullptr;  // allgather_i64 staging (device)
  int64_t scratchCap = 0;
  int64_t calls = 0, bytesIn = 0;
};

namespace {

int fail(const char* what, ncclResult_t r) {
  gs_set_error(std::string("rccl transport: ") + what + ": " + ncclGetErrorString(r));
  return GS_EDEVICE;
}
int failh(const char* what, hipError_t r) {
  gs_set_error(std::string("rccl transport: ") + what + ": " + hipGetErrorString(r));
  return GS_EDEVICE;
}

#define NCHK(x, what)                  \
  do {                                 \
    ncclResult_t r_ = (x);             \
    if (r_ != ncclSuccess) return fail(what, r_); \
  } while (0)
#define HCHK(x, what)                  \
  do {                                 \
    hipError_t r_ = (x);               \
    if (r_ != hipSuccess) return failh(what, r_); \
  } while (0)

int cb_allgather_i64(void* user, const int64_t* mine, int32_t n, int64_t* all) {
  gs_rccl* c = static_cast<gs_rccl*>(user);
  HCHK(hipSetDevice(c->device), "hipSetDevice");
  const int64_t need = (int64_t)n * (c->world + 1);
  if (need > c->scratchCap) {
    if (c->scratch) HCHK(hipFree(c->scratch), "hipFree");
    c->scratch = nullptr;
    HCHK(hipMalloc(&c->scratch, (size_t)need * 8), "hipMalloc");
    c->scratchCap = need;
  }
  int64_t* dMine = c->scratch + (int64_t)n * c->world;
  HCHK(hipMemcpyAsync(dMine, mine, (size_t)n * 8, hipMemcpyHostToDevice, c->stream), "H2D");
  NCHK(ncclAllGather(dMine, c->scratch, (size_t)n, ncclInt64, c->comm, c->stream), "ncclAllGather(i64)");
  HCHK(hipMemcpyAsync(all, c->scratch, (size_t)n * c->world * 8, hipMemcpyDeviceToHost, c->stream), "D2H");
  HCHK(hipStreamSynchronize(c->stream), "sync");
  c->calls++;
  return 0;
}

int cb_allgather(void* user, const void* send, void* recv, int64_t bytes) {
  gs_rccl* c = static_cast<gs_rccl*>(user);
  HCHK(hipSetDevice(c->device), "hipSetDevice");
  if (bytes > 0) {
    NCHK(ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c->comm, c->stream), "ncclAllGather");
    HCHK(hipStreamSynchronize(c->stream), "sync");
  }
  c->calls++;
  c->bytesIn += bytes * (c->world - 1);
  return 0;
}

int cb_alltoallv(void* user, const void* send, const int64_t* send_bytes, void* recv, const int64_t* recv_bytes) {
  gs_rccl* c = static_cast<gs_rccl*>(user);
  HCHK(hipSetDevice(c->device), "hipSetDevice");
  std::vector<int64_t> so(c->world + 1, 0), ro(c->world + 1, 0);
  for (int r = 0; r < c->world; ++r) {
    so[r + 1] = so[r] + send_bytes[r];
    ro[r + 1] = ro[r] + recv_bytes[r];
  }
  const uint8_t* s = static_cast<const uint8_t*>(send);
  uint8_t* d = static_cast<uint8_t*>(recv);
  if (send_bytes[c->rank] != recv_bytes[c->rank]) {
    gs_set_error("rccl transport: alltoallv: own block sizes differ");
    return GS_EINVAL;
  }
  if (send_bytes[c->rank] > 0)
    HCHK(hipMemcpyAsync(d + ro[c->rank], s + so[c->rank], (size_t)send_bytes[c->rank], hipMemcpyDeviceToDevice,
                        c->stream),
         "self copy");
  NCHK(ncclGroupStart(), "ncclGroupStart");
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) continue;
    if (send_bytes[p] > 0) NCHK(ncclSend(s + so[p], (size_t)send_bytes[p], ncclUint8, p, c->comm, c->stream), "ncclSend");
    if (recv_bytes[p] > 0) NCHK(ncclRecv(d + ro[p], (size_t)recv_bytes[p], ncclUint8, p, c->comm, c->stream), "ncclRecv");
  }
  NCHK(ncclGroupEnd(), "ncclGroupEnd");
  HCHK(hipStreamSynchronize(c->stream), "sync");
  c->calls++;
  c->bytesIn += ro[c->world] - recv_bytes[c->rank];
  return 0;
}

}  // namespace

extern "C" {

int gs_rccl_get_unique_id(uint8_t id[GS_RCCL_ID_BYTES]) {
  if (!id) {
    gs_set_error("gs_rccl_get_unique_id: NULL id");
    return GS_EINVAL;
  }
  static_assert(sizeof(ncclUniqueId) == GS_RCCL_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  NCHK(ncclGetUniqueId(&u), "ncclGetUniqueId");
  std::memcpy(id, u.internal, GS_RCCL_ID_BYTES);
  return GS_OK;
}

int gs_rccl_create(int32_t rank, int32_t world, const uint8_t id[GS_RCCL_ID_BYTES], int32_t device, gs_rccl** out) {
  if (!out || !id || world < 1 || rank < 0 || rank >= world || device < 0) {
    gs_set_error("gs_rccl_create: bad arguments");
    return GS_EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
    gs_set_error("gs_rccl_create: no HIP device " + std::to_string(device));
    return GS_EDEVICE;
  }
  auto* c = new gs_rccl();
  c->rank = rank;
  c->world = world;
  c->device = device;
  hipError_t h = hipSetDevice(device);
  if (h == hipSuccess) h = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (h != hipSuccess) {
    delete c;
    return failh("stream", h);
  }
  ncclUniqueId u;
  std::memcpy(u.internal, id, GS_RCCL_ID_BYTES);
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return fail("ncclCommInitRank", r);
  }
  *out = c;
  return GS_OK;
}

int gs_rccl_transport(gs_rccl* comm, gs_transport* out) {
  if (!comm || !out) {
    gs_set_error("gs_rccl_transport: NULL argument");
    return GS_EINVAL;
  }
  out->user = comm;
  out->allgather_i64 = cb_allgather_i64;
  out->allgather = cb_allgather;
  out->alltoallv = cb_alltoallv;
  return GS_OK;
}

int gs_rccl_stats(const gs_rccl* comm, int64_t* calls, int64_t* bytes_in) {
  if (!comm) {
    gs_set_error("gs_rccl_stats: NULL communicator");
    return GS_EINVAL;
  }
  if (calls) *calls = comm->calls;
  if (bytes_in) *bytes_in = comm->bytesIn;
  return GS_OK;
}

int gs_rccl_destroy(gs_rccl* comm) {
  if (!comm) return GS_OK;
  (void)hipSetDevice(comm->device);
  if (comm->stream) (void)hipStreamSynchronize(comm->stream);
  if (comm->comm) (void)ncclCommDestroy(comm->comm);
  if (comm->scratch) (void)hipFree(comm->scratch);
  if (comm->stream) (void)hipStreamDestroy(comm->stream);
  delete comm;
  return GS_OK;
}

}  // extern "C"
