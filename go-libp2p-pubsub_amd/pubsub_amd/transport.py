"""gs_transport over torch.distributed: the per-hop exchange of a partitioned
engine (gossip_engine.h).

In the reference every host runs its own router and the only traffic between
hosts is RPCs (pubsub.go:902-970).  A partitioned engine simulates one node
range per GPU, and at the end of every hop it hands the RPCs its nodes sent to
other ranks' nodes to this transport:

  allgather_i64  a handful of sizes per rank (host memory);
  allgather      each rank's frontier lists, IWANT arena segment and, after a
                 heartbeat, its IHAVE payload rows (equal-size device chunks);
  alltoallv      per-edge records (forwarding sets + control outbox) to the
                 rank owning the receiving node.

With the "nccl" backend (RCCL on ROCm, over xGMI between the GPUs of a node)
the collectives run directly on the engine's device buffers.  With "gloo" the
buffers are staged through host memory, which lets several ranks share one GPU
(tests) or run with no GPU at all (`memory="host"`: the buffers are host
pointers, used by the CPU tests of this module).
"""
import ctypes as C
import traceback

import numpy as np
import torch
import torch.distributed as dist

from . import _abi


class _DevicePtr:
    """A raw device pointer seen as a uint8 tensor (zero-copy)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {
            "shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False), "version": 2}


class TorchTransport:
    """Implements gs_transport with torch.distributed collectives.

    memory: "device" — the engine passes HIP device pointers (product engine);
            "host"   — host pointers (CPU tests of the transport itself).
    """

    def __init__(self, group=None, memory="device", device=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.memory = memory
        if device is None and memory == "device":
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.on_device = self.backend == "nccl"  # collectives need device tensors
        self.calls = 0
        self.c = _abi.TransportC()
        self.c.user = None
        # keep the ctypes callback objects alive as long as the transport
        self._cb = (_abi.ALLGATHER_I64(self._allgather_i64), _abi.ALLGATHER(self._allgather),
                    _abi.ALLTOALLV(self._alltoallv))
        self.c.allgather_i64, self.c.allgather, self.c.alltoallv = self._cb

    # ---------------------------------------------------------------- buffers
    def _view(self, ptr, nbytes):
        """The engine's buffer as a uint8 tensor sharing its memory."""
        nbytes = int(nbytes)
        if nbytes == 0 or not ptr:
            dev = self.device if self.memory == "device" else "cpu"
            return torch.empty(0, dtype=torch.uint8, device=dev)
        if self.memory == "host":
            arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(int(ptr)))
            return torch.from_numpy(arr)
        return torch.as_tensor(_DevicePtr(ptr, nbytes), device=self.device)

    def _sync(self):
        if self.memory == "device" or self.on_device:
            torch.cuda.current_stream().synchronize()

    # ---------------------------------------------------------------- callbacks
    def _guard(fn):
        def run(self, *a):
            try:
                fn(self, *a)
                self.calls += 1
                return 0
            except Exception:  # never unwind through the C caller
                traceback.print_exc()
                return -1
        return run

    @_guard
    def _allgather_i64(self, _user, mine, n, out):
        src = np.ctypeslib.as_array(mine, shape=(n,)).copy()
        t = torch.from_numpy(src)
        if self.on_device:
            t = t.to(self.device)
        res = torch.empty(self.world * n, dtype=torch.int64, device=t.device)
        if self.on_device:
            dist.all_gather_into_tensor(res, t, group=self.group)
        else:
            dist.all_gather(list(res.chunk(self.world)), t, group=self.group)
        np.ctypeslib.as_array(out, shape=(self.world * n,))[:] = res.cpu().numpy()

    @_guard
    def _allgather(self, _user, send, recv, nbytes):
        s = self._view(send, nbytes)
        r = self._view(recv, nbytes * self.world)
        if self.on_device:
            dist.all_gather_into_tensor(r, s, group=self.group)
        else:
            rc = torch.empty(nbytes * self.world, dtype=torch.uint8)
            dist.all_gather(list(rc.chunk(self.world)), s.cpu(), group=self.group)
            r.copy_(rc)
        self._sync()

    @_guard
    def _alltoallv(self, _user, send, send_bytes, recv, recv_bytes):
        sb = [int(x) for x in np.ctypeslib.as_array(send_bytes, shape=(self.world,))]
        rb = [int(x) for x in np.ctypeslib.as_array(recv_bytes, shape=(self.world,))]
        s = self._view(send, sum(sb))
        r = self._view(recv, sum(rb))
        if self.on_device:
            dist.all_to_all_single(r, s, output_split_sizes=rb, input_split_sizes=sb, group=self.group)
        else:
            rc = torch.empty(sum(rb), dtype=torch.uint8)
            _alltoallv_p2p(rc, s.cpu(), rb, sb, self.rank, self.world, self.group)
            r.copy_(rc)
        self._sync()


def _alltoallv_p2p(out, inp, out_splits, in_splits, rank, world, group):
    """all-to-all-v as paired send/recv (gloo has no uneven all_to_all)."""
    ro = np.concatenate([[0], np.cumsum(out_splits)]).astype(np.int64)
    so = np.concatenate([[0], np.cumsum(in_splits)]).astype(np.int64)
    out[ro[rank]:ro[rank + 1]].copy_(inp[so[rank]:so[rank + 1]])
    reqs = []
    for peer in range(world):
        if peer == rank:
            continue
        if in_splits[peer]:
            reqs.append(dist.isend(inp[so[peer]:so[peer + 1]].contiguous(), _global(peer, group), group=group))
        if out_splits[peer]:
            reqs.append(dist.irecv(out[ro[peer]:ro[peer + 1]], _global(peer, group), group=group))
    for q in reqs:
        q.wait()


def _global(rank, group):
    return rank if group is None else dist.get_global_rank(group, rank)


class RcclTransport:
    """The product library's native RCCL transport (include/gs_transport.h):
    the same gs_transport semantics as TorchTransport with the collectives
    issued by C++ (ncclAllGather, grouped ncclSend / ncclRecv) on the engine's
    device buffers — what a cgo host uses.  The communicator
    id is made on rank 0 and handed to the other ranks through `group`
    (torch.distributed, any backend) or given as `uid` (bytes)."""

    def __init__(self, rank, world, device=0, group=None, uid=None, lib=None):
        from .engine import PRODUCT_LIB
        self.lib = C.CDLL(lib or PRODUCT_LIB, mode=C.RTLD_LOCAL)
        for name, res, args in _abi.RCCL_FUNCTIONS + [("gs_last_error", C.c_char_p, [])]:
            fn = getattr(self.lib, name)  # AttributeError = missing export: fail loudly
            fn.restype, fn.argtypes = res, args
        n = _abi.GS_RCCL_ID_BYTES
        idbuf = (C.c_uint8 * n)()
        if uid is None:
            if rank == 0:
                self._check(self.lib.gs_rccl_get_unique_id(idbuf))
            if world > 1:
                obj = [bytes(idbuf)]
                dist.broadcast_object_list(obj, src=0, group=group)
                C.memmove(idbuf, obj[0], n)
        else:
            C.memmove(idbuf, bytes(uid), n)
        self.uid = bytes(idbuf)
        self.h = C.c_void_p()
        self._check(self.lib.gs_rccl_create(int(rank), int(world), idbuf, int(device), C.byref(self.h)))
        self.c = _abi.TransportC()
        self._check(self.lib.gs_rccl_transport(self.h, C.byref(self.c)))
        self.rank, self.world = rank, world

    def _check(self, rc):
        if rc != _abi.GS_OK:
            from .engine import GossipEngineError
            raise GossipEngineError(rc, self.lib.gs_last_error().decode(errors="replace"))

    @property
    def calls(self):
        c, b = C.c_int64(), C.c_int64()
        self._check(self.lib.gs_rccl_stats(self.h, C.byref(c), C.byref(b)))
        return c.value

    def close(self):
        if self.h:
            self.lib.gs_rccl_destroy(self.h)
            self.h = C.c_void_p()
