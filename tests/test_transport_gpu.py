"""The native RCCL transport (include/gs_transport.h) on the GPU: the three
gs_transport callbacks on device buffers, driven exactly as the engine drives
them.  One GPU per box, so one rank (RCCL refuses two ranks on one device):
the collectives, the staging of allgather_i64 and the own-block copy of
alltoallv run for real; cross-rank traffic is covered by the torch transport's
multi-rank tests (same semantics, test_partition_gpu.py / test_transport_cpu.py)."""
import ctypes as C

import numpy as np
import pytest
import torch

from pubsub_amd import _abi
from pubsub_amd.transport import RcclTransport

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl():
    torch.cuda.set_device(0)
    t = RcclTransport(0, 1, device=0)
    yield t
    t.close()


def test_allgather_i64(rccl):
    mine = np.array([7, -3, 1 << 40], np.int64)
    out = np.zeros(3, np.int64)
    rc = rccl.c.allgather_i64(rccl.c.user, mine.ctypes.data_as(C.POINTER(C.c_int64)), 3,
                              out.ctypes.data_as(C.POINTER(C.c_int64)))
    assert rc == 0
    assert np.array_equal(out, mine)


def test_allgather_device(rccl):
    src = torch.arange(1000, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(1000, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert rccl.c.allgather(rccl.c.user, src.data_ptr(), dst.data_ptr(), 1000) == 0
    assert torch.equal(src, dst)


def test_alltoallv_own_block(rccl):
    src = torch.randint(0, 255, (4096,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    sb = np.array([4096], np.int64)
    rb = np.array([4096], np.int64)
    rc = rccl.c.alltoallv(rccl.c.user, src.data_ptr(), sb.ctypes.data_as(C.POINTER(C.c_int64)),
                          dst.data_ptr(), rb.ctypes.data_as(C.POINTER(C.c_int64)))
    assert rc == 0
    assert torch.equal(src, dst)
    assert rccl.calls >= 1
    bad = np.array([10], np.int64)
    rc = rccl.c.alltoallv(rccl.c.user, src.data_ptr(), sb.ctypes.data_as(C.POINTER(C.c_int64)),
                          dst.data_ptr(), bad.ctypes.data_as(C.POINTER(C.c_int64)))
    assert rc == _abi.GS_EINVAL
