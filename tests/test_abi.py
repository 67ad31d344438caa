"""The product library loads without a GPU, exports every function declared in
include/gossip_engine.h, mirrors the reference's parameter validation, and
refuses to run (GS_EDEVICE) when no HIP device is present — there is no CPU
fallback in the product path."""
import ctypes as C
import os
import re

import pytest

from pubsub_amd import PRODUCT_LIB, _abi
from pubsub_amd.params import GossipSubParams, Hour

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(REPO, "include", "gossip_engine.h")).read()
    return sorted(set(re.findall(r"^[a-z_0-9 \*]+?\b(gs_[a-z_0-9]+)\(", src, re.M)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(n for n, _, _ in _abi.ABI_FUNCTIONS)


@pytest.mark.parametrize("which", ["product", "oracle"])
def test_library_exports_every_symbol(which, oracle_path):
    path = PRODUCT_LIB if which == "product" else oracle_path
    if which == "product" and not os.path.exists(path):
        pytest.skip("product library not built (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name in declared_functions():
        assert hasattr(lib, name), f"{which} library does not export {name}"


def test_product_exports_rpc_header():
    """include/gs_rpc.h (host-side RPC fragmentation) is product-only."""
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    src = open(os.path.join(REPO, "include", "gs_rpc.h")).read()
    names = set(re.findall(r"^[a-z_0-9 \*]+?\b(gs_[a-z_0-9]+)\(", src, re.M))
    assert {"gs_rpc_size", "gs_fragment_rpc"} <= names
    lib = C.CDLL(PRODUCT_LIB)
    for name in names:
        assert hasattr(lib, name), f"product library does not export {name}"


def test_product_params_match_oracle(oracle_path):
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    prod, orac = _abi.bind(PRODUCT_LIB), _abi.bind(oracle_path)
    a, b = _abi.GossipSubParamsC(), _abi.GossipSubParamsC()
    prod.gs_default_gossipsub_params(C.byref(a))
    orac.gs_default_gossipsub_params(C.byref(b))
    assert bytes(a) == bytes(b) == bytes(GossipSubParams().to_c())
    assert prod.gs_score_parameter_decay(Hour) == .9987216039048303
    ga, gb = _abi.PeerGaterParamsC(), _abi.PeerGaterParamsC()
    prod.gs_default_peer_gater_params(C.byref(ga))
    orac.gs_default_peer_gater_params(C.byref(gb))
    assert bytes(ga) == bytes(gb)


def test_product_validation_tables(oracle_path):
    """score_params_test.go tables against the product's validate() mirrors."""
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    import test_oracle_params as t
    lib = _abi.bind(PRODUCT_LIB)
    t.test_thresholds_validation(lib)
    t.test_topic_score_params_validation(lib)
    t.test_peer_score_params_validation(lib)


def test_product_fails_loudly_without_gpu():
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    from pubsub_amd import GossipEngineError, NewFloodSub, graphs
    g = graphs.dense_connect(10, 1)
    with pytest.raises(GossipEngineError) as ei:
        NewFloodSub(10, 1, g, graphs.all_subscribed(10, 1))
    assert ei.value.code == _abi.GS_EDEVICE


def test_product_exports_transport_header():
    """include/gs_transport.h (native RCCL transport) is product-only and bound
    by pubsub_amd.transport.RcclTransport."""
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    src = open(os.path.join(REPO, "include", "gs_transport.h")).read()
    names = set(re.findall(r"^[a-z_0-9 \*]+?\b(gs_[a-z_0-9]+)\(", src, re.M))
    assert names == {n for n, _, _ in _abi.RCCL_FUNCTIONS}
    lib = C.CDLL(PRODUCT_LIB)
    for name in names:
        assert hasattr(lib, name), f"product library does not export {name}"


def test_rccl_transport_refuses_bad_arguments_and_no_gpu():
    if not os.path.exists(PRODUCT_LIB):
        pytest.skip("product library not built")
    import torch
    lib = C.CDLL(PRODUCT_LIB)
    for name, res, args in _abi.RCCL_FUNCTIONS:
        getattr(lib, name).restype, getattr(lib, name).argtypes = res, args
    idb = (C.c_uint8 * _abi.GS_RCCL_ID_BYTES)()
    h = C.c_void_p()
    assert lib.gs_rccl_create(2, 2, idb, 0, C.byref(h)) == _abi.GS_EINVAL  # rank >= world
    assert lib.gs_rccl_create(0, 0, idb, 0, C.byref(h)) == _abi.GS_EINVAL
    assert lib.gs_rccl_transport(None, None) == _abi.GS_EINVAL
    assert lib.gs_rccl_destroy(None) == _abi.GS_OK
    if torch.cuda.device_count() == 0:
        assert lib.gs_rccl_create(0, 1, idb, 0, C.byref(h)) == _abi.GS_EDEVICE
