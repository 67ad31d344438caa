import ctypes as C
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "go-libp2p-pubsub_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

ORACLE_LIB = os.path.join(REPO, "oracle", "_build", "libgossip_oracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _ensure_oracle():
    src_dir = os.path.join(REPO, "oracle")
    srcs = [os.path.join(src_dir, f) for f in ("oracle_sim.cpp", "oracle_objects.cpp", "oracle_core.hpp")]
    stale = not os.path.exists(ORACLE_LIB) or any(os.path.getmtime(s) > os.path.getmtime(ORACLE_LIB) for s in srcs)
    if stale:
        subprocess.check_call(["make", "-s", "-C", src_dir])
    return ORACLE_LIB


@pytest.fixture(scope="session")
def oracle_path():
    return _ensure_oracle()


@pytest.fixture(scope="session")
def olib(oracle_path):
    """The oracle's object-level exports (ops_/omc_/ogt_/opg_/orng_)."""
    from pubsub_amd import _abi
    lib = C.CDLL(oracle_path, mode=C.RTLD_LOCAL)
    P = C.c_void_p
    i32, i64, u32, u64, f64 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
    sigs = {
        "ops_new": (P, [C.POINTER(_abi.PeerScoreParamsC)]), "ops_free": (None, [P]),
        "ops_set_app_score": (None, [P, i32, f64]),
        "ops_set_topic": (None, [P, i32, C.POINTER(_abi.TopicScoreParamsC)]),
        "ops_set_topic_score_params": (None, [P, i32, C.POINTER(_abi.TopicScoreParamsC)]),
        "ops_add_whitelist": (None, [P, u32, u32]), "ops_add_peer": (None, [P, i32]),
        "ops_remove_peer": (None, [P, i32, i64]), "ops_set_ips": (None, [P, i32, i32, C.POINTER(u32)]),
        "ops_score": (f64, [P, i32]), "ops_graft": (None, [P, i32, i32, i64]), "ops_prune": (None, [P, i32, i32]),
        "ops_add_penalty": (None, [P, i32, i32]), "ops_refresh": (None, [P, i64]),
        "ops_validate": (None, [P, i64, i32, i32, i64]), "ops_deliver": (None, [P, i64, i32, i32, i64]),
        "ops_duplicate": (None, [P, i64, i32, i32, i64]), "ops_reject": (None, [P, i64, i32, i32, i32, i64]),
        "ops_gc": (None, [P, i64]), "ops_expire_head": (None, [P, i64]),
        "ops_topic_stats": (C.c_int, [P, i32, i32, C.POINTER(f64)]),
        "ops_set_stats": (None, [P, i32, i32, i32, i64, i64, f64, f64, f64, f64]),
        "ops_set_behaviour_penalty": (None, [P, i32, f64]),
        "omc_new": (P, [i32, i32]), "omc_free": (None, [P]), "omc_put": (None, [P, i64, i32]),
        "omc_get": (C.c_int, [P, i64]), "omc_get_for_peer": (C.c_int, [P, i64, i32]),
        "omc_gossip_ids": (C.c_int, [P, i32, C.POINTER(i64), i32]), "omc_len": (C.c_int, [P]),
        "omc_shift": (None, [P]),
        "ogt_new": (P, [i64]), "ogt_free": (None, [P]),
        "ogt_add_promise": (None, [P, i32, i32, C.POINTER(i64), i32, i64]),
        "ogt_broken": (C.c_int, [P, i64, C.POINTER(C.c_int), C.POINTER(C.c_int), i32]),
        "ogt_deliver": (None, [P, i64]), "ogt_throttle": (None, [P, i32]),
        "opg_new": (P, [C.POINTER(_abi.PeerGaterParamsC), C.POINTER(u32), i32]), "opg_free": (None, [P]),
        "opg_add_peer": (None, [P, i32]), "opg_remove_peer": (None, [P, i32, i64]),
        "opg_accept_from": (C.c_int, [P, i32, i64, f64]), "opg_validate": (None, [P]),
        "opg_deliver": (None, [P, i32]), "opg_duplicate": (None, [P, i32]),
        "opg_reject": (None, [P, i32, i32, i64]), "opg_decay": (None, [P, i64]),
        "opg_has_peer_stats": (C.c_int, [P, i32]), "opg_has_ip_stats": (C.c_int, [P, u32]),
        "opg_set_ip_expire": (None, [P, u32, i64]),
        "orng_key64": (u64, [u32, u32, u32, u32, u32, u32]),
        "orng_key64_mid": (u64, [u32, u32, u32, u32, u32, u32]),
        "orng_philox": (None, [C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
