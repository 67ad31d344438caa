"""RPC size accounting and fragmentation through the product library
(include/gs_rpc.h, csrc/gs_rpc.cpp).

Mirrors fragmentRPC / fragmentMessageIds (gossipsub.go:1158-1272): sendRPC
(gossipsub.go:1101-1156) cuts an outgoing RPC that reaches the stream's maximum
message size into RPCs that each fit.  The caller describes the RPC by the sizes
of its parts (``RpcShape``); ``fragment_rpc`` returns which fragment every part
lands in and each fragment's encoded size.  Errors follow the reference: a
published message over the limit raises ``GossipEngineError`` with the
reference's text "message with len=%d exceeds limit %d".
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .engine import PRODUCT_LIB, GossipEngineError

GS_RPC_IHAVE = 0
GS_RPC_IWANT = 1
_GS_ECAPACITY = -5

_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


class _Shape(C.Structure):
    _fields_ = [("n_sub", C.c_int32), ("sub_size", _i64p),
                ("n_pub", C.c_int32), ("pub_size", _i64p),
                ("has_control", C.c_int32),
                ("n_ihave", C.c_int32), ("ihave_topic_len", _i64p), ("ihave_nids", _i32p),
                ("n_iwant", C.c_int32), ("iwant_nids", _i32p),
                ("id_len", _i64p),
                ("n_graft", C.c_int32), ("graft_size", _i64p),
                ("n_prune", C.c_int32), ("prune_size", _i64p)]


class _Frags(C.Structure):
    _fields_ = [("sub_frag", _i32p), ("pub_frag", _i32p), ("graft_frag", _i32p),
                ("prune_frag", _i32p), ("id_bucket", _i32p), ("bucket_cap", C.c_int32),
                ("bucket_frag", _i32p), ("bucket_kind", _i32p), ("bucket_src", _i32p),
                ("frag_cap", C.c_int32), ("frag_size", _i64p),
                ("n_bucket", C.c_int32), ("n_frag", C.c_int32), ("control_whole", C.c_int32)]


_lib = None


def _library():
    global _lib
    if _lib is None:
        lib = C.CDLL(PRODUCT_LIB)
        lib.gs_rpc_size.restype = C.c_int64
        lib.gs_rpc_size.argtypes = [C.POINTER(_Shape)]
        lib.gs_fragment_rpc.restype = C.c_int
        lib.gs_fragment_rpc.argtypes = [C.POINTER(_Shape), C.c_int64, C.POINTER(_Frags)]
        lib.gs_last_error.restype = C.c_char_p
        _lib = lib
    return _lib


@dataclass
class RpcShape:
    """The sizes fragmentRPC looks at (pb/rpc.proto).  ``*_size`` are the parts'
    Size(); ``ihave_ids`` / ``iwant_ids`` hold the length of every message id of
    each entry; ``ihave_topic_len`` is len(TopicID) or None when it is nil."""
    sub_size: List[int] = field(default_factory=list)
    pub_size: List[int] = field(default_factory=list)
    has_control: bool = False
    ihave_topic_len: List[Optional[int]] = field(default_factory=list)
    ihave_ids: List[List[int]] = field(default_factory=list)
    iwant_ids: List[List[int]] = field(default_factory=list)
    graft_size: List[int] = field(default_factory=list)
    prune_size: List[int] = field(default_factory=list)

    def _c(self):
        def a64(x):
            return np.ascontiguousarray(np.asarray(x, dtype=np.int64).reshape(-1))

        def a32(x):
            return np.ascontiguousarray(np.asarray(x, dtype=np.int32).reshape(-1))

        keep = {
            "sub": a64(self.sub_size), "pub": a64(self.pub_size),
            "tl": a64([-1 if t is None else t for t in self.ihave_topic_len]),
            "hn": a32([len(x) for x in self.ihave_ids]), "wn": a32([len(x) for x in self.iwant_ids]),
            "ids": a64([l for x in self.ihave_ids for l in x] + [l for x in self.iwant_ids for l in x]),
            "g": a64(self.graft_size), "p": a64(self.prune_size),
        }
        if len(self.ihave_topic_len) != len(self.ihave_ids):
            raise ValueError("ihave_topic_len and ihave_ids differ in length")
        s = _Shape(len(keep["sub"]), keep["sub"].ctypes.data_as(_i64p),
                   len(keep["pub"]), keep["pub"].ctypes.data_as(_i64p),
                   int(self.has_control),
                   len(keep["hn"]), keep["tl"].ctypes.data_as(_i64p), keep["hn"].ctypes.data_as(_i32p),
                   len(keep["wn"]), keep["wn"].ctypes.data_as(_i32p),
                   keep["ids"].ctypes.data_as(_i64p),
                   len(keep["g"]), keep["g"].ctypes.data_as(_i64p),
                   len(keep["p"]), keep["p"].ctypes.data_as(_i64p))
        return s, keep


@dataclass
class Fragments:
    """Where every part went.  ``id_bucket`` follows the id order of RpcShape
    (ihave ids, then iwant ids); bucket b is entry ``bucket_src[b]`` of kind
    ``bucket_kind[b]`` (a fresh entry without TopicID unless ``control_whole``
    or a single fragment), placed in fragment ``bucket_frag[b]``."""
    frag_size: np.ndarray
    sub_frag: np.ndarray
    pub_frag: np.ndarray
    graft_frag: np.ndarray
    prune_frag: np.ndarray
    id_bucket: np.ndarray
    bucket_frag: np.ndarray
    bucket_kind: np.ndarray
    bucket_src: np.ndarray
    control_whole: bool

    @property
    def n_frag(self):
        return len(self.frag_size)


def rpc_size(shape: RpcShape) -> int:
    """RPC.Size() of the shape."""
    s, _keep = shape._c()
    n = _library().gs_rpc_size(C.byref(s))
    if n < 0:
        raise GossipEngineError(int(n), _library().gs_last_error().decode())
    return int(n)


def fragment_rpc(shape: RpcShape, limit: int) -> Fragments:
    """fragmentRPC(rpc, limit), gossipsub.go:1158."""
    lib = _library()
    s, _keep = shape._c()
    n_ids = len(_keep["ids"])
    frag_cap = bucket_cap = 16
    while True:
        o = {k: np.full(n, -1, np.int32) for k, n in (
            ("sub", s.n_sub), ("pub", s.n_pub), ("g", s.n_graft), ("p", s.n_prune), ("ids", n_ids),
            ("bf", bucket_cap), ("bk", bucket_cap), ("bs", bucket_cap))}
        fs = np.zeros(frag_cap, np.int64)
        f = _Frags(o["sub"].ctypes.data_as(_i32p), o["pub"].ctypes.data_as(_i32p),
                   o["g"].ctypes.data_as(_i32p), o["p"].ctypes.data_as(_i32p),
                   o["ids"].ctypes.data_as(_i32p), bucket_cap,
                   o["bf"].ctypes.data_as(_i32p), o["bk"].ctypes.data_as(_i32p),
                   o["bs"].ctypes.data_as(_i32p), frag_cap, fs.ctypes.data_as(_i64p), 0, 0, 0)
        rc = lib.gs_fragment_rpc(C.byref(s), int(limit), C.byref(f))
        if rc == _GS_ECAPACITY:
            frag_cap, bucket_cap = max(frag_cap, f.n_frag), max(bucket_cap, f.n_bucket)
            continue
        if rc != 0:
            raise GossipEngineError(rc, lib.gs_last_error().decode())
        nb = f.n_bucket
        return Fragments(fs[:f.n_frag].copy(), o["sub"], o["pub"], o["g"], o["p"], o["ids"],
                         o["bf"][:nb].copy(), o["bk"][:nb].copy(), o["bs"][:nb].copy(),
                         bool(f.control_whole))
