"""ctypes binding of oracle/build/liboracle.so (TEST INFRASTRUCTURE ONLY).

The C restatement of vecengine + vecfc keyed by dense Add-order indices.
"""

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.orc_create.restype = ctypes.c_void_p
        L.orc_create.argtypes = [ctypes.c_uint32, u32p]
        L.orc_destroy.argtypes = [ctypes.c_void_p]
        L.orc_add.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p]
        L.orc_add_batch.restype = ctypes.c_int64
        L.orc_add_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u32p, u32p, u64p, u32p, ctypes.c_int]
        L.orc_flush.argtypes = [ctypes.c_void_p]
        L.orc_drop_not_flushed.argtypes = [ctypes.c_void_p]
        L.orc_num_events.restype = ctypes.c_uint64
        L.orc_num_events.argtypes = [ctypes.c_void_p]
        L.orc_num_branches.restype = ctypes.c_uint32
        L.orc_num_branches.argtypes = [ctypes.c_void_p]
        L.orc_get_branch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, u32p]
        for f in (L.orc_get_hb, L.orc_get_la, L.orc_get_merged_hb):
            f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, u8p, ctypes.c_uint32, u32p]
        L.orc_forkless_cause.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_forkless_cause_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u32p, u32p, u8p]
        _lib = L
    return _lib


def _p(arr, t):
    return arr.ctypes.data_as(t)


class OracleIndex:
    """Dense-index C oracle.  weights in validator idx order."""

    def __init__(self, weights):
        self.L = lib()
        w = np.ascontiguousarray(weights, dtype=np.uint32)
        self.h = self.L.orc_create(len(w), _p(w, u32p))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_destroy(self.h)
            self.h = None

    def add(self, creator_idx, seq, parents):
        p = np.ascontiguousarray(parents, dtype=np.uint32)
        return self.L.orc_add(self.h, creator_idx, seq, len(p), _p(p, u32p))

    def add_batch(self, creator, seq, poff, parents, flush_each=False):
        creator = np.ascontiguousarray(creator, dtype=np.uint32)
        seq = np.ascontiguousarray(seq, dtype=np.uint32)
        poff = np.ascontiguousarray(poff, dtype=np.uint64)
        parents = np.ascontiguousarray(parents, dtype=np.uint32)
        return self.L.orc_add_batch(self.h, len(creator), _p(creator, u32p), _p(seq, u32p),
                                    _p(poff, u64p), _p(parents, u32p), int(flush_each))

    def flush(self):
        self.L.orc_flush(self.h)

    def drop_not_flushed(self):
        self.L.orc_drop_not_flushed(self.h)

    def num_events(self):
        return self.L.orc_num_events(self.h)

    def num_branches(self):
        return self.L.orc_num_branches(self.h)

    def branch(self, ev):
        out = ctypes.c_uint32()
        if self.L.orc_get_branch(self.h, ev, ctypes.byref(out)) != 0:
            return None
        return out.value

    def _row(self, f, ev):
        n = ctypes.c_uint32()
        if f(self.h, ev, None, 0, ctypes.byref(n)) != 0:
            return None
        buf = (ctypes.c_uint8 * max(n.value, 1))()
        f(self.h, ev, buf, n.value, ctypes.byref(n))
        return bytes(buf[:n.value])

    def hb(self, ev):
        return self._row(self.L.orc_get_hb, ev)

    def la(self, ev):
        return self._row(self.L.orc_get_la, ev)

    def merged_hb(self, ev):
        return self._row(self.L.orc_get_merged_hb, ev)

    def forkless_cause(self, a, b):
        return self.L.orc_forkless_cause(self.h, a, b)

    def forkless_cause_batch(self, a, b):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros(len(a), dtype=np.uint8)
        self.L.orc_forkless_cause_batch(self.h, len(a), _p(a, u32p), _p(b, u32p), _p(out, u8p))
        return out
