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
        L.orc_get_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, u32p, u64p, u8p, ctypes.c_uint64]
        L.orc_forkless_cause_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u32p, u32p, u8p]
        L.orc_forkless_cause_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u32p, u32p, u8p, ctypes.c_int]
        # abft_oracle.c
        L.abo_create.restype = ctypes.c_void_p
        L.abo_create.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_void_p]
        L.abo_destroy.argtypes = [ctypes.c_void_p]
        L.abo_process_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, u32p, u32p, u64p, u32p, u32p, u32p, u32p]
        L.abo_build.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p]
        for f in (L.abo_epoch, L.abo_last_decided_frame, L.abo_num_events):
            f.restype = ctypes.c_uint32
            f.argtypes = [ctypes.c_void_p]
        L.abo_event_frame.restype = ctypes.c_uint32
        L.abo_event_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.abo_trace.argtypes = [ctypes.c_void_p, u64p]
        L.abo_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.abo_fc_seconds.restype = ctypes.c_double
        L.abo_fc_seconds.argtypes = [ctypes.c_void_p]
        L.abo_set_fc_cache.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.abo_frame_roots.restype = ctypes.c_uint32
        L.abo_frame_roots.argtypes = [ctypes.c_void_p, ctypes.c_uint32, u32p, ctypes.c_uint32]
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

    def rows(self, mode, evs):
        """Rows of many events at once (mode 0 HighestBefore, 1 LowestAfter):
        (offsets[n + 1], bytes) as numpy arrays."""
        evs = np.ascontiguousarray(evs, dtype=np.uint32)
        off = np.zeros(len(evs) + 1, dtype=np.uint64)
        assert self.L.orc_get_rows(self.h, mode, len(evs), _p(evs, u32p), _p(off, u64p), None, 0) == 0
        buf = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
        assert self.L.orc_get_rows(self.h, mode, len(evs), _p(evs, u32p), _p(off, u64p), _p(buf, u8p), len(buf)) == 0
        return off, buf[:int(off[-1])]

    def forkless_cause(self, a, b):
        return self.L.orc_forkless_cause(self.h, a, b)

    def forkless_cause_batch(self, a, b):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros(len(a), dtype=np.uint8)
        self.L.orc_forkless_cause_batch(self.h, len(a), _p(a, u32p), _p(b, u32p), _p(out, u8p))
        return out

    def c_funcs(self):
        """This index as C function pointers (handle, add, flush, drop, fc,
        merged_hb) for lachesis_hip.dropin.replay(kind="cpu") -- the bench's
        cpu_baseline leg and the tests drive the same caller restatement over
        this CPU index."""
        f = lambda fn: ctypes.cast(fn, ctypes.c_void_p).value
        L = self.L
        return {"owner": self, "h": self.h, "add": f(L.orc_add), "flush": f(L.orc_flush), "drop": f(L.orc_drop_not_flushed),
                "fc": f(L.orc_forkless_cause), "merged_hb": f(L.orc_get_merged_hb)}

    def forkless_cause_batch_mt(self, a, b, threads):
        """The same over OpenMP threads (CPU baseline; results identical)."""
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros(len(a), dtype=np.uint8)
        self.L.orc_forkless_cause_batch_mt(self.h, len(a), _p(a, u32p), _p(b, u32p), _p(out, u8p), int(threads))
        return out


_BEGIN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32)
_APPLY = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32)
_END = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, u32p, ctypes.POINTER(u32p))


class _Cb(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("begin_block", _BEGIN), ("apply_event", _APPLY), ("end_block", _END)]


class AbftOracle:
    """Dense-index C restatement of abft.IndexedLachesis (abft_oracle.c), with
    the batch semantics of lx_abft_process_batch.  Records every block as
    (epoch, frame, atropos, cheaters, confirmed events); ``seal(epoch, frame)``
    may return new weights (idx order) to seal the epoch."""

    def __init__(self, weights, epoch=1, seal=None):
        self.L = lib()
        self.blocks = []
        self.seal = seal
        self._cur = None
        self._keep_w = None
        self._cb = _Cb(None, _BEGIN(self._begin), _APPLY(self._apply), _END(self._end))
        w = np.ascontiguousarray(weights, dtype=np.uint32)
        self.h = self.L.abo_create(epoch, len(w), _p(w, u32p), ctypes.cast(ctypes.pointer(self._cb), ctypes.c_void_p))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.abo_destroy(self.h)
            self.h = None

    def _begin(self, user, frame, atropos, cheaters, n):
        self._cur = [self.epoch(), frame, atropos, tuple(cheaters[k] for k in range(n)), []]

    def _apply(self, user, ev):
        self._cur[4].append(ev)

    def _end(self, user, n_out, w_out):
        b = self._cur
        self.blocks.append((b[0], b[1], b[2], b[3], tuple(b[4])))
        nw = self.seal(b[0], b[1]) if self.seal else None
        if nw is None:
            return 0
        self._keep_w = np.ascontiguousarray(nw, dtype=np.uint32)
        n_out[0] = len(self._keep_w)
        w_out[0] = _p(self._keep_w, u32p)
        return 1

    def process_batch(self, creator, seq, poff, par, claimed=None):
        creator = np.ascontiguousarray(creator, dtype=np.uint32)
        seq = np.ascontiguousarray(seq, dtype=np.uint32)
        poff = np.ascontiguousarray(poff, dtype=np.uint64)
        par = np.ascontiguousarray(par if len(par) else [0], dtype=np.uint32)
        n = len(creator)
        out = np.zeros(n, dtype=np.uint32)
        cl = None if claimed is None else np.ascontiguousarray(claimed, dtype=np.uint32)
        consumed = ctypes.c_uint32()
        rc = self.L.abo_process_batch(self.h, n, _p(creator, u32p), _p(seq, u32p), _p(poff, u64p), _p(par, u32p),
                                      None if cl is None else _p(cl, u32p), _p(out, u32p), ctypes.byref(consumed))
        return rc, consumed.value, out

    def trace(self):
        """The caller's call sequence on the index so far: {"hash", "fc_calls",
        "fc_lru_hits", "adds", "flushes", "drops"} (abo_trace)."""
        out = np.zeros(6, dtype=np.uint64)
        self.L.abo_trace(self.h, _p(out, u64p))
        return dict(zip(("hash", "fc_calls", "fc_lru_hits", "adds", "flushes", "drops"), map(int, out)))

    def set_fc_cache(self, pairs):
        """The reference's ForklessCause LRU (DefaultConfig: 20000 pairs); 0 = none."""
        self.L.abo_set_fc_cache(self.h, pairs)

    def set_timing(self, on=True):
        self.L.abo_set_timing(self.h, int(on))

    def fc_seconds(self):
        return self.L.abo_fc_seconds(self.h)

    def epoch(self):
        return self.L.abo_epoch(self.h)

    def last_decided_frame(self):
        return self.L.abo_last_decided_frame(self.h)

    def frame_roots(self, f):
        n = self.L.abo_frame_roots(self.h, f, None, 0)
        out = np.zeros(max(n, 1), dtype=np.uint32)
        self.L.abo_frame_roots(self.h, f, _p(out, u32p), n)
        return out[:n]
