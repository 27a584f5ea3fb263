"""Level-synchronous DAG batcher over include/lachesis_batcher.h.

The GPU-side counterpart of gossip/dagordering.EventsBuffer
(event_buffer.go:53-110): events arrive in any order; an event waits until
every parent is known; ``pop`` releases everything releasable as one
parents-first batch in topological levels, ready for ``lx_add_batch``
(bit-exact to the reference's per-event Add in the released order).

:class:`LevelBatcher` names events by any hashable id (a ``hash.Event`` in the
reference) and keeps the id <-> uint64 handle map the cgo shim would keep.
:meth:`LevelBatcher.drain_into` feeds a :class:`~lachesis_hip.VecfcIndex`.
"""

import ctypes

import numpy as np

from .capi import LxError, _p, load_library, u8p, u32p, u64p, vp

PUSH_QUEUED, PUSH_DUPLICATE, PUSH_CONNECTED = 0, 1, 2


class LevelBatcher:
    def __init__(self, capacity=0):
        """``capacity``: expected events per epoch (lx_batcher_reserve; a hint)."""
        self.L = load_library()
        h = vp()
        rc = self.L.lx_batcher_create(ctypes.byref(h))
        if rc != 0:
            raise LxError(rc, "lx_batcher_create failed")
        self.h = h
        if capacity:
            self._chk(self.L.lx_batcher_reserve(h, capacity))
        self._handle = {}      # event id -> uint64 handle
        self._event = {}       # uint64 handle -> event

    def close(self):
        if getattr(self, "h", None):
            self.L.lx_batcher_destroy(self.h)
            self.h = None

    __del__ = close

    def _chk(self, rc):
        if rc != 0:
            raise LxError(rc, self.L.lx_batcher_last_error(self.h).decode())

    def _h(self, eid):
        k = self._handle.get(eid)
        if k is None:
            k = len(self._handle) + 1
            self._handle[eid] = k
        return k

    def reset(self):
        """New epoch (with the index's lx_reset)."""
        self._chk(self.L.lx_batcher_reset(self.h))
        self._handle.clear()
        self._event.clear()

    def push(self, events, validators):
        """Push events (``id``, ``creator``, ``seq``, ``parents``; any order).
        Returns the LX_PUSH_* status per event."""
        n = len(events)
        if not n:
            return np.zeros(0, dtype=np.uint8)
        ids = np.array([self._h(e.id) for e in events], dtype=np.uint64)
        cr = np.array([validators.idxs[e.creator] for e in events], dtype=np.uint32)
        sq = np.array([e.seq for e in events], dtype=np.uint32)
        off = np.zeros(n + 1, dtype=np.uint64)
        flat = []
        for i, e in enumerate(events):
            flat.extend(self._h(p) for p in e.parents)
            off[i + 1] = len(flat)
        par = np.array(flat if flat else [0], dtype=np.uint64)
        st = np.zeros(n, dtype=np.uint8)
        self._chk(self.L.lx_batcher_push(self.h, n, _p(ids, u64p), _p(cr, u32p), _p(sq, u32p), _p(off, u64p),
                                         _p(par, u64p), _p(st, u8p)))
        for e, s in zip(events, st):
            if s == PUSH_QUEUED:
                self._event[self._handle[e.id]] = e
        return st

    def peek(self):
        """(events, parent entries, levels, still waiting) of the next pop."""
        ne, nl, nw = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        npar = ctypes.c_uint64()
        self._chk(self.L.lx_batcher_peek(self.h, ctypes.byref(ne), ctypes.byref(npar), ctypes.byref(nl),
                                         ctypes.byref(nw)))
        return ne.value, npar.value, nl.value, nw.value

    def pop(self):
        """Release the ready levels: (events, creator, seq, parent_off,
        parent_idx, level_off, first_dense) -- the arrays lx_add_batch takes."""
        ne, npar, nl, _ = self.peek()
        ids = np.zeros(max(ne, 1), dtype=np.uint64)
        cr = np.zeros(max(ne, 1), dtype=np.uint32)
        sq = np.zeros(max(ne, 1), dtype=np.uint32)
        off = np.zeros(ne + 1, dtype=np.uint64)
        par = np.zeros(max(npar, 1), dtype=np.uint32)
        lev = np.zeros(nl + 1, dtype=np.uint32)
        first = ctypes.c_uint64()
        self._chk(self.L.lx_batcher_pop(self.h, _p(ids, u64p), _p(cr, u32p), _p(sq, u32p), _p(off, u64p),
                                        _p(par, u32p), _p(lev, u32p), ctypes.byref(first)))
        events = [self._event.pop(int(k)) for k in ids[:ne]]
        return events, cr[:ne], sq[:ne], off, par[:npar], lev, first.value

    def unpop(self, events):
        """Forget the last pop after the index rejected it."""
        self._chk(self.L.lx_batcher_unpop(self.h))

    def drain_into(self, index):
        """Pop and index with one lx_add_batch (index: VecfcIndex of the same
        epoch, fed only through this batcher).  Returns the released events."""
        events, cr, sq, off, par, lev, first = self.pop()
        if not events:
            return events
        assert first == len(index.ids), "index and batcher out of step"
        try:
            index.ix.add_batch(cr, sq, off, par)
        except LxError:
            self.unpop(events)
            raise
        for e in events:
            index.pos[e.id] = len(index.ids)
            index.ids.append(e.id)
        self.last_levels = lev
        return events

    def drain_all(self, index, validators, on_reject=None):
        """Index everything releasable, one lx_add_batch per pop.  A batch is
        all-or-nothing, but the reference processes events one at a time and
        rejects only the bad one (abft/indexed_lachesis.go:69-82): when the
        index refuses a batch at event k (its first offending event), the batch
        is un-popped, event k is handed to ``on_reject(event, error)`` and
        every other event is pushed back -- the next pop releases them again,
        except k's descendants, which stay pending like events with a missing
        parent in dagordering.EventsBuffer.  Returns the events indexed."""
        done = []
        while True:
            if self.peek()[0] == 0:
                return done
            events, cr, sq, off, par, lev, first = self.pop()
            assert first == len(index.ids), "index and batcher out of step"
            try:
                index.ix.add_batch(cr, sq, off, par)
            except LxError as err:
                self.unpop(events)
                k = getattr(err, "index", 0xFFFFFFFF)
                if k >= len(events):
                    raise
                if on_reject:
                    on_reject(events[k], err)
                self.push(events[:k] + events[k + 1:], validators)
                continue
            for e in events:
                index.pos[e.id] = len(index.ids)
                index.ids.append(e.id)
            self.last_levels = lev
            done.extend(events)
