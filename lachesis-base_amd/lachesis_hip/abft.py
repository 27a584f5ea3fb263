"""abft.IndexedLachesis over the HIP library (include/lachesis_abft.h).

Mirrors the reference's consensus surface so the parity tests drive it like
abft/common_test.go drives FakeLachesis:

* ``IndexedLachesis(validators, epoch)``   -- NewIndexedLachesis + ApplyGenesis
  (abft/indexed_lachesis.go:42-51, abft/apply_genesis.go:17-44)
* ``bootstrap(begin_block)``               -- Bootstrap with
  lachesis.ConsensusCallbacks: ``begin_block(block) -> (apply_event, end_block)``
  (lachesis/consensus.go:21-44); ``end_block()`` returns the next epoch's
  validators to seal the epoch, or None
* ``build(e)`` / ``process(e)``            -- Build / Process
  (abft/indexed_lachesis.go:53-82); ``process_batch(events)`` processes many
  events in one call with the same results
* ``reset(epoch, validators)``             -- Orderer.Reset (abft/bootstrap.go:54-65)
* ``store``                                -- the bits of abft.Store the tests read
  (GetEpoch, GetValidators, GetLastDecidedFrame, GetFrameRoots,
  GetEventConfirmedOn)

``validators`` is any object with ``ids`` (idx order), ``weights`` (idx
order) and ``idxs`` (ID -> idx), like pos.Validators.  Events carry ``id``,
``creator``, ``seq``, ``parents`` (ids, self-parent first) and ``frame``.
All computation is on the GPU; there is no CPU path.
"""

import ctypes

import numpy as np

from .capi import Index, LxError, _p, u32p, u64p, vp

FRAME_BUILD = 0xFFFFFFFF
ERR_FRAME = -7
ERR_BYZANTINE = -8


class Block:
    """lachesis.Block {Atropos, Cheaters} (lachesis/block.go)."""

    def __init__(self, atropos, cheaters):
        self.atropos = atropos
        self.cheaters = cheaters

    def __eq__(self, o):
        return (self.atropos, self.cheaters) == (o.atropos, o.cheaters)

    def __repr__(self):
        return "Block(%r, cheaters=%r)" % (self.atropos, self.cheaters)


class WrongFrameError(RuntimeError):
    """ErrWrongFrame (abft/event_processing.go:11-13)."""


class _Validators:
    """Minimal pos.Validators built from weights by ID (sorted as
    inter/pos/sort.go:16-22) for validator sets returned by end_block."""

    def __init__(self, ids, weights):
        self.ids = list(ids)
        self.weights = list(weights)
        self.idxs = {v: i for i, v in enumerate(self.ids)}


BEGIN_BLOCK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32)
APPLY_EVENT = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32)
END_BLOCK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                             ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)))


class Callbacks(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("begin_block", BEGIN_BLOCK), ("apply_event", APPLY_EVENT),
                ("end_block", END_BLOCK)]


class AbftStats(ctypes.Structure):
    _fields_ = [("ms_index", ctypes.c_float), ("ms_frames", ctypes.c_float), ("ms_election", ctypes.c_float),
                ("ms_blocks", ctypes.c_float), ("frame_steps", ctypes.c_uint32), ("fc_launches", ctypes.c_uint32),
                ("vote_launches", ctypes.c_uint32), ("blocks", ctypes.c_uint32), ("fc_pairs", ctypes.c_uint64),
                ("fc_pair_cols", ctypes.c_uint64), ("ms_root_fc_gpu", ctypes.c_float),
                ("fc_lane_ops", ctypes.c_uint64), ("elections_ahead", ctypes.c_uint32)]


class _StoreView:
    def __init__(self, lch):
        self._l = lch

    def get_epoch(self):
        return self._l.L.lx_abft_epoch(self._l.h)

    def get_validators(self):
        return self._l.validators

    @property
    def last_decided_frame(self):
        return self._l.L.lx_abft_last_decided_frame(self._l.h)

    def get_frame_roots(self, f):
        """Root event ids of frame f (abft/store_roots.go:52-93)."""
        n = ctypes.c_uint32()
        self._l._chk(self._l.L.lx_abft_frame_roots(self._l.h, f, None, 0, ctypes.byref(n)))
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        self._l._chk(self._l.L.lx_abft_frame_roots(self._l.h, f, _p(out, u32p), n.value, ctypes.byref(n)))
        return [self._l.evs[i].id for i in out[:n.value]]

    def get_event_confirmed_on(self, eid):
        i = self._l.pos.get(eid)
        if i is None:
            return 0
        out = ctypes.c_uint32()
        self._l._chk(self._l.L.lx_abft_event_confirmed_on(self._l.h, i, ctypes.byref(out)))
        return out.value


class IndexedLachesis:
    def __init__(self, validators, epoch=1, device=0, event_capacity=0):
        self.ix = Index(device=device, event_capacity=event_capacity)
        self.L = self.ix.L
        h = vp()
        rc = self.L.lx_abft_create(self.ix.h, ctypes.byref(h))
        if rc != 0:
            raise LxError(rc, "lx_abft_create failed")
        self.h = h
        self.validators = validators
        self.genesis_epoch = epoch
        self.pos = {}
        self.evs = []
        self.store = _StoreView(self)
        self._begin_block = None
        self._cur = None
        self._sealed_with = None
        self._keep = None

    def close(self):
        if getattr(self, "h", None):
            self.L.lx_abft_destroy(self.h)
            self.h = None
        if getattr(self, "ix", None) is not None:
            self.ix.close()

    __del__ = close

    def _chk(self, rc):
        if rc != 0:
            raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
        return rc

    # callbacks -----------------------------------------------------------------
    def _on_begin(self, user, frame, atropos, cheaters, n):
        block = Block(self.evs[atropos].id, [self.validators.ids[cheaters[k]] for k in range(n)])
        res = self._begin_block(block) if self._begin_block is not None else None
        self._cur = res if res is not None else (None, None)

    def _on_apply(self, user, ev):
        apply_event = self._cur[0] if self._cur else None
        if apply_event is not None:
            apply_event(self.evs[ev])

    def _on_end(self, user, n_out, w_out):
        end_block = self._cur[1] if self._cur else None
        self._cur = None
        nv = end_block() if end_block is not None else None
        if nv is None:
            return 0
        self._sealed_with = nv
        self._seal_w = np.ascontiguousarray(nv.weights, dtype=np.uint32)
        n_out[0] = len(self._seal_w)
        w_out[0] = self._seal_w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        return 1

    def bootstrap(self, begin_block=None):
        """Bootstrap (abft/indexed_lachesis.go:84-99, abft/lachesis.go:88-100)."""
        self._begin_block = begin_block
        cb = Callbacks(None, BEGIN_BLOCK(self._on_begin) if begin_block is not None else BEGIN_BLOCK(),
                       APPLY_EVENT(self._on_apply), END_BLOCK(self._on_end))
        self._keep = cb
        w = np.ascontiguousarray(self.validators.weights, dtype=np.uint32)
        self._chk(self.L.lx_abft_bootstrap(self.h, self.genesis_epoch, len(w), _p(w, u32p), ctypes.byref(cb)))

    def reset(self, epoch, validators):
        """Orderer.Reset (abft/bootstrap.go:54-65)."""
        w = np.ascontiguousarray(validators.weights, dtype=np.uint32)
        self._chk(self.L.lx_abft_reset(self.h, epoch, len(w), _p(w, u32p)))
        self.validators = validators
        self.pos = {}
        self.evs = []

    # events --------------------------------------------------------------------
    def _dense(self, events):
        creator, seq, off, flat = [], [], [0], []
        local = {}
        base = len(self.evs)
        for k, e in enumerate(events):
            creator.append(self.validators.idxs[e.creator])
            seq.append(e.seq)
            for p in e.parents:
                q = self.pos.get(p)
                if q is None:
                    q = local.get(p)
                if q is None:
                    raise KeyError(p)
                flat.append(q)
            off.append(len(flat))
            local[e.id] = base + k
        return (np.array(creator, dtype=np.uint32), np.array(seq, dtype=np.uint32),
                np.array(off, dtype=np.uint64), np.array(flat if flat else [0], dtype=np.uint32))

    def build(self, e):
        """Build (indexed_lachesis.go:53-63): sets e.frame."""
        creator, seq, off, flat = self._dense([e])
        out = ctypes.c_uint32()
        n = int(off[1])
        self._chk(self.L.lx_abft_build(self.h, int(creator[0]), int(seq[0]), n, _p(flat, u32p), ctypes.byref(out)))
        e.frame = out.value

    def process(self, e):
        """Process (indexed_lachesis.go:65-82): None or the error."""
        consumed, err = self.process_batch([e])
        return err

    def process_batch(self, events, claimed=True):
        """Processes events in order; returns (consumed, error).  ``claimed``
        False trusts the computed frames (Build then Process).  consumed <
        len(events) without error means a block sealed the epoch."""
        events = list(events)
        if not events:
            return 0, None
        try:
            creator, seq, off, flat = self._dense(events)
        except KeyError as k:
            # Add fails for an unknown parent (vecengine/index.go:159-161):
            # process the events before the first such event
            bad = next(i for i, e in enumerate(events)
                       if any(p not in self.pos and p not in {x.id for x in events[:i]} for p in e.parents))
            c, err = self.process_batch(events[:bad], claimed) if bad else (0, None)
            if err is not None or c < bad:
                return c, err
            return c, LxError(-2, "processed out of order, parent not found (inconsistent DB), parent=%r" % (k.args[0],))
        frames = np.array([e.frame if claimed else FRAME_BUILD for e in events], dtype=np.uint32)
        out = np.zeros(len(events), dtype=np.uint32)
        consumed = ctypes.c_uint32()
        base = len(self.evs)
        for k, e in enumerate(events):
            self.pos[e.id] = base + k
            self.evs.append(e)
        epoch0 = self.store.get_epoch()
        self._sealed_with = None
        rc = self.L.lx_abft_process_batch(self.h, len(events), _p(creator, u32p), _p(seq, u32p), _p(off, u64p),
                                          _p(flat, u32p), _p(frames, u32p), _p(out, u32p), ctypes.byref(consumed))
        c = consumed.value
        if not claimed:
            for k in range(c):
                events[k].frame = int(out[k])
        if self.store.get_epoch() != epoch0:
            # sealed: a new, empty epoch (frame_decide.go:52-58)
            self.validators = self._sealed_with
            self.pos = {}
            self.evs = []
        else:
            for e in events[c:]:
                del self.pos[e.id]
            del self.evs[base + c:]
        if rc == ERR_FRAME:
            return c, WrongFrameError("claimed frame mismatched with calculated")
        if rc != 0:
            raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
        return c, None

    def frame_of(self, eid):
        out = ctypes.c_uint32()
        self._chk(self.L.lx_abft_event_frame(self.h, self.pos[eid], ctypes.byref(out)))
        return out.value

    def last_stats(self):
        st = AbftStats()
        self._chk(self.L.lx_abft_last_stats(self.h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in AbftStats._fields_}

    def set_option(self, name, value):
        """lx_abft_set_option (path selection; results never change)."""
        self._chk(self.L.lx_abft_set_option(self.h, name.encode(), int(value)))


class DenseLachesis:
    """Dense-index handle over lx_abft_* (what a cgo shim binds 1:1): events
    are Add-order indices of the current epoch, validators are idx-ordered
    weights.  Records blocks as (epoch, frame, atropos, cheaters, confirmed);
    ``apply_events=False`` skips the per-event ApplyEvent callback (the
    confirmation DFS still runs; GetEventConfirmedOn still answers).
    ``seal(epoch, frame)`` may return the next epoch's weights.
    ``block_log=True``: no callbacks at all -- the library logs each decided
    block itself (option block_log, with the confirmed events when
    apply_events) and the blocks are read after each batch; never seals."""

    def __init__(self, weights, epoch=1, device=0, event_capacity=0, apply_events=True, seal=None, block_log=False):
        self.ix = Index(device=device, event_capacity=event_capacity)
        self.L = self.ix.L
        h = vp()
        rc = self.L.lx_abft_create(self.ix.h, ctypes.byref(h))
        if rc != 0:
            raise LxError(rc, "lx_abft_create failed")
        self.h = h
        self.blocks = []
        self.seal = seal
        self._cur = None
        self._seal_w = None
        self.block_log = bool(block_log)
        if self.block_log and seal is not None:
            raise ValueError("block_log never seals: no seal callback")
        self._cb = None if self.block_log else Callbacks(
            None, BEGIN_BLOCK(self._begin), APPLY_EVENT(self._apply) if apply_events else APPLY_EVENT(),
            END_BLOCK(self._end))
        w = np.ascontiguousarray(weights, dtype=np.uint32)
        rc = self.L.lx_abft_bootstrap(self.h, epoch, len(w), _p(w, u32p),
                                      None if self._cb is None else ctypes.byref(self._cb))
        if rc != 0:
            raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
        if self.block_log:
            self.set_option("block_log", 2 if apply_events else 1)

    def close(self):
        if getattr(self, "h", None):
            self.L.lx_abft_destroy(self.h)
            self.h = None
        if getattr(self, "ix", None) is not None:
            self.ix.close()

    __del__ = close

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
        self._seal_w = np.ascontiguousarray(nw, dtype=np.uint32)
        n_out[0] = len(self._seal_w)
        w_out[0] = self._seal_w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        return 1

    def process_batch(self, creator, seq, poff, par, claimed=None):
        """Returns (rc, consumed, frames)."""
        creator = np.ascontiguousarray(creator, dtype=np.uint32)
        seq = np.ascontiguousarray(seq, dtype=np.uint32)
        poff = np.ascontiguousarray(poff, dtype=np.uint64)
        par = np.ascontiguousarray(par if len(par) else [0], dtype=np.uint32)
        n = len(creator)
        out = np.zeros(n, dtype=np.uint32)
        cl = None if claimed is None else np.ascontiguousarray(claimed, dtype=np.uint32)
        consumed = ctypes.c_uint32()
        rc = self.L.lx_abft_process_batch(self.h, n, _p(creator, u32p), _p(seq, u32p), _p(poff, u64p),
                                          _p(par, u32p), None if cl is None else _p(cl, u32p), _p(out, u32p),
                                          ctypes.byref(consumed))
        if rc not in (0, ERR_FRAME):
            raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
        if self.block_log:
            self._read_block_log()
        return rc, consumed.value, out

    def _read_block_log(self):
        nb = ctypes.c_uint32()
        ptr = [ctypes.POINTER(ctypes.c_uint32)() for _ in range(6)]
        rc = self.L.lx_abft_block_log(self.h, ctypes.byref(nb), *[ctypes.byref(q) for q in ptr])
        if rc != 0:
            raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
        n = nb.value
        if not n:
            return
        fr, at, co, ch, fo, cf = ptr
        ep = self.epoch()
        for k in range(n):
            self.blocks.append((ep, fr[k], at[k], tuple(ch[i] for i in range(co[k], co[k + 1])),
                                tuple(cf[i] for i in range(fo[k], fo[k + 1]))))

    def epoch(self):
        return self.L.lx_abft_epoch(self.h)

    def confirmed_on(self, n):
        """GetEventConfirmedOn of events [0, n) of the epoch (0 = not confirmed)."""
        out = np.zeros(n, dtype=np.uint32)
        f = ctypes.c_uint32()
        for i in range(n):
            rc = self.L.lx_abft_event_confirmed_on(self.h, i, ctypes.byref(f))
            if rc != 0:
                raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
            out[i] = f.value
        return out

    def last_decided_frame(self):
        return self.L.lx_abft_last_decided_frame(self.h)

    def frame_roots(self, f):
        n = ctypes.c_uint32()
        self.L.lx_abft_frame_roots(self.h, f, None, 0, ctypes.byref(n))
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        self.L.lx_abft_frame_roots(self.h, f, _p(out, u32p), n.value, ctypes.byref(n))
        return out[:n.value]

    def last_stats(self):
        st = AbftStats()
        self.L.lx_abft_last_stats(self.h, ctypes.byref(st))
        return {f: getattr(st, f) for f, _ in AbftStats._fields_}

    def set_option(self, name, value):
        """lx_abft_set_option (path selection; results never change)."""
        rc = self.L.lx_abft_set_option(self.h, name.encode(), int(value))
        if rc != 0:
            raise LxError(rc, self.L.lx_abft_last_error(self.h).decode())
