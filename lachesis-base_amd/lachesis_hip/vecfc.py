"""Hash-keyed facade with the reference's vecfc.Index surface.

Mirrors what the cgo shim of INTEGRATION.md does in Go: it keeps the
event-ID -> dense-index map and forwards to the C ABI.  Method names follow
vecfc/index.go, vecfc/forkless_cause.go and vecengine/index.go; error
behaviour follows the reference (``crit`` for unknown events, ``add`` raises
for out-of-order parents, vecengine/index.go:159-161).
"""

import struct

from .capi import Index

MAX_INT32 = 0x7FFFFFFF


class BranchSeq(tuple):
    """vecfc.BranchSeq {Seq, MinSeq} (vecfc/vector.go:21-25)."""

    def __new__(cls, seq, min_seq):
        return super().__new__(cls, (seq, min_seq))

    @property
    def seq(self):
        return self[0]

    @property
    def min_seq(self):
        return self[1]

    def is_fork_detected(self):                       # vector.go:99-102
        return self[0] == 0 and self[1] == MAX_INT32


class HighestBeforeSeq:
    """Byte-encoded HighestBefore vector (vecfc/vector.go:63-90)."""

    def __init__(self, raw):
        self.raw = bytes(raw)

    def size(self):
        return len(self.raw) // 8

    def get(self, i):
        if i >= self.size():
            return BranchSeq(0, 0)
        return BranchSeq(*struct.unpack_from("<II", self.raw, 8 * i))

    def is_fork_detected(self, i):                    # vector_ops.go:31-33
        return self.get(i).is_fork_detected()

    def to_bytes(self):
        return self.raw


class LowestAfterSeq:
    """Byte-encoded LowestAfter vector (vecfc/vector.go:39-61)."""

    def __init__(self, raw):
        self.raw = bytes(raw)

    def size(self):
        return len(self.raw) // 4

    def get(self, i):
        if i >= self.size():
            return 0
        return struct.unpack_from("<I", self.raw, 4 * i)[0]

    def to_bytes(self):
        return self.raw


class Ratio:
    """cachescale.Ratio (utils/cachescale/ratio.go:8-44): v * Target / Base, rounded up."""

    def __init__(self, base=1, target=1):
        self.base, self.target = base, target

    def U64(self, v):
        m = v * self.target
        return m // self.base + (1 if m % self.base else 0)

    I = U = U32 = U64


IDENTITY = Ratio(1, 1)


class IndexCacheConfig:
    """vecfc.IndexCacheConfig (vecfc/index.go:15-20)."""

    def __init__(self, forkless_cause_pairs, highest_before_seq_size, lowest_after_seq_size):
        self.forkless_cause_pairs = forkless_cause_pairs
        self.highest_before_seq_size = highest_before_seq_size
        self.lowest_after_seq_size = lowest_after_seq_size


class IndexConfig:
    """vecfc.IndexConfig (vecfc/index.go:22-25).  The reference sizes its LRU
    caches from it; the device planes replace those caches (vectors live in
    HBM, ForklessCause(a, b) is never recomputed wrongly because it is
    immutable once a is indexed), so it changes nothing here -- it is kept so
    callers written against vecfc construct the index unchanged."""

    def __init__(self, caches):
        self.caches = caches


def default_config(scale=IDENTITY):
    """vecfc.DefaultConfig (vecfc/index.go:52-61)."""
    return IndexConfig(IndexCacheConfig(scale.I(20000), scale.U(160 * 1024), scale.U(160 * 1024)))


def lite_config():
    """vecfc.LiteConfig (vecfc/index.go:63-66): DefaultConfig scaled 1/100."""
    return default_config(Ratio(100, 1))


def new_index(crit, config=None, device=0, event_capacity=0):
    """vecfc.NewIndex (vecfc/index.go:68-78)."""
    return VecfcIndex(device=device, event_capacity=event_capacity, crit=crit, config=config)


def new_index_with_engine(crit, config, engine):
    """vecfc.NewIndexWithEngine (vecfc/index.go:80-89): an index over an
    existing engine -- here a :class:`lachesis_hip.Index` handle, which the
    new facade shares (its epoch state is the engine's)."""
    return VecfcIndex(crit=crit, config=config, engine=engine)


class _EngineState:
    """The epoch state a vecengine.Engine owns: the device handle, the event-ID
    <-> dense-index map, the flush point, validators and the getEvent
    callback.  Every vecfc.Index over one engine (NewIndexWithEngine) shares
    this object, so a Reset / Flush / DropNotFlushed / restore through one
    facade is what the others see (vecfc/index.go:80-89 shares its Engine)."""

    def __init__(self, ix):
        self.ix = ix
        self.pos = {}
        self.ids = []
        self.n_flushed = 0
        self.validators = None
        self.get_event_fn = None


def _shared(name):
    return property(lambda self: getattr(self._st, name), lambda self, v: setattr(self._st, name, v))


class VecfcIndex:
    """vecfc.Index over the HIP library.  ``validators`` needs ``ids``,
    ``weights`` (idx order) and ``idxs`` (ValidatorID -> idx)."""

    ix = _shared("ix")
    pos = _shared("pos")
    ids = _shared("ids")
    n_flushed = _shared("n_flushed")
    validators = _shared("validators")
    get_event_fn = _shared("get_event_fn")

    def __init__(self, device=0, event_capacity=0, crit=None, config=None, engine=None):
        self.crit = crit or self._panic
        self.cfg = config or default_config()
        if isinstance(engine, VecfcIndex):
            # a second vecfc.Index over the same engine: one shared epoch state
            self._st = engine._st
        else:
            self._st = _EngineState(engine if engine is not None else Index(device=device, event_capacity=event_capacity))

    @staticmethod
    def _panic(err):
        raise err

    # vecfc/index.go:98-105
    def reset(self, validators, get_event=None):
        self.validators = validators
        self.get_event_fn = get_event
        self.ix.reset(validators.weights)
        self.pos = {}
        self.ids = []
        self.n_flushed = 0

    # vecengine/index.go:71-75
    def add(self, e):
        parents = []
        for p in e.parents:
            if p not in self.pos:
                raise ValueError("processed out of order, parent not found (inconsistent DB), parent=%r" % (p,))
            parents.append(self.pos[p])
        self.ix.add(self.validators.idxs[e.creator], e.seq, parents)
        self.pos[e.id] = len(self.ids)
        self.ids.append(e.id)

    def add_events(self, events):
        """Batched Add of many events (same result as add() one by one)."""
        import numpy as np
        base = len(self.ids)
        local = {e.id: base + k for k, e in enumerate(events)}
        creator, seq, off, flat = [], [], [0], []
        for e in events:
            creator.append(self.validators.idxs[e.creator])
            seq.append(e.seq)
            for p in e.parents:
                q = self.pos.get(p, local.get(p))
                if q is None:
                    raise ValueError("processed out of order, parent not found, parent=%r" % (p,))
                flat.append(q)
            off.append(len(flat))
        self.ix.add_batch(creator, seq, np.array(off, dtype=np.uint64), flat)
        for e in events:
            self.pos[e.id] = len(self.ids)
            self.ids.append(e.id)

    # vecengine/index.go:78-96
    def flush(self, db=None):
        """Flush.  With ``db`` (a dict of tables standing in for the index's
        kvdb.Store) the write-back Puts go into the reference's tables keyed
        by event id -- db["S"] HighestBefore bytes, db["s"] LowestAfter
        bytes, db["b"] 4-B big-endian branch IDs, db["B"][b"c"]
        RLP(BranchesInfo) (vecfc/index.go:38-41, vecengine/index.go:39-42) --
        and nothing else: ``restore`` works from exactly these tables."""
        if db is not None:
            wb = self.ix.writeback()
            for t in ("S", "s", "b", "B"):
                db.setdefault(t, {})
            for k, v in wb["S"].items():
                eid = self.ids[k]
                db["S"][eid] = v
                db["b"][eid] = wb["b"][k]
            for k, v in wb["s"].items():
                db["s"][self.ids[k]] = v
            db["B"][b"c"] = wb["B"]
        self.ix.flush()
        self.n_flushed = len(self.ids)

    def restore(self, validators, db, get_event, chunk=4096):
        """Restart over persisted tables (abft/restart_test.go:156-188 builds a
        fresh index over a copy of the DB): the events of table "b" are loaded
        in a parents-first order with their table S / s / b bytes and table B's
        RLP(BranchesInfo) (lx_load_rows / lx_load_finish) -- no replay of Add.
        Tables that do not form one consistent epoch call crit ("inconsistent
        DB", as vecengine/store_branches_info.go:83)."""
        from .capi import LxError
        self.reset(validators, get_event)
        ids = list(db.get("b", {}))
        if not ids and not db.get("B"):
            return                              # nothing flushed yet: an empty epoch
        events = {eid: get_event(eid) for eid in ids}
        order, state = [], {}
        for root in sorted(ids, key=lambda x: (getattr(events[x], "lamport", 0), x)):
            stack = [(root, False)]
            while stack:
                eid, done = stack.pop()
                if done:
                    if state.get(eid) != 2:
                        state[eid] = 2
                        order.append(eid)
                    continue
                if state.get(eid):
                    continue
                state[eid] = 1
                stack.append((eid, True))
                for p in reversed(events[eid].parents):
                    if p not in events:
                        self.crit(RuntimeError("inconsistent DB: parent %r of %r not persisted" % (p, eid)))
                        return
                    if not state.get(p):
                        stack.append((p, False))
        pos = {eid: k for k, eid in enumerate(order)}
        try:
            for lo in range(0, len(order), chunk):
                part = order[lo:lo + chunk]
                creator, seq, off, flat = [], [], [0], []
                for eid in part:
                    e = events[eid]
                    creator.append(validators.idxs[e.creator])
                    seq.append(e.seq)
                    flat.extend(pos[p] for p in e.parents)
                    off.append(len(flat))
                self.ix.load_rows(creator, seq, off, flat, b"".join(db["b"][eid] for eid in part),
                                  [db["S"][eid] for eid in part], [db["s"][eid] for eid in part])
            self.ix.load_finish(db.get("B", {}).get(b"c", b""))
        except (LxError, KeyError) as err:
            self.crit(RuntimeError("inconsistent DB: %s" % (err,)))
            return
        self.ids = order
        self.pos = pos
        self.n_flushed = len(order)

    def drop_not_flushed(self):
        self.ix.drop_not_flushed()
        for eid in self.ids[self.n_flushed:]:
            del self.pos[eid]
        del self.ids[self.n_flushed:]

    def _idx(self, eid):
        return self.pos.get(eid)

    # vecfc/forkless_cause.go:28-38
    def forkless_cause(self, a_id, b_id):
        a, b = self._idx(a_id), self._idx(b_id)
        if a is None or b is None:
            self.crit(RuntimeError("Event A=%r or B=%r not found" % (a_id, b_id)))
            return False
        return self.ix.forkless_cause(a, b)

    # vecfc/store_vectors.go:26-51 (nil if unknown)
    def get_highest_before(self, eid):
        i = self._idx(eid)
        return None if i is None else HighestBeforeSeq(self.ix.highest_before(i))

    def get_lowest_after(self, eid):
        i = self._idx(eid)
        return None if i is None else LowestAfterSeq(self.ix.lowest_after(i))

    # vecfc/index.go:143-145
    def get_merged_highest_before(self, eid):
        i = self._idx(eid)
        return None if i is None else HighestBeforeSeq(self.ix.merged_highest_before(i))

    # vecengine/store_branches_info.go:83-88
    def get_event_branch_id(self, eid):
        i = self._idx(eid)
        if i is None:
            self.crit(RuntimeError("failed to read event's branch ID (inconsistent DB)"))
            return 0
        return self.ix.branch(i)

    def at_least_one_fork(self):
        return self.ix.at_least_one_fork()

    # vecengine/branches_info.go:15-25 (InitBranchesInfo): the library keeps
    # BranchesInfo live on the device and the host (restored by restore())
    def init_branches_info(self):
        pass

    # vecfc/index.go:107-130: the callbacks the reference's Engine calls.  The
    # GPU engine computes and stores the vectors itself, so the setters are
    # not part of its contract (crit); getters and constructors behave as the
    # reference's.
    def get_engine_callbacks(self):
        def unsupported(*_):
            self.crit(RuntimeError("the GPU engine stores vectors itself (Set* callbacks are not used)"))
        return {
            "GetHighestBefore": self.get_highest_before,
            "GetLowestAfter": self.get_lowest_after,
            "SetHighestBefore": unsupported,
            "SetLowestAfter": unsupported,
            "NewHighestBefore": lambda size: HighestBeforeSeq(bytes(8 * size)),
            "NewLowestAfter": lambda size: LowestAfterSeq(bytes(4 * size)),
            "OnDbReset": lambda db: None,
            "OnDropNotFlushed": lambda: None,
        }

    def get_event(self, eid):
        return self.get_event_fn(eid) if self.get_event_fn else None

    # vecengine/traversal.go:13-37: iterative DFS over parents, `walk` decides
    # whether to descend (host traversal through the get_event callback)
    def dfs_subgraph(self, head, walk):
        stack = list(head.parents)
        while stack:
            cur = stack.pop()
            if not walk(cur):
                continue
            ev = self.get_event(cur)
            if ev is None:
                raise RuntimeError("event not found %r" % (cur,))
            stack.extend(ev.parents)

    def branches_info(self):
        last_seq, creators = self.ix.branches_info()
        by = [[] for _ in range(len(self.validators.weights))]
        for b, c in enumerate(creators):
            by[int(c)].append(b)
        return list(map(int, last_seq)), list(map(int, creators)), by
