"""Faithful CPU restatement of vecengine + vecfc (TEST INFRASTRUCTURE ONLY).

Every method cites the reference function it restates.  Vectors are kept in the
reference's byte encodings (vecfc/vector.go:14-102):

* LowestAfterSeq  : bytes, 4 B per branch, LE uint32 seq
* HighestBeforeSeq: bytes, 8 B per branch, LE Seq || LE MinSeq
* fork marker     : {Seq: 0, MinSeq: MaxInt32}             (vector.go:91-97)

Storage mirrors ``flushable.WrapWithDrop`` over the ``v|b``, ``v|B``, ``v|S``,
``v|s`` tables: writes go to a dirty overlay, ``flush`` merges them,
``drop_not_flushed`` discards them (vecengine/index.go:56-96).  The LRU caches
of vecfc/index.go:43-47 only change speed, never results, so
they are omitted; the ForklessCause pair cache is likewise omitted (its
results are immutable once ``a`` is indexed).

BranchesInfo is persisted on ``flush`` as a Python tuple copy instead of the
go-ethereum RLP bytes (byte-exact RLP is "parity unpinned").
"""

import struct

from .pos import WeightCounter

MAX_INT32 = 0x7FFFFFFF
FORK_DETECTED = (0, MAX_INT32)


# ----------------------------------------------------------------------------
# vecfc/vector.go + vecfc/vector_ops.go

class LowestAfterSeq:
    __slots__ = ("b",)

    def __init__(self, size=0, raw=None):
        self.b = bytearray(raw) if raw is not None else bytearray(4 * size)

    def size(self):                                   # vector.go:48-51
        return len(self.b) // 4

    def get(self, i):                                 # vector.go:39-46
        if i >= self.size():
            return 0
        return struct.unpack_from("<I", self.b, 4 * i)[0]

    def set(self, i, seq):                            # vector.go:53-61
        while i >= self.size():
            self.b.extend(b"\0\0\0\0")
        struct.pack_into("<I", self.b, 4 * i, seq)

    def init_with_event(self, i, e):                  # vector_ops.go:9-11
        self.set(i, e.seq)

    def visit(self, i, e):                            # vector_ops.go:13-20
        if self.get(i) != 0:
            return False
        self.set(i, e.seq)
        return True

    def to_bytes(self):
        return bytes(self.b)


class HighestBeforeSeq:
    __slots__ = ("b",)

    def __init__(self, size=0, raw=None):
        self.b = bytearray(raw) if raw is not None else bytearray(8 * size)

    def size(self):                                   # vector.go:63-66
        return len(self.b) // 8

    def get(self, i):                                 # vector.go:68-80
        if i >= self.size():
            return (0, 0)
        return struct.unpack_from("<II", self.b, 8 * i)

    def set(self, i, bs):                             # vector.go:82-90
        while i >= self.size():
            self.b.extend(b"\0" * 8)
        struct.pack_into("<II", self.b, 8 * i, bs[0], bs[1])

    def init_with_event(self, i, e):                  # vector_ops.go:22-24
        self.set(i, (e.seq, e.seq))

    def is_empty(self, i):                            # vector_ops.go:26-29
        s = self.get(i)
        return s != FORK_DETECTED and s[0] == 0

    def is_fork_detected(self, i):                    # vector_ops.go:31-33
        return self.get(i) == FORK_DETECTED

    def seq(self, i):
        return self.get(i)[0]

    def min_seq(self, i):
        return self.get(i)[1]

    def set_fork_detected(self, i):                   # vector_ops.go:45-47
        self.set(i, FORK_DETECTED)

    def collect_from(self, other, num):               # vector_ops.go:49-79
        for branch in range(num):
            his = other.get(branch)
            if his[0] == 0 and his != FORK_DETECTED:
                continue
            my = self.get(branch)
            if my == FORK_DETECTED:
                continue
            if his == FORK_DETECTED:
                self.set_fork_detected(branch)
            else:
                my_seq, my_min = my
                if my_seq == 0 or my_min > his[1]:
                    my_min = his[1]
                    self.set(branch, (my_seq, my_min))
                if my_seq < his[0]:
                    my_seq = his[0]
                    self.set(branch, (my_seq, my_min))

    def gather_from(self, to, other, branches):       # vector_ops.go:81-96
        highest = (0, 0)
        for b in branches:
            bs = other.get(b)
            if bs == FORK_DETECTED:
                highest = bs
                break
            if bs[0] > highest[0]:
                highest = bs
        self.set(to, highest)

    def to_bytes(self):
        return bytes(self.b)


# ----------------------------------------------------------------------------
# flushable kv (kvdb/flushable/flushable.go:48-62,188-227, semantics only)

class FlushableTable:
    def __init__(self):
        self.flushed = {}
        self.dirty = {}

    def get(self, k):
        if k in self.dirty:
            return self.dirty[k]
        return self.flushed.get(k)

    def put(self, k, v):
        self.dirty[k] = v

    def not_flushed(self):
        return len(self.dirty)

    def flush(self):
        self.flushed.update(self.dirty)
        self.dirty = {}

    def drop(self):
        self.dirty = {}


class BranchesInfo:
    """vecengine/branches_info.go:9-14."""

    def __init__(self, last_seq, creator_idxs, by_creators):
        self.last_seq = last_seq
        self.creator_idxs = creator_idxs
        self.by_creators = by_creators

    @classmethod
    def initial(cls, n):                              # branches_info.go:27-45
        return cls([0] * n, list(range(n)), [[i] for i in range(n)])

    def copy(self):
        return BranchesInfo(list(self.last_seq), list(self.creator_idxs),
                            [list(x) for x in self.by_creators])


class Index:
    """vecfc.Index with its embedded vecengine.Engine."""

    def __init__(self):
        self.validators = None

    # vecengine/index.go:56-68 + vecfc/index.go:98-105
    def reset(self, validators, get_event):
        self.validators = validators
        self.get_event = get_event
        self.tbl_branch = FlushableTable()    # table "b"
        self.tbl_binfo = FlushableTable()     # table "B"
        self.tbl_hb = FlushableTable()        # table "S"
        self.tbl_la = FlushableTable()        # table "s"
        self.bi = None

    def _tables(self):
        return (self.tbl_branch, self.tbl_binfo, self.tbl_hb, self.tbl_la)

    # branches_info.go:16-25
    def init_branches_info(self):
        if self.bi is None:
            stored = self.tbl_binfo.get(b"c")
            self.bi = stored.copy() if stored is not None else BranchesInfo.initial(len(self.validators))

    def at_least_one_fork(self):                      # branches_info.go:47-49
        return len(self.bi.creator_idxs) > len(self.validators)

    def branches_info(self):
        return self.bi

    # vecengine/index.go:78-85
    def flush(self):
        if self.bi is not None:
            self.tbl_binfo.put(b"c", self.bi.copy())
        for t in self._tables():
            t.flush()

    # vecengine/index.go:88-96
    def drop_not_flushed(self):
        self.bi = None
        if any(t.not_flushed() for t in self._tables()):
            for t in self._tables():
                t.drop()

    # store_branches_info.go:75-88
    def get_event_branch_id(self, eid):
        b = self.tbl_branch.get(eid)
        if b is None:
            raise RuntimeError("failed to read event's branch ID (inconsistent DB)")
        return b

    # vecfc/store_vectors.go:26-65
    def get_lowest_after(self, eid):
        b = self.tbl_la.get(eid)
        return None if b is None else LowestAfterSeq(raw=b)

    def get_highest_before(self, eid):
        b = self.tbl_hb.get(eid)
        return None if b is None else HighestBeforeSeq(raw=b)

    def set_lowest_after(self, eid, v):
        self.tbl_la.put(eid, v.to_bytes())

    def set_highest_before(self, eid, v):
        self.tbl_hb.put(eid, v.to_bytes())

    # vecengine/index.go:71-75
    def add(self, e):
        self.init_branches_info()
        self._fill_event_vectors(e)

    # vecengine/index.go:98-103
    def _set_fork_detected(self, before, branch_id):
        creator = self.bi.creator_idxs[branch_id]
        for b in self.bi.by_creators[creator]:
            before.set_fork_detected(b)

    # vecengine/index.go:105-141
    def _fill_global_branch_id(self, e, me):
        bi = self.bi
        if len(bi.creator_idxs) != len(bi.last_seq) or len(bi.creator_idxs) < len(self.validators):
            raise RuntimeError("inconsistent BranchIDCreators len (inconsistent DB)")
        sp = e.self_parent()
        if sp is None:
            if bi.last_seq[me] == 0:
                bi.last_seq[me] = e.seq
                return me
        else:
            spb = self.get_event_branch_id(sp)
            if bi.last_seq[spb] + 1 == e.seq:
                bi.last_seq[spb] = e.seq
                return spb
        bi.last_seq.append(e.seq)
        bi.creator_idxs.append(me)
        nb = len(bi.last_seq) - 1
        bi.by_creators[me].append(nb)
        return nb

    # vecengine/index.go:144-233
    def _fill_event_vectors(self, e):
        me = self.validators.idxs[e.creator]
        n_before = len(self.bi.creator_idxs)
        before = HighestBeforeSeq(n_before)
        after = LowestAfterSeq(n_before)
        me_branch = self._fill_global_branch_id(e, me)

        parents_vecs = []
        for p in e.parents:
            self.get_event_branch_id(p)                 # result unused (index.go:155)
            pv = self.get_highest_before(p)
            if pv is None:
                raise ValueError("processed out of order, parent not found (inconsistent DB), parent=%r" % (p,))
            parents_vecs.append(pv)

        after.init_with_event(me_branch, e)
        before.init_with_event(me_branch, e)
        n_branches = len(self.bi.creator_idxs)
        for pv in parents_vecs:
            before.collect_from(pv, n_branches)

        if self.at_least_one_fork():
            V = len(self.validators)
            for n in range(V):
                if len(self.bi.by_creators[n]) <= 1:
                    continue
                for b in self.bi.by_creators[n]:
                    if before.is_fork_detected(b):
                        self._set_fork_detected(before, n)
                        break
            for n in range(V):
                if before.is_fork_detected(n):
                    continue
                done = False
                for a in self.bi.by_creators[n]:
                    for b in self.bi.by_creators[n]:
                        if a == b:
                            continue
                        if before.is_empty(a) or before.is_empty(b):
                            continue
                        if before.min_seq(a) <= before.seq(b) and before.min_seq(b) <= before.seq(a):
                            self._set_fork_detected(before, n)
                            done = True
                            break
                    if done:
                        break

        # DFS (vecengine/traversal.go:13-37) with onWalk (index.go:212-225)
        stack = list(e.parents)
        while stack:
            cur = stack.pop()
            la = self.get_lowest_after(cur)
            if not la.visit(me_branch, e):
                continue
            self.set_lowest_after(cur, la)
            ev = self.get_event(cur)
            if ev is None:
                raise RuntimeError("event not found %r" % (cur,))
            stack.extend(ev.parents)

        self.set_highest_before(e.id, before)
        self.set_lowest_after(e.id, after)
        self.tbl_branch.put(e.id, me_branch)

    # vecengine/index.go:235-250 (+ vecfc/index.go:143-145)
    def get_merged_highest_before(self, eid):
        self.init_branches_info()
        if self.at_least_one_fork():
            scattered = self.get_highest_before(eid)
            merged = HighestBeforeSeq(len(self.validators))
            for creator, branches in enumerate(self.bi.by_creators):
                merged.gather_from(creator, scattered, branches)
            return merged
        return self.get_highest_before(eid)

    # vecfc/forkless_cause.go:28-82
    def forkless_cause(self, a_id, b_id):
        self.init_branches_info()
        a = self.get_highest_before(a_id)
        if a is None:
            raise RuntimeError("Event A=%r not found" % (a_id,))
        if self.at_least_one_fork():
            bb = self.get_event_branch_id(b_id)
            if a.is_fork_detected(bb):
                return False
        b = self.get_lowest_after(b_id)
        if b is None:
            raise RuntimeError("Event B=%r not found" % (b_id,))
        yes = WeightCounter(self.validators)
        for branch, creator in enumerate(self.bi.creator_idxs):
            la = b.get(branch)
            hb = a.get(branch)
            if la <= hb[0] and la != 0 and hb != FORK_DETECTED:
                yes.count_by_idx(creator)
        return yes.has_quorum()

    # test helper mirroring Engine.DfsSubgraph (traversal.go:13-37)
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
