"""Test-DAG tools (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates the parts of ``inter/dag/tdag`` the index tests use:

* ``ascii_scheme_for_each``  -- ``ASCIIschemeForEach`` (ascii_scheme.go:25-211)
  with the filler rule of ascii_scheme.go:332-334.  Validator IDs are
  ``BE32(sha256(name)[0:4])`` of the first event drawn in each column
  (ascii_scheme.go:124, hash/event_hash.go:288-298, inter/idx/index.go:96-98).
* ``rand_fork_dag``          -- the structure of ``ForEachRandFork``
  (test_common.go:37-136) driven by a portable splitmix64 PRNG instead of Go's
  ``math/rand`` (whose seeded stream cannot be reproduced without Go, SURVEY
  section 4).  The same generator is implemented bit-identically in
  ``oracle/csrc/oracle.c`` and ``lachesis-base_amd/csrc/dag_gen.cpp``.
* ``by_parents``             -- ``ByParents`` topological order (events.go:24-50).

Event IDs: the index only uses event IDs as opaque keys (the DFS visiting
order does not change its result), so events are keyed
by their creation index instead of the RLP/sha256 ID of
serialization.go:27-38.
"""

import hashlib
import re


class Event:
    __slots__ = ("id", "creator", "seq", "lamport", "parents", "name", "frame", "epoch")

    def __init__(self, eid, creator, seq, lamport, parents, name=""):
        self.id = eid
        self.creator = creator
        self.seq = seq
        self.lamport = lamport
        self.parents = list(parents)
        self.name = name
        self.frame = 0        # consensus fields set by abft Build (inter/dag/event.go:20-24)
        self.epoch = 0

    def self_parent(self):
        # inter/dag/event.go:87-92: parents[0] iff seq > 1
        if self.seq <= 1 or not self.parents:
            return None
        return self.parents[0]

    def __repr__(self):
        return "Event(%s c=%d s=%d p=%s)" % (self.name or self.id, self.creator,
                                             self.seq, self.parents)


def validator_id_of_name(name):
    return int.from_bytes(hashlib.sha256(name.encode()).digest()[:4], "big")


_FILLER = re.compile("[ ─═]+")   # ' ', '─', '═'  (ascii_scheme.go:332-334)


def ascii_scheme_for_each(scheme, process=None):
    """Returns (nodes, events_by_node, names, ordered_events)."""
    nodes = []
    events = {}
    names = {}
    ordered = []
    cur_far = {}
    for line in scheme.strip().split("\n"):
        n_names, n_creators, n_links = [], [], []
        prev_ref = 0
        prev_far, cur_far = cur_far, {}
        col = 0
        for symbol in [s for s in _FILLER.split(line.strip()) if s]:
            symbol = symbol.strip()
            if symbol.startswith("//"):
                break
            if symbol in ("╠", "║╠", "╠╫"):      # ╠ ║╠ ╠╫
                refs = [0] * (col + 1)
                refs[col] = 1
                n_links.append(refs)
            elif symbol in ("║╚", "╚"):                    # ║╚ ╚
                refs = [0] * (col + 1)
                refs[col] = prev_far.get(col, 2)
                n_links.append(refs)
            elif symbol in ("╣", "╣║", "╫╣", "╬"):  # ╣ ╣║ ╫╣ ╬
                last = n_links[-1]
                last.extend([0] * (col + 1 - len(last)))
                last[col] = 1
            elif symbol in ("╝║", "╝", "╩╫", "╫╩"):  # ╝║ ╝ ╩╫ ╫╩
                last = n_links[-1]
                last.extend([0] * (col + 1 - len(last)))
                last[col] = prev_far.get(col, 2)
            elif symbol in ("╫", "║", "║║"):          # ╫ ║ ║║
                pass
            else:
                if symbol.startswith("║") or symbol.endswith("║"):
                    cur_far[col] = int(symbol.strip("║"))
                else:
                    if symbol in names:
                        raise ValueError("event '%s' already exists" % symbol)
                    n_creators.append(col)
                    n_names.append(symbol)
                    if len(n_links) < len(n_names):
                        n_links.append([0] * (col + 1))
            if symbol not in ("╚", "╝"):
                col += 1
            else:
                prev_ref = prev_far[col] - 1 if col in prev_far else 1

        for i, name in enumerate(n_names):
            if len(nodes) <= n_creators[i]:
                v = validator_id_of_name(name)
                nodes.append(v)
                events[v] = []
            creator = nodes[n_creators[i]]
            parents = []
            last = len(events[creator]) - prev_ref - 1
            if last >= 0:
                sp = events[creator][last]
                seq = sp.seq + 1
                parents.append(sp.id)
                max_lamport = sp.lamport
            else:
                seq = 1
                max_lamport = 0
            for c, ref in enumerate(n_links[i]):
                if ref < 1:
                    continue
                other = nodes[c]
                lst = len(events[other]) - ref
                if lst < 0:
                    break
                p = events[other][lst]
                if p.id in parents:
                    continue
                parents.append(p.id)
                max_lamport = max(max_lamport, p.lamport)
            e = Event(name, creator, seq, max_lamport + 1, parents, name)
            events[creator].append(e)
            names[name] = e
            ordered.append(e)
            if process is not None:
                process(e, name)
    return nodes, events, names, ordered


# ----------------------------------------------------------------------------
# portable PRNG + seeded fork-DAG generator

MASK64 = (1 << 64) - 1


class SplitMix64:
    """splitmix64; below(n) = (next() >> 11) % n (bias irrelevant for tests,
    identical in the C and C++ generators)."""

    def __init__(self, seed):
        self.s = seed & MASK64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def below(self, n):
        return (self.next() >> 11) % n


def rand_fork_dag(n_nodes, events_per_node, parent_count, cheaters=0,
                  forks_count=0, seed=1, node_ids=None, rng=None, build=None, eid_base=0):
    """Structure of tdag.ForEachRandFork (test_common.go:37-136).

    Node ``k`` (0-based generation column) is a cheater iff ``k < cheaters``.
    Other parents: ``parent_count-1`` distinct other nodes drawn by rejection
    sampling (stand-in for ``r.Perm(nodeCount)`` minus self).
    ``build(e)`` (optional) mirrors the ForEachEvent.Build callback
    (test_common.go:110-116): returning False drops the event (it is neither
    kept as a parent nor returned).  ``rng`` lets several epochs share one
    stream, as the reference's epoch tests share ``r``.
    Returns (node_ids, events_in_creation_order).
    """
    if rng is None:
        rng = SplitMix64(seed)
    if node_ids is None:
        node_ids = [k + 1 for k in range(n_nodes)]
    evs_by_node = [[] for _ in range(n_nodes)]
    forks_done = [0] * n_nodes
    out = []
    n_other = min(parent_count - 1, n_nodes - 1)
    for i in range(n_nodes * events_per_node):
        me = i % n_nodes
        others = []
        while len(others) < n_other:
            u = rng.below(n_nodes - 1)
            cand = u if u < me else u + 1
            if cand not in others:
                others.append(cand)
        ee = evs_by_node[me]
        parent = None
        if ee:
            parent = ee[-1]
            flipped = (rng.below(events_per_node) <= forks_count or
                       i < (n_nodes - 1) * events_per_node)
            if me < cheaters and len(ee) > 1 and forks_done[me] < forks_count and flipped:
                parent = ee[rng.below(len(ee) - 1)]
                if rng.below(len(ee)) == 0:
                    parent = None
                forks_done[me] += 1
        parents = []
        if parent is None:
            seq, lamport = 1, 1
        else:
            seq, lamport = parent.seq + 1, parent.lamport + 1
            parents.append(parent.id)
        for o in others:
            oe = evs_by_node[o]
            if oe:
                p = oe[-1]
                parents.append(p.id)
                if lamport <= p.lamport:
                    lamport = p.lamport + 1
        e = Event(eid_base + i, node_ids[me], seq, lamport, parents,
                  "%s%03d" % (chr(ord("a") + me) if me < 26 else "n%d_" % me, len(ee)))
        if build is not None and build(e) is False:
            continue
        ee.append(e)
        out.append(e)
    return node_ids, out


def by_parents(events):
    """tdag.ByParents (events.go:24-50): repeatedly take the first event whose
    in-set parents are all ready."""
    unsorted = list(events)
    exists = {e.id for e in events}
    ready = set()
    res = []
    while unsorted:
        for i, e in enumerate(unsorted):
            if all((p not in exists) or (p in ready) for p in e.parents):
                res.append(e)
                del unsorted[i]
                ready.add(e.id)
                break
    return res


def shuffle(events, rng):
    """Fisher-Yates with SplitMix64 (stand-in for r.Perm)."""
    arr = list(events)
    for i in range(len(arr) - 1, 0, -1):
        j = rng.below(i + 1)
        arr[i], arr[j] = arr[j], arr[i]
    return arr


def to_dense(events, validators):
    """Dense arrays for the C ABI: (creator_idx, seq, parent_off, parent_idx),
    parents as Add-order positions (self-parent first, as in the input)."""
    import numpy as np
    pos = {e.id: i for i, e in enumerate(events)}
    creator = np.array([validators.idxs[e.creator] for e in events], dtype=np.uint32)
    seq = np.array([e.seq for e in events], dtype=np.uint32)
    off = np.zeros(len(events) + 1, dtype=np.uint64)
    flat = []
    for i, e in enumerate(events):
        flat.extend(pos[p] for p in e.parents)
        off[i + 1] = len(flat)
    return creator, seq, off, np.array(flat, dtype=np.uint32)
